# round 4: residual GEMMs with K = 512 (out_proj, pw2) on co-resident 64x128 tiles - forward A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04r
mkdir -p $O
for t in none 16 5 none 16 5; do
  if [ $t = none ]; then TL=""; else TL="3:14@0k1024,3:$t@0k0"; fi
  CFM_TILES=$TL timeout -k 10 300 python3 tools/fwd_ab.py "resid_k512_tile=$t" 20 >> $O/ab.txt 2>> $O/err.txt || exit 1
done
cat $O/ab.txt
CFM_TILES="3:14@0k1024,3:16@0k0" timeout -k 10 300 python3 tools/fwd_stages.py "k512_t16" > $O/stages.txt 2>> $O/err.txt || exit 1
timeout -k 10 300 python3 tools/fwd_stages.py "default" >> $O/stages.txt 2>> $O/err.txt || exit 1
grep -E "out_proj|pw2|sum" $O/stages.txt
# joint logits GEMM tile re-measured with the one-instruction head/tail stores
for t in 11 5 0 1 11; do
  CFM_TILES="4:$t@100000" timeout -k 10 300 python3 bench.py --mode joint --steps 5 --warmup 2 > $O/joint_t$t.$RANDOM.json 2>> $O/err.txt || exit 1
done
for f in $O/joint_t*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['ms_per_step'],d.get('breakdown',{}).get('joint'))"; done
