# round 4: tile A/B for the RNN-T joint output GEMM and the 256-byte K-step residual tile
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 200 python3 tools/gemm_probe.py 14,18 ffn_down,out > $O/probe_t18.txt 2>&1; echo probe_rc=$?
for t in 3:18@4096 none 3:18@4096 none; do
  CFM_TILES=$t timeout -k 10 200 python3 bench.py --no-train --cpu-budget 0 --no-parity > $O/fwd_${t/:/_}.$RANDOM.json 2>> $O/fwd.err || break
done
for t in none 4:13@100000 4:5@100000 4:0@100000 4:11@100000 4:1@100000; do
  CFM_TILES=$t timeout -k 10 200 python3 bench.py --mode joint --steps 6 --warmup 2 > $O/joint_${t/:/_}.json 2>> $O/joint.err || break
done
echo done_e
