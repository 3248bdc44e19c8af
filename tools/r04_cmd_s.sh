# round 4: two-blocks-per-CU tiles for ffn_up (tile 0, 128x128 one group) and ffn_down (tile 16) - forward A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04s
mkdir -p $O
for t in none up0 down16 none up0 down16; do
  case $t in none) TL="";; up0) TL="2:0@4096";; down16) TL="3:16@0k0";; esac
  CFM_TILES=$TL timeout -k 10 300 python3 tools/fwd_ab.py "tiles=$t" 20 >> $O/ab.txt 2>> $O/err.txt || exit 1
done
cat $O/ab.txt
