set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05lab}
mkdir -p $O
for s in ffn_up ffn_up_store ffn_down; do
  timeout -k 10 120 tools/lab/ffn_lab $s 20 7 > $O/$s.txt 2>&1 || { cat $O/$s.txt; exit 1; }
  cat $O/$s.txt
done
