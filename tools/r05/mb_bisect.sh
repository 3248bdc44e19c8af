# fold2 micro-batch nondeterminism: first layer count at which it shows; tile 10 probe for ffn_up
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05mbb
mkdir -p $O
for n in 1 2 3; do
  echo "== layers $n"
  CFM_LN_FOLD2=1 CFM_DBG_LAYERS=$n MB_ONLY3=1 timeout -k 10 200 python3 tools/mb_check.py "L$n" 2>>$O/err.txt | cut -c1-150 || exit 1
done
timeout -k 10 200 python3 tools/gemm_probe.py 10,11 ffn_up 2>>$O/err.txt || exit 1
for i in 1 2; do
  CFM_TILES=2:10 timeout -k 10 300 python3 tools/fwd_ab.py t10 10 2>>$O/err.txt || exit 1
  timeout -k 10 300 python3 tools/fwd_ab.py t11 10 2>>$O/err.txt || exit 1
done
