# fold2 micro-batch nondeterminism: which kernel path does it depend on?
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05mb
mkdir -p $O
run() { echo "== $1"; env $2 timeout -k 10 200 python3 tools/mb_check.py "$1" 2>>$O/err.txt | cut -c1-200; }
run base "CFM_LN_FOLD2=1"
run noqa "CFM_LN_FOLD2=1 CFM_QKV_ATTN=0"
run noglu "CFM_LN_FOLD2=1 CFM_GLU_DW=0"
run noc12 "CFM_LN_FOLD2=1 CFM_CONV12=0"
run wt0 "CFM_LN_FOLD2=1 CFM_GEMM_WT=0"
run tiles "CFM_LN_FOLD2=1 CFM_TILES=2:5,3:5"
run f0 "CFM_LN_FOLD2=0"
