set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05mbc
mkdir -p $O
run() { echo "== $1"; env $2 timeout -k 10 200 python3 tools/mb_check.py "$1" 2>>$O/err.txt | cut -c1-130; }
run L2 "CFM_LN_FOLD2=1 CFM_DBG_LAYERS=2"
run L2-no-ln2in "CFM_LN_FOLD2=1 CFM_DBG_LAYERS=2 CFM_FOLD2_DBG=1"
run L2-no-xln "CFM_LN_FOLD2=1 CFM_DBG_LAYERS=2 CFM_FOLD2_DBG=2"
run L2-neither "CFM_LN_FOLD2=1 CFM_DBG_LAYERS=2 CFM_FOLD2_DBG=3"
run L2-bigtiles "CFM_LN_FOLD2=1 CFM_DBG_LAYERS=2 CFM_TILES=2:11,3:14"
