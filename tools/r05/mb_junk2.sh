set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05mbj2
mkdir -p $O
run() { echo "== $1"; env $2 timeout -k 10 200 python3 tools/mb_check.py "$1" 2>>$O/err.txt | cut -c1-130; }
for i in 1 2; do
run swish5 "CFM_LN_FOLD2=1 MB_JUNK2=1 CFM_TILES=2:5"
run resid16 "CFM_LN_FOLD2=1 MB_JUNK2=1 CFM_TILES=3:16"
run swish5-noxln "CFM_LN_FOLD2=1 MB_JUNK2=1 CFM_TILES=2:5 CFM_FOLD2_DBG=2"
run swish1 "CFM_LN_FOLD2=1 MB_JUNK2=1 CFM_TILES=2:1"
done
