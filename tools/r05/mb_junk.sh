set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05mbj
mkdir -p $O
run() { echo "== $1"; env $2 timeout -k 10 200 python3 tools/mb_check.py "$1" 2>>$O/err.txt | cut -c1-130; }
for i in 1 2; do
run f2-junk2-smalltiles "CFM_LN_FOLD2=1 MB_JUNK2=1 CFM_TILES=2:5,3:16"
run f0-junk2-smalltiles "CFM_LN_FOLD2=0 MB_JUNK2=1 CFM_TILES=2:5,3:16"
run f2-junk2 "CFM_LN_FOLD2=1 MB_JUNK2=1"
done
