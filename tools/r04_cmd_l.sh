# round 4: bisect the micro-batch mismatch (norm_out fold): serialised parts / unrelated concurrent work
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04l
mkdir -p $O
CFM_MB_SERIAL=1 CFM_LN_FOLD2=1 timeout -k 10 300 python3 tools/mb_check.py "fold2=1,serial-parts" >> $O/mb8.txt 2>> $O/err.txt || exit 1
MB_JUNK=1 CFM_LN_FOLD2=1 timeout -k 10 300 python3 tools/mb_check.py "fold2=1,junk" >> $O/mb8.txt 2>> $O/err.txt || exit 1
cat $O/mb8.txt
