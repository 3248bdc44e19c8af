# round 4: forward A/B - read-ahead K-group loop, norm_out fold; stage tables
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04m
mkdir -p $O
for cfg in "1 0" "0 0" "1 1" "1 0" "0 0" "1 1"; do
  set -- $cfg
  CFM_GEMM_AHEAD=$1 CFM_LN_FOLD2=$2 timeout -k 10 300 python3 tools/fwd_ab.py "ahead=$1,fold2=$2" 20 >> $O/ab.txt 2>> $O/err.txt || exit 1
done
cat $O/ab.txt
CFM_GEMM_AHEAD=1 timeout -k 10 300 python3 tools/fwd_stages.py "ahead1" > $O/stages.txt 2>> $O/err.txt || exit 1
CFM_GEMM_AHEAD=0 timeout -k 10 300 python3 tools/fwd_stages.py "ahead0" >> $O/stages.txt 2>> $O/err.txt || exit 1
CFM_GEMM_AHEAD=1 CFM_LN_FOLD2=1 timeout -k 10 300 python3 tools/fwd_stages.py "fold2" >> $O/stages.txt 2>> $O/err.txt || exit 1
cat $O/stages.txt
timeout -k 10 300 python3 bench.py --mode joint --steps 5 --warmup 2 > $O/joint.json 2>> $O/err.txt || exit 1
cat $O/joint.json
