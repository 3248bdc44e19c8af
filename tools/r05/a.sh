# round 5 baseline on this round's box: forward bench + GEMM probes for the FFN pair
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-budget 0 > $O/bench.json 2> $O/err.txt || exit 1
python3 tools/show_bench.py $O/bench.json
timeout -k 10 200 python3 tools/gemm_probe.py 11,14 ffn_up,ffn_down,out > $O/probe.txt 2>> $O/err.txt || exit 1
cat $O/probe.txt
timeout -k 10 200 python3 tools/epi_probe.py > $O/epi.txt 2>> $O/err.txt || exit 1
cat $O/epi.txt
