#!/bin/bash
# Training-step check on one GPU: parity tests (train, DP, CTC), bench --mode train, rocprofv3 stats.
#   bash tools/train_prof.sh <tag>   -> gpurun_out/prof_train_<tag>/
R=${1:?tag}
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/prof_train_$R
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_dp.py tests/test_gpu_ctc.py -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo tests_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode train --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err; rc=$?; echo bench_rc=$rc
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
  python3 bench.py --mode train --steps 3 --warmup 1 > $O/bench_prof.json 2> $O/bench_prof.err; rc=$?; echo prof_rc=$rc
[ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py $O/run_kernel_stats.csv 40 > $O/summary.txt 2>&1
rm -f $O/run_kernel_trace.csv
