#!/bin/bash
# Round profile on one GPU:  bash tools/profile_round.sh r01b
#   0. bench.py without the profiler (its breakdown = chained dispatch-packet stop events)
#   1. rocprofv3 --kernel-trace --stats over bench.py (per-kernel durations; stages.txt compares
#      rocprof's per-dispatch averages of the breakdown forwards with step 0's numbers)
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE; kernel-trace only) over tools/traffic_driver.py
# Outputs under gpurun_out/prof_<tag>/ ; copy the summaries into profiles/ afterwards.
R=${1:?tag}
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_$R
mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-budget 0 > $O/bench_noprof.json 2> $O/bench_noprof.err; rc=$?; echo noprof_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
  python3 bench.py --steps 10 --warmup 3 --cpu-budget 0 > $O/bench.json 2> $O/bench.err; rc=$?; echo trace_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- \
  python3 tools/traffic_driver.py 2 > $O/fetch.log 2>&1; rc=$?; echo fetch_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- \
  python3 tools/traffic_driver.py 2 > $O/write.log 2>&1; rc=$?; echo write_rc=$rc
[ $rc -eq 0 ] || exit $rc
python3 tools/traffic_summary.py $(find $O/fetch -name '*counter_collection.csv' | head -1) \
  $(find $O/write -name '*counter_collection.csv' | head -1) $O/traffic.json > $O/traffic.txt 2>&1; echo summary_rc=$?
python3 tools/prof_summary.py $O/run_kernel_stats.csv 40 > $O/summary.txt 2>&1
python3 tools/prof_summary.py --trace $O/run_kernel_trace.csv 40 >> $O/summary.txt 2>&1
python3 tools/stage_trace.py $O/run_kernel_trace.csv $O/bench_noprof.json --burst 1 > $O/stages.txt 2>&1; echo stages_rc=$?
