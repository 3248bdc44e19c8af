#!/bin/bash
# In-forward profile of the north-star forward:  bash tools/forward_profile.sh TAG
#   1. bench.py (default line, no profiler)
#   2. rocprofv3 --kernel-trace --stats over bench.py --no-breakdown: in-forward per-kernel durations
#   3. rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE (kernel-trace only) over traffic_driver.py
#   4. FETCH_SIZE and WRITE_SIZE passes (one counter group per run)
# Outputs under gpurun_out/fprof_TAG/; tools/forward_profile.py writes stages.json / stages.txt.
R=${1:?tag}
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fprof_$R
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo bench_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --steps 10 --warmup 3 --cpu-budget 0 --no-breakdown --no-train --no-parity > $O/trace_bench.json 2> $O/trace_bench.err; rc=$?; echo trace_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/mfma -o run -- \
  python3 tools/traffic_driver.py 2 > $O/mfma.log 2>&1; rc=$?; echo mfma_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- \
  python3 tools/traffic_driver.py 2 > $O/fetch.log 2>&1; rc=$?; echo fetch_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- \
  python3 tools/traffic_driver.py 2 > $O/write.log 2>&1; rc=$?; echo write_rc=$rc
[ $rc -eq 0 ] || exit $rc
python3 tools/forward_profile.py $(find $O/trace -name '*kernel_trace.csv' | head -1) \
  $(find $O/mfma -name '*counter_collection.csv' | head -1) $O/stages.json > $O/stages.txt 2>&1; echo stages_rc=$?
python3 tools/traffic_summary.py $(find $O/fetch -name '*counter_collection.csv' | head -1) \
  $(find $O/write -name '*counter_collection.csv' | head -1) $O/traffic.json > $O/traffic.txt 2>&1; echo traffic_rc=$?
cp $(find $O/trace -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv 2>/dev/null
python3 tools/prof_summary.py $O/kernel_stats.csv 30 > $O/summary.txt 2>&1
ls $O
