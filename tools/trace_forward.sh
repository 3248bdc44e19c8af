#!/bin/bash
# Kernel trace of the timed forward loop only (no breakdown), single stream, for in-forward
# per-stage durations:  bash tools/trace_forward.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
O=gpurun_out/trace_$1; mkdir -p $O
CFM_MICROBATCH=${MB:-1} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
  python3 bench.py --steps 10 --warmup 3 --cpu-budget 0 --no-breakdown > $O/bench.json 2> $O/bench.err; rc=$?; echo trace_rc=$rc
[ $rc -eq 0 ] || exit $rc
python3 tools/stage_trace.py $O/run_kernel_trace.csv --burst 1 --forwards 5 > $O/stages.txt 2>&1; echo stages_rc=$?
