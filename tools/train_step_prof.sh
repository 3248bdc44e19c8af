#!/bin/bash
# Kernel trace of one timed training step (after 2 warm-ups) summarised per kernel: bash tools/train_step_prof.sh tag
R=${1:?tag}
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/train_step_$R
mkdir -p $O
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- \
  python3 bench.py --mode ${MODE:-train} --steps 2 --warmup 2 > $O/bench.json 2> $O/bench.err; rc=$?; echo trace_rc=$rc
[ $rc -eq 0 ] || exit $rc
T=$(find $O -name '*kernel_trace.csv' | head -1)
python3 tools/train_step_trace.py $T 70 > $O/step.txt; rc=$?
rm -f $T
exit $rc
