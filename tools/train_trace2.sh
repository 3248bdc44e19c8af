#!/bin/bash
# Kernel trace of 2 training steps (1 warm-up) grouped per kernel and grid: bash tools/train_trace2.sh tag
R=${1:?tag}
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
O=gpurun_out/trace_train_$R
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- \
  python3 bench.py --mode train --steps 1 --warmup 1 > $O/bench.json 2> $O/bench.err; rc=$?; echo trace_rc=$rc
[ $rc -eq 0 ] || exit $rc
T=$(find $O -name '*kernel_trace.csv' | head -1)
python3 tools/tn_trace.py $T tn_glds > $O/tn.txt
python3 tools/tn_trace.py $T gemm_kernel gemm8 bgemm attn_bwd rel_attn > $O/gemm.txt
python3 tools/tn_trace.py $T "" > $O/all.txt
rm -f $T
