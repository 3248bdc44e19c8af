#!/bin/bash
# One GPU session: GPU tests, then the bench (default tile policy), then per-tile breakdowns.
# Every GPU step has its own time limit; a crash/timeout ends the script.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -le 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest_rc=$rc
ok $rc || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget ${CPU_BUDGET:-5} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; echo bench_rc=$rc
[ $rc -eq 0 ] || exit $rc
for t in ${TILES:-}; do
  CFM_GEMM_TILE=$t timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-budget 0 > gpurun_out/bench_tile$t.json 2>> gpurun_out/bench.err; rc=$?; echo tile${t}_rc=$rc
  [ $rc -eq 0 ] || exit $rc
done
