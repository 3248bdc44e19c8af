#!/bin/bash
# Quick GPU check: the given pytest selection, then the default bench line (forward + train leg + CPU baseline).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "$1" ]; then
  timeout -k 10 300 python -u -m pytest $1 -x -v --timeout 120 --timeout-method thread > gpurun_out/quick_pytest.log 2>&1; rc=$?; echo pytest_rc=$rc
  [ $rc -eq 0 ] || { tail -30 gpurun_out/quick_pytest.log; exit $rc; }
fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err; rc=$?; echo bench_rc=$rc
[ $rc -eq 0 ] || tail -20 gpurun_out/quick_bench.err
exit $rc
