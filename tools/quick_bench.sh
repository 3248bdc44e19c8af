#!/bin/bash
# Quick A/B on one GPU: forward bench (breakdown) + encoder parity tests.
#   bash tools/quick_bench.sh <tag> [extra pytest files...]
T=${1:-q}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 > gpurun_out/$T.json 2> gpurun_out/$T.err; rc=$?; echo bench_rc=$rc
[ $rc -eq 0 ] || exit $rc
python tools/show_bench.py gpurun_out/$T.json 2>/dev/null | head -40
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu "$@" > gpurun_out/$T.pytest.log 2>&1; rc=$?; echo pytest_rc=$rc
  tail -3 gpurun_out/$T.pytest.log
fi
exit $rc
