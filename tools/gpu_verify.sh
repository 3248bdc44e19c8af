#!/bin/bash
# Round verification: all GPU tests, smoke(), then the default bench (N=1) and the train bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/verify_pytest.log 2>&1; rc=$?; echo pytest_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/verify_smoke.log 2>&1; rc=$?; echo smoke_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/verify_bench.json 2> gpurun_out/verify_bench.err; rc=$?; echo bench_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode train --steps 5 --warmup 2 > gpurun_out/verify_train.json 2> gpurun_out/verify_train.err; rc=$?; echo train_rc=$rc
exit $rc
