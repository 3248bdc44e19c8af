#!/bin/bash
# All GPU tests (one process), log under gpurun_out/.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo pytest_rc=$rc; tail -4 gpurun_out/gpu_tests.log; exit $rc
