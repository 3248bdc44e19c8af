#!/bin/bash
# Training-step A/B over values of one environment variable:  bash tools/env_train_ab.sh VAR "v1 v2 ..." [rounds]
#   the training GPU tests first (default settings), then bench --mode train per value, alternating
V=${1:?var}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_comm.py tests/test_gpu_dp.py tests/test_gpu_train_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?; echo tests_rc=$rc
[ $rc -eq 0 ] || exit $rc
for r in $(seq 1 ${3:-2}); do
  for v in $2; do
    env $V=$v timeout -k 10 300 python bench.py --mode train --steps 5 --warmup 2 > gpurun_out/ab_${v}_$r.json 2>> gpurun_out/ab.err; rc=$?
    [ $rc -eq 0 ] || exit $rc
    python -c "import json;d=json.load(open('gpurun_out/ab_${v}_$r.json'));print('$V=$v run $r', d['ms_per_step'], 'ms/step')"
  done
done
