#!/bin/bash
# Weight-gradient TN tile A/B on the training step:  bash tools/tn_ab.sh "11 21 12 22"
#   every GPU test on the default tile, the training tests on each candidate, then bench --mode train per tile
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tn_pytest.log 2>&1; rc=$?; echo pytest_rc=$rc
[ $rc -eq 0 ] || exit $rc
for t in ${1:-11 21 12 22}; do
  CFM_TN_TILE=$t timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tn_test_$t.log 2>&1; rc=$?; echo test_${t}_rc=$rc
  [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for t in ${1:-11 21 12 22}; do
    CFM_TN_TILE=$t timeout -k 10 300 python bench.py --mode train --steps 5 --warmup 2 > gpurun_out/tn_train_${t}_$r.json 2>> gpurun_out/tn_train.err; rc=$?
    [ $rc -eq 0 ] || exit $rc
    python -c "import json;d=json.load(open('gpurun_out/tn_train_${t}_$r.json'));print('tile $t run $r', d['ms_per_step'], 'ms/step')"
  done
done
