#!/bin/bash
# Round-end verification: all GPU tests, smoke(), the default bench (N=1), then every other bench mode.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_verify.sh || exit $?
for m in joint rnnt_train stream cache_stream mel decode; do
  timeout -k 10 300 python bench.py --mode $m > gpurun_out/verify_$m.json 2> gpurun_out/verify_$m.err; rc=$?; echo ${m}_rc=$rc
  [ $rc -eq 0 ] || exit $rc
done
