# Encoder GPU tests, then the default bench (forward, N=1) with its per-stage breakdown.
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_ops.py tests/test_gpu_train.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fwd.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 > gpurun_out/bench_fwd.json 2> gpurun_out/bench_fwd.err
