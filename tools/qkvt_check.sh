cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_ops.py tests/test_gpu_stream.py tests/test_gpu_joint.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_qkvt.log 2>&1 || exit $?
timeout -k 10 200 python tools/qkv_probe.py > gpurun_out/qkv_probe.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-budget 0 > gpurun_out/bench_qkvt.json 2> gpurun_out/bench_qkvt.err
