# Training-path GPU tests, then the config-3 train bench and a rocprofv3 kernel summary of it.
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_ops.py tests/test_gpu_dp.py tests/test_gpu_ctc.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_train.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --mode train --steps 5 --warmup 2 > gpurun_out/bench_train.json 2> gpurun_out/bench_train.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train_c -o run -- python bench.py --mode train --steps 2 --warmup 2 > gpurun_out/bench_train_prof.json 2>> gpurun_out/bench_train.err
