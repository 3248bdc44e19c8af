# Attention-backward GPU tests, the fused-vs-materialised op timing and the config-3 train bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_ops.py -k "rel_attention" -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_attn_bwd.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/attn_bwd_bench.py > gpurun_out/attn_bwd_bench.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_train.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --mode train --steps 5 --warmup 2 > gpurun_out/bench_train.json 2> gpurun_out/bench_train.err || exit $?
CFM_ATTN_BWD_FUSED=0 timeout -k 10 300 python bench.py --mode train --steps 5 --warmup 2 > gpurun_out/bench_train_unfused.json 2>> gpurun_out/bench_train.err
