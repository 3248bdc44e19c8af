# A/B of write-through GEMM output stores: encoder tests, then the default bench with CFM_GEMM_WT=1 and 0.
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_wt.log 2>&1 || exit $?
for w in 1 0 1 0; do
  CFM_GEMM_WT=$w timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-budget 0 > gpurun_out/bench_wt$w.json 2>> gpurun_out/bench_wt.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_wt$w.json')); print('wt=$w', d['ms_per_step'])" >> gpurun_out/wt_ab.txt
done
