cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || exit 1
for mb in 1 2 3; do CFM_MICROBATCH=$mb timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-budget 0 > gpurun_out/bench_mb$mb.json 2>>gpurun_out/bench.err || exit 1; done
