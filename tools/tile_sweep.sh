#!/bin/bash
# In-forward per-stage timings for each forced GEMM tile:  bash tools/tile_sweep.sh "0 1 5 9 10 11"
cd "$GRAFT_REPO_ROOT" || exit 1
for t in ${1:-0 1 5 9 10 11}; do
  CFM_GEMM_TILE=$t timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-budget 0 > gpurun_out/sweep_t$t.json 2>>gpurun_out/sweep.err || exit 1
done
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-budget 0 > gpurun_out/sweep_auto.json 2>>gpurun_out/sweep.err
