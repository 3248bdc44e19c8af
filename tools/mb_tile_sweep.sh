#!/bin/bash
# Forward A/B over micro-batch count x tile rules (no profiler):  bash tools/mb_tile_sweep.sh
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sweep
run() {   # name mb tiles
  CFM_MICROBATCH=$2 CFM_TILES="$3" timeout -k 10 120 python bench.py --steps 30 --warmup 5 --cpu-budget 0 \
    --no-breakdown --no-train --no-parity > gpurun_out/sweep/$1.json 2>gpurun_out/sweep/$1.err || { echo "$1 failed"; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sweep/$1.json')); print('$1 mb=$2 tiles=$3', d['ms_per_step'])" | tee -a gpurun_out/sweep/summary.txt
}
run base 1 "" && run mb2 2 "" && run mb2_small 2 "2:0,3:13,0:0" && run mb1_small 1 "2:0,3:13,0:0" \
  && run mb2_up256x128 2 "2:1,3:13,0:0" && run mb2_k4 2 "2:11,3:14" && run mb4_small 4 "2:0,3:13,0:0" && run base2 1 ""
