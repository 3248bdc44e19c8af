#!/bin/bash
# Forward A/B over CFM_TILES rules for the FFN GEMMs (2 = linear1 + Swish, 3 = residual GEMMs):  bash tools/ffn_tile_sweep.sh
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sw
for r in 1 2; do for t in "" "2:7" "2:10" "2:15" "2:1" "3:17@4096" "3:12@4096" "3:9@4096" "3:13@4096"; do
  CFM_TILES="$t" timeout -k 10 120 python bench.py --steps 30 --warmup 5 --cpu-budget 0 --no-breakdown --no-train --no-parity > gpurun_out/sw/o.json 2>gpurun_out/sw/e.txt || { echo "tiles=$t failed"; tail -3 gpurun_out/sw/e.txt; exit 1; }
  python3 -c "import json; print('tiles=$t', json.load(open('gpurun_out/sw/o.json'))['ms_per_step'])"
done; done
