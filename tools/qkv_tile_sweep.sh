#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sw
for r in 1 2; do for t in "" "0:12" "0:13" "0:14" "0:1" "0:15" "0:16" "0:8"; do
  CFM_TILES="$t" timeout -k 10 120 python bench.py --steps 30 --warmup 5 --cpu-budget 0 --no-breakdown --no-train --no-parity > gpurun_out/sw/o.json 2>gpurun_out/sw/e.txt || { echo "tiles=$t failed"; tail -3 gpurun_out/sw/e.txt; exit 1; }
  python3 -c "import json; print('tiles=$t', json.load(open('gpurun_out/sw/o.json'))['ms_per_step'])"
done; done
