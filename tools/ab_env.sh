#!/bin/bash
# Forward A/B of one environment switch, alternating runs (no profiler):  bash tools/ab_env.sh VAR "A B" [reps]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
VAR=$1; VALS=$2; REPS=${3:-2}
for r in $(seq 1 $REPS); do for v in $VALS; do
  env $VAR=$v timeout -k 10 120 python bench.py --steps 30 --warmup 5 --cpu-budget 0 --no-breakdown --no-train --no-parity \
    > gpurun_out/ab/${VAR}_$v.json 2>gpurun_out/ab/${VAR}_$v.err || { echo "$VAR=$v failed"; tail -5 gpurun_out/ab/${VAR}_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/${VAR}_$v.json')); print('$VAR=$v', d['ms_per_step'])" | tee -a gpurun_out/ab/summary.txt
done; done
