#!/bin/bash
# Forward attention probes: bench breakdown of rel_attention under CFM_ATTN_PROBE bits
#   bash tools/attn_probe.sh "0 1 2 4 8"
cd "$GRAFT_REPO_ROOT" || exit 1
for pb in ${1:-0 1 2 4 8}; do
  us=$(CFM_ATTN_PROBE=$pb timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-budget 0 --no-parity 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); b=d['breakdown']['rel_attention']; print(round(b['ms_per_launch']*1000,2), d['ms_per_step'])"); rc=$?
  [ $rc -eq 0 ] || { echo "probe $pb failed rc=$rc"; exit $rc; }
  echo "probe $pb: rel_attention us/launch, forward ms = $us"
done
