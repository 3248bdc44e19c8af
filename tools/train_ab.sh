#!/bin/bash
# Training-step A/B over environment configurations: bash tools/train_ab.sh "LABEL|ENV=.. ENV=.." ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in "$@"; do
  label=${cfg%%|*}; envs=${cfg#*|}
  [ "$envs" = "$cfg" ] && envs=""
  ms=$(env $envs timeout -k 10 200 python bench.py --mode train --steps 5 --warmup 2 2>/dev/null | python3 -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])"); rc=$?
  [ $rc -eq 0 ] || { echo "$label failed rc=$rc"; exit $rc; }
  echo "$label $ms"
done
