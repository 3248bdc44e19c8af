#!/bin/bash
# Forward A/B over environment configurations: bash tools/fwd_ab.sh "LABEL|ENV=.. ENV=.." ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in "$@"; do
  label=${cfg%%|*}; envs=${cfg#*|}
  [ "$envs" = "$cfg" ] && envs=""
  env $envs timeout -k 10 120 python tools/fwd_ab.py "$label" 10 2>/dev/null; rc=$?
  [ $rc -eq 0 ] || { echo "$label failed rc=$rc"; exit $rc; }
done
