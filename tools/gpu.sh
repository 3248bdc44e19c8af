#!/bin/bash
# gpurun wrapper: re-submits ONLY when the infrastructure reports a transient failure before the
# command started (status "transient": no box, nothing ran).  Never retries a command that ran.
for attempt in 1 2 3 4; do
  /usr/local/graft/bin/gpurun "$@" > /tmp/gpurun_last.txt 2>&1
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ] && ! grep -q "backing off" /tmp/gpurun_last.txt; then
    tail -3 /tmp/gpurun_last.txt; exit $rc
  fi
  echo "[gpu.sh] transient infrastructure failure (attempt $attempt), waiting"; sleep 90
done
tail -3 /tmp/gpurun_last.txt; exit $rc
