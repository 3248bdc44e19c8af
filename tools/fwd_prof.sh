#!/bin/bash
# rocprofv3 kernel trace of the bf16 forward (tools/fwd_ab.py): per-kernel summary -> gpurun_out/fprof_<tag>/
T=${1:-x}
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fprof_$T; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 tools/fwd_ab.py prof 4 > $O/log.txt 2>&1; rc=$?; echo prof_rc=$rc
[ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py $(find $O -name '*kernel_stats.csv' | head -1) 30 > $O/summary.txt 2>&1
cat $O/summary.txt | head -40
