# fused joint logits: probe decomposition + kernel stats (csv)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05jb}
mkdir -p $O
timeout -k 10 300 python3 tools/joint_probe.py > $O/probe.txt 2>&1; rc=$?; cat $O/probe.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --mode joint --steps 3 --warmup 1 --cpu-budget 0 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY' | tee $O/kernel_stats.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:16]:
    print(f'{r["Name"][:100]:100s} {r["Calls"]:>6s} {float(r["TotalDurationNs"])/1e6:9.3f} ms {float(r["AverageNs"])/1e3:9.2f} us')
PY
