# fused joint logits kernel: parity tests, same-box A/B against the hidden kernel + GEMM path, kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05ja}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_joint.py > $O/pytest.txt 2>&1; rc=$?
tail -30 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for f in 0 1; do
    CFM_JOINT_FUSED=$f timeout -k 10 300 python3 bench.py --mode joint --steps 20 --warmup 5 --cpu-budget 0 > $O/joint_f${f}_r$r.json 2>> $O/err.txt || exit 1
    python3 - $O/joint_f${f}_r$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d["ms_per_step"], d["breakdown"]["joint"])
PY
  done
done
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --mode joint --steps 3 --warmup 1 --cpu-budget 0 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print(f'{r["Name"][:90]:90s} {r["Calls"]:>6s} {float(r["TotalDurationNs"])/1e6:9.3f} ms {float(r["AverageNs"])/1e3:9.2f} us')
PY
