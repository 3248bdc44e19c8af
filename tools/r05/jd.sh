# fused joint logits: joint / RNN-T training parity, same-box bench A/B (CFM_JOINT_FUSED 0/1), kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05jd}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_joint.py tests/test_gpu_rnnt_train.py tests/test_gpu_fullsize.py > $O/pytest.txt 2>&1; rc=$?
tail -4 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for f in 0 1; do
    for m in joint rnnt_train; do
      CFM_JOINT_FUSED=$f timeout -k 10 300 python3 bench.py --mode $m --steps 20 --warmup 5 --cpu-budget 0 > $O/${m}_f${f}_r$r.json 2>> $O/err.txt || exit 1
      python3 - $O/${m}_f${f}_r$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d["ms_per_step"], d.get("breakdown", {}).get("joint", ""))
PY
    done
  done
done
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --mode joint --steps 3 --warmup 1 --cpu-budget 0 > $O/prof.log 2>&1 || exit 1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY' | tee $O/kernel_stats.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:16]:
    print(f'{r["Name"][:100]:100s} {r["Calls"]:>6s} {float(r["TotalDurationNs"])/1e6:9.3f} ms {float(r["AverageNs"])/1e3:9.2f} us')
PY
