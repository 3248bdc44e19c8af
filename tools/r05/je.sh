# one-pass joint activation backward: parity, same-box RNN-T training A/B (CFM_JOINT_ACT_FUSED 0/1)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05je}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_joint.py tests/test_gpu_rnnt_train.py tests/test_gpu_fullsize.py > $O/pytest.txt 2>&1; rc=$?
tail -4 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for f in 0 1; do
    CFM_JOINT_ACT_FUSED=$f timeout -k 10 300 python3 bench.py --mode rnnt_train --steps 20 --warmup 5 --cpu-budget 0 > $O/rnnt_train_a${f}_r$r.json 2>> $O/err.txt || exit 1
    python3 - $O/rnnt_train_a${f}_r$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d["ms_per_step"])
PY
  done
done
