# round 4: denominator kernel with early row loads and register-held blank / label logits (CFM_RNNT_DENOM_EARLY) - parity + A/B + traces
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04a7
mkdir -p $O
export TMPDIR=/tmp
for m in 0 1; do
  CFM_RNNT_DENOM_EARLY=$m timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rnnt_loss.py -x -q --timeout 300 --timeout-method thread > $O/pytest_e$m.txt 2>&1; echo pytest_e$m rc=$?
  tail -1 $O/pytest_e$m.txt
  grep -q " passed" $O/pytest_e$m.txt && ! grep -q "failed\|rror" $O/pytest_e$m.txt || exit 1
done
for m in 0 1 0 1; do
  CFM_RNNT_DENOM_EARLY=$m timeout -k 10 300 python3 bench.py --mode rnnt_train --steps 5 --warmup 2 > $O/rnnt_train_e$m.$RANDOM.json 2>> $O/err.txt || exit 1
done
for m in 0 1; do
  CFM_RNNT_DENOM_EARLY=$m timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof$m -o run -- python3 bench.py --mode rnnt_train --steps 2 --warmup 1 > $O/prof_bench$m.json 2>> $O/err.txt || exit 1
done
for f in $O/rnnt_train_e*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['ms_per_step'],d['loss'])"; done
