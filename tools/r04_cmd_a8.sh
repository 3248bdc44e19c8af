# round 4: bf16 row-run pack with four columns per lane (CFM_PACK_ROWS=2) vs two (=1) - parity + A/B + traces
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04a8
mkdir -p $O
export TMPDIR=/tmp
CFM_PACK_ROWS=2 timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; echo pytest_rc=$?
tail -1 $O/pytest.txt
grep -q " passed" $O/pytest.txt && ! grep -q "failed\|rror" $O/pytest.txt || exit 1
for m in 1 2 1 2; do
  CFM_PACK_ROWS=$m timeout -k 10 300 python3 bench.py --mode rnnt_train --steps 5 --warmup 2 > $O/rnnt_train_p$m.$RANDOM.json 2>> $O/err.txt || exit 1
done
for m in 1 2; do
  CFM_PACK_ROWS=$m timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof$m -o run -- python3 bench.py --mode rnnt_train --steps 2 --warmup 1 > $O/prof_bench$m.json 2>> $O/err.txt || exit 1
done
for f in $O/rnnt_train_p*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['ms_per_step'],d['loss'])"; done
