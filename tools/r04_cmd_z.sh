# round 4: row-run pack kernel (CFM_PACK_ROWS) + NT=1 LSTM steps - full GPU suite, smoke, train/rnnt_train A/B, trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; echo pytest_rc=$?
tail -3 $O/pytest.txt
grep -q " passed" $O/pytest.txt && ! grep -q "failed\|rror" $O/pytest.txt || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
for m in 0 1 0 1; do
  CFM_PACK_ROWS=$m timeout -k 10 300 python3 bench.py --mode rnnt_train --steps 5 --warmup 2 > $O/rnnt_train_p$m.$RANDOM.json 2>> $O/err.txt || exit 1
done
for m in 0 1; do
  CFM_PACK_ROWS=$m timeout -k 10 300 python3 bench.py --mode train --steps 5 --warmup 2 > $O/train_p$m.json 2>> $O/err.txt || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 bench.py --mode rnnt_train --steps 3 --warmup 1 > $O/prof_bench.json 2>> $O/err.txt || exit 1
for f in $O/*train_p*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['ms_per_step'])"; done
for m in 1 0; do
  CFM_SYNC_LABEL_CHECK=$m timeout -k 10 300 python3 bench.py --mode rnnt_train --steps 5 --warmup 2 > $O/rnnt_train_sync$m.json 2>> $O/err.txt || exit 1
done
timeout -k 10 300 python3 tools/rnnt_host_profile.py --steps 3 > $O/host_profile.txt 2>> $O/err.txt || exit 1
for f in $O/rnnt_train_sync*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['ms_per_step'])"; done
head -30 $O/host_profile.txt
