# round 4 final verification: full GPU suite, smoke, every bench mode the round touched
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04fin
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; echo pytest_rc=$?
tail -3 $O/pytest.txt
grep -q " passed" $O/pytest.txt && ! grep -q "failed\|rror" $O/pytest.txt || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench.json 2>> $O/err.txt || exit 1
for m in joint rnnt_train train decode; do
  timeout -k 10 300 python3 bench.py --mode $m --steps 5 --warmup 2 > $O/bench_$m.json 2>> $O/err.txt || exit 1
done
cat $O/smoke.txt | tail -1
for f in $O/bench*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'],d.get('roofline',{}).get('frac'))"; done
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 bench.py --mode rnnt_train --steps 3 --warmup 1 > $O/prof_bench.json 2>> $O/err.txt || exit 1
