# round 4 end: the committed tree once more - full GPU suite, smoke, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04fin2
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; echo pytest_rc=$?
tail -1 $O/pytest.txt
grep -q " passed" $O/pytest.txt && ! grep -q "failed\|rror" $O/pytest.txt || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
tail -1 $O/smoke.txt
timeout -k 10 300 python3 bench.py > $O/bench.json 2>> $O/err.txt || exit 1
timeout -k 10 300 python3 bench.py --mode rnnt_train --steps 5 --warmup 2 > $O/bench_rnnt_train.json 2>> $O/err.txt || exit 1
for f in $O/bench*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'])"; done
