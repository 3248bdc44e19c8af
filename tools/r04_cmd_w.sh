# round 4: embedding gradient with LDS-staged labels - RNN-T train parity + rnnt_train bench + kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rnnt_train.py tests/test_gpu_rnnt_decode.py -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; echo pytest_rc=$?
tail -3 $O/pytest.txt
grep -q " passed" $O/pytest.txt && ! grep -q "failed\|rror" $O/pytest.txt || exit 1
timeout -k 10 300 python3 bench.py --mode rnnt_train --steps 5 --warmup 2 > $O/rnnt_train.json 2>> $O/err.txt || exit 1
timeout -k 10 300 python3 bench.py --mode joint --steps 5 --warmup 2 > $O/joint.json 2>> $O/err.txt || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --mode rnnt_train --steps 3 --warmup 1 > $O/prof_bench.json 2>> $O/err.txt || exit 1
cat $O/rnnt_train.json $O/joint.json
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if 'embed_grad' in r['Name'] or 'lstm' in r['Name']: print(r['Name'][:90], r['Calls'], r['AverageNs'])
PY
