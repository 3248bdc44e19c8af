# round 4: LSTM cell backward fused into the recurrent-product epilogue (CFM_LSTM_BWD_FUSE) - parity + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04a6
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rnnt_train.py tests/test_gpu_rnnt_decode.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; echo pytest_rc=$?
tail -3 $O/pytest.txt
grep -q " passed" $O/pytest.txt && ! grep -q "failed\|rror" $O/pytest.txt || exit 1
for m in 0 1 0 1; do
  CFM_LSTM_BWD_FUSE=$m timeout -k 10 300 python3 bench.py --mode rnnt_train --steps 5 --warmup 2 > $O/rnnt_train_b$m.$RANDOM.json 2>> $O/err.txt || exit 1
done
for f in $O/rnnt_train_b*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['ms_per_step'],d['loss'])"; done
