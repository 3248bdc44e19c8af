# round 4: LSTM BPTT recurrent product on the matrix cores: parity, rnnt_train A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rnnt_train.py tests/test_gpu_rnnt_decode.py -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; echo pytest_rc=$?
tail -2 $O/pytest.txt
grep -q " passed" $O/pytest.txt && ! grep -q "failed\|rror" $O/pytest.txt || exit 1
for m in 1 0 1 0; do
  CFM_LSTM_MFMA=$m timeout -k 10 300 python3 bench.py --mode rnnt_train --steps 4 --warmup 2 > $O/rnnt_$m.$RANDOM.json 2>> $O/bench.err || exit 1
done
echo done_j
