# round 4: the prediction network's LSTM step on the matrix cores: parity, then joint / decode / rnnt_train A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_rnnt_decode.py tests/test_gpu_rnnt_train.py tests/test_gpu_joint.py -x -q --timeout 300 --timeout-method thread > $O/pytest_lstm.txt 2>&1; echo pytest_rc=$?
tail -2 $O/pytest_lstm.txt
grep -q " passed" $O/pytest_lstm.txt && ! grep -q "failed\|rror" $O/pytest_lstm.txt || exit 1
for m in 1 0; do
  CFM_LSTM_MFMA=$m timeout -k 10 200 python3 bench.py --mode joint --steps 6 --warmup 2 > $O/joint_$m.json 2>> $O/bench.err || exit 1
  CFM_LSTM_MFMA=$m timeout -k 10 300 python3 bench.py --mode decode --steps 3 --warmup 1 > $O/decode_$m.json 2>> $O/bench.err || exit 1
  CFM_LSTM_MFMA=$m timeout -k 10 300 python3 bench.py --mode rnnt_train --steps 4 --warmup 2 > $O/rnnt_$m.json 2>> $O/bench.err || exit 1
done
echo done_h
