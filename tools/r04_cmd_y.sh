# round 4: prediction net as one cooperative launch (lstm_seq_mfma_kernel) + MFMA steps for H < 128 - parity + A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04y
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rnnt_decode.py tests/test_gpu_rnnt_train.py tests/test_gpu_joint.py -x -v --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; echo pytest_rc=$?
tail -3 $O/pytest.txt
grep -q " passed" $O/pytest.txt && ! grep -q "failed\|rror" $O/pytest.txt || exit 1
for m in 0 1 0 1; do
  CFM_LSTM_SEQ=$m timeout -k 10 300 python3 bench.py --mode joint --steps 5 --warmup 2 > $O/joint_s$m.$RANDOM.json 2>> $O/err.txt || exit 1
done
CFM_LSTM_SEQ=1 timeout -k 10 300 python3 bench.py --mode decode --steps 3 --warmup 1 > $O/decode.json 2>> $O/err.txt || exit 1
for f in $O/joint_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['ms_per_step'],d.get('breakdown'))"; done
cat $O/decode.json
