# round 4: layer-0 LSTM input table (gathered embedding projection) - prediction-net parity + joint/decode A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04u
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_rnnt_decode.py tests/test_gpu_rnnt_train.py tests/test_gpu_joint.py -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; echo pytest_rc=$?
tail -3 $O/pytest.txt
grep -q " passed" $O/pytest.txt && ! grep -q "failed\|rror" $O/pytest.txt || exit 1
for m in 0 1 0 1; do
  CFM_LSTM_XTAB=$m timeout -k 10 300 python3 bench.py --mode joint --steps 5 --warmup 2 > $O/joint_x$m.$RANDOM.json 2>> $O/err.txt || exit 1
done
for m in 0 1; do
  CFM_LSTM_XTAB=$m timeout -k 10 300 python3 bench.py --mode decode --steps 3 --warmup 1 > $O/decode_x$m.json 2>> $O/err.txt || exit 1
done
for f in $O/joint_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['ms_per_step'],d.get('breakdown'))"; done
for f in $O/decode_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'])"; done
