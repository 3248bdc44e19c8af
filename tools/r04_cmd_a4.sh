# round 4: RNN-T gradient over flat aligned spans (rnnt_grad_flat_kernel) + float4 denominators - loss/train parity + rnnt_train A/B + trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04a4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rnnt_loss.py tests/test_gpu_rnnt_train.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; echo pytest_rc=$?
tail -3 $O/pytest.txt
grep -q " passed" $O/pytest.txt && ! grep -q "failed\|rror" $O/pytest.txt || exit 1
for m in 0 1 0 1; do
  CFM_RNNT_GRAD_FLAT=$m timeout -k 10 300 python3 bench.py --mode rnnt_train --steps 5 --warmup 2 > $O/rnnt_train_f$m.$RANDOM.json 2>> $O/err.txt || exit 1
done
for m in 0 1; do
  CFM_RNNT_DENOM_V4=$m timeout -k 10 300 python3 bench.py --mode rnnt_train --steps 5 --warmup 2 > $O/rnnt_train_v$m.json 2>> $O/err.txt || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 bench.py --mode rnnt_train --steps 3 --warmup 1 > $O/prof_bench.json 2>> $O/err.txt || exit 1
for f in $O/rnnt_train_[fv]*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['ms_per_step'],d['loss'])"; done
