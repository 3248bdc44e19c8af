set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_rnnt_train.py tests/test_gpu_train_ops.py tests/test_gpu_attn_bwd_fused.py tests/test_gpu_fullsize.py > $O/pytest.txt 2>&1; rc=$?
tail -2 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
bash tools/train_lib_ab.sh 3 train > $O/train_ab.txt 2>&1 || { cat $O/train_ab.txt; exit 1; }
cat $O/train_ab.txt
bash tools/train_lib_ab.sh 2 rnnt_train > $O/rnnt_ab.txt 2>&1 || { cat $O/rnnt_ab.txt; exit 1; }
cat $O/rnnt_ab.txt
