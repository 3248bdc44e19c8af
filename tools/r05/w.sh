set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05w2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_encoder.py tests/test_gpu_ops.py tests/test_gpu_train.py tests/test_gpu_train_ops.py > $O/pytest.txt 2>&1; rc=$?
tail -2 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
TAG=r05w2 ROUNDS=4 bash tools/r05/libab.sh
