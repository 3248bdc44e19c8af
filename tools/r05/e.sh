set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_encoder.py tests/test_gpu_ops.py tests/test_gpu_train_ops.py > $O/pytest.txt 2>&1; rc=$?
tail -2 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
TAG=r05e ROUNDS=4 bash tools/r05/libab.sh
