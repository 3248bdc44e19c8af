# GPU tests touched by the ADVICE / linear-pack changes, then the conv2 study
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_submodules.py tests/test_gpu_rnnt_loss.py tests/test_gpu_rnnt_decode.py tests/test_gpu_ops.py > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
bash tools/r05/conv2a.sh
