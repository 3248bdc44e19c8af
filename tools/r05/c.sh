set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05c
mkdir -p $O
bash tools/r05/mb_junk2.sh > $O/junk2.txt 2>&1; cat $O/junk2.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_fullsize.py > $O/pytest.txt 2>&1; rc=$?
tail -2 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
bash tools/train_lib_ab.sh 3 train 2>&1 | tee $O/train_ab.txt
