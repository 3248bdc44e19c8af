set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_encoder.py tests/test_gpu_fullsize.py tests/test_gpu_ops.py > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?
cat $O/bench.json
exit $rc
