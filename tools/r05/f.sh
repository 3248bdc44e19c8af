set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05f
mkdir -p $O
for r in 1 2; do
for sp in 0 1; do
CFM_G8_SPREAD=$sp CFM_GEMM8_DENSE=1 timeout -k 10 200 python3 tools/op_driver.py gemm 10 -1 ref4096s,conv2s 2>/dev/null | sed "s/^/spread$sp /" || exit 1
done
done
for r in 1 2; do
for sp in 0 1; do
CFM_G8_SPREAD=$sp CFM_CONV12=0 timeout -k 10 120 python3 tools/fwd_ab.py "conv12=0 spread=$sp" 10 2>/dev/null || exit 1
done
done
CFM_G8_SPREAD=1 CFM_CONV12=0 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_encoder.py -k "full_size" > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; exit $rc
