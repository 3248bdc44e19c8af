# A/B of the swapped-operand GEMM epilogues (CFM_GEMM_SWAP) + the GPU tests they touch
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05sw}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_encoder.py tests/test_gpu_submodules.py tests/test_gpu_ops.py tests/test_gpu_rnnt_loss.py tests/test_gpu_rnnt_decode.py > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for sw in 1 0; do
    CFM_GEMM_SWAP=$sw timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --cpu-budget 0 > $O/b_sw${sw}_$i.json 2>> $O/err.txt || exit 1
  done
done
python3 tools/show_bench.py $O/b_sw*.json | grep -E "==|ffn|out_proj|pw2|pos"
timeout -k 10 200 python3 tools/gemm_probe.py 11,14 ffn_up,ffn_down > $O/probe_sw1.txt 2>> $O/err.txt || exit 1
CFM_GEMM_SWAP=0 timeout -k 10 200 python3 tools/gemm_probe.py 11,14 ffn_up,ffn_down > $O/probe_sw0.txt 2>> $O/err.txt || exit 1
cat $O/probe_sw1.txt $O/probe_sw0.txt
