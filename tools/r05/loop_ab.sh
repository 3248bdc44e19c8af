# GEMM main-loop change: GPU encoder tests + forward bench x2 + probes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05lp}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_encoder.py tests/test_gpu_submodules.py tests/test_gpu_train.py > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --cpu-budget 0 > $O/b_$i.json 2>> $O/err.txt || exit 1
done
python3 tools/show_bench.py $O/b_*.json
timeout -k 10 200 python3 tools/gemm_probe.py 11,14,16 ffn_up,ffn_down,out > $O/probe.txt 2>> $O/err.txt || exit 1
cat $O/probe.txt
