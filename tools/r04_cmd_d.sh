# round 4: direct-epilogue store-policy A/B, then the joint / training / rnnt traces (r04_cmd_c.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04d
mkdir -p $O
for v in "1 0" "0 1"; do
  set -- $v
  CFM_GEMM_DIRECT=$1 CFM_GEMM_WT=$2 timeout -k 10 200 python3 tools/gemm_probe.py 11 ffn_up > $O/probe_d$1_wt$2.txt 2>&1 && \
  CFM_GEMM_DIRECT=$1 CFM_GEMM_WT=$2 timeout -k 10 200 python3 tools/gemm_probe.py 14 ffn_down,out >> $O/probe_d$1_wt$2.txt 2>&1 && \
  CFM_GEMM_DIRECT=$1 CFM_GEMM_WT=$2 timeout -k 10 300 python3 bench.py --no-train --cpu-budget 0 --no-parity > $O/bench_d$1_wt$2.json 2> $O/bench_d$1_wt$2.err || exit 1
done
bash tools/r04_cmd_c.sh
O=gpurun_out/r04d
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_encoder.py -x -v -k conv12 --timeout 200 --timeout-method thread > $O/pytest_conv12.txt 2>&1; echo conv12_pytest_rc=$?
grep -q "passed" $O/pytest_conv12.txt && ! grep -q "failed\|error" $O/pytest_conv12.txt && \
for c in 1 0 1 0; do CFM_CONV12=$c timeout -k 10 300 python3 bench.py --no-train --cpu-budget 0 --no-parity > $O/bench_c12_$c.$RANDOM.json 2>> $O/bench_c12.err || break; done
echo done_d
