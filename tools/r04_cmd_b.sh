set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 300 python3 tools/gemm_probe.py 11 ffn_up > $O/probe_direct.txt 2>&1 && \
timeout -k 10 300 python3 tools/gemm_probe.py 14 ffn_down,out >> $O/probe_direct.txt 2>&1 && \
CFM_GEMM_DIRECT=0 timeout -k 10 300 python3 tools/gemm_probe.py 11 ffn_up > $O/probe_old.txt 2>&1 && \
CFM_GEMM_DIRECT=0 timeout -k 10 300 python3 tools/gemm_probe.py 14 ffn_down,out >> $O/probe_old.txt 2>&1 && \
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_encoder.py -x -q --timeout 120 --timeout-method thread > $O/pytest_enc.txt 2>&1 ; echo pytest_rc=$? && \
timeout -k 10 300 python3 bench.py --no-train --cpu-budget 0 > $O/bench_direct.json 2> $O/bench_direct.err && \
CFM_GEMM_DIRECT=0 timeout -k 10 300 python3 bench.py --no-train --cpu-budget 0 --no-parity > $O/bench_old.json 2> $O/bench_old.err
echo done
