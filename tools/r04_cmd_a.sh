set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/gemm_probe.py 11 ffn_up > gpurun_out/probe_a.txt 2>&1 && \
timeout -k 10 300 python3 tools/gemm_probe.py 14 ffn_down,out >> gpurun_out/probe_a.txt 2>&1 && \
bash tools/forward_profile.sh r04a
