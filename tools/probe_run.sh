cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python tools/gemm_probe.py ${1:-11,7,1,5,9} ${2:-qkvs} > gpurun_out/probe.txt 2>&1; echo rc=$?
cat gpurun_out/probe.txt
