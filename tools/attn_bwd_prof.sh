# Kernel breakdown of the fused attention backward op at the config-3 shape.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export CFM_ATTN_BWD_FUSED=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab -o run -- python tools/attn_bwd_bench.py --child 32 250 8 64 /tmp/ab.npz > gpurun_out/prof_ab.log 2>&1
