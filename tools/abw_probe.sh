#!/bin/bash
# attn_bwd_scores_kernel time per probe build (CFM_ABW_PROBE in attn_bwd.hip; probe_libs/ built by hand)
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for P in base p1 p6 p8 p15; do
  L=$PWD/conformer-nemo_amd/conformer_amd/libcfm.so
  [ $P != base ] && L=$PWD/conformer-nemo_amd/probe_libs/libcfm_$P.so
  CFM_LIB_PATH=$L CFM_ATTN_BWD_FUSED=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abw_$P -o run -- \
    python3 tools/attn_bwd_bench.py --child 32 250 8 64 /tmp/abw.npz > gpurun_out/abw_$P.log 2>&1 || exit 1
  S=$(find gpurun_out/abw_$P -name '*kernel_stats.csv' | head -1)
  echo "$P $(grep attn_bwd_scores $S | cut -c1-200)"
done
