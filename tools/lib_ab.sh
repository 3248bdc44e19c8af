#!/bin/bash
# Same-box forward A/B between two builds of the library: bash tools/lib_ab.sh [rounds]
# (conformer_amd/libcfm_base.so = the reference build, libcfm.so = the candidate)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B=conformer-nemo_amd/conformer_amd/libcfm_base.so
for r in $(seq 1 ${1:-3}); do
  CFM_LIB_PATH=$PWD/$B timeout -k 10 120 python tools/fwd_ab.py base 10 2>/dev/null || exit 1
  timeout -k 10 120 python tools/fwd_ab.py new 10 2>/dev/null || exit 1
done
