#!/bin/bash
# Same-box training-step A/B between two library builds: bash tools/train_lib_ab.sh [rounds] [mode]
# (conformer_amd/libcfm_base.so = the reference build, libcfm.so = the candidate)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B=$PWD/conformer-nemo_amd/conformer_amd/libcfm_base.so
M=${2:-train}
for r in $(seq 1 ${1:-3}); do
  CFM_LIB_PATH=$B timeout -k 10 200 python bench.py --mode $M --steps 10 --warmup 3 > gpurun_out/ab_base.json 2>/dev/null || exit 1
  python3 -c "import json; print('base', json.load(open('gpurun_out/ab_base.json'))['ms_per_step'])"
  timeout -k 10 200 python bench.py --mode $M --steps 10 --warmup 3 > gpurun_out/ab_new.json 2>/dev/null || exit 1
  python3 -c "import json; print('new ', json.load(open('gpurun_out/ab_new.json'))['ms_per_step'])"
done
