set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05u
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_encoder.py -k "conv12 or batch_invariance" > $O/pytest.txt 2>&1; rc=$?
tail -2 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
B=$PWD/conformer-nemo_amd/conformer_amd/libcfm_base.so
for r in 1 2 3; do
  CFM_LIB_PATH=$B timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --cpu-budget 0 --no-train --no-parity > $O/base.json 2>> $O/err.txt || exit 1
  python3 -c "import json; d=json.load(open('$O/base.json')); b=d['breakdown']['conv2_gemm']; print('base', d['ms_per_step'], 'ms  conv2_gemm', round(b['ms_total']*1000,1), 'us')"
  for v in 0 1; do
  CFM_CONV12B=$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --cpu-budget 0 --no-train --no-parity > $O/new.json 2>> $O/err.txt || exit 1
  python3 -c "import json; d=json.load(open('$O/new.json')); b=d['breakdown']['conv2_gemm']; print('new conv12b=$v', d['ms_per_step'], 'ms  conv2_gemm', round(b['ms_total']*1000,1), 'us')"
  done
done
