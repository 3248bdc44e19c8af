set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_encoder.py -k "conv12" > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for v in 0 1; do
  CFM_CONV12B=$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --cpu-budget 0 --no-train --no-parity > $O/b_$v.json 2>> $O/err.txt || exit 1
  python3 -c "import json; d=json.load(open('$O/b_$v.json')); b=d['breakdown']['conv2_gemm']; print('conv12b=$v', d['ms_per_step'], 'ms/step  conv2_gemm', round(b['ms_total']*1000,1), 'us')"
done
done
