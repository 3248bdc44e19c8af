set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05v
mkdir -p $O
for r in 1 2; do
for pb in 0 8 16 24 32 64 88 256 376; do
  CFM_GEMM_PROBE=$pb timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --cpu-budget 0 --no-train --no-parity > $O/b_$pb.json 2>> $O/err.txt || exit 1
  python3 -c "import json; d=json.load(open('$O/b_$pb.json')); b=d['breakdown']['conv2_gemm']; print('probe $pb conv2_gemm', round(b['ms_total']*1000,1), 'us')"
done
done
