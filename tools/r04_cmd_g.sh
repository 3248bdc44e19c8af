# round 4: conv12 XCD column split A/B + full GPU test suite
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04g
mkdir -p $O
for c in 1 0 1 0; do CFM_C12_XCD_COLS=$c timeout -k 10 300 python3 bench.py --no-train --cpu-budget 0 --no-parity > $O/bench_xc_$c.$RANDOM.json 2>> $O/bench.err || break; done
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; echo pytest_rc=$?
tail -3 $O/pytest_gpu.txt
