cd "$GRAFT_REPO_ROOT" || exit 1
for t in 0 1 8; do
  CFM_GEMM_TILE=$t timeout -k 10 200 python bench.py --mode train --steps 4 --warmup 2 > gpurun_out/train_tile$t.json 2>> gpurun_out/train_tile.err || exit $?
done
