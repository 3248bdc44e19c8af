# Train-step time per weight-gradient tile (CFM_WGRAD_TILE) for the M-row layer gradients.
cd "$GRAFT_REPO_ROOT" || exit 1
for t in -1 11 8 1 0 10 9; do
  CFM_WGRAD_TILE=$t timeout -k 10 200 python bench.py --mode train --steps 5 --warmup 2 > gpurun_out/wg_$t.json 2>> gpurun_out/wg.err || exit $?
done
