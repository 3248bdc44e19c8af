cd "$GRAFT_REPO_ROOT" || exit 1
for mb in 2 3 4 2; do
  CFM_MICROBATCH=$mb timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-budget 0 --no-breakdown > gpurun_out/bench_mb$mb.json 2>>gpurun_out/bench_mb.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/bench_mb$mb.json')); print('mb=$mb', d['ms_per_step'])" >> gpurun_out/mb.txt
done
