# round 4: two-stream micro-batching with co-resident (<= 80 KB LDS) GEMM tiles: does a second stream's
# main loop overlap the first stream's store-bound epilogue on the same CU?
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04i
mkdir -p $O
run() { env "$@" timeout -k 10 200 python3 bench.py --no-train --cpu-budget 0 --no-parity --no-breakdown > $O/$(echo "$@" | tr ' =:,@' '_____').json 2>> $O/err.txt; }
for r in 1 2; do
run X=$r
run X=$r CFM_MICROBATCH=2
run X=$r CFM_MICROBATCH=2 CFM_TILES=2:5,3:16,0:5,6:5
run X=$r CFM_MICROBATCH=2 CFM_TILES=2:0,3:0,0:5,6:5
run X=$r CFM_MICROBATCH=4 CFM_TILES=2:5,3:16,0:5,6:5
run X=$r CFM_MICROBATCH=2 CFM_TILES=2:5,3:16,0:5,6:5 CFM_QKV_ATTN=0
done
ls $O
