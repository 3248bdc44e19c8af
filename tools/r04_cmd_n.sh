# round 4: config-4 joint mode kernel trace (per-kernel durations of encoder T'=400 + prediction net + joint)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --mode joint --steps 3 --warmup 1 --no-breakdown > $O/joint_trace.json 2> $O/trace.err; echo trace_rc=$?
find $O/trace -name '*kernel_stats.csv' | head -1
