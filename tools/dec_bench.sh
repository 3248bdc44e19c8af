# Greedy-decode bench sweep over the blank-logit bias, then a rocprofv3 kernel summary of one run.
cd "$GRAFT_REPO_ROOT" || exit 1
for bb in ${BIASES:-1.1 1.2 1.3}; do
  BLANK_BIAS=$bb timeout -k 10 200 python bench.py --mode decode --steps 3 --warmup 1 > gpurun_out/bench_decode_$bb.json 2> gpurun_out/bench_decode.err || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BLANK_BIAS=${PROF_BIAS:-1.2} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_decode -o run -- python bench.py --mode decode --steps 2 --warmup 1 > gpurun_out/bench_decode_prof.json 2>> gpurun_out/bench_decode.err
