cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tr_trace -o run -- python3 bench.py --mode train --steps 1 --warmup 1 > gpurun_out/prof_tr_trace.json 2> gpurun_out/prof_tr_trace.err
