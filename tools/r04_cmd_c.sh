# round 4: joint / training / rnnt-training kernel traces, training host timing, L2->LDS rate curve
set -o pipefail
cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 300 tools/l2lds_rate > $O/l2lds_rate.txt 2>&1; echo l2lds_rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/joint -o run -- \
  python3 bench.py --mode joint --steps 4 --warmup 2 > $O/joint.json 2> $O/joint.err; echo joint_rc=$?
timeout -k 10 300 python3 tools/train_host_timing.py 6 > $O/train_host.txt 2>&1; echo host_rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train -o run -- \
  python3 bench.py --mode train --steps 3 --warmup 2 > $O/train.json 2> $O/train.err; echo train_rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rnnt -o run -- \
  python3 bench.py --mode rnnt_train --steps 3 --warmup 2 > $O/rnnt.json 2> $O/rnnt.err; echo rnnt_rc=$?
for d in joint train rnnt; do
  f=$(find $O/$d -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && python3 tools/prof_summary.py $f 40 > $O/${d}_summary.txt 2>&1
  f=$(find $O/$d -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && python3 tools/train_step_trace.py $f > $O/${d}_steptrace.txt 2>&1
done
echo done
