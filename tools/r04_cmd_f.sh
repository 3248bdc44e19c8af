# round 4: joint tail columns + 256x256 logits tile, pipelined conv12: parity then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_joint.py tests/test_gpu_rnnt_train.py tests/test_gpu_rnnt_loss.py -x -q --timeout 200 --timeout-method thread > $O/pytest_joint.txt 2>&1; echo joint_pytest_rc=$?
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_encoder.py -x -q -k conv12 --timeout 200 --timeout-method thread > $O/pytest_conv12.txt 2>&1; echo conv12_pytest_rc=$?
grep -q " passed" $O/pytest_joint.txt && ! grep -q "failed\|rror" $O/pytest_joint.txt && \
  timeout -k 10 200 python3 bench.py --mode joint --steps 6 --warmup 2 > $O/joint.json 2> $O/joint.err
grep -q " passed" $O/pytest_conv12.txt && ! grep -q "failed\|rror" $O/pytest_conv12.txt && \
for c in 1 0 1 0; do CFM_CONV12=$c timeout -k 10 300 python3 bench.py --no-train --cpu-budget 0 --no-parity > $O/bench_c12_$c.$RANDOM.json 2>> $O/bench_c12.err || break; done
echo done_f
