# round 4: encoder parity (halo conv tiles, attention query split) + config-4 joint A/B + joint kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_encoder.py -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; echo pytest_rc=$?
tail -3 $O/pytest.txt
grep -q " passed" $O/pytest.txt && ! grep -q "failed\|rror" $O/pytest.txt || exit 1
for cfg in "1 1" "0 0" "1 0" "0 1"; do
  set -- $cfg
  CFM_ATTN_QSPLIT=$1 CFM_GLU_DW=$2 timeout -k 10 300 python3 bench.py --mode joint --steps 5 --warmup 2 > $O/joint_q$1_g$2.json 2>> $O/err.txt || exit 1
done
for f in $O/joint_*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f',d['ms_per_step'],d.get('breakdown'))"; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --mode joint --steps 3 --warmup 1 --no-breakdown > $O/joint_trace.json 2> $O/trace.err; echo trace_rc=$?
