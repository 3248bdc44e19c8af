# round 4: chunked joint (hidden + logits GEMM per chunk of utterances) and non-temporal logits stores -
# parity + joint-mode A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04t
mkdir -p $O
CFM_JOINT_CHUNK=2 CFM_LOGITS_NT=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_joint.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; echo pytest_rc=$?
tail -3 $O/pytest.txt
grep -q " passed" $O/pytest.txt && ! grep -q "failed\|rror" $O/pytest.txt || exit 1
for cfg in "0 0" "2 0" "4 0" "0 1" "2 1" "0 0" "2 0" "4 0" "0 1" "2 1"; do
  set -- $cfg
  CFM_JOINT_CHUNK=$1 CFM_LOGITS_NT=$2 timeout -k 10 300 python3 bench.py --mode joint --steps 5 --warmup 2 > $O/joint_c$1_nt$2.$RANDOM.json 2>> $O/err.txt || exit 1
done
for f in $O/joint_c*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f',d['ms_per_step'],d.get('breakdown',{}).get('joint'))"; done
