# fused joint logits: parity tests + timing (probe decomposition, split / unfused A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05jc}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_joint.py ${EXTRA_TESTS:-} > $O/pytest.txt 2>&1; rc=$?
tail -4 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/joint_probe.py > $O/probe.txt 2>&1; rc=$?; cat $O/probe.txt; exit $rc
