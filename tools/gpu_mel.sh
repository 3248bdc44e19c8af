cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mel.py -v -rf -x --timeout 120 --timeout-method thread -s > gpurun_out/pytest_mel.log 2>&1; echo pytest_rc=$?
