# round 4: norm_out fold (ln_fold2) parity + forward A/B + stage tables with GEMM probes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_encoder.py -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; echo pytest_rc=$?
tail -3 $O/pytest.txt
grep -q " passed" $O/pytest.txt && ! grep -q "failed\|rror" $O/pytest.txt || exit 1
for m in 1 0 1 0; do
  CFM_LN_FOLD2=$m timeout -k 10 300 python3 tools/fwd_ab.py "ln_fold2=$m" 20 >> $O/ab.txt 2>> $O/err.txt || exit 1
done
cat $O/ab.txt
for pr in 0 2 1; do
  CFM_GEMM_PROBE=$pr timeout -k 10 300 python3 tools/fwd_stages.py "probe$pr" >> $O/stages.txt 2>> $O/err.txt || exit 1
done
echo done_k
