# PMC passes over the fused attention backward (config-3 shape), one counter group per pass
set -o pipefail
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_attn_bwd_fused.py tests/test_gpu_train.py > gpurun_out/r05n_pytest.txt 2>&1 || { tail -20 gpurun_out/r05n_pytest.txt; exit 1; }; tail -1 gpurun_out/r05n_pytest.txt
cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05n
mkdir -p $O
export CFM_ATTN_BWD_FUSED=1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 tools/attn_bwd_bench.py --child 32 250 8 64 /tmp/ab.npz > $O/t.log 2>&1 || exit 1
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p$i -o run -- python3 tools/attn_bwd_bench.py --child 32 250 8 64 /tmp/ab.npz > $O/p$i.log 2>&1; rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, collections
O = "gpurun_out/r05n"
for f in sorted(glob.glob(O + "/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "attn_bwd_scores" not in k:
            continue
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for c, v in sorted(acc.items()):
        print(f"{f.split('/')[2]} {c:32s} mean/dispatch {sum(v)/len(v):.4g}  (n={len(v)})")
PY
grep -h "attn_bwd_scores\|bgemm\|tn_glds" $(find $O/t -name '*kernel_stats.csv') | cut -d, -f1-5 | head
