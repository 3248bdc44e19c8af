# SQ counters per forward kernel (one counter group per pass, kernel-trace only) over the north-star forward
set -o pipefail
cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05z
mkdir -p $O
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p$i -o run -- python3 tools/traffic_driver.py 2 > $O/p$i.log 2>&1; rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, collections
O = "gpurun_out/r05z"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
names = {}
for f in sorted(glob.glob(O + "/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        short = k.replace("(anonymous namespace)::", "").split("(")[0][:70]
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
rows = []
for k, d in acc.items():
    n = len(d.get("SQ_WAVES", [1]))
    if n < 10: continue
    m = {c: sum(v) / len(v) for c, v in d.items()}
    w = m.get("SQ_WAVES", 1)
    rows.append((m.get("SQ_WAVE_CYCLES", 0), k, m, w))
rows.sort(reverse=True)
for _, k, m, w in rows[:14]:
    wc = m.get("SQ_WAVE_CYCLES", 0)
    print(f"{k}")
    print(f"   waves {w:.0f}  per-wave: cycles(q) {wc/w:.0f} valu {m.get('SQ_INSTS_VALU',0)/w:.0f} lds {m.get('SQ_INSTS_LDS',0)/w:.0f} salu {m.get('SQ_INSTS_SALU',0)/w:.0f} vmem_rd {m.get('SQ_INSTS_VMEM_RD',0)/w:.0f} vmem_wr {m.get('SQ_INSTS_VMEM_WR',0)/w:.0f}"
          f"  wait_any {m.get('SQ_WAIT_ANY',0)/max(wc,1):.2f} wait_inst {m.get('SQ_WAIT_INST_ANY',0)/max(wc,1):.2f} active {m.get('SQ_ACTIVE_INST_ANY',0)/max(wc,1):.2f} lds_stall {m.get('SQ_WAIT_INST_LDS',0)/max(wc,1):.2f} bankconf {m.get('SQ_LDS_BANK_CONFLICT',0)/max(m.get('SQ_INSTS_LDS',1),1):.2f}")
PY
