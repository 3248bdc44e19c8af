#!/bin/bash
# PMC passes (one rocprofv3 run each, kernel-trace only) over the bf16 forward (tools/fwd_ab.py):
#   bash tools/fwd_pmc.sh TAG [passes]   -> gpurun_out/fpmc_TAG/summary.txt
T=${1:-x}
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fpmc_$T; mkdir -p $O
i=0
for set in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU" \
           "TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  case ",${2:-1,2,3,4,5,6,7}," in *",$i,"*) ;; *) continue ;; esac
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p$i -o run -- python3 tools/fwd_ab.py pmc 2 > $O/p$i.log 2>&1; rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $(find $O -name '*counter_collection.csv') > $O/summary.txt 2>&1
cat $O/summary.txt
