#!/bin/bash
# PMC passes on GEMM kernels:  bash tools/pmc_gemm.sh TAG TILE SHAPES [PASSES]   (e.g. t11 11 ref4096,ffn_up 1,2,3)
# (TA_* counters are not collected: a TA pass ran past its 120 s limit on MI355X.)
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmcg_$1; mkdir -p $O
i=0
for set in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU" \
           "TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  case ",${4:-1,2,3,4,5}," in *",$i,"*) ;; *) continue ;; esac
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p$i -o run -- python3 tools/op_driver.py gemm 5 $2 $3 > $O/p$i.log 2>&1; rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
