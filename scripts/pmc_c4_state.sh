#!/bin/bash
# C4's two states in one process (scripts/c4_state_probe.py: "plain" then "c3first"), one PMC
# pass per counter set with the kernel trace beside it, so every k_lane_q dispatch carries its
# duration and counters.  scripts/pmc_c4_state.py splits the dispatches at the C3 work.
#   bash scripts/pmc_c4_state.sh            (all sets)      SETS="tlb tcc" bash ... (some)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
declare -A C
C[tlb]="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_GUI_ACTIVE"
C[tcc]="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TA_BUSY_avr GRBM_GUI_ACTIVE"
C[lat]="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_SERIALIZATION_STALL_sum TD_BUSY_avr GRBM_GUI_ACTIVE"
C[sq]="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES"
C[ea]="TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE"
for s in ${SETS:-tlb tcc lat sq ea}; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc ${C[$s]} -d $OUT/c4state_$s -o pmc --output-format csv \
    -- python scripts/c4_state_probe.py ${MODES:-plain c3first} > $OUT/c4state_$s.log 2>&1
  rc=$?; echo "[c4state $s] rc=$rc" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done
