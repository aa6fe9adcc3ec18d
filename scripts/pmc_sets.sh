#!/bin/bash
# Experiments only: counter passes (one rocprofv3 --pmc run each) for library variants
# scripts/ab/lib_<v>.so on one config.  VARS="old quad" CFG=c4 PASSES="A B"
#   A: SQ instruction mix and waits      B: TA / TD / TCP pipeline
#   F: FETCH_SIZE                         W: WRITE_SIZE
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
CFG=${CFG:-c4}
for v in ${VARS:-old quad}; do
  for p in ${PASSES:-A B}; do
    case $p in
      A) ctr="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" ;;
      B) ctr="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE" ;;
      F) ctr="FETCH_SIZE" ;;
      W) ctr="WRITE_SIZE" ;;
    esac
    AM_LIB=$PWD/scripts/ab/lib_$v.so timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/pm_${CFG}_${v}_$p -o pmc --output-format csv -- python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pm_${CFG}_${v}_$p.log 2>&1
    rc=$?; echo "[pmc $CFG $v $p] rc=$rc" | tee -a $OUT/steps.log
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
echo done
