#!/bin/bash
# SQ stall breakdown (SQ_WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY, instruction
# mix) of whole-library variants scripts/ab/lib_<V>.so on one config, one PMC pass each.
#   VARS="old new" CFG=c4 bash scripts/pmc_sq.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
CFG=${CFG:-c4}
CTRS=${CTRS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"}
for v in $VARS; do
  cp scripts/ab/lib_$v.so antidote_amd/libantidote_mat.so
  timeout -s KILL 300 rocprofv3 --pmc $CTRS -d $OUT/pmcsq_${CFG}_$v -o pmc --output-format csv -- python bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmcsq_${CFG}_$v.log 2>&1
  rc=$?; echo "[pmcsq $CFG $v] rc=$rc" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done
