#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over a short bench of $CFG (default c3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
CFG=${CFG:-c3}
PASSES=${PASSES:-"FETCH_SIZE WRITE_SIZE SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU"}
i=0
for p in $PASSES; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc ${p//,/ } -d $OUT/pmc${i}_$CFG -o pmc --output-format csv -- python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc${i}_$CFG.log 2>&1
  rc=$?; echo "[pmc $i $p] rc=$rc" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done | tee -a $OUT/steps.log
