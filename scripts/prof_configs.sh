#!/bin/bash
# rocprofv3 kernel-trace stats for each config in $CFGS (default: c3 c4 c5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
for c in ${CFGS:-c3 c4 c5}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof_$c.log 2>&1
  rc=$?; echo "[prof $c] rc=$rc" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done
