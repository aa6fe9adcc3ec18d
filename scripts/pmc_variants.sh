#!/bin/bash
# Experiments only: FETCH_SIZE / WRITE_SIZE of the C3 wave kernel for library variants
# (antidote_amd/lib_<v>.so built with -DAMK_SKIP=<mask>), one rocprofv3 pass per counter.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
for v in ${VARS:-s2 s3 s7}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    AM_LIB=$PWD/antidote_amd/lib_$v.so timeout -s KILL 300 rocprofv3 --pmc $c -d $OUT/pv_${v}_$c -o pmc --output-format csv -- python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pv_${v}_$c.log 2>&1
    rc=$?; echo "[$v $c] rc=$rc" | tee -a $OUT/steps.log
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
