#!/bin/bash
# A/B whole-library variants (scripts/ab/lib_<V>.so, built with different compile-time
# kernel parameters) on one config: each variant is copied over the in-tree library of this
# box's scratch copy and timed by bench.py, ROUNDS interleaved rounds.  VARS="A B ..." CFG=c4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
CFG=${CFG:-c4}
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARS; do
    cp scripts/ab/lib_$v.so antidote_amd/libantidote_mat.so
    timeout -k 10 300 python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-secondary ${BENCH_EXTRA:-} > $OUT/ab_${CFG}_${v}_$r.json 2> $OUT/ab_${CFG}_${v}_$r.err
    rc=$?; echo "[ab $CFG $v $r] rc=$rc $(python -c "import json;d=json.load(open('$OUT/ab_${CFG}_${v}_$r.json'));print(round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))" 2>/dev/null)" | tee -a $OUT/steps.log
    if [ $rc -ge 124 ]; then exit $rc; fi  # a time limit or a signal: stop; an error: next variant
  done
done
echo done
