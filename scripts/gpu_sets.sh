#!/bin/bash
# Parity tests, then the set-heavy bench configs (c3, c4, c5) with kernel stats for c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1; shift; "$@"; local rc=$?; echo "[$name] rc=$rc" | tee -a $OUT/steps.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
for c in ${CFGS:-c3 c5 c4}; do
  step bench_$c bash -c "timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline ${BARGS:-} > $OUT/bench_$c.json 2> $OUT/bench_$c.err"
done
if [ -n "${PROF:-}" ]; then
  for c in $PROF; do
    step prof_$c timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof_$c.log 2>&1
  done
fi
echo done
