#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Stops at the first step that faults/aborts/times out (exit >= 2 other than pytest's 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STEPS="${STEPS:-pytest smoke bench prof}"
ok() { local rc=$1 name=$2; echo "[$name] rc=$rc" | tee -a $OUT/steps.log; if [ $rc -ge 2 ] || [ $rc -lt 0 ]; then echo "stopping after $name" | tee -a $OUT/steps.log; exit $rc; fi; }
for s in $STEPS; do
  case $s in
    pytest) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; ok $? pytest ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; ok $? smoke ;;
    bench) timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err; ok $? bench ;;
    gc) timeout -k 10 300 python scripts/bench_gc.py > $OUT/gc_bench.json 2> $OUT/gc_bench.err; ok $? gc ;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1; ok $? prof ;;
  esac
done
echo done | tee -a $OUT/steps.log
