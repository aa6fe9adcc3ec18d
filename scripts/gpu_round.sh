#!/bin/bash
# One GPU-box session for the round's record: parity tests, smoke, the default bench (C3),
# C2/C4/C5 bench lines, the GC bench, kernel-trace stats of every config and PMC HBM
# traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the configs in $PMC_CFGS.
# Every step runs under its own time limit; the first GPU failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STEPS="${STEPS:-pytest smoke bench benches gc prof pmc}"
ok() { local rc=$1 name=$2; echo "[$name] rc=$rc" | tee -a $OUT/steps.log; if [ $rc -ne 0 ] && [ "$name" != pytest ]; then echo "stopping after $name" | tee -a $OUT/steps.log; exit $rc; fi; if [ $rc -ge 2 ]; then exit $rc; fi; }
for s in $STEPS; do
  case $s in
    pytest) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; ok $? pytest ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; ok $? smoke ;;
    bench) timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err; ok $? bench ;;
    benches) for c in ${BENCH_CFGS:-c2 c4 c5}; do timeout -k 10 400 python bench.py --config $c ${BENCH_ARGS:-} > $OUT/bench_$c.json 2> $OUT/bench_$c.err; ok $? bench_$c; done ;;
    gc) timeout -k 10 300 python scripts/bench_gc.py > $OUT/gc_bench.json 2> $OUT/gc_bench.err; ok $? gc ;;
    cached) timeout -k 10 600 python bench.py --base cached > $OUT/bench_c3_cached.json 2> $OUT/bench_c3_cached.err; ok $? cached ;;
    profcached) timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3_cached -o run --output-format csv -- python bench.py --base cached --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_c3_cached.json 2> $OUT/prof_c3_cached.log; ok $? profcached ;;
    pmccached)
           timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmcf_c3_cached -o pmc --output-format csv -- python bench.py --base cached --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmcf_c3_cached.log 2>&1; ok $? pmcf_c3_cached
           timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw_c3_cached -o pmc --output-format csv -- python bench.py --base cached --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmcw_c3_cached.log 2>&1; ok $? pmcw_c3_cached ;;
    escape) for spec in ${ESC_SPECS:-c3:0.01 c3:0.1 c2:0.1 c4:0.1 c5:0.1}; do c=${spec%%:*}; e=${spec#*:}; timeout -k 10 300 python bench.py --config $c --escape $e --no-secondary --no-cpu-baseline > $OUT/esc_${c}_$e.json 2> $OUT/esc_${c}_$e.err; ok $? esc_${c}_$e; done ;;
    ingest) timeout -k 10 400 python scripts/bench_ingest.py ${INGEST_ARGS:-} > $OUT/ingest.json 2> $OUT/ingest.err; ok $? ingest ;;
    prof) for c in ${PROF_CFGS:-c2 c3 c4 c5}; do timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline ${PROF_ARGS:-} > $OUT/prof_$c.json 2> $OUT/prof_$c.log; ok $? prof_$c; done ;;
    pmc) for c in ${PMC_CFGS:-c4 c5}; do
           timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmcf_$c -o pmc --output-format csv -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/pmcf_$c.log 2>&1; ok $? pmcf_$c
           timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw_$c -o pmc --output-format csv -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > $OUT/pmcw_$c.log 2>&1; ok $? pmcw_$c
         done ;;
  esac
done
echo done | tee -a $OUT/steps.log
