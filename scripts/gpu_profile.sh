#!/bin/bash
# Bench + kernel-trace stats + PMC traffic passes for one config (default c2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
CFG=${CFG:-c2}
run() { local name=$1; shift; "$@"; local rc=$?; echo "[$name] rc=$rc" >> $OUT/steps.log; echo "[$name] rc=$rc" >&2; if [ $rc -ne 0 ]; then exit $rc; fi; }
run bench timeout -k 10 600 python bench.py --config $CFG --steps 20 --warmup 3 > $OUT/bench_$CFG.json 2> $OUT/bench_$CFG.err
run stats timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$CFG -o run --output-format csv -- python bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_$CFG.log 2>&1
run pmc_fetch timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmcf_$CFG -o pmc --output-format csv -- python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmcf_$CFG.log 2>&1
run pmc_write timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw_$CFG -o pmc --output-format csv -- python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmcw_$CFG.log 2>&1
echo done | tee -a $OUT/steps.log
