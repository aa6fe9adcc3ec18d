#!/bin/bash
# Kernel-trace stats of library variants (scripts/ab/lib_<V>.so) on one config:
#   VARS="cur new" CFG=c5 bash scripts/prof_variants.sh  -> gpurun_out/pv_<CFG>_<V>/run_kernel_stats.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp antidote_amd/libantidote_mat.so /tmp/intree.so
for v in $VARS; do
  cp scripts/ab/lib_$v.so antidote_amd/libantidote_mat.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pv_${CFG}_$v -o run --output-format csv -- python bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-secondary ${BENCH_EXTRA:-} > gpurun_out/pv_${CFG}_$v.json 2> gpurun_out/pv_${CFG}_$v.err || exit 1
done
cp /tmp/intree.so antidote_amd/libantidote_mat.so
