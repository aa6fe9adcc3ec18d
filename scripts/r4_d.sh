#!/bin/bash
# round-4 iteration D: GPU tests (in-tree), cached C3 A/B (zone skip off / on), C5 A/B (bounded
# counters through k_big_chunk / k_big_run, bcounter wave limit 32768 / 4096), kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/steps.log
if [ $rc -ge 2 ]; then exit $rc; fi
cp antidote_amd/libantidote_mat.so /tmp/intree.so
VARS="nozone z7" CFG=c3 ROUNDS=2 BENCH_EXTRA="--base cached" bash scripts/ab_libs.sh || exit $?
VARS="chunkbc bcw32k z7" CFG=c5 ROUNDS=2 bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
CFGS="c5" bash scripts/prof_configs.sh || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3c -o run --output-format csv -- python bench.py --config c3 --base cached --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c3c.log 2>&1 || exit $?
echo done >> gpurun_out/steps.log
