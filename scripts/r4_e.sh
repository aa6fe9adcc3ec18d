#!/bin/bash
# round-4 iteration E: GPU tests (in-tree), cached C3 A/B (per-tile zone test / one round per
# read / + entry-major cache), C4 A/B (4 / 2 quad phases in flight).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/steps.log
if [ $rc -ge 2 ]; then exit $rc; fi
cp antidote_amd/libantidote_mat.so /tmp/intree.so
VARS="z7 zb em" CFG=c3 ROUNDS=2 BENCH_EXTRA="--base cached" bash scripts/ab_libs.sh || exit $?
VARS="em q2" CFG=c4 ROUNDS=3 bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3c -o run --output-format csv -- python bench.py --config c3 --base cached --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c3c.log 2>&1 || exit $?
echo done >> gpurun_out/steps.log
