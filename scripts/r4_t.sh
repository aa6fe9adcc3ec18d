#!/bin/bash
# round-4 iteration T: cached reads skip the records of their leading zones inside the base
# (in-tree, lib_cs) -- tests, then C3 cached A/B against lib_gs8 and C3 fresh once.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_zones.py tests/test_gpu_bigview.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_zones.log 2>&1
rc=$?; echo "pytest zones(cs) rc=$rc" >> gpurun_out/steps.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=4 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest(cs) rc=$rc" >> gpurun_out/steps.log
if [ $rc -ge 2 ]; then exit $rc; fi
cp antidote_amd/libantidote_mat.so /tmp/intree.so
BENCH_EXTRA="--base cached" VARS="gs8 cs" CFG=c3 ROUNDS=2 bash scripts/ab_libs.sh || exit $?
VARS="gs8 cs" CFG=c3 ROUNDS=1 bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
echo done >> gpurun_out/steps.log
