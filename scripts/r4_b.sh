#!/bin/bash
# round-4 iteration B: GPU tests, cached C3 A/B (hints only vs hints + split copy), kernel
# stats of c5 / c4 / c3 with the in-tree library, SQ counters of c4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/steps.log
if [ $rc -ge 2 ]; then exit $rc; fi
cp antidote_amd/libantidote_mat.so /tmp/intree.so
VARS="sep tee" CFG=c3 ROUNDS=2 BENCH_EXTRA="--base cached" bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
CFGS="c5 c4" bash scripts/prof_configs.sh || exit $?
VARS="tee" CFG=c4 bash scripts/pmc_sq.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
echo done >> gpurun_out/steps.log
