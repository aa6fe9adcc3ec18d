#!/bin/bash
# round-4 iteration on one box: GPU tests (in-tree library), then A/B of library variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/steps.log
if [ $rc -ge 2 ]; then exit $rc; fi
cp antidote_amd/libantidote_mat.so /tmp/intree.so
VARS="${C4_VARS:-old cur gm2}" CFG=c4 ROUNDS=2 bash scripts/ab_libs.sh || exit $?
VARS="${C5_VARS:-cur big}" CFG=c5 ROUNDS=1 bash scripts/ab_libs.sh || exit $?
if [ -n "${PMC_VARS:-}" ]; then VARS="$PMC_VARS" CFG=c4 bash scripts/pmc_sq.sh || exit $?; fi
cp /tmp/intree.so antidote_amd/libantidote_mat.so
echo done >> gpurun_out/steps.log
