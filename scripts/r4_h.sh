#!/bin/bash
# round-4 iteration H: GPU tests (in-tree: exact zones in the big-read run kernel), C5 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/steps.log
if [ $rc -ge 2 ]; then exit $rc; fi
cp antidote_amd/libantidote_mat.so /tmp/intree.so
VARS="ez zr" CFG=c5 ROUNDS=2 bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
CFGS="c5" bash scripts/prof_configs.sh || exit $?
echo done >> gpurun_out/steps.log
