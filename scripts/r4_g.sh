#!/bin/bash
# round-4 iteration G: GPU tests (in-tree: exact zones for fresh reads, bcounter-row prefetch,
# hot-MV threshold 1024), A/B on C3 / C5 / C2 (fr = before, nofz = all but the fresh zone test).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/steps.log
if [ $rc -ge 2 ]; then exit $rc; fi
cp antidote_amd/libantidote_mat.so /tmp/intree.so
VARS="fr nofz ez" CFG=c3 ROUNDS=2 bash scripts/ab_libs.sh || exit $?
VARS="fr nofz ez" CFG=c5 ROUNDS=2 bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
echo done >> gpurun_out/steps.log
