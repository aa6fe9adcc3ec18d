#!/bin/bash
# round-4 iteration M: the early bounded-counter chain only over logs with such keys (in-tree, lib_bt)
# -- the whole GPU suite, then C5 A/B against the per-type-stream library (lib_ms), C4 too.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=4 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest(bt) rc=$rc" >> gpurun_out/steps.log
if [ $rc -ge 2 ]; then exit $rc; fi
cp antidote_amd/libantidote_mat.so /tmp/intree.so
VARS="ms bt" CFG=c5 ROUNDS=2 bash scripts/ab_libs.sh || exit $?
VARS="ms bt" CFG=c4 ROUNDS=2 bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
echo done >> gpurun_out/steps.log
