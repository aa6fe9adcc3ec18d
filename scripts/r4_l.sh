#!/bin/bash
# round-4 iteration L: the bounded-counter chain planned on its own stream beside the lane tier (in-tree, lib_bc)
# -- the whole GPU suite, then C5 A/B against the per-type-stream library (lib_ms), C4 too.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=4 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest(bc) rc=$rc" >> gpurun_out/steps.log
if [ $rc -ge 2 ]; then exit $rc; fi
cp antidote_amd/libantidote_mat.so /tmp/intree.so
VARS="ms bc" CFG=c5 ROUNDS=2 bash scripts/ab_libs.sh || exit $?
VARS="ms bc" CFG=c4 ROUNDS=2 bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
echo done >> gpurun_out/steps.log
