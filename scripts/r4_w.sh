#!/bin/bash
# round-4 iteration W: the lane tier waits for the early bounded-counter planner (in-tree,
# lib_bo) -- mixed-batch tests, then C5 A/B against lib_cur.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_readbatch.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bo.log 2>&1
rc=$?; echo "pytest(bo) rc=$rc" >> gpurun_out/steps.log
if [ $rc -ne 0 ]; then exit $rc; fi
cp antidote_amd/libantidote_mat.so /tmp/intree.so
VARS="cur bo" CFG=c5 ROUNDS=3 bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
echo done >> gpurun_out/steps.log
