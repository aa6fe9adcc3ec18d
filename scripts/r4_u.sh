#!/bin/bash
# round-4 iteration U: the leading zones' summary words stored after the tile loop, so their
# loads overlap the records and tile loads (in-tree, lib_sl) -- zone tests, then C3 A/B against
# lib_cur.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_zones.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_zones.log 2>&1
rc=$?; echo "pytest zones(sl) rc=$rc" >> gpurun_out/steps.log
if [ $rc -ne 0 ]; then exit $rc; fi
cp antidote_amd/libantidote_mat.so /tmp/intree.so
VARS="cur sl" CFG=c3 ROUNDS=3 bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
echo done >> gpurun_out/steps.log
