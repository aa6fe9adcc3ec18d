#!/bin/bash
# round-4 iteration S: zone group summaries -- a fresh read takes its leading whole zones'
# born / killed words from the summaries and streams only the later records (in-tree, lib_gs8;
# ABI 8) -- the zone and parity tests, the whole GPU suite, then C3 A/B against the same tree
# without summaries (lib_ng8), C3 cached once.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_zones.py tests/test_gpu_bigview.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_zones.log 2>&1
rc=$?; echo "pytest zones(gs8) rc=$rc" >> gpurun_out/steps.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=4 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest(gs8) rc=$rc" >> gpurun_out/steps.log
if [ $rc -ge 2 ]; then exit $rc; fi
cp antidote_amd/libantidote_mat.so /tmp/intree.so
VARS="ng8 gs8" CFG=c3 ROUNDS=3 bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
echo done >> gpurun_out/steps.log
