#!/bin/bash
# round-4 iteration J: grouped MV big reads in two passes, inclusion then records (lib_gs) --
# its parity tests, then C5 A/B against the in-tree library (ez).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp antidote_amd/libantidote_mat.so /tmp/intree.so
cp scripts/ab/lib_gs.so antidote_amd/libantidote_mat.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_bigview.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -q --maxfail=4 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest(gs) rc=$rc" >> gpurun_out/steps.log
cp /tmp/intree.so antidote_amd/libantidote_mat.so
if [ $rc -ge 2 ]; then exit $rc; fi
VARS="ez gs" CFG=c5 ROUNDS=2 bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
echo done >> gpurun_out/steps.log
