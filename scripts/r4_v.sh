#!/bin/bash
# round-4 iteration V: the group wave kernel at 5 waves per SIMD on the final code (lib_o5) --
# zone / config tests with it, then C3 fresh and cached A/B against lib_cur.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp antidote_amd/libantidote_mat.so /tmp/intree.so
cp scripts/ab/lib_o5.so antidote_amd/libantidote_mat.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_zones.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_o5.log 2>&1
rc=$?; echo "pytest(o5) rc=$rc" >> gpurun_out/steps.log
cp /tmp/intree.so antidote_amd/libantidote_mat.so
if [ $rc -ne 0 ]; then exit $rc; fi
VARS="cur o5" CFG=c3 ROUNDS=3 bash scripts/ab_libs.sh || exit $?
BENCH_EXTRA="--base cached" VARS="cur o5" CFG=c3 ROUNDS=1 bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
echo done >> gpurun_out/steps.log
