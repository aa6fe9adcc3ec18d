#!/bin/bash
# round-4 iteration R: big-read prep initializes bounded-counter slots one thread per slot; the grouped finish scans 8 bitmap words per thread
# (in-tree, lib_bf) -- the big-read tests first, the whole GPU suite, then C5 A/B
# against lib_cur.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bigview.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_bigview.log 2>&1
rc=$?; echo "pytest bigview(bf) rc=$rc" >> gpurun_out/steps.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=4 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest(bf) rc=$rc" >> gpurun_out/steps.log
if [ $rc -ge 2 ]; then exit $rc; fi
cp antidote_amd/libantidote_mat.so /tmp/intree.so
VARS="cur bf" CFG=c5 ROUNDS=3 bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
echo done >> gpurun_out/steps.log
