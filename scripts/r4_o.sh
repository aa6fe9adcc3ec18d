#!/bin/bash
# round-4 iteration O: group wave kernel at 5 waves per SIMD (lib_o5) and with 1024-record
# chunks (lib_v16) -- their set-read parity tests, then C3 fresh and cached A/B against lib_cur.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp antidote_amd/libantidote_mat.so /tmp/intree.so
for v in o5 v16; do
  cp scripts/ab/lib_$v.so antidote_amd/libantidote_mat.so
  timeout -k 10 400 python -u -m pytest tests/test_gpu_zones.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_snapcache.py -m gpu -q --maxfail=4 --timeout 120 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1
  rc=$?; echo "pytest($v) rc=$rc" >> gpurun_out/steps.log
  if [ $rc -ge 2 ]; then cp /tmp/intree.so antidote_amd/libantidote_mat.so; exit $rc; fi
done
VARS="cur o5 v16" CFG=c3 ROUNDS=2 bash scripts/ab_libs.sh || exit $?
BENCH_EXTRA="--base cached" VARS="cur o5 v16" CFG=c3 ROUNDS=1 bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
echo done >> gpurun_out/steps.log
