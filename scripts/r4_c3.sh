#!/bin/bash
# round-4 iteration for the cached C3 path: GPU tests on the in-tree library, A/B of the
# cached read against the previous library, and a kernel-trace profile of the new one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/steps.log
  if [ $rc -ge 2 ]; then exit $rc; fi
fi
cp antidote_amd/libantidote_mat.so /tmp/intree.so
VARS="${C3_VARS:-cur hint}" CFG=c3 ROUNDS=${ROUNDS:-2} BENCH_EXTRA="--base cached" bash scripts/ab_libs.sh || exit $?
cp /tmp/intree.so antidote_amd/libantidote_mat.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3c -o run -- python bench.py --config c3 --base cached --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c3c.json 2> gpurun_out/prof_c3c.err || exit $?
echo done >> gpurun_out/steps.log
