#!/bin/bash
# One GPU iteration on one box: optional GPU tests of the in-tree library, then interleaved A/B
# rounds of library variants (scripts/build_variant.sh -> scripts/ab/lib_<V>.so) per config.
#   TESTS="tests/test_gpu_zones.py ..."   pytest targets first (empty: skip; "all": tests -m gpu)
#   AB="c3:cur,new:2 c4:cur,new:1:--base=cached,--index=summaries"   CFG:VARIANTS:ROUNDS[:bench args, comma-separated]
#   PMC="c4:cur,new"                       optional SQ counter passes (scripts/pmc_sq.sh)
# Every step is time-limited; a failing test run stops the iteration; the in-tree library is
# restored at the end.  Results land in gpurun_out/ (steps.log, ab_*.json).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  if [ "$TESTS" = all ]; then T="tests -m gpu"; else T="$TESTS -m gpu"; fi
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest $T -q --maxfail=4 --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
cp antidote_amd/libantidote_mat.so /tmp/intree.so
for spec in ${AB:-}; do
  IFS=: read -r cfg vars rounds extra <<< "$spec"
  VARS="${vars//,/ }" CFG=$cfg ROUNDS=${rounds:-2} BENCH_EXTRA="${extra//,/ }" bash scripts/ab_libs.sh || exit $?
done
for spec in ${PMC:-}; do
  IFS=: read -r cfg vars <<< "$spec"
  VARS="${vars//,/ }" CFG=$cfg bash scripts/pmc_sq.sh || exit $?
done
cp /tmp/intree.so antidote_amd/libantidote_mat.so
echo done >> gpurun_out/steps.log
