#!/bin/bash
# One GPU iteration (edited per experiment): parity of the set paths with the in-tree library
# (record-pass kernel), then each prefetch variant's parity on the zone tests and a C3 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_zones.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_bigview.py -m gpu > gpurun_out/t10.log 2>&1 || exit 1
cp antidote_amd/libantidote_mat.so scripts/ab/lib_cur.so
for v in xr3 xr4; do
  cp scripts/ab/lib_$v.so antidote_amd/libantidote_mat.so
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_zones.py tests/test_gpu_configs.py -m gpu > gpurun_out/t10_$v.log 2>&1 || exit 2
done
cp scripts/ab/lib_cur.so antidote_amd/libantidote_mat.so
AB="c3:cur,xr3,xr4:2" bash scripts/ab_round.sh || exit 3
