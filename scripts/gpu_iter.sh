#!/bin/bash
# One GPU iteration (edited per experiment): parity of the touched paths (in-tree library), then
# C3 A/B of the in-tree library against scripts/ab/lib_db.so, then kernel stats of the better.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_zones.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu > gpurun_out/t8.log 2>&1 || exit 1
cp antidote_amd/libantidote_mat.so scripts/ab/lib_cur.so
AB="c3:cur,db:2" bash scripts/ab_round.sh || exit 2
cp scripts/ab/lib_db.so antidote_amd/libantidote_mat.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/prof8.json 2> gpurun_out/prof8.err || exit 3
