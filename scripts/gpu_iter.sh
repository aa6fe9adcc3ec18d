#!/bin/bash
# One GPU iteration (edited per experiment): kernel trace + FETCH/WRITE bytes of the C3 read kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof12 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/prof12.json 2> gpurun_out/prof12.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc12f -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > gpurun_out/pmc12f.log 2>&1 || exit 2
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc12w -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > gpurun_out/pmc12w.log 2>&1 || exit 3
