cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "[pytest] rc=$rc" | tee -a gpurun_out/steps.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/prof_c3.json 2> gpurun_out/prof_c3.log
rc=$?; echo "[prof_c3] rc=$rc" | tee -a gpurun_out/steps.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 1000 bash scripts/pmc_c4_state.sh
