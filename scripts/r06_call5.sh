cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for c in c5_hot c5_mv_bc_zipf c4_mixed; do
  timeout -k 10 300 python -u scripts/debug_mixed.py $c 3 > gpurun_out/dbg_$c.log 2>&1
  rc=$?; echo "[dbg $c] rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "[pytest] rc=$rc" | tee -a gpurun_out/steps.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "[bench] rc=$?" | tee -a gpurun_out/steps.log
