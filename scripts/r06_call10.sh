cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "[pytest] rc=$rc" | tee -a gpurun_out/steps.log
if [ $rc -gt 1 ]; then exit $rc; fi
for spec in c3:0 c3:0.01 c3:0.1 c4:0 c4:0.01 c4:0.1 c5:0 c5:0.1 c2:0 c2:0.1; do
  c=${spec%%:*}; e=${spec#*:}
  timeout -k 10 300 python bench.py --config $c --escape $e --no-secondary --no-cpu-baseline > gpurun_out/esc_${c}_$e.json 2> gpurun_out/esc_${c}_$e.err
  rc=$?; echo "[esc $c $e] rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/esc_${c}_$e.json'));print(round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))" 2>/dev/null)" | tee -a gpurun_out/steps.log
  if [ $rc -ge 124 ]; then exit $rc; fi
done
