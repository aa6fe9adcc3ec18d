cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T="tests/test_gpu_configs.py -k mixed_batch"
for v in cur cur old old cur; do
  if [ $v = old ]; then export AM_LIB=scripts/ab/lib_oldplan.so; else unset AM_LIB; fi
  timeout -k 10 300 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_$v.log 2>&1
  rc=$?; echo "[mixed $v] rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -gt 1 ]; then exit $rc; fi
done
unset AM_LIB
AM_LIB=scripts/ab/lib_ph.so timeout -k 10 300 python scripts/phase_prof.py --c4 > gpurun_out/phase_c4.txt 2>&1
echo "[phase] rc=$?" | tee -a gpurun_out/steps.log
