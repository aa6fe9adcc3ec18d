cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in cur old; do
  if [ $v = old ]; then export AM_LIB=scripts/ab/lib_oldplan.so; else unset AM_LIB; fi
  timeout -k 10 300 python -u scripts/debug_mixed.py c5_hot 3 > gpurun_out/dbg_$v.log 2>&1
  rc=$?; echo "[dbg $v] rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
