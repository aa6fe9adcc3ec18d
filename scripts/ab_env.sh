#!/bin/bash
# A/B runtime knobs on one config: each entry of ENVS ("NAME=V,NAME2=V2" or "-" for none) is
# exported for one bench.py run, ROUNDS interleaved rounds.  ENVS="- AM_LANE_OCC=7" CFG=c4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
CFG=${CFG:-c4}
for r in $(seq 1 ${ROUNDS:-2}); do
  for e in $ENVS; do
    tag=$(echo "$e" | tr ',=' '__')
    if [ "$e" = "-" ]; then envs=(); else IFS=',' read -ra envs <<< "$e"; fi
    timeout -k 10 300 env "${envs[@]}" python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline \
      > $OUT/abe_${CFG}_${tag}_$r.json 2> $OUT/abe_${CFG}_${tag}_$r.err
    rc=$?; echo "[abe $CFG $e $r] rc=$rc $(python -c "import json;d=json.load(open('$OUT/abe_${CFG}_${tag}_$r.json'));print(round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))" 2>/dev/null)" | tee -a $OUT/steps.log
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
echo done
