#!/bin/bash
# Wave issue priority of the main decode kernel while it runs beside the FSST
# kernel (FLS_OVERLAP_DECODE_PRIO, s_setprio): same-buffer A/B at the 8-GPU
# share (SF12.5) and at SF100.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/abenv_overlap_prio.txt
: > $OUT
for SC in ${SCALES:-12.5 100}; do
  echo "== SF$SC" >> $OUT
  timeout -k 10 500 python scripts/ab_env.py --workload lineitem_full --scale $SC --rounds 5 --cols all --arms \
    p0: p1:FLS_OVERLAP_DECODE_PRIO=1 p2:FLS_OVERLAP_DECODE_PRIO=2 p3:FLS_OVERLAP_DECODE_PRIO=3 \
    serial:FLS_OVERLAP_FSST_WPC=0 >> $OUT 2>&1 || exit $?
done
grep -v amdgpu $OUT
