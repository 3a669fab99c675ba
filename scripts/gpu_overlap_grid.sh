#!/bin/bash
# Overlap grid split A/B (same buffers, interleaved) at the per-GPU share of
# an 8-GPU run (SF12.5) and at SF100: narrow decode blocks per CU (d) x FSST
# waves per CU (f), against serial (f = 0).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/abenv_overlap_grid.txt
: > $OUT
for SC in ${SCALES:-12.5 100}; do
  echo "== SF$SC" >> $OUT
  timeout -k 10 500 python scripts/ab_env.py --workload lineitem_full --scale $SC --rounds 5 --cols all --arms \
    d1f12: serial:FLS_OVERLAP_FSST_WPC=0 d4f24:FLS_OVERLAP_DECODE_BPC=4,FLS_OVERLAP_FSST_WPC=24 \
    d1f6:FLS_OVERLAP_FSST_WPC=6 d1f4:FLS_OVERLAP_FSST_WPC=4 d3f8:FLS_OVERLAP_DECODE_BPC=3,FLS_OVERLAP_FSST_WPC=8 \
    >> $OUT 2>&1 || exit $?
done
grep -v amdgpu $OUT
