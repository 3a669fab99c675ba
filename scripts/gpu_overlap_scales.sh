#!/bin/bash
# Overlap vs serial FSST at the per-GPU shares of 1/2/4/8-GPU runs.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/abenv_overlap_scales.txt
for SC in ${SCALES:-25 50 100}; do
  echo "== SF$SC" >> gpurun_out/abenv_overlap_scales.txt
  timeout -k 10 400 python scripts/ab_env.py --workload lineitem_full --scale $SC --rounds 5 --cols all --arms \
    d1f16: d1f12:FLS_OVERLAP_FSST_WPC=12 serial:FLS_OVERLAP_FSST_WPC=0 >> gpurun_out/abenv_overlap_scales.txt 2>&1 || exit $?
done
grep -v amdgpu gpurun_out/abenv_overlap_scales.txt
