#!/bin/bash
# FSST occupancy: the zero-at-flush kernel at 6 (default build, variant 12),
# 7 and 8 waves per SIMD (separate builds, variant 4), l_comment SF10,
# interleaved separate processes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for arm in "libflsgpu.so 12" "libflsgpu_w7.so 4" "libflsgpu_w8.so 4"; do
    set -- $arm
    r=$(FLS_LIB=$1 FLS_FSST_VARIANT=$2 timeout -k 10 120 python scripts/fsst_prof.py --reps 20 2>&1 | grep "per launch") || exit 1
    echo "$1 v$2: $r"
  done
done
