#!/bin/bash
# The per-GPU share of an 8-GPU run (SF12.5): overlap-split A/B and a kernel trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python scripts/ab_env.py --workload lineitem_full --scale 12.5 --rounds 7 --cols all --arms \
  d1f16: d1f8:FLS_OVERLAP_FSST_WPC=8 d1f12:FLS_OVERLAP_FSST_WPC=12 d1f24:FLS_OVERLAP_FSST_WPC=24 \
  d2f16:FLS_OVERLAP_DECODE_BPC=2 d2f8:FLS_OVERLAP_DECODE_BPC=2,FLS_OVERLAP_FSST_WPC=8 serial:FLS_OVERLAP_FSST_WPC=0 \
  > gpurun_out/abenv_sf12p5.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/abenv_sf12p5.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_sf12p5 -o prof -- python3 bench.py --scale 12.5 --steps 10 --warmup 2 --cpu-seconds 0 --e2e-scale 0 --no-verify --no-traffic > gpurun_out/bench_prof_sf12p5.json 2> gpurun_out/bench_prof_sf12p5.log
echo "prof rc=$?"
