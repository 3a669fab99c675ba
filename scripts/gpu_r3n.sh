# round 3n: the 8-GPU share (lineitem_full SF12.5 on one GPU): FSST after vs beside the main kernel
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u scripts/ab_env.py --workload lineitem_full --scale 12.5 --cols all --rounds 9 \
   --arms "serial:FLS_OVERLAP_MIN_VECS_PER_CU=400" "overlap:FLS_OVERLAP_MIN_VECS_PER_CU=0" "overlap8:FLS_OVERLAP_MIN_VECS_PER_CU=0,FLS_OVERLAP_FSST_WPC=8" "overlap16:FLS_OVERLAP_MIN_VECS_PER_CU=0,FLS_OVERLAP_FSST_WPC=16" > gpurun_out/r3/abenv_sf12p5_r3n.txt 2>&1
