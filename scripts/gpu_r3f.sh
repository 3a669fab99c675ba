# round 3f: is the segmented FSST kernel occupancy(latency)-bound?  waves per CU A/B
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/ab_env.py --workload lineitem_full --scale 10 --cols 15 --rounds 7 \
   --arms "w21:FLS_FSST_VARIANT=109" "w16:FLS_FSST_VARIANT=109,FLS_FSST_WPC=16" "w12:FLS_FSST_VARIANT=109,FLS_FSST_WPC=12" "w8:FLS_FSST_VARIANT=109,FLS_FSST_WPC=8" "wide:FLS_FSST_VARIANT=125" "wide16:FLS_FSST_VARIANT=125,FLS_FSST_WPC=16" "cp:FLS_FSST_SEG=0" "cp16:FLS_FSST_SEG=0,FLS_FSST_WPC=16" > gpurun_out/r3/abenv_fsst_wpc_r3f.txt 2>&1
