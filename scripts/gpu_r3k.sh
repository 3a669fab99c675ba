# round 3k: where the segmented FSST kernel's time goes (cost ablations, wrong output, same buffers)
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u scripts/ab_env.py --workload lineitem_full --scale 10 --cols 15 --rounds 7 \
   --arms "w4k:FLS_FSST_VARIANT=125" "no_records:FLS_FSST_VARIANT=637" "no_flush:FLS_FSST_VARIANT=1149" "no_write:FLS_FSST_VARIANT=2173" "cp:FLS_FSST_SEG=0" > gpurun_out/r3/abenv_fsst_ablate_r3k.txt 2>&1
