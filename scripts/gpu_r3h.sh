# round 3h (5-wave budget): segmented FSST kernel: two segments per lane per round (cap 4096 / 6144)
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/ab_env.py --workload lineitem_full --scale 10 --cols 15 --rounds 7 \
   --arms "spl:FLS_FSST_VARIANT=109" "wide:FLS_FSST_VARIANT=125" "double:FLS_FSST_VARIANT=253" "double6k:FLS_FSST_VARIANT=253,FLS_FSST_SEG_CAP=6144" "cp:FLS_FSST_SEG=0" > gpurun_out/r3/abenv_fsst_double_r3h.txt 2>&1 &&
FLS_FSST_VARIANT=253 FLS_FSST_SEG_CAP=6144 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_alp_fsst.py -m gpu > gpurun_out/r3/pt_fsst_r3h.log 2>&1
