# round 3l: segmented FSST kernel with two-batch records + pipelined flush
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_alp_fsst.py -m gpu > gpurun_out/r3/pt_fsst_r3l.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_env.py --workload lineitem_full --scale 10 --cols 15 --rounds 7 \
   --arms "w4k:FLS_FSST_VARIANT=125" "wb5k:FLS_FSST_VARIANT=381" "no_records:FLS_FSST_VARIANT=637" "no_flush:FLS_FSST_VARIANT=1149" "cp:FLS_FSST_SEG=0" > gpurun_out/r3/abenv_fsst_r3l.txt 2>&1
