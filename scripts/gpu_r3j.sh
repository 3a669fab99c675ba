# round 3j: segmented FSST kernel: per-round records (non-batched) vs batched, caps, double
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_alp_fsst.py -m gpu > gpurun_out/r3/pt_fsst_r3j.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_env.py --workload lineitem_full --scale 10 --cols 15 --rounds 7 \
   --arms "w4k:FLS_FSST_VARIANT=125" "w5k:FLS_FSST_VARIANT=125,FLS_FSST_SEG_CAP=5120" "wb5k:FLS_FSST_VARIANT=381" "d6k:FLS_FSST_VARIANT=253" "base4k:FLS_FSST_VARIANT=76" "cp:FLS_FSST_SEG=0" > gpurun_out/r3/abenv_fsst_r3j.txt 2>&1 &&
FLS_FSST_VARIANT=253 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_alp_fsst.py -m gpu -k "escape or agree or corrupt or full_fidelity" > gpurun_out/r3/pt_fsst_d_r3j.log 2>&1
