# round 3i: segmented FSST kernel with batched records: variants x ring caps (same buffers)
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_alp_fsst.py -m gpu > gpurun_out/r3/pt_fsst_r3i.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_env.py --workload lineitem_full --scale 10 --cols 15 --rounds 7 \
   --arms "w6k:FLS_FSST_VARIANT=125" "w5k:FLS_FSST_VARIANT=125,FLS_FSST_SEG_CAP=5120" "d6k:FLS_FSST_VARIANT=253" "d5k:FLS_FSST_VARIANT=253,FLS_FSST_SEG_CAP=5120" "base6k:FLS_FSST_VARIANT=76" "cp:FLS_FSST_SEG=0" > gpurun_out/r3/abenv_fsst_batch_r3i.txt 2>&1 &&
FLS_FSST_VARIANT=253 timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_alp_fsst.py -m gpu -k "escape or agree or corrupt or full_fidelity" > gpurun_out/r3/pt_fsst_d_r3i.log 2>&1
