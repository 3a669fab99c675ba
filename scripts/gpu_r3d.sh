# round 3d: segmented FSST kernel, accumulator vs sparse (complete-qword) stores (same buffers)
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/ab_env.py --workload lineitem_full --scale 10 --cols 15 --rounds 7 \
   --arms "seg:FLS_FSST_SEG=1" "seg_sparse:FLS_FSST_VARIANT=77" "cp:FLS_FSST_SEG=0" > gpurun_out/r3/abenv_fsst_sparse_r3d.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_alp_fsst.py -m gpu -k "escape or agree or corrupt" > gpurun_out/r3/pt_fsst_r3d.log 2>&1
