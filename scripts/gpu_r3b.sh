# round 3b: segmented FSST kernel on escape-free l_comment (encoder: one-byte
# symbol for every byte present): A/B vs the code-parallel kernel + SQ counters
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_alp_fsst.py -m gpu > gpurun_out/r3/pt_fsst_r3b.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_env.py --workload lineitem_full --scale 10 --cols 15 --rounds 7 \
   --arms "seg:FLS_FSST_SEG=1" "seg3072:FLS_FSST_SEG_CAP=3072" "cp:FLS_FSST_SEG=0" > gpurun_out/r3/abenv_fsst_seg_r3b.txt 2>&1 &&
bash scripts/gpu_fsst_sq.sh fsst_kernelILi16 seg_r3b > gpurun_out/r3/fsst_sq_seg_r3b.txt 2>&1
