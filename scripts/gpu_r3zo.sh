# round 3zo: FSST segmented kernel with a 4-wave register budget (kFsstSegW4,
# 101 VGPRs against 96): parity with the variant forced, same-buffer A/B
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
FLS_FSST_VARIANT=37245 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_alp_fsst.py -m gpu > gpurun_out/r3/pt_fsst_w4_r3zo.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_env.py --workload lineitem_full --scale 10 --cols 15 --rounds 9 \
   --arms "lean:FLS_FSST_VARIANT=4477" "w4:FLS_FSST_VARIANT=37245" > gpurun_out/r3/abenv_fsst_w4_r3zo.txt 2>&1
rc=$?; tail -2 gpurun_out/r3/pt_fsst_w4_r3zo.log; grep -v amdgpu gpurun_out/r3/abenv_fsst_w4_r3zo.txt | tail -1; exit $rc
