# round 3za: lean FSST writer (lengths in bits, tagged entries) -- parity with
# the variant forced, then same-buffer A/B against the default
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
FLS_FSST_VARIANT=4477 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_alp_fsst.py tests/test_gpu_random.py -m gpu > gpurun_out/r3/pt_fsst_lean_r3za.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_env.py --workload lineitem_full --scale 10 --cols 15 --rounds 7 \
   --arms "wb5k:FLS_FSST_VARIANT=381" "lean:FLS_FSST_VARIANT=4477" "cp:FLS_FSST_SEG=0" > gpurun_out/r3/abenv_fsst_lean_r3za.txt 2>&1
rc=$?; tail -3 gpurun_out/r3/pt_fsst_lean_r3za.log; cat gpurun_out/r3/abenv_fsst_lean_r3za.txt | grep -v amdgpu | tail -5; exit $rc
