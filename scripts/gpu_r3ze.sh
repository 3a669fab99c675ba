# round 3ze: 8 KB-per-wave FSST variant (kFsstSegD8, 20 waves per CU):
# parity with the variant forced, then same-buffer A/B against the default
# on l_comment SF10 and on the SF12.5 table (serial)
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
FLS_FSST_VARIANT=12669 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_alp_fsst.py tests/test_gpu_random.py -m gpu > gpurun_out/r3/pt_fsst_d8_r3ze.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_env.py --workload lineitem_full --scale 10 --cols 15 --rounds 9 \
   --arms "lean:FLS_FSST_VARIANT=4477" "d8:FLS_FSST_VARIANT=12669" > gpurun_out/r3/abenv_fsst_d8_r3ze.txt 2>&1 &&
timeout -k 10 400 python -u scripts/ab_env.py --workload lineitem_full --scale 12.5 --rounds 9 \
   --arms "lean:FLS_FSST_VARIANT=4477" "d8:FLS_FSST_VARIANT=12669" > gpurun_out/r3/abenv_sf12_d8_r3ze.txt 2>&1
rc=$?; tail -3 gpurun_out/r3/pt_fsst_d8_r3ze.log; grep -v amdgpu gpurun_out/r3/abenv_*_r3ze.txt | tail -6; exit $rc
