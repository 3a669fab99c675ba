# round 3zg: FSST waves per CU between 16 and 20 (the 8 KB variant fits 20;
# 20 measured 27 % slower than 16 in r3ze/r3zf), with and without lazy
# ring compaction
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
FLS_FSST_VARIANT=29053 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_alp_fsst.py -m gpu > gpurun_out/r3/pt_fsst_d8lazy_r3zg.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_env.py --workload lineitem_full --scale 10 --cols 15 --rounds 9 \
   --arms "lean16:FLS_FSST_VARIANT=4477" "d8_17:FLS_FSST_VARIANT=12669,FLS_FSST_WPC=17" "d8_18:FLS_FSST_VARIANT=12669,FLS_FSST_WPC=18" \
          "d8_19:FLS_FSST_VARIANT=12669,FLS_FSST_WPC=19" "d8_20:FLS_FSST_VARIANT=12669" "d8lazy_16:FLS_FSST_VARIANT=29053,FLS_FSST_WPC=16" "d8lazy_18:FLS_FSST_VARIANT=29053,FLS_FSST_WPC=18" "lazy:FLS_FSST_VARIANT=20861" > gpurun_out/r3/abenv_fsst_wpc_r3zg.txt 2>&1
rc=$?; tail -2 gpurun_out/r3/pt_fsst_d8lazy_r3zg.log; grep -v amdgpu gpurun_out/r3/abenv_fsst_wpc_r3zg.txt | tail -3; exit $rc
