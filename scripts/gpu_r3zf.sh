# round 3zf: FSST waves per CU (standalone launch, FLS_FSST_WPC) on the lean
# kernel, and the 8 KB variant at the lean kernel's 16 waves per CU
set -o pipefail
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
FLS_FSST_VARIANT=20861 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_alp_fsst.py tests/test_gpu_random.py -m gpu > gpurun_out/r3/pt_fsst_lazy_r3zf.log 2>&1 &&
timeout -k 10 400 python -u scripts/ab_env.py --workload lineitem_full --scale 10 --cols 15 --rounds 9 \
   --arms "lean16:FLS_FSST_VARIANT=4477" "lean12:FLS_FSST_VARIANT=4477,FLS_FSST_WPC=12" "lean14:FLS_FSST_VARIANT=4477,FLS_FSST_WPC=14" \
          "lean8:FLS_FSST_VARIANT=4477,FLS_FSST_WPC=8" "d8_16:FLS_FSST_VARIANT=12669,FLS_FSST_WPC=16" "lazy:FLS_FSST_VARIANT=20861" "lazy12:FLS_FSST_VARIANT=20861,FLS_FSST_WPC=12" > gpurun_out/r3/abenv_fsst_wpc_r3zf.txt 2>&1
rc=$?; tail -2 gpurun_out/r3/pt_fsst_lazy_r3zf.log; grep -v amdgpu gpurun_out/r3/abenv_fsst_wpc_r3zf.txt | tail -3; exit $rc
