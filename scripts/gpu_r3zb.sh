# round 3zb: SQ counters of the lean segmented FSST kernel (l_comment SF10)
set -o pipefail
mkdir -p gpurun_out/r3
export FLS_FSST_VARIANT=4477
bash scripts/gpu_fsst_sq.sh fsst_kernel lean > gpurun_out/r3/fsst_sq_lean_r3zb.txt 2>&1
rc=$?; cat gpurun_out/r3/fsst_sq_lean_r3zb.txt | grep -v amdgpu; exit $rc
