# round 3zm: overlapped vs serial FSST at SF50 and SF100 with the round-3
# FSST kernel (same-buffer A/B), to place FLS_OVERLAP_MIN_VECS_PER_CU
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3
timeout -k 10 500 python -u scripts/ab_env.py --workload lineitem_full --scale 50 --rounds 5 \
   --arms "ovl:FLS_OVERLAP_MIN_VECS_PER_CU=0" "ser:FLS_OVERLAP_FSST_WPC=0" > gpurun_out/r3/abenv_sf50_split_r3zm.txt 2>&1 &&
timeout -k 10 600 python -u scripts/ab_env.py --workload lineitem_full --scale 100 --rounds 5 \
   --arms "ovl:FLS_OVERLAP_MIN_VECS_PER_CU=0" "ser:FLS_OVERLAP_FSST_WPC=0" > gpurun_out/r3/abenv_sf100_split_r3zm.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/r3/abenv_sf50_split_r3zm.txt | tail -1; grep -v amdgpu gpurun_out/r3/abenv_sf100_split_r3zm.txt | tail -1; exit $rc
