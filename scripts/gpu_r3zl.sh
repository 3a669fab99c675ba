# round 3zl: SF12.5 (8-GPU per-GPU share) serial vs overlapped splits with
# the round-3 FSST kernel (same-buffer A/B), and the same at SF25
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3
timeout -k 10 500 python -u scripts/ab_env.py --workload lineitem_full --scale 12.5 --rounds 9 \
   --arms "ser:FLS_OVERLAP_MIN_VECS_PER_CU=100000" "ovl12:FLS_OVERLAP_MIN_VECS_PER_CU=0" \
          "ovl8:FLS_OVERLAP_MIN_VECS_PER_CU=0,FLS_OVERLAP_FSST_WPC=8" "ovl4:FLS_OVERLAP_MIN_VECS_PER_CU=0,FLS_OVERLAP_FSST_WPC=4" \
          "ovl12b2:FLS_OVERLAP_MIN_VECS_PER_CU=0,FLS_OVERLAP_DECODE_BPC=2" > gpurun_out/r3/abenv_sf12_split_r3zl.txt 2>&1 &&
timeout -k 10 500 python -u scripts/ab_env.py --workload lineitem_full --scale 25 --rounds 7 \
   --arms "ovl:FLS_OVERLAP_MIN_VECS_PER_CU=0" "ser:FLS_OVERLAP_FSST_WPC=0" > gpurun_out/r3/abenv_sf25_split_r3zl.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/r3/abenv_sf12_split_r3zl.txt | tail -2; grep -v amdgpu gpurun_out/r3/abenv_sf25_split_r3zl.txt | tail -2; exit $rc
