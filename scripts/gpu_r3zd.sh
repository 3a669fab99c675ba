# round 3zd: SF12.5 (8-GPU per-GPU share) kernel traces with the lean FSST
# kernel, overlapped vs serial, and a same-buffer A/B of the two
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
export PYTHONUNBUFFERED=1
ARMS="ovl ser" timeout -k 10 500 bash scripts/gpu_sf12_trace.sh sf12zd &&
python3 scripts/trace_span.py $(find gpurun_out/tr_sf12zd_ovl -name "*kernel_trace.csv" | head -1) > gpurun_out/r3/spans_sf12_ovl_r3zd.txt 2>&1 ;
python3 scripts/trace_span.py $(find gpurun_out/tr_sf12zd_ser -name "*kernel_trace.csv" | head -1) > gpurun_out/r3/spans_sf12_ser_r3zd.txt 2>&1 ;
timeout -k 10 400 python -u scripts/ab_env.py --workload lineitem_full --scale 12.5 --rounds 9 \
   --arms "ser:FLS_OVERLAP_MIN_VECS_PER_CU=400" "ovl:FLS_OVERLAP_MIN_VECS_PER_CU=0" "ovl16:FLS_OVERLAP_MIN_VECS_PER_CU=0,FLS_OVERLAP_FSST_WPC=16" > gpurun_out/r3/abenv_sf12_ovl_r3zd.txt 2>&1
rc=$?; tail -3 gpurun_out/r3/spans_sf12_*_r3zd.txt; grep -v amdgpu gpurun_out/r3/abenv_sf12_ovl_r3zd.txt | tail -4; exit $rc
