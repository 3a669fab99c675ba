#!/bin/bash
# FSST kernels overlapped with the main decode kernel: GPU parity, then a
# same-buffer A/B of overlap splits on lineitem_full (SCALE, default 100).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=tests; [ -n "$QUICK" ] && T="tests/test_alp_fsst.py tests/test_gpu_decode.py"
timeout -k 10 600 python -u -m pytest $T -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_overlap.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/pt_overlap.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pt_overlap.log | head -30; tail -40 gpurun_out/pt_overlap.log; exit $rc; }
timeout -k 10 900 python scripts/ab_env.py --workload lineitem_full --scale ${SCALE:-100} --rounds 5 --cols all --arms \
  ser:FLS_OVERLAP_FSST_WPC=0 d1f12:FLS_OVERLAP_DECODE_BPC=1,FLS_OVERLAP_FSST_WPC=12 d2f8:FLS_OVERLAP_DECODE_BPC=2,FLS_OVERLAP_FSST_WPC=8 \
  d1f16:FLS_OVERLAP_DECODE_BPC=1,FLS_OVERLAP_FSST_WPC=16 d2f12:FLS_OVERLAP_DECODE_BPC=2,FLS_OVERLAP_FSST_WPC=12 \
  d1f20:FLS_OVERLAP_DECODE_BPC=1,FLS_OVERLAP_FSST_WPC=20 > gpurun_out/abenv_overlap.txt 2>&1
rc=$?; echo "== ab"; grep -v amdgpu gpurun_out/abenv_overlap.txt; exit $rc
