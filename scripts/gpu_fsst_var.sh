#!/bin/bash
# FSST code-parallel kernel variants (FLS_FSST_VARIANT bits, fls_decode.hpp):
# FSST parity under every variant, then a same-buffer A/B on l_comment (SF10)
# and on the whole lineitem_full table (SF100, FSST overlapped).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in ${VARS:-0 1 3 5 7}; do
  FLS_FSST_VARIANT=$V timeout -k 10 300 python -u -m pytest tests/test_alp_fsst.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_fsst_v$V.log 2>&1
  rc=$?; echo "variant $V parity: $(tail -1 gpurun_out/pt_fsst_v$V.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pt_fsst_v$V.log; exit $rc; }
done
ARMS=""; for V in ${VARS:-0 1 3 5 7}; do ARMS="$ARMS v$V:FLS_FSST_VARIANT=$V"; done
timeout -k 10 400 python scripts/ab_env.py --workload lineitem_full --scale 10 --arms $ARMS --cols 15 > gpurun_out/abenv_fsst_var.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/abenv_fsst_var.txt; [ $rc -eq 0 ] || exit $rc
[ -n "$QUICK" ] && exit 0
timeout -k 10 500 python scripts/ab_env.py --workload lineitem_full --scale 100 --rounds 5 --arms $ARMS --cols all > gpurun_out/abenv_fsst_var_full.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/abenv_fsst_var_full.txt; exit $rc
