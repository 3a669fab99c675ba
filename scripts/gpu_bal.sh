#!/bin/bash
# balanced split (policy 32): parity of every distribution policy, then
# same-buffer A/B against the work queue (policy 0) on lineitem, c3, c4.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_bal.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/pt_bal.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pt_bal.log; exit $rc; }
ARMS="q:FLS_DECODE_POLICY=0 s100:FLS_DECODE_POLICY=32 s85:FLS_DECODE_POLICY=32,FLS_STATIC_PCT=85 s70p4:FLS_DECODE_POLICY=32,FLS_STATIC_PCT=70,FLS_TAIL_PIECES=4 s100b3:FLS_DECODE_POLICY=32,FLS_BLOCKS_PER_CU=3 qb3:FLS_DECODE_POLICY=0,FLS_BLOCKS_PER_CU=3"
for wl in ${WLS:-lineitem c3 c4}; do
  COLS=all; [ "$wl" = lineitem ] && COLS=all,0,8
  timeout -k 10 600 python scripts/ab_env.py --workload $wl --arms $ARMS --cols $COLS --rounds 7 > gpurun_out/abenv_bal_$wl.txt 2>&1
  rc=$?; echo "== $wl"; grep -v amdgpu gpurun_out/abenv_bal_$wl.txt; [ $rc -eq 0 ] || exit $rc
done
