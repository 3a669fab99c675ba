#!/bin/bash
# parity under each decode policy, then same-buffer A/B of the policies
# usage: gpu_abenv.sh "pol1 pol2 ..." [workloads]
POLS=${1:-"0 4 8"}
WLS=${2:-"lineitem c3"}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in $POLS; do
  FLS_DECODE_POLICY=$p timeout -k 10 600 python -m pytest tests/test_gpu_decode.py tests/test_gpu_fullsize.py -q -x -p no:cacheprovider > gpurun_out/pt_pol$p.log 2>&1
  rc=$?; echo "parity policy $p: $(tail -1 gpurun_out/pt_pol$p.log)"; [ $rc -eq 0 ] || exit $rc
done
ARMS=""
for p in $POLS; do ARMS="$ARMS p$p:FLS_DECODE_POLICY=$p"; done
for wl in $WLS; do
  COLS=all; [ "$wl" = lineitem ] && COLS=all,0,3,5,8,10
  timeout -k 10 600 python scripts/ab_env.py --workload $wl --arms $ARMS --cols $COLS > gpurun_out/abenv_$wl.txt 2>&1
  rc=$?; echo "== $wl"; grep -v amdgpu gpurun_out/abenv_$wl.txt; [ $rc -eq 0 ] || exit $rc
done
