#!/bin/bash
# FSST kernel: parity under both round sizes, then same-buffer A/B on lineitem_full SF10
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in 0 16; do
  FLS_DECODE_POLICY=$p timeout -k 10 600 python -m pytest tests/test_alp_fsst.py tests/test_filter.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pt_fsst$p.log 2>&1
  rc=$?; echo "parity policy $p: $(tail -1 gpurun_out/pt_fsst$p.log)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python scripts/ab_env.py --workload lineitem_full --scale 10 --arms bpl8:FLS_DECODE_POLICY=0 bpl16:FLS_DECODE_POLICY=16 --cols all,15 > gpurun_out/abenv_fsst.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/abenv_fsst.txt; exit $rc
