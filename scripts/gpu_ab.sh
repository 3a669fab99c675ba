#!/bin/bash
# A/B round: quick GPU parity, then interleaved variant pairs at SF100.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_decode.py -q -x -p no:cacheprovider > gpurun_out/pt_ab.log 2>&1
rc=$?; tail -2 gpurun_out/pt_ab.log; [ $rc -eq 0 ] || exit $rc
for v in "$@"; do
  timeout -k 10 300 python scripts/ab.py --variants base,$v --cols all,0,3,6,8,10 > gpurun_out/ab_$v.txt 2>&1
  rc=$?; echo "== base vs $v (rc=$rc)"; cat gpurun_out/ab_$v.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
done
