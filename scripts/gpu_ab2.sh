#!/bin/bash
# A/B of prebuilt variant libraries: parity of each variant (decode tests),
# then interleaved SF100 timing against base.  usage: gpu_ab2.sh v1 v2 ...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  FLS_LIB=libflsgpu_$v.so timeout -k 10 600 python -m pytest tests/test_gpu_decode.py tests/test_gpu_fullsize.py -q -x -p no:cacheprovider > gpurun_out/pt_ab_$v.log 2>&1
  rc=$?; echo "parity $v: $(tail -1 gpurun_out/pt_ab_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
V=$(echo "$@" | tr ' ' ',')
timeout -k 10 600 python scripts/ab.py --variants base,$V --cols all,0,3,6,8,10 --rounds 9 > gpurun_out/ab_multi.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_multi.txt; exit $rc
