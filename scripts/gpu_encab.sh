#!/bin/bash
# Encoder A/B: parity of the default build (test_encode), then device-resident
# encode rates for base and each variant, interleaved twice.
# usage: gpu_encab.sh <tag> v1 [v2 ...]
TAG=$1; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_encode.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_encab_$TAG.log 2>&1
rc=$?; echo "encode parity: $(tail -1 gpurun_out/pt_encab_$TAG.log)"; [ $rc -eq 0 ] || exit $rc
for v in "$@"; do
  FLS_LIB=libflsgpu_$v.so timeout -k 10 300 python -u -m pytest tests/test_encode.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_encab_${TAG}_$v.log 2>&1
  rc=$?; echo "encode parity $v: $(tail -1 gpurun_out/pt_encab_${TAG}_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for round in 1 2; do
  for v in base "$@"; do
    lib=libflsgpu.so; [ $v = base ] || lib=libflsgpu_$v.so
    FLS_LIB=$lib timeout -k 10 200 python scripts/encode_bench.py --no-writer --reps 7 > gpurun_out/encab_${TAG}_${v}_$round.txt 2>&1
    rc=$?; echo "== $v round $round rc=$rc"; grep -v amdgpu gpurun_out/encab_${TAG}_${v}_$round.txt | python3 -c "import sys,json;[print(d['case'],d['kernel_ms'],d['frac_of_8TBps']) for d in map(json.loads,sys.stdin)]"; [ $rc -eq 0 ] || exit $rc
  done
done
