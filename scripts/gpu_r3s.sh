# round 3s: encoder with a scalar wave index -- parity, the mixed-file comparison once for
# the default (5-wave) and once for the 6-wave build, then encode rates vs the round-2 code (vw)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_encode.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_enc_r3s.log 2>&1
rc=$?; echo "encode parity: $(tail -1 gpurun_out/pt_enc_r3s.log)"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_enc_diag.sh base n6 > gpurun_out/encode_diag_r3s.txt 2>&1
rc=$?; cat gpurun_out/encode_diag_r3s.txt | tail -20; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for v in base n6 vw; do
    lib=libflsgpu.so; [ $v = base ] || lib=libflsgpu_$v.so
    FLS_LIB=$lib timeout -k 10 200 python scripts/encode_bench.py --no-writer --reps 7 > gpurun_out/encab_r3s_${v}_$round.txt 2>&1
    rc=$?; echo "== $v round $round rc=$rc"; grep -v amdgpu gpurun_out/encab_r3s_${v}_$round.txt | python3 -c "import sys,json;[print(d['case'],d['kernel_ms'],d['frac_of_8TBps']) for d in map(json.loads,sys.stdin)]"; [ $rc -eq 0 ] || exit $rc
  done
done
