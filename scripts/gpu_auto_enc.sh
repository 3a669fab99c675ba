#!/bin/bash
# GPU ENC_AUTO: encoder GPU tests, the mixed-file byte diagnostic, then the
# write-path rates with the GPU arm (byte-identity checked) and COPY.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_encode.py tests/test_copy.py tests/test_writer.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pt_auto_enc.log 2>&1
rc=$?; echo "encoder/writer gpu tests: $(tail -1 gpurun_out/pt_auto_enc.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pt_auto_enc.log | head -20; exit $rc; }
bash scripts/gpu_enc_diag.sh base > gpurun_out/encode_diag_auto.txt 2>&1
rc=$?; cat gpurun_out/encode_diag_auto.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/writer_bench.py --scale ${SCALE:-10} --threads 16 --gpu --copy > gpurun_out/writer_auto.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/writer_auto.txt; exit $rc
