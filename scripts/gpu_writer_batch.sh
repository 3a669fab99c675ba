#!/bin/bash
# Batched row-group intake (fls_writer_add_rowgroups, the COPY sink's
# batches): GPU writer / COPY parity tests, then the writer and COPY rates on
# lineitem SF10 (CPU threads, GPU encoder, per-row-group vs batched calls).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_encode.py tests/test_copy.py tests/test_extension.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_writer_batch.log 2>&1
rc=$?; echo "parity: $(tail -1 gpurun_out/pt_writer_batch.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pt_writer_batch.log; exit $rc; }
timeout -k 10 500 python -u scripts/writer_bench.py --scale 10 --threads 16 --gpu --copy > gpurun_out/writer_batch.txt 2>&1
rc=$?; cat gpurun_out/writer_batch.txt; exit $rc
