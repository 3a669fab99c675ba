# round 3zh: GPU FSST compression in the writer -- byte identity against the
# host compressor (tests), the encoder / COPY GPU suites, and the writer and
# COPY rates on lineitem_full (l_comment FSST)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encode.py tests/test_copy.py tests/test_writer.py -m gpu > gpurun_out/r3/pt_fsst_gpu_enc_r3zh.log 2>&1
rc=$?; tail -3 gpurun_out/r3/pt_fsst_gpu_enc_r3zh.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/writer_bench.py --workload lineitem_full --scale 2 --threads 16 --gpu > gpurun_out/r3/writer_full_gpu_r3zh.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/r3/writer_full_gpu_r3zh.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/writer_bench.py --workload lineitem_full --scale 10 --threads 16 --copy --copy-only > gpurun_out/r3/copy_full_gpu_r3zh.txt 2>&1
rc=$?; grep COPY gpurun_out/r3/copy_full_gpu_r3zh.txt; exit $rc
