# round 3z: writer and COPY rates with l_comment (FSST encode on the CPU threads, the faster matcher)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python scripts/writer_bench.py --workload lineitem_full --scale 2 --threads 16 > gpurun_out/writer_full_r3z.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/writer_full_r3z.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/writer_bench.py --workload lineitem_full --scale 10 --threads 16 --copy --copy-only > gpurun_out/copy_full_r3z.txt 2>&1
rc=$?; grep COPY gpurun_out/copy_full_r3z.txt; exit $rc
