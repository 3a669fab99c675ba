# round 3zi: same-box A/B of GPU FSST compression in the writer
# (FLS_WRITER_FSST_GPU=0 keeps FSST on the host threads): C-ABI writer and
# COPY on lineitem_full, and the writer's phase profile with it on
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3
for arm in gpu host; do
  if [ $arm = host ]; then export FLS_WRITER_FSST_GPU=0; else unset FLS_WRITER_FSST_GPU; fi
  timeout -k 10 500 python scripts/writer_bench.py --workload lineitem_full --scale 4 --threads 16 --gpu > gpurun_out/r3/writer_full_${arm}_r3zi.txt 2>&1
  rc=$?; echo "== $arm"; grep 'GPU 0' gpurun_out/r3/writer_full_${arm}_r3zi.txt; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 500 python scripts/writer_bench.py --workload lineitem_full --scale 10 --threads 16 --copy --copy-only > gpurun_out/r3/copy_full_${arm}_r3zi.txt 2>&1
  rc=$?; grep COPY gpurun_out/r3/copy_full_${arm}_r3zi.txt; [ $rc -eq 0 ] || exit $rc
done
unset FLS_WRITER_FSST_GPU
FLS_WRITER_PROFILE=1 timeout -k 10 500 python scripts/writer_bench.py --workload lineitem_full --scale 4 --threads 16 --gpu > gpurun_out/r3/writer_full_prof_r3zi.txt 2>&1
rc=$?; grep -i 'profile' gpurun_out/r3/writer_full_prof_r3zi.txt | tail -4; exit $rc
