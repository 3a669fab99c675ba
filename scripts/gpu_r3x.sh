# round 3x: COPY throughput (ordered / unordered) on the current build, lineitem SF10
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python scripts/writer_bench.py --scale 10 --threads 16 --copy > gpurun_out/copy_sf10_r3x.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/copy_sf10_r3x.txt | tail -8; exit $rc
