# c3 (DELTA64, 1e9 INT64 keys): store cache-policy combinations; balanced split vs queue
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 600 python -u scripts/ab_builds.py --variants base,cp18,cp3,cp19 --workload c3 --scale 1 --rounds 6 --verify > $O/ab_builds_c3_cpol_r6s.txt 2>&1; echo "ab rc=$?"; tail -1 $O/ab_builds_c3_cpol_r6s.txt
timeout -k 10 600 python -u scripts/ab_env.py --workload c3 --scale 1 --arms "queue:" "balanced:FLS_DECODE_POLICY=32" > $O/abenv_c3_policy_r6s.txt 2>&1; echo "abenv rc=$?"; grep -v amdgpu $O/abenv_c3_policy_r6s.txt | tail -2
