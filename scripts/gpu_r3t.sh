# round 3t: full GPU suite, smoke, default bench + rocprof (QUICK round)
QUICK=1 bash scripts/gpu_round.sh r3t
