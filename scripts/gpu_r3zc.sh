# round 3zc: checkpoint of the round-3 HEAD after the re-entry (full GPU suite,
# smoke, default bench + rocprof kernel stats)
QUICK=1 bash scripts/gpu_round.sh r3zc
