"""oracle/ -- CPU restatement of the FastLanes decode path.  TEST INFRASTRUCTURE
ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).  Parity with
upstream cwida/FastLanes bytes is UNPINNED (see flsref.h)."""
