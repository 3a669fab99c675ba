#!/bin/bash
# GPU encoder vs CPU writer, byte for byte, on mixed files (every integer
# type x FFOR / DELTA) at several sizes and row-group sizes, 5 repeats each.
# usage: gpu_enc_diag.sh [variant ...]  (default: the in-tree build)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in ${@:-base}; do lib=libflsgpu_$v.so; [ $v = base ] && lib=libflsgpu.so; echo "== $v"
  for cfg in "--n 20000 --rowgroup 4096" "--n 200000 --rowgroup 1024" "--n 400000 --rowgroup 4096" "--n 300000 --rowgroup 65536"; do
    FLS_LIB=$lib timeout -k 10 120 python scripts/enc_diag.py $cfg --reps 5 --mixed-only 2>&1 | grep -v amdgpu || exit 1; done; done
