# the bench command at round 4 (50dc1cf), round 5 (44928df) and HEAD, interleaved in one lease
export TMPDIR=/tmp; mkdir -p gpurun_out; O=$PWD/gpurun_out
F="--steps 20 --cpu-seconds 0 --e2e-scale 0 --no-traffic --no-verify"
for sc in 100 12.5; do
  for i in 1 2 3; do
    for tree in abtree_r4 abtree_r5 .; do
      tag=$(basename $(cd $tree && pwd)); [ "$tree" = "." ] && tag=head
      (cd $tree && timeout -k 10 300 python3 bench.py --scale $sc $F > $O/abr_${tag}_sf${sc}_$i.json 2> $O/abr_${tag}_sf${sc}_$i.log) || exit 1
      python3 -c "import json;d=json.load(open('$O/abr_${tag}_sf${sc}_$i.json'));print('$tag sf$sc run $i', round(d['ms_per_step'],4), round(d['roofline']['frac'],4))"
    done
  done
done
