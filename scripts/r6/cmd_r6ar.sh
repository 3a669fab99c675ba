# pinned allocation rate by thread count and chunk size, fresh process each
mkdir -p gpurun_out; O=gpurun_out/pin_alloc_r6ar.txt; : > $O
for cfg in "1 8" "4 8" "8 8" "16 8" "1 64" "4 64" "8 64" "1 2" "8 2"; do
  timeout -k 10 60 ./scripts/pin_alloc_probe $cfg 2048 >> $O 2>&1 || exit 1
done
cat $O
