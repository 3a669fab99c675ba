export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 200 ./scripts/membw7 10 0 > $O/membw7_default_r6e.txt 2>&1 || exit 1
timeout -k 10 200 ./scripts/membw7 10 4 > $O/membw7_contig_r6e.txt 2>&1
echo "contig rc=$?"
timeout -k 10 200 ./scripts/membw7 10 0 > $O/membw7_default2_r6e.txt 2>&1 || exit 1
