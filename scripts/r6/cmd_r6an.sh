# PCIe copy rates per fresh process, SDMA against kernel copies
mkdir -p gpurun_out; O=gpurun_out/d2h_probe_r6an.txt; : > $O
for i in 1 2 3 4 5 6; do echo -n "sdma run $i: " >> $O; timeout -k 10 60 ./scripts/d2h_probe >> $O 2>&1 || exit 1; done
for i in 1 2 3; do echo -n "HSA_ENABLE_SDMA=0 run $i: " >> $O; HSA_ENABLE_SDMA=0 timeout -k 10 60 ./scripts/d2h_probe >> $O 2>&1 || exit 1; done
cat $O
