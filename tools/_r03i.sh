B="--no-cpu-baseline --no-host-pipeline --steps 20 --warmup 5"
A=$GRAFT_REPO_ROOT/tools/ab/librns_checksum_
steps=()
for cfg in c5_imix d576B d1000B; do
  for v in main out1 out2 ks2; do
    if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
    steps+=(${cfg}_$v 200 "$E python bench.py $B --config $cfg")
  done
done
bash tools/gpu_steps.sh r03i "${steps[@]}" && bash tools/pmc_issue.sh r03i_pmc c5_imix
