B="--no-cpu-baseline --no-host-pipeline --warmup 5 --steps 200"
A=$GRAFT_REPO_ROOT/tools/ab/librns_checksum_
steps=()
for rep in 1 2; do
  for v in main tg1024 tg4096 tg8192; do
    if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
    steps+=(c2_${v}_$rep 200 "$E python bench.py $B --config c2_64B")
  done
done
bash tools/gpu_steps.sh r03p "${steps[@]}"
