B="--no-cpu-baseline --no-host-pipeline --steps 20 --warmup 5"
A=$GRAFT_REPO_ROOT/tools/ab/librns_checksum_
steps=(py_o3a17 300 "RNS_CHECKSUM_LIB=${A}o3a17.so python -u -m pytest tests/test_gpu_packed.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread")
for rep in 1 2; do
  for cfg in c5_imix d576B; do
    for v in main o3a1 o3a3 o3a16 o3a17 o3a18; do
      if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
      steps+=(${cfg}_${v}_$rep 200 "$E python bench.py $B --config $cfg")
    done
  done
done
bash tools/gpu_steps.sh r03o "${steps[@]}"
