B="--no-cpu-baseline --no-host-pipeline --warmup 5"
A=$GRAFT_REPO_ROOT/tools/ab/librns_checksum_
steps=(py_ks2 300 "RNS_CHECKSUM_LIB=${A}ks2.so python -u -m pytest tests/test_gpu_packed.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
       py_tv11 300 "RNS_CHECKSUM_LIB=${A}tv11.so python -u -m pytest tests/test_gpu_parity.py -k 'strided or full_size' -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread")
for rep in 1 2; do
  for cfg in c5_imix d576B; do
    for v in main ks2; do
      if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
      steps+=(${cfg}_${v}_$rep 200 "$E python bench.py $B --steps 20 --config $cfg")
    done
  done
  for v in main tv11; do
    if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
    steps+=(c2_${v}_$rep 200 "$E python bench.py $B --steps 200 --config c2_64B")
  done
done
bash tools/gpu_steps.sh r03r "${steps[@]}"
