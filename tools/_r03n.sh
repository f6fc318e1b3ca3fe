B="--no-cpu-baseline --no-host-pipeline --steps 20 --warmup 5"
A=$GRAFT_REPO_ROOT/tools/ab/librns_checksum_
steps=()
for v in d6 d8; do
  steps+=(py_$v 300 "RNS_CHECKSUM_LIB=$A$v.so python -u -m pytest tests/test_gpu_packed.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread")
done
steps+=(py_rxo8 300 "RNS_CHECKSUM_LIB=${A}rxo8.so python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread")
for rep in 1 2; do
  for cfg in c5_imix d576B; do
    for v in main d6 d8; do
      if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
      steps+=(${cfg}_${v}_$rep 200 "$E python bench.py $B --config $cfg")
    done
  done
  for v in main rxo8; do
    if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
    steps+=(v_c2_${v}_$rep 200 "$E python bench.py $B --config c2_64B --op verify --steps 200")
    steps+=(v_c5_${v}_$rep 200 "$E python bench.py $B --config c5_imix --op verify")
  done
  for v in main s16; do
    if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
    steps+=(c3_${v}_$rep 200 "$E python bench.py $B --config c3_1500B")
  done
done
bash tools/gpu_steps.sh r03n "${steps[@]}"
