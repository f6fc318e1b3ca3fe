B="--no-cpu-baseline --no-host-pipeline --warmup 5"
A=$GRAFT_REPO_ROOT/tools/ab/librns_checksum_
steps=(py_rxo4 300 "RNS_CHECKSUM_LIB=${A}rxo4.so python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread")
for rep in 1 2; do
  for v in main rxo4 rxo5; do
    if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
    steps+=(v_c2_${v}_$rep 200 "$E python bench.py $B --steps 200 --config c2_64B --op verify")
    steps+=(v_c5_${v}_$rep 200 "$E python bench.py $B --steps 20 --config c5_imix --op verify")
    steps+=(v_c3_${v}_$rep 200 "$E python bench.py $B --steps 20 --config c3_1500B --op verify")
  done
done
bash tools/gpu_steps.sh r03s "${steps[@]}"
