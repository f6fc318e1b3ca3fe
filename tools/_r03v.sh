B="--no-cpu-baseline --no-host-pipeline --warmup 5 --steps 20"
A=$GRAFT_REPO_ROOT/tools/ab/librns_checksum_
steps=(py_upw2 300 "RNS_CHECKSUM_LIB=${A}upw2.so python -u -m pytest tests/test_gpu_packed.py tests/test_gpu_rx.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread")
for rep in 1 2; do
  for cfg in c5_imix d576B; do
    for v in main upw2 upw4; do
      if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
      steps+=(${cfg}_${v}_$rep 200 "$E python bench.py $B --config $cfg")
    done
  done
  for v in main upw2; do
    if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
    steps+=(v_c2_${v}_$rep 200 "$E python bench.py --no-cpu-baseline --no-host-pipeline --warmup 5 --steps 200 --config c2_64B --op verify")
  done
done
bash tools/gpu_steps.sh r03v "${steps[@]}" && \
bash tools/pmc_configs.sh r03u c5_imix
