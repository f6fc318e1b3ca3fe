B="--no-cpu-baseline --no-host-pipeline --steps 20 --warmup 5"
A=$GRAFT_REPO_ROOT/tools/ab/librns_checksum_
steps=(pytest 900 "python -u -m pytest tests -m gpu -q -p no:cacheprovider --maxfail 5 --timeout 300 --timeout-method thread")
for v in p8; do
  steps+=(py_$v 300 "RNS_CHECKSUM_LIB=$A$v.so python -u -m pytest tests/test_gpu_packed.py tests/test_gpu_parity.py -k 'packed or full_size' -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread")
done
for cfg in c5_imix d576B d1000B; do
  for v in main p8; do
    if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
    steps+=(${cfg}_$v 200 "$E python bench.py $B --config $cfg")
  done
done
for v in main p8; do
  if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
  steps+=(sh0_$v 200 "$E python bench.py $B --config c5_imix --shard 0/8")
done
for v in main rnt; do
  if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
  steps+=(c2_$v 200 "$E python bench.py $B --config c2_64B --steps 200")
done
steps+=(py_rxp8 300 "RNS_CHECKSUM_LIB=${A}rxp8.so python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_packed.py tests/test_gpu_bench_verify.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread")
for v in main rxnt rxp8; do
  if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
  steps+=(v_c2_$v 200 "$E python bench.py $B --config c2_64B --op verify --steps 200")
done
for v in main mnt s16p8; do
  if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
  steps+=(c3_$v 200 "$E python bench.py $B --config c3_1500B")
done
steps+=(ops_main 400 "python tools/bench_ops.py --ops csum,chain --configs c3_1500B,c5_imix --out gpurun_out/r03l/ops_main.json")
steps+=(prof_c2 300 "prof:python @ROOT@/bench.py $B --config c2_64B --steps 200")
bash tools/gpu_steps.sh r03l "${steps[@]}"
