B="--no-cpu-baseline --no-host-pipeline --steps 20 --warmup 5"
A=$GRAFT_REPO_ROOT/tools/ab/librns_checksum_
steps=(pytest 900 "python -u -m pytest tests/test_gpu_packed.py tests/test_gpu_rx.py tests/test_c_caller.py tests/test_gpu_parity.py tests/test_gpu_bench_shard.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
       smoke 200 "python -c 'import __graft_entry__ as g; g.smoke()'")
for cfg in c5_imix c3_1500B c2_64B; do
  st=20; [ $cfg = c2_64B ] && st=200
  for v in main d2 d6 d8 tmp nostream; do
    if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
    steps+=(${cfg}_$v 200 "$E python bench.py $B --config $cfg --steps $st")
  done
done
steps+=(c4_main 200 "python bench.py $B --config c4_9000B --desc packed" c4_nostream 200 "RNS_CHECKSUM_LIB=${A}nostream.so python bench.py $B --config c4_9000B")
bash tools/gpu_steps.sh r03c "${steps[@]}"
