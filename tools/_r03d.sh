B="--no-cpu-baseline --no-host-pipeline --steps 20 --warmup 5"
A=$GRAFT_REPO_ROOT/tools/ab/librns_checksum_
steps=(pytest 600 "python -u -m pytest tests/test_gpu_packed.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
       pyw4 300 "RNS_CHECKSUM_LIB=${A}w4.so python -u -m pytest tests/test_gpu_packed.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k 'random or stream_rows or unaligned'"
       pyd8b4w4 300 "RNS_CHECKSUM_LIB=${A}d8b4w4.so python -u -m pytest tests/test_gpu_packed.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k 'random or stream_rows or unaligned'")
for cfg in c5_imix c3_1500B c2_64B; do
  st=20; [ $cfg = c2_64B ] && st=200
  for v in main b4 d8b4 w4 d8b4w4 d8 d12b4 nostream; do
    if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
    steps+=(${cfg}_$v 200 "$E python bench.py $B --config $cfg --steps $st")
  done
done
bash tools/gpu_steps.sh r03d "${steps[@]}"
