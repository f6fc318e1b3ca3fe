B="--no-cpu-baseline --no-host-pipeline --steps 20 --warmup 5"
A=$GRAFT_REPO_ROOT/tools/ab/librns_checksum_
steps=(pytest 600 "python -u -m pytest tests/test_gpu_packed.py tests/test_gpu_rx.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
       pyk4 300 "RNS_CHECKSUM_LIB=${A}k4.so python -u -m pytest tests/test_gpu_packed.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread")
for cfg in c5_imix c3_1500B c2_64B; do
  st=20; [ $cfg = c2_64B ] && st=200
  for v in main k2 k4 k16 k2w4 nostream; do
    if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
    steps+=(${cfg}_$v 200 "$E python bench.py $B --config $cfg --steps $st")
  done
done
for cfg in d40B d576B d1000B; do
  for v in main nostream; do
    if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
    steps+=(${cfg}_$v 200 "$E python bench.py $B --config $cfg")
  done
done
bash tools/gpu_steps.sh r03e "${steps[@]}"
