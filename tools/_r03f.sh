B="--no-cpu-baseline --no-host-pipeline --steps 20 --warmup 5"
A=$GRAFT_REPO_ROOT/tools/ab/librns_checksum_
steps=(pytest 600 "python -u -m pytest tests/test_gpu_packed.py tests/test_gpu_rx.py tests/test_c_caller.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread")
for v in ks1 ks2 ks4; do
  steps+=(py$v 300 "RNS_CHECKSUM_LIB=${A}$v.so python -u -m pytest tests/test_gpu_packed.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread")
done
for cfg in c5_imix c2_64B d40B d576B c3_1500B; do
  st=20; [ $cfg = c2_64B ] && st=200
  for v in main ks1 ks2 ks4 ks4o5 nostream; do
    [ $cfg = c3_1500B ] && [ $v != main ] && [ $v != nostream ] && [ $v != ks2 ] && continue
    if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
    steps+=(${cfg}_$v 200 "$E python bench.py $B --config $cfg --steps $st")
  done
done
bash tools/gpu_steps.sh r03f "${steps[@]}"
