# Final validation of the committed defaults + the tiny-grid A/B for c2.
D="--gpus 1 --steps 20 --warmup 5"
B="--no-cpu-baseline --no-host-pipeline --warmup 5 --steps 200"
A=$GRAFT_REPO_ROOT/tools/ab/librns_checksum_
steps=(pytest 900 "python -u -m pytest tests -m gpu -q -p no:cacheprovider --maxfail 5 --timeout 300 --timeout-method thread"
       smoke 200 "python -c 'import __graft_entry__ as g; g.smoke()'"
       bench_c5_imix 300 "prof:python @ROOT@/bench.py $D --config c5_imix"
       bench_c3_1500B 300 "prof:python @ROOT@/bench.py $D --config c3_1500B")
for r in 0 7; do
  steps+=(shard${r}_c5_imix 300 "prof:python @ROOT@/bench.py $D --config c5_imix --shard $r/8 --no-host-pipeline")
done
for rep in 1 2; do
  for v in main tg1024 tg4096 tg8192; do
    if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
    steps+=(c2_${v}_$rep 200 "$E python bench.py $B --config c2_64B")
  done
done
bash tools/gpu_steps.sh r03q "${steps[@]}"
