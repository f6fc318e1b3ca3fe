B="--no-cpu-baseline --no-host-pipeline --steps 20 --warmup 5"
A=$GRAFT_REPO_ROOT/tools/ab/librns_checksum_
steps=(pytest 900 "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
       smoke 200 "python -c 'import __graft_entry__ as g; g.smoke()'")
for v in main chainold; do
  if [ $v = main ]; then E=""; else E="RNS_CHECKSUM_LIB=$A$v.so"; fi
  steps+=(ops_$v 400 "$E python tools/bench_ops.py --ops csum,chain --configs c3_1500B,c5_imix --out gpurun_out/r03h/ops_$v.json")
done
for cfg in c2_64B c3_1500B c5_imix; do
  st=20; [ $cfg = c2_64B ] && st=200
  steps+=(cs_${cfg} 200 "python bench.py $B --config $cfg --steps $st")
  [ $cfg = c2_64B ] && steps+=(cs_${cfg}_strided 200 "python bench.py $B --config $cfg --steps $st --desc strided")
  steps+=(v_${cfg} 200 "python bench.py $B --config $cfg --op verify --steps $st")
done
bash tools/gpu_steps.sh r03h "${steps[@]}"
