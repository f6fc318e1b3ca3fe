bash tools/gpu_steps.sh r03a \
 pytest 600 "python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
 smoke 200 "python -c 'import __graft_entry__ as g; g.smoke()'" \
 c5 300 "prof:python3 @ROOT@/bench.py --gpus 1 --steps 20 --warmup 5 --config c5_imix --no-host-pipeline --cpu-seconds 4" \
 c5_s2 200 "python bench.py --steps 20 --warmup 5 --config c5_imix --no-host-pipeline --no-cpu-baseline --graph-streams 2" \
 c5_s3 200 "python bench.py --steps 20 --warmup 5 --config c5_imix --no-host-pipeline --no-cpu-baseline --graph-streams 3" \
 c5_s4 200 "python bench.py --steps 20 --warmup 5 --config c5_imix --no-host-pipeline --no-cpu-baseline --graph-streams 4" \
 c5_sh0 200 "prof:python3 @ROOT@/bench.py --steps 20 --warmup 5 --config c5_imix --shard 0/8 --no-host-pipeline --cpu-seconds 2" \
 c5_sh7 200 "prof:python3 @ROOT@/bench.py --steps 20 --warmup 5 --config c5_imix --shard 7/8 --no-host-pipeline --cpu-seconds 2" \
 c3 300 "prof:python3 @ROOT@/bench.py --gpus 1 --steps 20 --warmup 5 --config c3_1500B" \
 c2 200 "prof:python3 @ROOT@/bench.py --gpus 1 --steps 200 --warmup 5 --config c2_64B --no-host-pipeline --cpu-seconds 2"
