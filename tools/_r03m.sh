# Round-3 final measurements on the tree as committed: GPU tests, smoke, the driver's bench
# command for every config under rocprofv3 (line + trace of ONE run, reconciled), the verify
# lines, the N=8 shard of c5, the widened ops, and PMC traffic of the bench kernels.
D="--gpus 1 --steps 20 --warmup 5"
steps=(pytest 900 "python -u -m pytest tests -m gpu -q -p no:cacheprovider --maxfail 5 --timeout 300 --timeout-method thread"
       smoke 200 "python -c 'import __graft_entry__ as g; g.smoke()'")
for cfg in c3_1500B c5_imix c4_9000B; do
  steps+=(bench_$cfg 300 "prof:python @ROOT@/bench.py $D --config $cfg")
done
steps+=(bench_c2_64B 300 "prof:python @ROOT@/bench.py --gpus 1 --steps 200 --warmup 5 --config c2_64B")
for r in 0 7; do
  steps+=(shard${r}_c5_imix 300 "prof:python @ROOT@/bench.py $D --config c5_imix --shard $r/8 --no-host-pipeline")
done
steps+=(verify_c2 200 "python bench.py --steps 200 --warmup 5 --config c2_64B --op verify"
        verify_c3 200 "python bench.py $D --config c3_1500B --op verify"
        verify_c5 200 "python bench.py $D --config c5_imix --op verify"
        ops 600 "python tools/bench_ops.py --out gpurun_out/r03m/ops.json")
bash tools/gpu_steps.sh r03m "${steps[@]}" && bash tools/pmc_configs.sh r03m_pmc c3_1500B,c5_imix,c2_64B
