B="--no-cpu-baseline --no-host-pipeline --steps 20 --warmup 5"
NS=RNS_CHECKSUM_LIB=$GRAFT_REPO_ROOT/tools/ab/librns_checksum_nostream.so
bash tools/gpu_steps.sh r03b \
 pytest 600 "python -u -m pytest tests/test_gpu_packed.py tests/test_c_caller.py tests/test_gpu_parity.py tests/test_gpu_rx.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
 smoke 200 "python -c 'import __graft_entry__ as g; g.smoke()'" \
 c5_new 200 "python bench.py $B --config c5_imix" \
 c5_old 200 "$NS python bench.py $B --config c5_imix" \
 c3_new 200 "python bench.py $B --config c3_1500B" \
 c3_old 200 "$NS python bench.py $B --config c3_1500B" \
 c2_new 200 "python bench.py $B --config c2_64B --steps 200" \
 c2_old 200 "$NS python bench.py $B --config c2_64B --steps 200" \
 c4_new 200 "python bench.py $B --config c4_9000B --desc packed" \
 c4_old 200 "$NS python bench.py $B --config c4_9000B" \
 c5_new2 200 "python bench.py $B --config c5_imix" \
 pmcw 900 "bash tools/pmc_write.sh r03b_pmcw"
