set -u
bash tools/gpu_all.sh r02q
for c in c3_1500B c2_64B; do
  timeout -k 10 200 python bench.py --config $c --graph off --no-cpu-baseline --no-host-pipeline --steps 40 > gpurun_out/r02q_off_$c.log 2>&1 || exit 1
done
RNS_CHECKSUM_LIB=tools/ab/librns_checksum_inr.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fill.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02q_inr_tests.log 2>&1; tail -1 gpurun_out/r02q_inr_tests.log
for rep in 1 2; do for L in product inr; do
  if [ $L = product ]; then LIBV=""; else LIBV=tools/ab/librns_checksum_$L.so; fi
  RNS_CHECKSUM_LIB=$LIBV timeout -k 10 300 python tools/bench_ops.py --ops fill --chain-layouts packed --out gpurun_out/r02q_fill_${L}_$rep.json > gpurun_out/r02q_fill_$L.log 2>&1 || exit 1
  echo "$L $rep $(tail -1 gpurun_out/r02q_fill_$L.log)"
done; done
bash tools/multi_rehearsal.sh r02q_mr
