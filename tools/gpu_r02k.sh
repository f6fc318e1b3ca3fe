set -u
O=gpurun_out/r02k; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_packed.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/packed.log 2>&1 || { tail -30 $O/packed.log; exit 1; }
tail -1 $O/packed.log
timeout -k 10 200 python tools/probe_thermal.py --seconds 20 --out $O/ab.json > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
grep -v smi $O/ab.log | tail -4
cd /tmp && timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r02k/counters.txt 2>&1; cd $GRAFT_REPO_ROOT
grep -i -E "DRAM|MALL|EA0_RD|EA_RD|HBM|UMC" gpurun_out/r02k/counters.txt | head -40
for L in product chnt u2; do
  if [ $L = product ]; then LIBV=""; else LIBV=tools/ab/librns_checksum_$L.so; fi
  RNS_CHECKSUM_LIB=$LIBV timeout -k 10 300 python tools/bench_ops.py --ops csum,chain --out gpurun_out/r02k/ops_$L.json > gpurun_out/r02k/ops_$L.log 2>&1 || { tail gpurun_out/r02k/ops_$L.log; exit 1; }
  echo "== $L"; grep '^c' gpurun_out/r02k/ops_$L.log
done
