set -u
O=gpurun_out/r02d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chains.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/chains.log 2>&1 || { tail -30 $O/chains.log; exit 1; }
tail -2 $O/chains.log
timeout -k 10 300 python tools/bench_ops.py --ops csum,chain --out $O/ops_chain.json > $O/ops.log 2>&1 || { tail $O/ops.log; exit 1; }
tail -3 $O/ops.log
RNS_CHECKSUM_LIB=tools/ab/librns_checksum_c32.so timeout -k 10 300 python tools/bench_ops.py --ops csum,chain --out $O/ops_chain_c32.json > $O/ops_c32.log 2>&1 || { tail $O/ops_c32.log; exit 1; }
tail -3 $O/ops_c32.log
