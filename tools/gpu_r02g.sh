set -u
O=gpurun_out/r02g; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_packed.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/probe_c2.py --label product --out $O/c2_product.json > $O/c2_product.log 2>&1 || { tail $O/c2_product.log; exit 1; }
cat $O/c2_product.log
RNS_CHECKSUM_LIB=tools/ab/librns_checksum_ppf.so timeout -k 10 300 python tools/probe_c2.py --label ppf --out $O/c2_ppf.json > $O/c2_ppf.log 2>&1 || { tail $O/c2_ppf.log; exit 1; }
grep packed $O/c2_ppf.log; tail -1 $O/c2_ppf.log
