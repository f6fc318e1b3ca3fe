set -u
O=gpurun_out/r02f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_packed.py tests/test_gpu_chains.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/packed.log 2>&1 || { tail -30 $O/packed.log; exit 1; }
tail -2 $O/packed.log
timeout -k 10 300 python tools/probe_layouts.py --skip-align --out $O/probe_layouts.json > $O/probe.log 2>&1 || { tail $O/probe.log; exit 1; }
cat $O/probe.log
