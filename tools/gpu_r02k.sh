set -u
O=gpurun_out/r02k; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_packed.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/packed.log 2>&1 || { tail -30 $O/packed.log; exit 1; }
tail -1 $O/packed.log
timeout -k 10 200 python tools/probe_thermal.py --seconds 20 --out $O/ab.json > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
grep -v smi $O/ab.log | tail -4
