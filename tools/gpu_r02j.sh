set -u
O=gpurun_out/r02j; mkdir -p $O
timeout -k 10 200 python tools/probe_thermal.py --seconds 100 --out $O/thermal.json > $O/thermal.log 2>&1 || { tail $O/thermal.log; exit 1; }
grep -v smi $O/thermal.log | head -3; grep -v smi $O/thermal.log | tail -3; grep smi $O/thermal.log | head -2 | cut -c1-600
