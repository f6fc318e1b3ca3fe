set -u
O=gpurun_out/r02m; mkdir -p $O
for rep in 1 2; do for d in packed 32 64; do
  timeout -k 10 200 python bench.py --config c5_imix --desc $d --no-cpu-baseline --no-host-pipeline --steps 20 --warmup 5 > $O/c5_${d}_$rep.log 2>&1 || { tail $O/c5_${d}_$rep.log; exit 1; }
  python -c "import json;l=[json.loads(x) for x in open('$O/c5_${d}_$rep.log') if x.startswith('{')][-1];print('c5 $d', l['roofline']['kernel_avg_us'])"
done; done
for g in on off; do
  timeout -k 10 200 python bench.py --config c2_64B --graph $g --no-cpu-baseline --no-host-pipeline --steps 60 --warmup 5 > $O/c2_$g.log 2>&1 || { tail $O/c2_$g.log; exit 1; }
  python -c "import json;l=[json.loads(x) for x in open('$O/c2_$g.log') if x.startswith('{')][-1];print('c2 graph $g', l['roofline']['kernel_avg_us'], l['ms_per_step'], l['value'])"
done
timeout -k 10 200 python tools/probe_thermal.py --seconds 10 > $O/th.log 2>&1; grep -v smi $O/th.log | tail -2
