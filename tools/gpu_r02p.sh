set -u
O=gpurun_out/r02p; mkdir -p $O
for c in c3_1500B c5_imix c4_9000B; do
for args in "--graph off" "--graph on --graph-streams 2" "--graph off" "--graph on --graph-streams 2"; do
  timeout -k 10 200 python bench.py --config $c $args --no-cpu-baseline --no-host-pipeline --steps 40 > $O/b.log 2>&1 || { tail $O/b.log; exit 1; }
  python -c "import json;l=[json.loads(x) for x in open('$O/b.log') if x.startswith('{')][-1];print('$c $args', l['steps'], l['roofline']['kernel_avg_us'], l['ms_per_step'], l['value'], l['roofline']['frac'])"
done; done
