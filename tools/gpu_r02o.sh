set -u
O=gpurun_out/r02o; mkdir -p $O
for args in "--graph off" "--graph on --graph-streams 1" "--graph on --graph-streams 2" "--graph on --graph-streams 3" "--graph on --graph-streams 2 --steps 120"; do
  timeout -k 10 200 python bench.py --config c2_64B $args --no-cpu-baseline --no-host-pipeline > $O/c2.log 2>&1 || { tail $O/c2.log; exit 1; }
  python -c "import json;l=[json.loads(x) for x in open('$O/c2.log') if x.startswith('{')][-1];print('$args', l['steps'], l['roofline']['kernel_avg_us'], l['ms_per_step'], l['value'], l['roofline']['frac'])"
done
