"""Print the key timing fields of bench.py JSON lines found in log files:
python tools/lines.py gpurun_out/<tag>/*.log"""
import json
import sys

for f in sys.argv[1:]:
    for ln in open(f, errors="replace"):
        if not ln.startswith("{\"metric\""):
            continue
        d = json.loads(ln)
        r = d["roofline"]
        iso = r.get("isolated") or {}
        print(f"{f.split('/')[-1]:40s} step {d['ms_per_step']*1e3:8.2f} us  kern {r['kernel_avg_us']:8.2f}  frac {r['frac']:.4f}"
              f"  iso {iso.get('kernel_avg_us', 0):8.2f} / {iso.get('frac', 0):.4f}  "
              f"{(d.get('verify') or {}).get('rejected_total', '')}/{(d.get('verify') or {}).get('rejected_expected', '')}"
              f"  {r.get('kernel', '')[:60]}")
