"""The key timing fields of bench.py JSON lines found in log files.

    python tools/lines.py gpurun_out/<tag>/*.log             # one row per line
    python tools/lines.py --json gpurun_out/<tag>/*.log      # {log name: fields} as JSON
"""
import json
import os
import sys


def collect(paths):
    out = {}
    for f in paths:
        for ln in open(f, errors="replace"):
            if not ln.startswith("{\"metric\""):
                continue
            d = json.loads(ln)
            r = d["roofline"]
            iso = r.get("isolated") or {}
            out[os.path.basename(f).rsplit(".", 1)[0]] = {
                "ms_per_step": d["ms_per_step"], "value": d["value"], "kernel_avg_us": r["kernel_avg_us"],
                "frac": r["frac"], "isolated_us": iso.get("kernel_avg_us"), "isolated_frac": iso.get("frac"),
                "kernel": r.get("kernel"), "descriptors": d["config"].get("descriptors"),
                "verify": d.get("verify"), "shard": (d.get("shard") or {}).get("rank"),
                "cpu_baseline": (d.get("cpu_baseline") or {}).get("value"),
                "gpu_sample_bit_exact": (d.get("cpu_baseline") or {}).get("gpu_sample_bit_exact")}
    return out


def main():
    args = sys.argv[1:]
    as_json = bool(args) and args[0] == "--json"
    res = collect(args[1:] if as_json else args)
    if as_json:
        print(json.dumps(res, indent=1))
        return
    for k, v in res.items():
        ver = v["verify"] or {}
        print(f"{k:32s} step {v['ms_per_step'] * 1e3:8.2f} us  kern {v['kernel_avg_us']:8.2f}  frac {v['frac']:.4f}"
              f"  iso {v['isolated_us'] or 0:8.2f} / {v['isolated_frac'] or 0:.4f}  "
              f"{ver.get('rejected_total', '')}/{ver.get('rejected_expected', '')}  {(v['kernel'] or '')[:50]}")


if __name__ == "__main__":
    main()
