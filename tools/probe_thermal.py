"""Does the chip slow down under sustained load?  Alternates 20 launches of IMIX and
20 of c3 for --seconds, printing each burst's per-launch time with the elapsed time,
and samples the shader clock / temperature / power from rocm-smi every ~10 s.

    python tools/probe_thermal.py [--seconds 90] [--out gpurun_out/thermal.json]
"""
import argparse
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rustnetworkstack_amd.workloads import DeviceBatch, make_layout  # noqa: E402


def smi():
    try:
        r = subprocess.run(["rocm-smi", "--showclocks", "--showtemp", "--showpower", "--json"], capture_output=True,
                           text=True, timeout=20)
        d = json.loads(r.stdout)
        card = d[sorted(d)[0]]
        keep = {k: v for k, v in card.items() if any(t in k.lower() for t in ("sclk", "mclk", "fclk", "temperature",
                                                                            "power"))}
        return keep
    except Exception as e:  # noqa: BLE001
        return {"error": str(e)[:200]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=90)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cfgs = {}
    for name in ("c5_imix", "c3_1500B"):
        b = DeviceBatch(make_layout(name), dev)
        cfgs[name] = (b, b.launcher(complement=True, packed=True), b.launcher(complement=True, compact=True))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.time()
    rows, last_smi = [], -1e9
    while time.time() - t0 < args.seconds:
        row = {"t": round(time.time() - t0, 1)}
        for name, (b, fp, fc) in cfgs.items():
            for form, fn in (("packed", fp), ("compact", fc)):
                e0.record()
                for _ in range(20):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                row[f"{name}_{form}"] = round(e0.elapsed_time(e1) / 20 * 1e3, 1)
        if time.time() - last_smi > 10:
            row["smi"] = smi()
            last_smi = time.time()
        rows.append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
