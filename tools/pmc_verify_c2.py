"""Summarise tools/pmc_verify_c2.sh: per-dispatch counter means of the three 64-byte kernels
and the same per datagram (2^20 per dispatch), with the verify kernels' excess over the
strided tiny checksum of the same bytes.

    python tools/pmc_verify_c2.py gpurun_out/<tag> [--out profiles/r06_pmc_verify_c2.json]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

KERNELS = {"csum": "csum_strided_tiny_kernel", "verify": "csum_strided_rx_kernel",
           "verify_packed": "csum_stream_kernel"}
N = 1 << 20


def collect(root, who):
    per = defaultdict(dict)
    for d in sorted(glob.glob(os.path.join(root, f"{who}_p*"))):
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if KERNELS[who] not in row.get("Kernel_Name", ""):
                    continue
                key = (f, row["Dispatch_Id"])
                per[row["Counter_Name"]][key] = per[row["Counter_Name"]].get(key, 0.0) + float(row["Counter_Value"])
    return {c: sum(v.values()) / len(v) for c, v in per.items() if v}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    res = {}
    for who, k in KERNELS.items():
        r = collect(args.dir, who)
        res[who] = {"kernel": k, "per_dispatch": {c: round(v, 1) for c, v in sorted(r.items())},
                    "per_datagram": {c: round(v / N, 3) for c, v in sorted(r.items())}}
    base = res["csum"]["per_datagram"]
    for who in ("verify", "verify_packed"):
        res[who]["excess_over_csum_per_datagram"] = {c: round(v - base.get(c, 0.0), 3)
                                                     for c, v in res[who]["per_datagram"].items() if c in base}
    text = json.dumps({"tool": "tools/pmc_verify_c2.sh + tools/pmc_verify_c2.py", "datagrams_per_dispatch": N,
                       "kernels": res}, indent=1)
    print(text)
    if args.out:
        open(args.out, "w").write(text)


if __name__ == "__main__":
    main()
