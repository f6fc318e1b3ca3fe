"""Summarise tools/pmc_write.sh: per kernel (by name) and per pass, the mean counter
value per dispatch, with the gfx950 corrections of MI355X_MICROARCH.md §HBM
(FETCH_SIZE KiB x 2 for wide streaming reads; WRITE_SIZE KiB as is) and the
EA write requests in bytes (TCC_EA0_WRREQ counts 32-byte requests unless _64B).

    python tools/pmc_write.py gpurun_out/<tag> [--out profiles/archive/r03/r03_pmc_write.json]
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    res = defaultdict(lambda: defaultdict(dict))
    for d in sorted(glob.glob(os.path.join(args.dir, "*_p[0-9]"))):
        op = os.path.basename(d).rsplit("_p", 1)[0]
        vals = defaultdict(lambda: defaultdict(float))
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = row.get("Kernel_Name", "")
                    if "csum_" not in k:
                        continue
                    m = re.search(r"(csum_\w+<[^()]*>)", k)
                    key = m.group(1) if m else k
                    vals[(key, row["Counter_Name"])][row["Dispatch_Id"]] += float(row["Counter_Value"])
        for (k, c), per in vals.items():
            v = list(per.values())
            res[op][k][c] = {"mean_per_dispatch": sum(v) / len(v), "dispatches": len(v)}
    out = {}
    for op, ks in res.items():
        out[op] = {}
        for k, cs in ks.items():
            e = {c: round(x["mean_per_dispatch"], 1) for c, x in cs.items()}
            e["dispatches"] = {c: x["dispatches"] for c, x in cs.items()}
            if "WRITE_SIZE" in cs:
                e["write_bytes"] = int(cs["WRITE_SIZE"]["mean_per_dispatch"] * 1024)
            if "FETCH_SIZE" in cs:
                e["fetch_bytes_corrected"] = int(2 * cs["FETCH_SIZE"]["mean_per_dispatch"] * 1024)
            if "TCC_EA0_WRREQ_sum" in cs:
                n64 = cs.get("TCC_EA0_WRREQ_64B_sum", {"mean_per_dispatch": 0.0})["mean_per_dispatch"]
                n = cs["TCC_EA0_WRREQ_sum"]["mean_per_dispatch"]
                e["ea_write_bytes_32B_64B"] = int(64 * n64 + 32 * (n - n64))
            out[op][k] = e
    text = json.dumps({"tool": "tools/pmc_write.sh + tools/pmc_write.py", "per_kernel": out}, indent=1)
    print(text)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
