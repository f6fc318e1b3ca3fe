"""Summarise tools/pmc_detail.sh output: per-launch counter means for the checksum kernels."""
import csv, glob, json, os, sys
from collections import defaultdict
root = sys.argv[1]
res = {}
for d in sorted(glob.glob(os.path.join(root, "*_p*"))):
    if not os.path.isdir(d):
        continue
    cfg = os.path.basename(d).rsplit("_p", 1)[0]
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "csum_" not in row.get("Kernel_Name", ""):
                continue
            per[row["Counter_Name"]][(f, row["Dispatch_Id"])] += float(row["Counter_Value"])
    for ctr, vals in per.items():
        res.setdefault(cfg, {})[ctr] = sum(vals.values()) / max(len(vals), 1)
for cfg, r in res.items():
    n32, n64, n128 = (r.get(f"TCC_EA0_RDREQ_{k}B_sum", 0) for k in (32, 64, 128))
    r["read_bytes_by_size"] = 32 * n32 + 64 * n64 + 128 * n128
print(json.dumps(res, indent=1))
