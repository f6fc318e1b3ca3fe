"""Summarise tools/pmc_issue.sh: per-dispatch counter means of the bench kernel (csum_*)
for every config pass directory gpurun_out/<tag>/<config>_p<N>."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def collect(root, cfg):
    per = defaultdict(dict)
    for d in sorted(glob.glob(os.path.join(root, f"{cfg}_p*"))):
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if "csum_" not in row.get("Kernel_Name", ""):
                    continue
                key = (f, row["Dispatch_Id"])
                per[row["Counter_Name"]][key] = per[row["Counter_Name"]].get(key, 0.0) + float(row["Counter_Value"])
    return {c: sum(v.values()) / len(v) for c, v in per.items() if v}


def main():
    root = sys.argv[1]
    cfgs = sorted({os.path.basename(d).rsplit("_p", 1)[0] for d in glob.glob(os.path.join(root, "*_p*"))
                   if os.path.isdir(d)})
    out = {}
    for cfg in cfgs:
        r = collect(root, cfg)
        wc = max(r.get("SQ_WAVE_CYCLES", 1), 1)
        r["derived"] = {
            "wait_frac": r.get("SQ_WAIT_ANY", 0) / wc,
            "issue_stall_frac": r.get("SQ_WAIT_INST_ANY", 0) / wc,
            "active_frac": r.get("SQ_ACTIVE_INST_ANY", 0) / wc,
            "icache_miss_rate": r.get("SQC_ICACHE_MISSES", 0) / max(r.get("SQC_ICACHE_REQ", 1), 1),
            "ifetch_per_wave": r.get("SQ_IFETCH", 0) / max(r.get("SQ_WAVES", 1), 1),
            "avg_vmem_in_flight_per_wave": r.get("SQ_INST_LEVEL_VMEM", 0) / max(r.get("SQ_LEVEL_WAVES", 1), 1),
        }
        out[cfg] = r
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
