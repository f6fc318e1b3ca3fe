"""Summarise tools/pmc_compare.sh: per-dispatch counter means for the probe's streaming
read kernel and the c3 checksum kernel, plus per-KB and per-wave ratios."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = {"probe": "read_store<0, 2>", "c3": "csum_"}


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
    root = sys.argv[1]
    out = {}
    for who in KERNELS:
        r = collect(root, who)
        kb = (1577058304 if who == "probe" else 1504 * (1 << 20)) / 1024  # bytes each dispatch streams
        waves = r.get("SQ_WAVES", 0) or 1
        r["derived"] = {
            "VALU_per_KB": r.get("SQ_INSTS_VALU", 0) * 1.0 / kb,
            "VMEM_RD_per_KB": r.get("SQ_INSTS_VMEM_RD", 0) / kb,
            "wait_frac": r.get("SQ_WAIT_ANY", 0) / max(r.get("SQ_WAVE_CYCLES", 1), 1),
            "active_frac": r.get("SQ_ACTIVE_INST_ANY", 0) / max(r.get("SQ_WAVE_CYCLES", 1), 1),
            "wave_cycles_per_wave": r.get("SQ_WAVE_CYCLES", 0) / waves,
            "avg_vmem_in_flight_per_wave": r.get("SQ_INST_LEVEL_VMEM", 0) / max(r.get("SQ_LEVEL_WAVES", 1), 1),
            "tcp_tcc_read_latency": r.get("TCP_TCC_READ_REQ_LATENCY_sum", 0) / max(r.get("TCP_TCC_READ_REQ_sum", 1), 1),
            "tcp_tcc_read_req_per_KB": r.get("TCP_TCC_READ_REQ_sum", 0) / kb,
        }
        out[who] = r
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
