"""Per-launch HBM traffic of the checksum kernel from rocprofv3 PMC passes.

Collect the counters in SEPARATE passes (MI355X_MICROARCH.md §rocprofv3 PMC slots:
FETCH_SIZE and WRITE_SIZE do not fit one pass), kernel-trace only, e.g.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py ...
    python tools/pmc_traffic.py --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write \
        --config c3_1500B --out profiles/traffic_c3_1500B.json

Correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE is in KiB and on gfx950 reports
exactly half the bytes of a wide (16 B/lane) coalesced streaming read, so
    hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
Both the raw and the corrected values are written.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def per_dispatch(path: str, counter: str, kernel_substr: str):
    files = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {path}")
    vals = defaultdict(float)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_substr not in row.get("Kernel_Name", ""):
                    continue
                if row.get("Counter_Name") != counter:
                    continue
                vals[(f, row.get("Dispatch_Id"))] += float(row["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--config", required=True)
    ap.add_argument("--kernel", default="csum_rounds_kernel")
    ap.add_argument("--algo-bytes", type=float, default=None, help="algorithmic bytes per launch, for the ratio")
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    fetch = per_dispatch(args.fetch, "FETCH_SIZE", args.kernel)
    write = per_dispatch(args.write, "WRITE_SIZE", args.kernel)
    if not fetch or not write:
        raise SystemExit(f"no dispatches of {args.kernel} found")
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    hbm = 2 * f_kib * 1024 + w_kib * 1024
    res = {
        "config": args.config,
        "kernel": args.kernel,
        "dispatches": {"fetch_pass": len(fetch), "write_pass": len(write)},
        "FETCH_SIZE_KiB_per_launch_raw": round(f_kib, 1),
        "WRITE_SIZE_KiB_per_launch_raw": round(w_kib, 1),
        "hbm_bytes_per_launch": int(hbm),
        "correction": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halves wide streaming reads)",
        "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes ({args.fetch}, {args.write})",
    }
    if args.algo_bytes:
        res["traffic_over_algorithmic"] = round(hbm / args.algo_bytes, 4)
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
