"""Reconcile a bench line with the rocprofv3 kernel trace of THE SAME run.

On the GPU box (tools/gpu_session.sh does this):

    rocprofv3 --kernel-trace --stats --output-format csv -d <dir> -o run -- \\
        python3 bench.py --gpus 1 --steps 20 --warmup 5 > bench.log

then here (or there):

    python tools/profile_bench.py --trace <dir>/run_kernel_trace.csv --bench bench.log \\
        --out profiles/archive/r02/r02_rocprof_bench_c3_1500B.json

bench.py's own dispatches of the product kernel come first, in order: W warmup
launches, K timed launches (one event pair around all of them), then, with
--median-launches M, M launches each inside its own event pair.  Later
dispatches of the same kernel (the host-pipeline leg's chunks) have smaller
grids and are excluded by grid size.  Writes the per-dispatch mean and median of
the K timed launches next to the bench line's kernel_avg_us and the frac each
implies (and, if present, the event-pair launches' durations).
"""
import argparse
import csv
import json
import re
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--bench", required=True, help="log holding the bench JSON line")
    ap.add_argument("--stats", default="", help="run_kernel_stats.csv of the same run (copied into the summary)")
    ap.add_argument("--out", required=True)
    ap.add_argument("--timed-stats-out", default="",
                    help="write a rocprofv3-style stats CSV row for the K timed dispatches only")
    ap.add_argument("--kernel", default="csum_", help="substring of the product kernel's name")
    args = ap.parse_args()

    line = [ln for ln in open(args.bench) if ln.startswith("{")][-1]
    b = json.loads(line)
    W, K = b.get("launches_before_timed", b["warmup"]), b["steps"]
    M = b["roofline"].get("evpair_launches", 0)
    # the product kernel is the one the line names (e.g. verify mode's batch is built by the
    # transmit-finalize kernel first, which also matches "csum_"): its template name + "<"
    m = re.match(r"[A-Za-z_0-9]+", str(b["roofline"].get("kernel", "")))
    want = (m.group(0) + "<") if m else args.kernel
    rows = [r for r in csv.DictReader(open(args.trace)) if args.kernel in r["Kernel_Name"] and want in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    if not rows:
        raise SystemExit("no dispatch of the product kernel in the trace")
    grid = int(rows[0]["Grid_Size_X"])
    name = rows[0]["Kernel_Name"]
    mine = [r for r in rows if int(r["Grid_Size_X"]) == grid and r["Kernel_Name"] == name]
    rot = b["config"].get("rotating_batches", 1)
    iso = b["roofline"].get("isolated")
    n_iso = iso["launches"] if iso else 0
    need = W + K + n_iso + M
    if len(mine) < need:
        raise SystemExit(f"trace has {len(mine)} dispatches of the bench kernel, expected >= {need}")
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in mine[:need]]
    timed, iso_d, per = dur[W:W + K], dur[W + K:W + K + n_iso], dur[W + K + n_iso:need]
    algo = b["roofline"]["algorithmic_bytes_per_launch"]
    peak = b["roofline"]["peak"]

    def frac(us):
        return round(algo / (us * 1e-6) / 1e9 / peak, 4)

    gaps = [(int(mine[i + 1]["Start_Timestamp"]) - int(mine[i]["End_Timestamp"])) / 1e3 for i in range(W, W + K - 1)]
    # span of the K timed dispatches (first start to last end) / K: the per-step time when
    # consecutive steps overlap on several streams (bench.py graph mode)
    span = (max(int(r["End_Timestamp"]) for r in mine[W:W + K]) -
            min(int(r["Start_Timestamp"]) for r in mine[W:W + K])) / 1e3 / K

    out = {
        "command": "rocprofv3 --kernel-trace --stats --output-format csv -- python3 bench.py "
                   f"--gpus 1 --steps {K} --warmup {b['warmup']}",
        "untimed_launches_skipped": W,
        "kernel": name,
        "grid_size_x": grid,
        "rotating_batches": rot,
        "dispatches_used": {"warmup": W, "timed": K, "per_launch": M},
        "rocprof_timed_us": {"mean": round(statistics.mean(timed), 2), "median": round(statistics.median(timed), 2),
                             "min": round(min(timed), 2), "max": round(max(timed), 2)},
        "rocprof_evpair_launches_us": ({"mean": round(statistics.mean(per), 2),
                                        "median": round(statistics.median(per), 2)} if per else None),
        "rocprof_gap_between_timed_launches_us": {"median": round(statistics.median(gaps), 2) if gaps else None,
                                                  "max": round(max(gaps), 2) if gaps else None},
        "bench": {"kernel_avg_us": b["roofline"]["kernel_avg_us"], "evpair_median_us": b["roofline"].get("evpair_median_us"),
                  "frac": b["roofline"]["frac"], "value": b["value"], "ms_per_step": b["ms_per_step"]},
        "rocprof_timed_span_us_per_launch": round(span, 2),
        "frac_from_rocprof_timed_span": frac(span),
        "frac_from_rocprof_timed_median": frac(statistics.median(timed)),
        "bench_frac_vs_rocprof_timed_median": round(b["roofline"]["frac"] / frac(statistics.median(timed)) - 1, 4),
        "bench_frac_vs_rocprof_timed_span": round(b["roofline"]["frac"] / frac(span) - 1, 4),
    }
    if iso_d:
        out["isolated"] = {"bench_kernel_avg_us": iso["kernel_avg_us"], "bench_frac": iso["frac"],
                           "rocprof_per_dispatch_us": {"mean": round(statistics.mean(iso_d), 2),
                                                       "median": round(statistics.median(iso_d), 2)},
                           "frac_from_rocprof_median": frac(statistics.median(iso_d)),
                           "bench_vs_rocprof_median": round(iso["frac"] / frac(statistics.median(iso_d)) - 1, 4)}
    if args.stats:
        out["stats_csv"] = [r for r in csv.DictReader(open(args.stats))]
        out["stats_csv_note"] = ("whole-run --stats: the product kernel's row also counts the warmup launches and "
                                 "the host-pipeline leg's chunk launches (smaller grids); the timed launches alone "
                                 "are rocprof_timed_us")
    if args.timed_stats_out:
        ns = [round(d * 1e3) for d in timed]
        with open(args.timed_stats_out, "w", newline="") as f:
            w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MedianNs", "MinNs", "MaxNs", "StdDev"])
            w.writerow([name, len(ns), sum(ns), round(statistics.mean(ns), 3), statistics.median(ns), min(ns),
                        max(ns), round(statistics.pstdev(ns), 3)])
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out.get(k) for k in ("rocprof_timed_us", "rocprof_timed_span_us_per_launch", "bench",
                                              "frac_from_rocprof_timed_span", "bench_frac_vs_rocprof_timed_span",
                                              "frac_from_rocprof_timed_median", "isolated")}))


if __name__ == "__main__":
    main()
