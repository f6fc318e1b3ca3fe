"""Copy the judged evidence of one gpurun session (gpurun_out/<tag>/) into profiles/.

    python tools/collect_profiles.py r01i --round r01

Writes profiles/<round>_bench_<config>.json (the bench JSON lines),
profiles/<round>_rocprof_bench_<config>.json / _timed_stats.csv / _kernel_stats.csv
(tools/gpu_session.sh: rocprofv3 --kernel-trace --stats of that same bench command,
reconciled by tools/profile_bench.py), profiles/traffic_<config>.json (PMC
FETCH_SIZE/WRITE_SIZE per launch, read by bench.py) and the sweep JSON if present.
"""
import argparse
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--round", default="r01")
    args = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", args.tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    for name in sorted(os.listdir(src)):
        if name.startswith("bench") and name.endswith(".log"):
            lines = [ln for ln in open(os.path.join(src, name)) if ln.startswith("{")]
            if lines:
                d = json.loads(lines[-1])
                cfg = d["config"]["workload"].split(":")[0]
                with open(os.path.join(dst, f"{args.round}_bench_{cfg}.json"), "w") as f:
                    json.dump(d, f, indent=1)
    for name in os.listdir(src):
        if name.startswith("traffic_") and name.endswith(".json"):
            d = json.load(open(os.path.join(src, name)))
            d["source"] = (f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes over "
                           f"`bench.py --steps 5 --warmup 1` (gpurun_out/{args.tag}/pmc_fetch, pmc_write)")
            d["collected"] = f"{args.round} gpurun session {args.tag}"
            with open(os.path.join(dst, name), "w") as f:
                json.dump(d, f, indent=1)
    # tools/gpu_session.sh: the bench line and the rocprofv3 trace of that same command
    for name in os.listdir(src):
        if name.startswith("rocprof_bench_") and name.endswith(".json"):
            cfg = name[len("rocprof_bench_"):-len(".json")]
            d = json.load(open(os.path.join(src, name)))
            d["collected"] = f"{args.round} gpurun session {args.tag}"
            with open(os.path.join(dst, f"{args.round}_rocprof_bench_{cfg}.json"), "w") as f:
                json.dump(d, f, indent=1)
            for suffix, srcname in (("_timed_stats.csv", f"rocprof_bench_{cfg}_timed_stats.csv"),
                                    ("_kernel_stats.csv", os.path.join("prof", "run_kernel_stats.csv"))):
                sp = os.path.join(src, srcname)
                if os.path.exists(sp):
                    shutil.copy(sp, os.path.join(dst, f"{args.round}_rocprof_bench_{cfg}{suffix}"))
    sw = os.path.join(src, "sweep.log")
    if os.path.exists(sw):
        lines = [ln for ln in open(sw) if ln.startswith("{")]
        if lines:
            with open(os.path.join(dst, f"{args.round}_sweep_{args.tag}.json"), "w") as f:
                json.dump(json.loads(lines[-1]), f, indent=1)
    print(sorted(os.listdir(dst)))


if __name__ == "__main__":
    sys.exit(main())
