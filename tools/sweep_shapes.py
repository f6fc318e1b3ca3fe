"""Kernel-shape sweep on one GPU: average device time per launch (HIP events on the
launch stream), interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).

    python tools/sweep_shapes.py [--configs c3_1500B,...] [--rounds 5] [--iters 10]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rustnetworkstack_amd.workloads import DeviceBatch, make_layout  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3_1500B,c4_9000B,c2_64B,c5_imix,d40B,d576B")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default="")
    args = ap.parse_args()
    if args.shapes:
        shapes = [tuple(int(x) for x in s.split(",")) for s in args.shapes.split(";")]
    else:
        shapes = [(v, g, u, 0) for v in (0, 2) for g in (16, 64) for u in (2, 4)]
        shapes += [(v, g, u, 0) for v in (1, 3) for g in (4, 8, 16, 32, 64) for u in (1, 2, 4, 8)]
        shapes += [(v, 4, u, 2048) for v in (1, 3) for u in (1, 2)]
        shapes += [(v, 0, 0, mb) for v in (4, 6) for mb in (0, 1024, 2048, 4096)]
    results = {}
    for cfg in args.configs.split(","):
        lay = make_layout(cfg)
        b = DeviceBatch(lay, "cuda:0")
        b.run()
        ref = b.host_out()
        times = {s: [] for s in shapes}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(args.rounds):
            for s in shapes:
                launch = b.launcher(shape=s)   # pre-bound: one ctypes call per launch
                launch()
                launch()
                e0.record()                    # queued behind the warm-up launches: no idle gap
                for i in range(args.iters):
                    launch()
                e1.record()
                torch.cuda.synchronize()
                times[s].append(e0.elapsed_time(e1) / args.iters)
                assert (b.host_out() == ref).all(), s
        algo = lay.payload_bytes + 2 * lay.n
        rows = []
        for s in shapes:
            t = sorted(times[s])
            med = t[len(t) // 2]
            rows.append((med, s, algo / (med * 1e-3) / 1e9, t[0]))
        rows.sort()
        results[cfg] = [{"shape": list(s), "median_us": round(m * 1e3, 1), "min_us": round(mn * 1e3, 1),
                         "GBps": round(gbs, 1)} for m, s, gbs, mn in rows]
        print(cfg, json.dumps(results[cfg][:8]), flush=True)
        del b
        torch.cuda.empty_cache()
    print(json.dumps(results))


if __name__ == "__main__":
    main()
