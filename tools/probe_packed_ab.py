"""A/B of library builds on the packed descriptor form (rns_csum_batch_packed_dev,
what bench.py runs for c2, c3 and c5): device time of one launch over each batch,
one pair of HIP events around K back-to-back launches, median of R rounds.

Each config is timed with its natural kernel (len_hint = the batch's mean length)
and, for the diagnostic one-size batches, also forced through the size-class kernel
(len_hint 500) so its per-class cost shows.  Results carry a checksum of the
results so builds can be compared for equality.

    RNS_CHECKSUM_LIB=<lib.so> python tools/probe_packed_ab.py --label <name> [--out f.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rustnetworkstack_amd.batch import PackedBatch  # noqa: E402
from rustnetworkstack_amd.workloads import DeviceBatch, make_layout  # noqa: E402


def timed(fn, steps, rounds):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    res = []
    for _ in range(rounds):
        e0.record()
        for _ in range(steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / steps * 1e3)
    res.sort()
    return res[len(res) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default=os.path.basename(os.environ.get("RNS_CHECKSUM_LIB", "in-tree")))
    ap.add_argument("--configs", default="c5_imix,c3_1500B,d40B:500,d576B:500,c2_64B,c5_imix")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    res = {"label": args.label, "lib": os.environ.get("RNS_CHECKSUM_LIB", "in-tree")}
    cache = {}
    for item in args.configs.split(","):
        name, _, hint = item.partition(":")
        if name not in cache:
            cache.clear()
            torch.cuda.empty_cache()
            cache[name] = DeviceBatch(make_layout(name), dev)
        b = cache[name]
        lay = b.layout
        nat = b.launcher(complement=True, packed=True)  # uploads the packed descriptors once
        pb = nat if not hint else PackedBatch(b.arena, b.blk_off, b.len16, b.seed, align_log2=4, complement=True,
                                              out=b.out, len_hint=int(hint))
        us = timed(pb, args.steps, args.rounds)
        key = item if item not in res else item + "_again"
        res[key] = {"us": round(us, 2), "GBps": round((lay.payload_bytes + 2 * lay.n) / us / 1e3, 1),
                    "checksum_of_results": int(b.out.to(torch.int64).sum().item())}
        print(key, json.dumps(res[key]), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
