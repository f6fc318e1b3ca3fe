"""Layout diagnostics (device time per launch, median of rounds of back-to-back launches):

* IMIX (c5) with packet starts aligned to 16 / 32 / 64 / 128 bytes: at 128 no two
  packets share a 128-byte line, so the time against the lines each layout touches
  shows what the re-fetch of shared lines costs;
* c2 (1M x 64 B, rotated over enough batches to defeat the Infinity Cache) through the
  64-bit, compact (u32 offset) and strided (no offset/length arrays) entries.

    python tools/probe_layouts.py [--out gpurun_out/probe_layouts.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rustnetworkstack_amd.batch import csum_batch_strided  # noqa: E402
from rustnetworkstack_amd.workloads import DeviceBatch, make_layout  # noqa: E402


def timed(fns, steps=30, rounds=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for f in fns:
        f()
    res = []
    for _ in range(rounds):
        e0.record()
        for i in range(steps):
            fns[i % len(fns)]()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / steps * 1e3)
    return sorted(res)[len(res) // 2]


def lines_touched(lay):
    first = lay.off // np.uint64(128)
    last = (lay.off + lay.length.astype(np.uint64) - np.uint64(1)) // np.uint64(128)
    per = (last - first + np.uint64(1)).astype(np.int64)
    # lines shared with the previous packet are counted once
    shared = np.zeros(lay.n, dtype=np.int64)
    shared[1:] = (first[1:] == last[:-1])
    return int(per.sum() - shared.sum()), int(per.sum())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--skip-align", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    res = {"imix_align": [], "c2": [], "forms": []}
    for name in ("c3_1500B", "c4_9000B", "c5_imix"):
        lay = make_layout(name)
        b = DeviceBatch(lay, dev)
        small = lay.arena_bytes + 16 < 2 ** 32
        row = {"config": name}
        for form, fn in (("64-bit", b.launcher(complement=True)),
                         ("compact", b.launcher(complement=True, compact=True) if small else None),
                         ("packed", b.launcher(complement=True, packed=True))):
            if fn is not None:
                row[form] = round(timed([fn]), 1)
        res["forms"].append(row)
        print(json.dumps(row), flush=True)
        del b
        torch.cuda.empty_cache()
    for align in (() if args.skip_align else (16, 32, 64, 128)):
        lay = make_layout("c5_imix", align=align)
        b = DeviceBatch(lay, dev)
        fn = b.launcher(complement=True, compact=lay.arena_bytes + 16 < 2 ** 32)
        us = timed([fn])
        uniq, per_pkt = lines_touched(lay)
        row = {"align": align, "us": round(us, 1), "arena_bytes": lay.arena_bytes,
               "payload_GBps": round(lay.payload_bytes / us / 1e3, 1),
               "lines_unique": uniq, "lines_per_packet_sum": per_pkt,
               "unique_line_TBps": round(uniq * 128 / us / 1e6, 3),
               "per_packet_line_TBps": round(per_pkt * 128 / us / 1e6, 3)}
        res["imix_align"].append(row)
        print(json.dumps(row), flush=True)
        del b, fn
        torch.cuda.empty_cache()
    lays = [make_layout("c2_64B", data_seed=0x5EEDC0DE + r) for r in range(12)]
    bs = [DeviceBatch(lay, dev) for lay in lays]
    n, pay = lays[0].n, lays[0].payload_bytes
    for name, fns in [
        ("64-bit", [b.launcher(complement=True) for b in bs]),
        ("compact", [b.launcher(complement=True, compact=True) for b in bs]),
        ("packed", [b.launcher(complement=True, packed=True) for b in bs]),
        ("strided+seed", [(lambda b=b: csum_batch_strided(b.arena, n, 64, 64, seed=b.seed, complement=True,
                                                          out=b.out)) for b in bs]),
        ("strided noseed", [(lambda b=b: csum_batch_strided(b.arena, n, 64, 64, complement=True, out=b.out))
                            for b in bs]),
    ]:
        us = timed(fns, steps=60)
        row = {"form": name, "us": round(us, 2), "algo_GBps": round((pay + 2 * n) / us / 1e3, 1)}
        res["c2"].append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
