"""c2 (1M x 64 B) diagnostics: device time per launch over 12 rotating batches (the
Infinity Cache cannot hold them) for the descriptor forms and rounds-kernel shapes.
Run once per library build (RNS_CHECKSUM_LIB=... for A/B builds), --label names it.

    python tools/probe_c2.py [--label product] [--out gpurun_out/probe_c2.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rustnetworkstack_amd.batch import csum_batch_strided  # noqa: E402
from rustnetworkstack_amd.workloads import DeviceBatch, make_layout  # noqa: E402
from tools.probe_layouts import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--label", default="product")
    ap.add_argument("--out", default="")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lays = [make_layout("c2_64B", data_seed=0x5EEDC0DE + r) for r in range(12)]
    bs = [DeviceBatch(lay, dev) for lay in lays]
    n, pay = lays[0].n, lays[0].payload_bytes
    forms = [
        ("compact", [b.launcher(complement=True, compact=True) for b in bs]),
        ("packed", [b.launcher(complement=True, packed=True) for b in bs]),
        ("strided+seed", [(lambda b=b: csum_batch_strided(b.arena, n, 64, 64, seed=b.seed, complement=True,
                                                          out=b.out)) for b in bs]),
    ]
    for shape in [(3, 4, 1, 2048), (19, 4, 1, 2048), (19, 4, 1, 1024), (19, 4, 1, 4096), (19, 4, 1, 0),
                  (3, 4, 1, 0), (19, 8, 1, 2048), (19, 4, 2, 2048)]:
        forms.append((f"64-bit shape {list(shape)}", [b.launcher(complement=True, shape=shape) for b in bs]))
    ref = [b.launcher(complement=True)() for b in bs]
    ref = [r.clone() for r in ref]
    rows = {}
    for rep in range(args.reps):  # interleaved repetitions
        for name, fns in forms:
            us = timed(fns, steps=60)
            rows.setdefault(name, []).append(round(us, 2))
    ok = True
    for name, fns in forms:  # every form's results equal the default path's
        for b, f, r in zip(bs, fns, ref):
            out = f()
            ok = ok and torch.equal(out.view(torch.int16), r.view(torch.int16))
    res = {"label": args.label, "same_results": bool(ok), "algo_bytes": pay + 2 * n,
           "us": {k: sorted(v)[len(v) // 2] for k, v in rows.items()}, "us_all": rows}
    for k, v in res["us"].items():
        print(f"{args.label:10s} {k:32s} {v:7.2f} us  {(pay + 2 * n) / v / 1e3:7.1f} GB/s", flush=True)
    print("same results:", ok)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
