"""c3 diagnostics: explicit descriptors vs the strided entry (no descriptor loads),
with and without per-packet seeds, and a few shapes.  Device time per launch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from rustnetworkstack_amd.batch import PreparedBatch, csum_batch_strided  # noqa: E402
from rustnetworkstack_amd.workloads import DeviceBatch, make_layout  # noqa: E402


def timed(fn, steps=30, rounds=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(); fn()
    res = []
    for _ in range(rounds):
        e0.record()
        for _ in range(steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / steps * 1e3)
    return sorted(res)[len(res) // 2]


lay = make_layout("c3_1500B")
b = DeviceBatch(lay, "cuda:0")
ref = None
rows = []
for name, fn in [
    ("explicit+seed", PreparedBatch(b.arena, b.off, b.length, b.seed, complement=True, out=b.out, len_hint=1500)),
    ("explicit noseed", PreparedBatch(b.arena, b.off, b.length, None, complement=True, out=b.out, len_hint=1500)),
    ("strided+seed", lambda: csum_batch_strided(b.arena, lay.n, 1504, 1500, seed=b.seed, complement=True, out=b.out)),
    ("strided noseed", lambda: csum_batch_strided(b.arena, lay.n, 1504, 1500, complement=True, out=b.out)),
]:
    rows.append((name, timed(fn)))
for s in [(3, 32, 4, 0), (3, 64, 2, 0), (3, 16, 8, 0), (2, 64, 4, 0), (2, 32, 4, 0), (3, 32, 4, 8192), (3, 32, 4, 4096)]:
    rows.append((str(s), timed(PreparedBatch(b.arena, b.off, b.length, b.seed, complement=True, out=b.out,
                                             len_hint=1500, shape=s))))
for name, us in rows:
    print(f"{name:24s} {us:8.1f} us  {(lay.payload_bytes + 2 * lay.n) / us / 1e3:8.1f} GB/s")
