"""Flat kernel on small synthetic batches: which packets differ from the oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from oracle.oracle import get_oracle, splitmix64_bytes
from rustnetworkstack_amd.batch import csum_batch
orc = get_oracle()
arena_np = splitmix64_bytes(7, 1 << 20)
arena = torch.from_numpy(arena_np).to("cuda:0")
d = lambda a, v: torch.from_numpy(np.ascontiguousarray(a).view(v)).to("cuda:0")
def run(name, off, ln):
    off = np.asarray(off, dtype=np.uint64); ln = np.asarray(ln, dtype=np.uint32)
    exp = orc.batch(arena_np, off, ln, None)
    out = csum_batch(arena, d(off, np.int64), d(ln, np.int32), None, shape=(18, 64, 2, 0))
    torch.cuda.synchronize()
    got = out.view(torch.int16).cpu().numpy().view(np.uint16)
    bad = np.nonzero(got != exp)[0]
    print(f"{name:28s} bad {bad.size:4d}/{exp.size}  first {bad[:16].tolist()}")
n = 64
run("16B aligned", np.arange(n) * 16, [16] * n)
run("32B aligned", np.arange(n) * 32, [32] * n)
run("48B aligned (3 chunks)", np.arange(n) * 48, [48] * n)
run("1..64 B, 16B slots of 64", np.arange(n) * 64, np.arange(1, n + 1))
run("20B at stride 20 (unaligned)", np.arange(n) * 20, [20] * n)
run("1500B", np.arange(n) * 1504, [1500] * n)
run("lanes 0..19 1 chunk, rest 2", np.arange(n) * 32, [16] * 20 + [32] * 44)
run("lanes 0..15 1 chunk, rest 2", np.arange(n) * 32, [16] * 16 + [32] * 48)
run("lanes 0..31 1 chunk, rest 2", np.arange(n) * 32, [16] * 32 + [32] * 32)
run("one 2-chunk at lane 20", np.arange(n) * 32, [16] * 20 + [32] + [16] * 43)
