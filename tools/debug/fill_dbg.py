import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np, torch
from oracle import oracle as O
from rustnetworkstack_amd.batch import csum_fill
from rustnetworkstack_amd.workloads import make_layout
from test_gpu_fill import expected_fill, stored_be, dev, host_u16
oracle = O.get_oracle()
n = 50000
lay = make_layout("c5_imix", n=n)
w = O.splitmix64_words(0xF1E1D, n)
shift = (w & np.uint64(7)).astype(np.uint64)
off = lay.off + shift
ln = np.maximum(lay.length - 8, 20).astype(np.uint32)
field = np.array([2, 6, 10, 16, 3, 17], dtype=np.uint32)[(w >> np.uint64(8)) % np.uint64(6)]
arena_np = O.splitmix64_bytes(0xABBA, lay.arena_bytes + 16)
zeroed, expect = expected_fill(oracle, arena_np, off, ln, lay.seed, field)
arena = torch.from_numpy(arena_np.copy()).to("cuda:0")
out = torch.empty(n, dtype=torch.uint16, device="cuda:0")
csum_fill(arena, dev(off, np.int64), dev(ln, np.int32), dev(lay.seed, np.int16),
          field=dev(field.astype(np.uint16), np.int16), out=out)
got = arena.cpu().numpy()
o = host_u16(out)
print("out ok", np.array_equal(o, expect))
st = stored_be(got, off, field)
bad = np.nonzero(st != expect)[0]
print("bad", len(bad))
for i in bad[:20]:
    fp = int(off[i]) + int(field[i])
    print(i, "off%16", int(off[i]) % 16, "len", int(ln[i]), "field", int(field[i]), "fp%32", fp % 32,
          "stored %04x expect %04x orig %04x" % (st[i], expect[i], (arena_np[fp] << 8) | arena_np[fp + 1]),
          "i%64", i % 64)
# other bytes changed?
mask = np.ones(got.shape[0], dtype=bool)
idx = off.astype(np.int64) + field.astype(np.int64)
mask[idx] = False; mask[idx + 1] = False
ch = np.nonzero(got[mask] != arena_np[mask])[0]
print("other bytes changed", len(ch))
