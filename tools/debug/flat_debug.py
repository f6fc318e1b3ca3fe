"""Where does the flat kernel differ from the golden sweep?"""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import numpy as np, torch
from conftest import sweep_arena
from rustnetworkstack_amd.batch import csum_batch
sw = json.load(open("tests/golden/sweep_vectors.json"))
arena = torch.from_numpy(sweep_arena(sw)).to("cuda:0")
off = np.array(sw["offset"], dtype=np.uint64); ln = np.array(sw["length"], dtype=np.uint32)
sd = np.array(sw["pkt_seed"], dtype=np.uint16); exp = np.array(sw["expect"], dtype=np.uint16)
d = lambda a, v: torch.from_numpy(np.ascontiguousarray(a).view(v)).to("cuda:0")
for shape in [(18, 64, 2, 0), (18, 64, 4, 0), (16, 64, 2, 0)]:
    out = csum_batch(arena, d(off, np.int64), d(ln, np.int32), d(sd, np.int16), shape=shape)
    torch.cuda.synchronize()
    got = out.view(torch.int16).cpu().numpy().view(np.uint16)
    bad = np.nonzero(got != exp)[0]
    print(shape, "bad", bad.size, "of", exp.size)
    for i in bad[:12]:
        b = i // 64
        print("  pkt", i, "batch", b, "lane", i % 64, "off", off[i], "len", ln[i], "got", got[i], "exp", exp[i],
              "batch lens", ln[b*64:(b+1)*64].min(), ln[b*64:(b+1)*64].max(), int(((ln[b*64:(b+1)*64].astype(np.int64) + (off[b*64:(b+1)*64] & 15).astype(np.int64) + 15)//16).sum()))
