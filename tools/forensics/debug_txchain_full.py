"""Debug aid (round 6): the full-size chain-finalize check of tests/test_gpu_tx_chain.py for one
config, every datagram of the first SAMPLE compared with the oracle, mismatches described.
    python tools/forensics/debug_txchain_full.py c5_imix 512 [sample]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from rustnetworkstack_amd.batch import csum_chain, fill_splitmix64, tx_fill_chain  # noqa: E402
from rustnetworkstack_amd.workloads import tx_chain_layout  # noqa: E402

R4 = bytes([192, 168, 1, 1])
L4 = bytes([192, 168, 1, 2])


def main():
    name, frag = sys.argv[1], int(sys.argv[2])
    sample = int(sys.argv[3]) if len(sys.argv) > 3 else 3000
    DEV = "cuda:0"
    orc = O.get_oracle()
    lay = tx_chain_layout(name, head=40, frag=frag)
    a = torch.empty(lay.arena_bytes + 64, dtype=torch.uint8, device=DEV)
    fill_splitmix64(a, lay.data_seed)
    first = lay.first.astype(np.int64)
    hoff = lay.frag_off[first[:-1]].astype(np.int64)
    hdr = np.frombuffer(bytes.fromhex("4500000000004000400600000000000000000000"), dtype=np.uint8).copy()
    hdr[12:16] = np.frombuffer(R4, dtype=np.uint8)
    hdr[16:20] = np.frombuffer(L4, dtype=np.uint8)
    d_hoff = torch.from_numpy(hoff).to(DEV)
    idx = d_hoff.view(-1, 1) + torch.arange(20, device=DEV)
    a[idx.flatten()] = torch.from_numpy(hdr).to(DEV).repeat(lay.n)
    del idx
    # (the sample's fragments end anywhere below the last one's: a head-only datagram's last
    # fragment is its head, in the header region)
    s_end = int((lay.frag_off[:first[sample]] + lay.frag_len[:first[sample]].astype(np.uint64)).max())
    before = a[:s_end].cpu().numpy()
    d_off = torch.from_numpy(lay.frag_off.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lay.frag_len.view(np.int32)).to(DEV)
    d_first = torch.from_numpy(lay.first.view(np.int32)).to(DEV)
    st = tx_fill_chain(a, d_off, d_len, d_first).cpu().numpy()
    after = a[:s_end].cpu().numpy()
    print("lib", os.environ.get("RNS_CHECKSUM_LIB", "default"), "status != 3:", int((st != 3).sum()))
    changed = np.flatnonzero(before != after)
    heads_end = int(hoff[sample - 1] + 40)
    print("changed bytes in sample range:", changed.size, "outside head region:", int((changed >= heads_end).sum()))
    bad = 0
    for i in range(sample):
        fr = [bytes(before[int(o):int(o) + int(n)]) for o, n in
              zip(lay.frag_off[first[i]:first[i + 1]], lay.frag_len[first[i]:first[i + 1]])]
        h, s = O.tx_chain_fill_ref(fr, ones_comp=orc.compute_ones_comp)
        got = bytes(after[hoff[i]:hoff[i] + 40])
        if got != h:
            bad += 1
            if bad <= 12:
                # the same chain read from the AFTER bytes (payload unchanged?)
                fr2 = [bytes(after[int(o):int(o) + int(n)]) for o, n in
                       zip(lay.frag_off[first[i]:first[i + 1]], lay.frag_len[first[i]:first[i + 1]])]
                same_pay = fr2[1:] == fr[1:]
                d = [k for k in range(40) if got[k] != h[k]]
                print(f"i={i} wave={i // 64} lane={i % 64} L={sum(len(f) for f in fr)} frags={[len(f) for f in fr]} "
                      f"hoff={hoff[i]} diff_at={d} got={got[d[0]:d[-1] + 1].hex()} want={h[d[0]:d[-1] + 1].hex()} "
                      f"payload_unchanged={same_pay}")
    print("mismatching datagrams:", bad, "of", sample)
    # the receive-side chain check on the device for the sample
    off2 = lay.frag_off.copy()
    ln2 = lay.frag_len.copy()
    off2[first[:-1]] += 20
    ln2[first[:-1]] -= 20
    L = np.add.reduceat(lay.frag_len.astype(np.int64), first[:-1])
    segs, inv = np.unique(L - 20, return_inverse=True)
    ph = np.array([O.pseudo_header_py(R4, L4, int(s), 6) for s in segs], dtype=np.uint16)[inv]
    bad_t = torch.zeros(1, dtype=torch.int32, device=DEV)
    l4 = csum_chain(a, torch.from_numpy(off2.view(np.int64)).to(DEV), torch.from_numpy(ln2.view(np.int32)).to(DEV),
                    d_first, torch.from_numpy(ph.view(np.int16)).to(DEV), complement=True, bad=bad_t)
    l4h = l4.view(torch.int16).cpu().numpy().view(np.uint16)
    print("device L4 check: nonzero", int((l4h != 0).sum()), "bad", int(bad_t.item()))


if __name__ == "__main__":
    main()
