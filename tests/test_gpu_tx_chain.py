"""Transmit finalize of NetBuffer chains on the GPU (rns_tx_fill_chain_dev: the transmit-rows
kernel in FIN mode) against oracle.tx_chain_fill_ref — the reference's transmit path over the
layout it really sends: alloc_header's head fragment holding the IP header and the L4 header
(buf.rs:262-291), then the payload fragments (buf.rs:385-420); the L4 checksum folded per
fragment over [head[hdr:], payload...] (tcp.rs:957-973, udp.rs:151-171, icmp.rs:87-112) and the
IPv4 header checksum (ip.rs:140-160), both stored into the head.  Every arena byte after the
fill and the status per datagram are compared."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from rustnetworkstack_amd import _lib
from rustnetworkstack_amd.batch import csum_batch, csum_chain, fill_splitmix64, tx_fill_chain
from rustnetworkstack_amd.workloads import tx_chain_layout
from test_gpu_tx import outgoing
from test_gpu_tx_packed import edge_datagrams
from test_rx_oracle import L4, L6, R4, R6, ipv4, tcp_seg

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dev(a, view):
    return torch.from_numpy(np.ascontiguousarray(a).view(view)).to(DEV)


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or _lib.load().rns_device_count() == 0:
        pytest.fail("gpu tests need a GPU (the HIP path has no CPU fallback)")


def l4_header_len(p):
    """Bytes of the L4 header behind the IP header (what alloc_header put in the head)."""
    if not p:
        return 0
    v = p[0] >> 4
    hdr = (p[0] & 15) * 4 if v == 4 else 40
    proto = p[9] if v == 4 and len(p) > 9 else p[6] if len(p) > 6 else 0
    return hdr + {6: 20, 17: 8, 1: 8, 58: 8}.get(proto, 0)


def layout(pkts, seed, *, shape):
    """Cut every datagram into [head, payload pieces] and place them.  shape "tx": heads back to
    back in a header region, each payload a run of even non-final pieces at a 16-byte start
    (the rows); "any": odd pieces, scattered pieces, empty pieces, heads split at any point,
    whole datagrams as one fragment (the exact loop); "mixed": blocks of both."""
    n = len(pkts)
    w = O.splitmix64_words(seed, 6 * n)
    heads, pieces = [], []
    for i, p in enumerate(pkts):
        tx = shape == "tx" or (shape == "mixed" and (i // 64) % 3 != 2)
        hl = min(len(p), l4_header_len(p))
        if not tx:
            r = int(w[6 * i] % np.uint64(8))
            hl = len(p) if r == 0 else min(len(p), hl + int(w[6 * i + 1] % np.uint64(9))) if r < 6 else \
                min(len(p), int(w[6 * i + 1] % np.uint64(70)))
        rest = p[hl:]
        k = 1 + int(w[6 * i + 2] % np.uint64(4)) if rest else 0
        cuts = sorted({int(w[6 * i + 3 + j % 3] >> np.uint64(8 * j)) % (len(rest) + 1) for j in range(k - 1)}) \
            if rest else []
        if tx:
            cuts = sorted({c & ~1 for c in cuts})
        b = [0] + cuts + [len(rest)]
        pieces.append([rest[b[j]:b[j + 1]] for j in range(len(b) - 1)] if rest else [])
        heads.append(p[:hl])
    hpos = 3
    off, ln, first = [], [], [0]
    hoffs = []
    for h in heads:
        hoffs.append(hpos)
        hpos += len(h)
    ppos = (hpos + 4096) & ~15
    placed = []
    for i in range(n):
        tx = shape == "tx" or (shape == "mixed" and (i // 64) % 3 != 2)
        if i % 101 == 50:                                   # no fragments at all: malformed
            first.append(len(off))
            placed.append(None)
            continue
        off.append(hoffs[i])
        ln.append(len(heads[i]))
        pl = []
        for j, piece in enumerate(pieces[i]):
            if not tx:
                ppos += int(w[6 * i + 5] >> np.uint64(4 * j)) % 5
            off.append(ppos)
            ln.append(len(piece))
            pl.append((ppos, piece))
            ppos += len(piece)
        ppos = (ppos + 15) & ~15
        placed.append(pl)
        first.append(len(off))
    arena = O.splitmix64_bytes(seed ^ 0xF17, ppos + 64)
    for i in range(n):
        if placed[i] is None:
            continue
        arena[hoffs[i]:hoffs[i] + len(heads[i])] = np.frombuffer(heads[i], dtype=np.uint8)
        for o, piece in placed[i]:
            arena[o:o + len(piece)] = np.frombuffer(piece, dtype=np.uint8)
    return arena, heads, hoffs, placed, np.array(off, np.uint64), np.array(ln, np.uint32), np.array(first, np.uint32)


def expected(oracle, arena, heads, hoffs, placed):
    want = arena.copy()
    st = np.zeros(len(heads), dtype=np.uint8)
    for i in range(len(heads)):
        if placed[i] is None:
            st[i] = O.TX_MALFORMED
            continue
        h, s = O.tx_chain_fill_ref([heads[i]] + [p for _, p in placed[i]], ones_comp=oracle.compute_ones_comp)
        want[hoffs[i]:hoffs[i] + len(h)] = np.frombuffer(h, dtype=np.uint8)
        st[i] = s
    return want, st


def run(arena, off, ln, first, base_shift=0):
    big = torch.from_numpy(np.concatenate([np.zeros(base_shift, np.uint8), arena])).to(DEV)
    a = big[base_shift:]
    st = tx_fill_chain(a, dev(off, np.int64), dev(ln, np.int32), dev(first, np.int32))
    torch.cuda.synchronize()
    return a.cpu().numpy(), st.cpu().numpy()


def check(oracle, pkts, seed, shape, base_shift=0):
    arena, heads, hoffs, placed, off, ln, first = layout(pkts, seed, shape=shape)
    want, want_st = expected(oracle, arena, heads, hoffs, placed)
    got, got_st = run(arena, off, ln, first, base_shift)
    bad = np.flatnonzero(got_st != want_st)
    assert bad.size == 0, [(int(i), int(got_st[i]), int(want_st[i]), pkts[i][:24].hex()) for i in bad[:5]]
    diff = np.flatnonzero(got != want)
    assert diff.size == 0, [(int(d), int(got[d]), int(want[d])) for d in diff[:8]]
    return want_st


@pytest.mark.parametrize("shape,base_shift", [("tx", 0), ("any", 0), ("mixed", 0), ("tx", 5)])
def test_chain_finalize_matches_reference_transmit_path(oracle, shape, base_shift):
    """Every kind of outgoing datagram (TCP / UDP / ICMP over IPv4 and IPv6, options, any
    protocol, short segments, garbage, empty) as a chain; the rows (tx shape), the exact loop
    (odd and scattered pieces, odd head splits, whole datagrams as one fragment) and blocks of
    both; an unaligned arena base."""
    st = check(oracle, outgoing(5000, 0xC4A1 + len(shape) + base_shift), 0x11 + base_shift, shape, base_shift)
    assert len(set(st.tolist())) >= 4


@pytest.mark.parametrize("shape", ["tx", "any"])
def test_chain_finalize_edge_datagrams(oracle, shape):
    """IHL 5..15 against every field position and segment length, IPv6 with short segments
    for each protocol, 65535-byte datagrams, malformed and empty ones, as chains."""
    check(oracle, edge_datagrams(), 0x22, shape)


def test_chain_finalize_equals_contiguous_fill_for_even_pieces():
    """A datagram cut into [IP + L4 headers, even pieces] finalizes to exactly the bytes the
    whole-datagram finalize stores (tx_fill_ref == tx_chain_fill_ref there), and the receive
    path accepts it: IPv4 header checksum 0, and the chain's L4 checksum with the receiver's
    pseudo-header 0 (tcp.rs:838-850)."""
    pkts = [ipv4(6, tcp_seg(R4, L4, O.splitmix64_bytes(k, 1 + k % 1459).tobytes())) for k in range(3000)]
    arena, heads, hoffs, placed, off, ln, first = layout(pkts, 0x33, shape="tx")
    got, st = run(arena, off, ln, first)
    keep = np.array([p is not None for p in placed])
    assert (st[keep] == (_lib.RNS_TX_IP_FILLED | _lib.RNS_TX_L4_FILLED)).all()
    for i in np.flatnonzero(keep)[:400]:
        want, _ = O.tx_fill_ref(pkts[i])
        assert bytes(got[hoffs[i]:hoffs[i] + 40]) == want[:40]
    # the receive side of every chain on the device: IP header and L4 chains verify to 0
    a = torch.from_numpy(got).to(DEV)
    hidx = first[:-1][keep]
    ip = csum_batch(a, dev(off[hidx], np.int64), dev(np.full(hidx.size, 20, np.uint32), np.int32), complement=True)
    assert int(ip.view(torch.int16).ne(0).sum().item()) == 0
    off2, ln2 = off.copy(), ln.copy()
    off2[hidx] += 20
    ln2[hidx] -= 20
    seg = np.array([len(pkts[i]) - 20 for i in np.flatnonzero(keep)])
    seeds = np.array([O.pseudo_header_py(R4, L4, int(s), 6) for s in seg], dtype=np.uint16)
    cnt = (first[1:] - first[:-1])[keep].astype(np.int64)
    f2 = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint32)
    fr = np.repeat(hidx.astype(np.int64), cnt) + (np.arange(int(cnt.sum())) - np.repeat(f2[:-1].astype(np.int64), cnt))
    l4 = csum_chain(a, dev(off2[fr], np.int64), dev(ln2[fr], np.int32), dev(f2, np.int32), dev(seeds, np.int16),
                    complement=True)
    assert int(l4.view(torch.int16).ne(0).sum().item()) == 0


def test_chain_finalize_rejects():
    """Malformed CSR ranges, no fragments, a payload fragment outside the arena (past the first
    four too), heads that do not hold the IP header: RNS_TX_MALFORMED and nothing written."""
    pkt = ipv4(6, tcp_seg(L4, R4, b"z" * 200))
    arena = np.zeros(4096, dtype=np.uint8)
    arena[0:len(pkt)] = np.frombuffer(pkt, dtype=np.uint8)
    arena[1000:1000 + len(pkt)] = np.frombuffer(pkt, dtype=np.uint8)
    # chains: [ok], [head outside], [payload past 5th fragment outside], [head 19 bytes], [reversed]
    off = [0, 40, 9000, 1000, 1040, 1050, 1060, 1070, 1 << 40, 0, 19]
    ln = [40, 200, 40, 40, 10, 10, 10, 10, 10, 19, 221]
    first = [0, 2, 3, 9, 11, 10]
    a = torch.from_numpy(arena.copy()).to(DEV)
    st = tx_fill_chain(a, dev(np.array(off, np.uint64), np.int64), dev(np.array(ln, np.uint32), np.int32),
                       dev(np.array(first, np.uint32), np.int32)).cpu().numpy()
    assert st[0] == _lib.RNS_TX_IP_FILLED | _lib.RNS_TX_L4_FILLED
    assert (st[1:] == _lib.RNS_TX_MALFORMED).all(), st
    got = a.cpu().numpy()
    want = arena.copy()
    want[0:40] = np.frombuffer(O.tx_fill_ref(pkt)[0][:40], dtype=np.uint8)
    assert np.array_equal(got, want)
    with pytest.raises(ValueError):
        tx_fill_chain(a, dev(np.array(off, np.uint64), np.int64), dev(np.array(ln[:-1], np.uint32), np.int32),
                      dev(np.array(first, np.uint32), np.int32))
    with pytest.raises(ValueError):
        tx_fill_chain(a, dev(np.array(off, np.uint64), np.int64), dev(np.array(ln, np.uint32), np.int32),
                      dev(np.array(first, np.uint32), np.int32), status=torch.empty(3, dtype=torch.uint8, device=DEV))


@pytest.mark.parametrize("name,frag", [("c3_1500B", 0), ("c5_imix", 512)])
def test_chain_finalize_full_size_then_receive(oracle, name, frag):
    """The bench batches as the reference lays them out to send: 40-byte IPv4 + TCP head
    fragments back to back in a header region, the payload as one fragment or as 512-byte
    NetBuffer fragments.  One finalize: every status IP + L4 filled; then on the device every
    IP header checksums to 0 and every [TCP header, payload] chain with the receiver's
    pseudo-header to 0; a sample against the oracle."""
    lay = tx_chain_layout(name, head=40, frag=frag)
    a = torch.empty(lay.arena_bytes + 64, dtype=torch.uint8, device=DEV)
    fill_splitmix64(a, lay.data_seed)
    first = lay.first.astype(np.int64)
    hoff = lay.frag_off[first[:-1]].astype(np.int64)
    hl = lay.frag_len[first[:-1]].astype(np.int64)
    L = np.add.reduceat(lay.frag_len.astype(np.int64), first[:-1])
    assert (hl == 40).all()
    hdr = np.frombuffer(bytes.fromhex("4500000000004000400600000000000000000000"), dtype=np.uint8).copy()
    hdr[12:16] = np.frombuffer(R4, dtype=np.uint8)
    hdr[16:20] = np.frombuffer(L4, dtype=np.uint8)
    d_hoff = torch.from_numpy(hoff).to(DEV)
    idx = d_hoff.view(-1, 1) + torch.arange(20, device=DEV)
    a[idx.flatten()] = torch.from_numpy(hdr).to(DEV).repeat(lay.n)
    del idx
    sample = 3000
    # (the sample's fragments end anywhere below the last one's: a head-only datagram's last
    # fragment is its head, in the header region)
    s_end = int((lay.frag_off[:first[sample]] + lay.frag_len[:first[sample]].astype(np.uint64)).max())
    before = a[:s_end].cpu().numpy()
    d_off, d_len, d_first = dev(lay.frag_off, np.int64), dev(lay.frag_len, np.int32), dev(lay.first, np.int32)
    st = tx_fill_chain(a, d_off, d_len, d_first)
    assert int((st != (_lib.RNS_TX_IP_FILLED | _lib.RNS_TX_L4_FILLED)).sum().item()) == 0
    ip = csum_batch(a, d_hoff, torch.full((lay.n,), 20, dtype=torch.int32, device=DEV), complement=True)
    assert int(ip.view(torch.int16).ne(0).sum().item()) == 0
    off2 = lay.frag_off.copy()
    ln2 = lay.frag_len.copy()
    off2[first[:-1]] += 20
    ln2[first[:-1]] -= 20
    segs, inv = np.unique(L - 20, return_inverse=True)
    ph = np.array([O.pseudo_header_py(R4, L4, int(s), 6) for s in segs], dtype=np.uint16)[inv]
    l4 = csum_chain(a, dev(off2, np.int64), dev(ln2, np.int32), d_first, dev(ph, np.int16), complement=True)
    assert int(l4.view(torch.int16).ne(0).sum().item()) == 0
    after = a[:s_end].cpu().numpy()
    for i in range(0, sample, 7):
        fr = [bytes(before[int(o):int(o) + int(n)]) for o, n in
              zip(lay.frag_off[first[i]:first[i + 1]], lay.frag_len[first[i]:first[i + 1]])]
        h, s = O.tx_chain_fill_ref(fr, ones_comp=oracle.compute_ones_comp)
        assert bytes(after[hoff[i]:hoff[i] + 40]) == h and s == 3
    del a
    torch.cuda.empty_cache()
