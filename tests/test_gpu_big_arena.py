"""Parity past 4 GiB: every product kernel instantiation that serves arenas of 4 GiB or
more (the BUF=false forms: 64-bit global loads instead of buffer loads with 32-bit
offsets) against the oracle.

One 4 GiB + 64 MiB device arena.  Every batch lives in three windows of it: one near
the start, one straddling the 4 GiB line, one ending at the arena's last byte.  The
oracle runs over a host "mini arena" (the three windows back to back, descriptors
translated), and for the in-place fills every byte of every window is compared.

Entries covered: the packed checksum (rows kernel D = 8 and D = 16, the tiny rounds
kernel, the unaligned-packing class kernel, a first block at an odd offset), the strided
form, the packed and explicit transmit fills, packed, explicit and strided receive verify, the
explicit, packed and chain transmit finalize, fragment chains (nontemporal and temporal class passes, each through a
buffer window based at its pass's fragments and through 64-bit loads for passes spanning more
than 4 GiB; the runs hint, which is ignored past 4 GiB) and the head-fragment chain fill.  Reference: util.rs:88-119,
tcp.rs:838-850 / 957-973, udp.rs:158-171, icmp.rs:46-112, ip.rs:76-80 / 158-159.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from rustnetworkstack_amd import _lib
from rustnetworkstack_amd.batch import (csum_batch_packed, csum_batch_strided, csum_chain, csum_chain_fill,
                                        csum_fill, csum_fill_packed, fill_splitmix64, packed_layout, rx_verify,
                                        rx_verify_packed, rx_verify_strided, tx_fill, tx_fill_chain,
                                        tx_fill_packed)
from test_gpu_rx import make_packets
from test_gpu_tx import outgoing
from test_rx_oracle import L4, L6, ipv4, tcp_seg, R4

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
NBYTES = (4 << 30) + (64 << 20)
FOUR_G = 1 << 32
SPAN = 4 << 20  # bytes per window


def dev(a, view):
    return torch.from_numpy(np.ascontiguousarray(a).view(view)).to(DEV)


def host_u16(t):
    torch.cuda.synchronize()
    return t.view(torch.int16).cpu().numpy().view(np.uint16)


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or _lib.load().rns_device_count() == 0:
        pytest.fail("gpu tests need a GPU (the HIP path has no CPU fallback)")


class Windows:
    """Three windows of the big arena: near its start, across the 4 GiB line, at its end."""

    def __init__(self, arena):
        self.arena = arena
        self.starts = [4096, FOUR_G - SPAN // 2, NBYTES - SPAN]
        self.orig = self.snapshot()

    def snapshot(self):
        torch.cuda.synchronize()
        return [self.arena[s:s + SPAN].cpu().numpy() for s in self.starts]

    def write(self, host_windows):
        for s, h in zip(self.starts, host_windows):
            self.arena[s:s + SPAN].copy_(torch.from_numpy(np.ascontiguousarray(h)))
        torch.cuda.synchronize()

    def restore(self):
        self.write(self.orig)

    def to_mini(self, k, off):
        return np.asarray(off, dtype=np.uint64) - np.uint64(self.starts[k]) + np.uint64(k * SPAN)


@pytest.fixture(scope="module")
def win():
    arena = torch.empty(NBYTES, dtype=torch.uint8, device=DEV)
    fill_splitmix64(arena, 0xB16A)
    w = Windows(arena)
    assert arena.numel() >= FOUR_G  # the BUF=false instantiations
    yield w
    del w.arena, arena
    torch.cuda.empty_cache()


def packed_windows(win, lens_per_window, align_log2, shifts=(0, 0, 5)):
    """Packed layouts, one per window (blocks of 64 packets never span windows: every window
    but the last holds a multiple of 64 packets).  Returns device blk_off / len16, the
    absolute and mini-arena offsets, lengths."""
    blks, offs, minis, lens = [], [], [], []
    for k, ln in enumerate(lens_per_window):
        ln = np.asarray(ln, dtype=np.uint16)
        assert k == len(lens_per_window) - 1 or ln.size % 64 == 0
        blk, off, end = packed_layout(ln, align_log2, win.starts[k] + shifts[k])
        assert end <= win.starts[k] + SPAN
        blks.append(blk)
        offs.append(off)
        minis.append(win.to_mini(k, off))
        lens.append(ln)
    blk = np.concatenate(blks).astype(np.uint64)
    return (dev(blk, np.int64), np.concatenate(offs), np.concatenate(minis), np.concatenate(lens))


def imix_lengths(n, salt):
    w = O.splitmix64_words(0x1A1A + salt, n)
    return np.array([40, 40, 40, 40, 40, 40, 40, 576, 576, 576, 576, 1500], dtype=np.uint16)[w % np.uint64(12)]


def lengths_for(kind, salt):
    if kind == "imix":
        return [imix_lengths(64 * 30, salt + k) for k in range(2)] + [imix_lengths(64 * 30 + 17, salt + 2)]
    if kind == "mtu":
        out = []
        for k in range(3):
            ln = np.full(64 * 20 + (7 if k == 2 else 0), 1500, dtype=np.uint16)
            ln[3::17] = (O.splitmix64_words(salt + k, ln[3::17].size) % np.uint64(3000)).astype(np.uint16)
            ln[5::29] = 0
            out.append(ln)
        return out
    if kind == "tiny":
        return [np.full(64 * 200, 64, dtype=np.uint16) for _ in range(2)] + [np.full(64 * 200 + 9, 64, np.uint16)]
    raise ValueError(kind)


@pytest.mark.parametrize("kind,hint,align_log2", [
    ("imix", 340, 4),    # rows kernel, D = 8, BUF=false
    ("mtu", 1500, 4),    # rows kernel, D = 16, BUF=false
    ("tiny", 64, 4),     # rounds kernel (tiny), BUF=false
    ("imix", 340, 0),    # unaligned packing: class kernel, packed form, BUF=false
    ("mtu", 1500, 1),    # the same, nontemporal
])
def test_packed_checksum(oracle, win, kind, hint, align_log2):
    lens = lengths_for(kind, hint + align_log2)
    blk, _, mini_off, ln = packed_windows(win, lens, align_log2)
    seeds = (O.splitmix64_words(0x5EED + hint, ln.size) & np.uint64(0xFFFF)).astype(np.uint16)
    mini = np.concatenate(win.orig)
    want = oracle.batch(mini, mini_off, ln.astype(np.uint32), seeds, complement=True)
    bad = torch.zeros(1, dtype=torch.int32, device=DEV)
    got = host_u16(csum_batch_packed(win.arena, blk, dev(ln, np.int16), dev(seeds, np.int16), align_log2=align_log2,
                                     complement=True, len_hint=hint, bad=bad))
    diff = np.flatnonzero(got != want)
    assert diff.size == 0, [(int(i), int(got[i]), int(want[i])) for i in diff[:5]]
    assert int(bad.item()) == 0


@pytest.mark.parametrize("first_adj,stride,L", [(-3, 80, 64), (0, 64, 64), (0, 48, 40)])
def test_strided_across_the_line(oracle, win, first_adj, stride, L):
    """The strided forms past 4 GiB: the rounds kernel (an unaligned first packet) and the
    tiny kernel (16-byte-aligned starts and stride)."""
    n = 20_000
    first = FOUR_G - 64 * 10_000 + first_adj
    want_arena = win.arena[first:first + n * stride].cpu().numpy()
    off = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    want = oracle.batch(want_arena, off, np.full(n, L, dtype=np.uint32), None, complement=True)
    got = host_u16(csum_batch_strided(win.arena, n, stride, L, first_off=first, complement=True))
    assert np.array_equal(got, want)


def expected_fill(oracle, mini, mini_off, ln, seeds, field):
    """Zero each field that fits (alloc_header), 0xffff ^ ones_comp(seed, packet), the result
    stored big-endian; a packet too short for its field yields 0 and is untouched."""
    a = mini.copy()
    fits = field.astype(np.int64) + 2 <= ln.astype(np.int64)
    idx = mini_off.astype(np.int64) + field.astype(np.int64)
    a[idx[fits]] = 0
    a[idx[fits] + 1] = 0
    want = oracle.batch(a, mini_off, ln.astype(np.uint32), seeds, complement=True)
    want[~fits] = 0
    a[idx[fits]] = (want[fits] >> 8).astype(np.uint8)
    a[idx[fits] + 1] = (want[fits] & 0xFF).astype(np.uint8)
    return want, fits, a


@pytest.mark.parametrize("kind,hint", [("imix", 340), ("mtu", 1500)])
def test_packed_fill(oracle, win, kind, hint):
    lens = lengths_for(kind, 77 + hint)
    blk, _, mini_off, ln = packed_windows(win, lens, 4, shifts=(0, 16, 32))
    n = ln.size
    seeds = (O.splitmix64_words(0xF1 + hint, n) & np.uint64(0xFFFF)).astype(np.uint16)
    field = np.array([16, 6, 2, 10, 3, 17, 15, 31], dtype=np.uint16)[O.splitmix64_words(0xF2, n) % np.uint64(8)]
    mini = np.concatenate(win.orig)
    want, fits, want_arena = expected_fill(oracle, mini, mini_off, ln, seeds, field)
    out = torch.empty(n, dtype=torch.uint16, device=DEV)
    bad = torch.zeros(1, dtype=torch.int32, device=DEV)
    try:
        csum_fill_packed(win.arena, blk, dev(ln, np.int16), dev(seeds, np.int16), field=dev(field, np.int16), out=out,
                         len_hint=hint, bad=bad)
        assert np.array_equal(host_u16(out), want)
        assert int(bad.item()) == int((~fits).sum())
        got = np.concatenate(win.snapshot())
        diff = np.flatnonzero(got != want_arena)
        assert diff.size == 0, [(int(d), int(got[d]), int(want_arena[d])) for d in diff[:8]]
    finally:
        win.restore()


def explicit_windows(win, per_window, salt, max_len=1600, min_gap=0):
    """Packets at arbitrary offsets (any alignment) in every window."""
    offs, minis, lens = [], [], []
    for k in range(3):
        w = O.splitmix64_words(0xE0 + salt + k, 2 * per_window)
        ln = (w[:per_window] % np.uint64(max_len)).astype(np.int64)
        gap = (w[per_window:] % np.uint64(23)).astype(np.int64) + min_gap
        pos = np.cumsum(gap + np.concatenate([[0], ln[:-1]])) + 7 * k
        assert pos[-1] + ln[-1] <= SPAN
        off = (pos + win.starts[k]).astype(np.uint64)
        offs.append(off)
        minis.append(win.to_mini(k, off))
        lens.append(ln.astype(np.uint32))
    return np.concatenate(offs), np.concatenate(minis), np.concatenate(lens)


def test_explicit_fill(oracle, win):
    off, mini_off, ln = explicit_windows(win, 2000, 1)
    n = ln.size
    seeds = (O.splitmix64_words(0xF3, n) & np.uint64(0xFFFF)).astype(np.uint16)
    field = np.array([16, 6, 2, 10, 3, 17], dtype=np.uint16)[O.splitmix64_words(0xF4, n) % np.uint64(6)]
    mini = np.concatenate(win.orig)
    want, fits, want_arena = expected_fill(oracle, mini, mini_off, ln, seeds, field)
    out = torch.empty(n, dtype=torch.uint16, device=DEV)
    bad = torch.zeros(1, dtype=torch.int32, device=DEV)
    try:
        csum_fill(win.arena, dev(off, np.int64), dev(ln, np.int32), dev(seeds, np.int16), field=dev(field, np.int16),
                  out=out, bad=bad)
        assert np.array_equal(host_u16(out), want)
        assert int(bad.item()) == int((~fits).sum())
        got = np.concatenate(win.snapshot())
        diff = np.flatnonzero(got != want_arena)
        assert diff.size == 0, [(int(d), int(got[d]), int(want_arena[d])) for d in diff[:8]]
    finally:
        win.restore()


def place(win, pkts_per_window, offs_per_window):
    """Write datagrams into the windows (device and the host copies)."""
    host = [h.copy() for h in win.orig]
    for k, (pk, off) in enumerate(zip(pkts_per_window, offs_per_window)):
        for o, p in zip(off, pk):
            r = int(o) - win.starts[k]
            host[k][r:r + len(p)] = np.frombuffer(p, dtype=np.uint8)
    win.write(host)
    return host


def datagrams(seed):
    """Per window: 128 ACK-sized TCP/IPv4 datagrams (a unit that skips the rows) then a mix
    of every kind the receive path distinguishes."""
    out = []
    for k in range(3):
        acks = [ipv4(6, tcp_seg(R4, L4, bytes([k, i]) * (i % 3))) for i in range(128)]
        out.append(acks + make_packets(640 + (11 if k == 2 else 0), seed + k))
    return out


def test_packed_receive_verify(oracle, win):
    pk = datagrams(0x9A)
    lens = [np.array([len(p) for p in w], dtype=np.uint16) for w in pk]
    blk, off, _, ln = packed_windows(win, lens, 4, shifts=(0, 0, 0))
    cuts = np.cumsum([0] + [len(w) for w in pk])
    try:
        place(win, pk, [off[cuts[k]:cuts[k + 1]] for k in range(3)])
        flat = [p for w in pk for p in w]
        want = [O.rx_verify_ref(p, L4, L6, ones_comp=oracle.compute_ones_comp) for p in flat]
        l4 = torch.empty(len(flat), dtype=torch.uint16, device=DEV)
        st = rx_verify_packed(win.arena, blk, dev(ln, np.int16), L4, L6, l4_sum=l4)
        torch.cuda.synchronize()
        got = st.cpu().numpy()
        want_st = np.array([w[0] for w in want], dtype=np.uint8)
        assert len(set(want_st.tolist())) >= 5
        diff = np.flatnonzero(got != want_st)
        assert diff.size == 0, [(int(i), int(got[i]), int(want_st[i])) for i in diff[:5]]
        assert np.array_equal(host_u16(l4), np.array([w[1] for w in want], dtype=np.uint16))
    finally:
        win.restore()


def test_explicit_receive_verify(oracle, win):
    pk = datagrams(0x9B)
    offs = []
    for k, w in enumerate(pk):
        g = O.splitmix64_words(0x77 + k, len(w)) % np.uint64(16)
        pos = np.cumsum(np.array([len(p) for p in w], dtype=np.int64) + g.astype(np.int64)) - \
            np.array([len(p) for p in w], dtype=np.int64) + 3 * k
        offs.append((pos + win.starts[k]).astype(np.uint64))
    try:
        place(win, pk, offs)
        flat = [p for w in pk for p in w]
        off = np.concatenate(offs)
        ln = np.array([len(p) for p in flat], dtype=np.uint32)
        want = [O.rx_verify_ref(p, L4, L6, ones_comp=oracle.compute_ones_comp) for p in flat]
        l4 = torch.empty(len(flat), dtype=torch.uint16, device=DEV)
        st = rx_verify(win.arena, dev(off, np.int64), dev(ln, np.int32), L4, L6, l4_sum=l4)
        torch.cuda.synchronize()
        assert np.array_equal(st.cpu().numpy(), np.array([w[0] for w in want], dtype=np.uint8))
        assert np.array_equal(host_u16(l4), np.array([w[1] for w in want], dtype=np.uint16))
    finally:
        win.restore()


def test_transmit_finalize(oracle, win):
    pk = [outgoing(700, 0x7A + k) for k in range(3)]
    offs = []
    for k, w in enumerate(pk):
        g = O.splitmix64_words(0x78 + k, len(w)) % np.uint64(16)
        ln = np.array([len(p) for p in w], dtype=np.int64)
        pos = np.cumsum(ln + g.astype(np.int64)) - ln + 5 * k
        offs.append((pos + win.starts[k]).astype(np.uint64))
    try:
        host = place(win, pk, offs)
        want_st = []
        for k, (w, off) in enumerate(zip(pk, offs)):
            for o, p in zip(off, w):
                q, s = O.tx_fill_ref(p, ones_comp=oracle.compute_ones_comp)
                r = int(o) - win.starts[k]
                host[k][r:r + len(q)] = np.frombuffer(q, dtype=np.uint8)
                want_st.append(s)
        flat = [p for w in pk for p in w]
        off = np.concatenate(offs)
        ln = np.array([len(p) for p in flat], dtype=np.uint32)
        st = tx_fill(win.arena, dev(off, np.int64), dev(ln, np.int32))
        torch.cuda.synchronize()
        assert np.array_equal(st.cpu().numpy(), np.array(want_st, dtype=np.uint8))
        got = np.concatenate(win.snapshot())
        want = np.concatenate(host)
        diff = np.flatnonzero(got != want)
        assert diff.size == 0, [(int(d), int(got[d]), int(want[d])) for d in diff[:8]]
    finally:
        win.restore()


@pytest.mark.parametrize("hint", [0, 1500])
def test_packed_transmit_finalize(oracle, win, hint):
    """rns_tx_fill_packed_dev's BUF=false instantiations (D = 8 and 16): every kind of outgoing
    datagram packed in each window (the middle one across the 4 GiB line, the last one at an
    odd 16-byte offset: its units take the per-datagram path); every window byte and status
    against oracle.tx_fill_ref."""
    pk = [outgoing(640 + (9 if k == 2 else 0), 0x7C + k + hint) for k in range(3)]
    lens = [np.array([len(p) for p in w], dtype=np.uint16) for w in pk]
    blk, off, _, ln = packed_windows(win, lens, 4, shifts=(0, 16, 5))
    cuts = np.cumsum([0] + [len(w) for w in pk])
    try:
        host = place(win, pk, [off[cuts[k]:cuts[k + 1]] for k in range(3)])
        want_st = []
        for k, w in enumerate(pk):
            for o, p in zip(off[cuts[k]:cuts[k + 1]], w):
                q, st = O.tx_fill_ref(p, ones_comp=oracle.compute_ones_comp)
                r = int(o) - win.starts[k]
                host[k][r:r + len(q)] = np.frombuffer(q, dtype=np.uint8)
                want_st.append(st)
        st = tx_fill_packed(win.arena, blk, dev(ln, np.int16), len_hint=hint)
        torch.cuda.synchronize()
        assert np.array_equal(st.cpu().numpy(), np.array(want_st, dtype=np.uint8))
        got = np.concatenate(win.snapshot())
        want = np.concatenate(host)
        diff = np.flatnonzero(got != want)
        assert diff.size == 0, [(int(d), int(got[d]), int(want[d])) for d in diff[:8]]
    finally:
        win.restore()


@pytest.mark.parametrize("shape", ["tx", "any"])
def test_chain_transmit_finalize(oracle, win, shape):
    """rns_tx_fill_chain_dev's BUF=false instantiation: every kind of outgoing datagram as a
    [head, payload pieces] chain in each window (the middle layout across the 4 GiB line), in
    the transmit shape (the rows) and scattered (the exact loop); every window byte and status
    against oracle.tx_chain_fill_ref."""
    from test_gpu_tx_chain import expected, layout
    inp = [h.copy() for h in win.orig]
    want = [h.copy() for h in win.orig]
    offs, lns, firsts, want_st = [], [], [np.zeros(1, np.uint32)], []
    nf = 0
    for k in range(3):
        pk = outgoing(600 + (5 if k == 2 else 0), 0x7D0 + k)
        arena, heads, hoffs, placed, off, ln, first = layout(pk, 0x7D8 + k, shape=shape)
        w_arena, st = expected(oracle, arena, heads, hoffs, placed)
        size = arena.size
        assert size <= SPAN
        rel = (0, (SPAN // 2 - size // 2) & ~15, (SPAN - size) & ~15)[k]
        inp[k][rel:rel + size] = arena
        want[k][rel:rel + size] = w_arena
        offs.append(off + np.uint64(win.starts[k] + rel))
        lns.append(ln)
        firsts.append(first[1:] + np.uint32(nf))
        nf += off.size
        want_st.append(st)
    try:
        win.write(inp)
        st = tx_fill_chain(win.arena, dev(np.concatenate(offs), np.int64), dev(np.concatenate(lns), np.int32),
                           dev(np.concatenate(firsts), np.int32))
        torch.cuda.synchronize()
        assert np.array_equal(st.cpu().numpy(), np.concatenate(want_st))
        got = np.concatenate(win.snapshot())
        w = np.concatenate(want)
        diff = np.flatnonzero(got != w)
        assert diff.size == 0, [(int(d), int(got[d]), int(w[d])) for d in diff[:8]]
    finally:
        win.restore()


@pytest.mark.parametrize("stride,shift", [(64, 0), (2048, 0), (2048, 3)])
def test_strided_receive_verify(oracle, win, stride, shift):
    """rns_rx_verify_strided_dev's BUF=false instantiation: a ring of slots in each window
    (64-byte ACK slots: the quads' loads; 2048-byte MRU slots: the wave loop for the longer
    datagrams; an unaligned first slot: the per-datagram path)."""
    per = min(SPAN // stride - 2, 900)
    for k in range(3):
        pk = [p[:stride] for p in make_packets(per, 0x5C0 + k + stride)]
        first = win.starts[k] + shift + (16 if k == 1 else 0)
        if k == 1:  # the ring crosses the 4 GiB line
            first = FOUR_G - stride * (per // 2) + shift
        try:
            place(win, [pk if j == k else [] for j in range(3)], [np.array([first + i * stride for i in range(per)],
                                                                            dtype=np.uint64) if j == k else []
                                                                  for j in range(3)])
            ln = np.array([len(p) for p in pk], dtype=np.uint16)
            want = [O.rx_verify_ref(p, L4, L6, ones_comp=oracle.compute_ones_comp) for p in pk]
            l4 = torch.empty(per, dtype=torch.uint16, device=DEV)
            st = rx_verify_strided(win.arena, stride, dev(ln, np.int16), L4, L6, first_off=first, l4_sum=l4)
            torch.cuda.synchronize()
            assert np.array_equal(st.cpu().numpy(), np.array([w[0] for w in want], dtype=np.uint8))
            assert np.array_equal(host_u16(l4), np.array([w[1] for w in want], dtype=np.uint16))
        finally:
            win.restore()


def chain_windows(win, per_window, salt, max_frag, min_head=1):
    """Chains of 1-6 fragments scattered over every window (any alignment, odd sizes); a
    packet's first fragment has at least min_head bytes."""
    offs, minis, lens, first = [], [], [], [0]
    for k in range(3):
        w = O.splitmix64_words(0xC0 + salt + k, 3 * per_window)
        nfr = (w[:per_window] % np.uint64(6)).astype(np.int64) + 1
        tot = int(nfr.sum())
        heads = np.concatenate([[0], np.cumsum(nfr[:-1])])
        fl = (O.splitmix64_words(0xC8 + salt + k, tot) % np.uint64(max_frag)).astype(np.int64) + 1
        fl[heads] = np.maximum(fl[heads], min_head)
        gap = (O.splitmix64_words(0xC9 + salt + k, tot) % np.uint64(40)).astype(np.int64)
        order = np.argsort(O.splitmix64_words(0xCA + salt + k, tot))  # memory order: scattered fragments
        pos = np.cumsum(fl[order] + gap) - fl[order] + 9 * k
        assert pos[-1] + fl[order][-1] <= SPAN
        at = np.empty(tot, dtype=np.int64)
        at[order] = pos
        off = (at + win.starts[k]).astype(np.uint64)
        offs.append(off)
        minis.append(win.to_mini(k, off))
        lens.append(fl.astype(np.uint32))
        for c in nfr:
            first.append(first[-1] + int(c))
    return np.concatenate(offs), np.concatenate(minis), np.concatenate(lens), np.array(first, dtype=np.uint32)


@pytest.mark.parametrize("hint,runs", [(512, False), (100, False), (512, True)])
def test_chains(oracle, win, hint, runs):
    off, mini_off, ln, first = chain_windows(win, 1500, hint, 2 * hint)
    n = first.size - 1
    seeds = (O.splitmix64_words(0xCB + hint, n) & np.uint64(0xFFFF)).astype(np.uint16)
    mini = np.concatenate(win.orig)
    want = oracle.chain_batch(mini, mini_off, ln, first, seeds, complement=True)
    got = host_u16(csum_chain(win.arena, dev(off, np.int64), dev(ln, np.int32), dev(first, np.int32),
                              dev(seeds, np.int16), complement=True, frag_len_hint=hint, runs=runs))
    diff = np.flatnonzero(got != want)
    assert diff.size == 0, [(int(i), int(got[i]), int(want[i])) for i in diff[:5]]


def interleave_packets(off, mini_off, ln, first, order):
    """The same chains with the packets in a new order (fragment arrays rebuilt to match)."""
    nf = np.diff(first.astype(np.int64))
    idx = np.concatenate([np.arange(first[p], first[p + 1]) for p in order])
    new_first = np.concatenate([[0], np.cumsum(nf[order])]).astype(np.uint32)
    return off[idx], mini_off[idx], ln[idx], new_first


@pytest.mark.parametrize("hint", [512, 100])
def test_chains_far_apart(oracle, win, hint):
    """Consecutive packets alternate between the first and the last window: every 64-fragment
    pass spans more than 4 GiB, so none fits one buffer window (the 64-bit loads); then the
    same packets window by window (every pass in one window: buffer loads from its base)."""
    off, mini_off, ln, first = chain_windows(win, 1500, 3 + hint, 2 * hint)
    n = first.size - 1
    a = np.arange(0, 1500)
    c = np.arange(3000, 4500)
    order = np.empty(3000, dtype=np.int64)
    order[0::2] = a
    order[1::2] = c
    for o in (order, np.arange(n)):
        o_off, o_mini, o_ln, o_first = interleave_packets(off, mini_off, ln, first, o)
        m = o_first.size - 1
        seeds = (O.splitmix64_words(0xCD + hint, m) & np.uint64(0xFFFF)).astype(np.uint16)
        want = oracle.chain_batch(np.concatenate(win.orig), o_mini, o_ln, o_first, seeds, complement=True)
        got = host_u16(csum_chain(win.arena, dev(o_off, np.int64), dev(o_ln, np.int32), dev(o_first, np.int32),
                                  dev(seeds, np.int16), complement=True, frag_len_hint=hint))
        diff = np.flatnonzero(got != want)
        assert diff.size == 0, [(int(i), int(got[i]), int(want[i])) for i in diff[:5]]


@pytest.mark.parametrize("txp", [False, True])
def test_chain_fill(oracle, win, txp):
    """Head-fragment fill (rns_csum_chain_fill_dev): the chain folded like util.rs:112-119
    with the field counted as zero, stored big-endian into the head fragment (txp: the
    transmit-rows kernel's exact loop, these chains being scattered)."""
    off, mini_off, ln, first = chain_windows(win, 1500, 7, 600, min_head=20)  # heads hold a 20-byte header
    n = first.size - 1
    seeds = (O.splitmix64_words(0xCC, n) & np.uint64(0xFFFF)).astype(np.uint16)
    field = np.array([16, 6, 2, 10], dtype=np.uint16)[np.arange(n) % 4]
    mini = np.concatenate(win.orig)
    want_arena = mini.copy()
    heads = mini_off[first[:-1]].astype(np.int64) + field.astype(np.int64)
    want_arena[heads] = 0
    want_arena[heads + 1] = 0
    want = oracle.chain_batch(want_arena, mini_off, ln, first, seeds, complement=True)
    want_arena[heads] = (want >> 8).astype(np.uint8)
    want_arena[heads + 1] = (want & 0xFF).astype(np.uint8)
    out = torch.empty(n, dtype=torch.uint16, device=DEV)
    try:
        csum_chain_fill(win.arena, dev(off, np.int64), dev(ln, np.int32), dev(first, np.int32), dev(seeds, np.int16),
                        field=dev(field, np.int16), out=out, frag_len_hint=512, tx_packed=txp)
        assert np.array_equal(host_u16(out), want)
        got = np.concatenate(win.snapshot())
        diff = np.flatnonzero(got != want_arena)
        assert diff.size == 0, [(int(d), int(got[d]), int(want_arena[d])) for d in diff[:8]]
    finally:
        win.restore()
