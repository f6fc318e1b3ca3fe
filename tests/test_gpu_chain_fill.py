"""Transmit fill over fragment chains (rns_csum_chain_fill_dev): the shape tcp_output,
udp_output and icmp_output_* checksum (tcp.rs:957-973, udp.rs:158-171, icmp.rs:87-112).
alloc_header prepends a zero-filled head fragment (buf.rs:262-291); the chain is folded by
compute_buffer_ones_comp (util.rs:112-119); the result is set_be16 into the head fragment.
Expected values: oracle.chain_batch over the arena with each field zeroed, then the result
stored big-endian (the restatement of exactly those three steps).  Every other arena byte
must be unchanged."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from rustnetworkstack_amd import _lib
from rustnetworkstack_amd.batch import csum_chain, csum_chain_fill
from rustnetworkstack_amd.workloads import tx_chain_layout

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dev(a, view):
    return torch.from_numpy(np.ascontiguousarray(a).view(view)).to(DEV)


def host_u16(t):
    torch.cuda.synchronize()
    return t.view(torch.int16).cpu().numpy().view(np.uint16)


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or _lib.load().rns_device_count() == 0:
        pytest.fail("gpu tests need a GPU (the HIP path has no CPU fallback)")


def expected(oracle, arena, off, ln, first, seeds, field, complement=True):
    """(results, fits, arena after): the field zeroed (alloc_header), the chain folded
    (compute_buffer_ones_comp), the result stored big-endian (set_be16); packets with no
    fragments, a malformed range or a head fragment too short for the field: 0, untouched."""
    a = arena.copy()
    f0 = first[:-1].astype(np.int64)
    f1 = first[1:].astype(np.int64)
    nf = off.size
    ok_range = (f0 < f1) & (f1 <= nf)
    head = np.where(ok_range, f0, 0)
    hl = ln[head].astype(np.int64) if nf else np.zeros(f0.size, dtype=np.int64)
    fits = ok_range & (field.astype(np.int64) + 2 <= hl)
    # a fragment outside the arena rejects its packet
    frag_out = (off.astype(np.int64) + ln.astype(np.int64)) > arena.size
    cb = np.concatenate([[0], np.cumsum(frag_out)])
    fits &= ~(ok_range & (cb[np.minimum(f1, nf)] - cb[np.minimum(f0, nf)] > 0))
    idx = off[head].astype(np.int64) + field.astype(np.int64)
    a[idx[fits]] = 0
    a[idx[fits] + 1] = 0
    # the fitting packets' chains as a CSR list of their own (the others: empty ranges)
    cnt = np.where(fits, f1 - f0, 0)
    new_first = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    tot = int(new_first[-1])
    frag = np.repeat(f0, cnt) + (np.arange(tot) - np.repeat(new_first[:-1], cnt))
    want = oracle.chain_batch(a, off[frag], ln[frag], new_first.astype(np.uint32), seeds, complement=complement)
    want = np.where(fits, want, 0).astype(np.uint16)
    a[idx[fits]] = (want[fits] >> 8).astype(np.uint8)
    a[idx[fits] + 1] = (want[fits] & 0xFF).astype(np.uint8)
    return want, fits, a


def run_fill(arena_np, off, ln, first, seeds, field, *, hint=512, runs=False, per_packet=True, complement=True,
             tx_packed=False):
    a = torch.from_numpy(arena_np.copy()).to(DEV)
    n = first.size - 1
    out = torch.empty(n, dtype=torch.uint16, device=DEV)
    bad = torch.zeros(1, dtype=torch.int32, device=DEV)
    csum_chain_fill(a, dev(np.asarray(off, np.uint64), np.int64), dev(np.asarray(ln, np.uint32), np.int32),
                    dev(np.asarray(first, np.uint32), np.int32),
                    None if seeds is None else dev(np.asarray(seeds, np.uint16), np.int16),
                    field=dev(np.asarray(field, np.uint16), np.int16) if per_packet else None,
                    field_off=int(field[0]) if n else 16, complement=complement, out=out, bad=bad,
                    frag_len_hint=hint, runs=runs, tx_packed=tx_packed)
    return host_u16(out), int(bad.item()), a.cpu().numpy()


def check(oracle, arena_np, off, ln, first, seeds, field, **kw):
    field = np.asarray(field, dtype=np.uint16)
    seeds_arr = np.zeros(first.size - 1, np.uint16) if seeds is None else np.asarray(seeds, np.uint16)
    want, fits, want_arena = expected(oracle, arena_np, np.asarray(off, np.uint64), np.asarray(ln, np.uint32),
                                      np.asarray(first, np.uint32), seeds_arr, field,
                                      complement=kw.get("complement", True))
    got, bad, got_arena = run_fill(arena_np, off, ln, first, seeds, field, **kw)
    diff = np.flatnonzero(got != want)
    assert diff.size == 0, [(int(i), int(got[i]), int(want[i])) for i in diff[:5]]
    assert bad == int((~fits).sum())
    d = np.flatnonzero(got_arena != want_arena)
    assert d.size == 0, [(int(i), int(got_arena[i]), int(want_arena[i])) for i in d[:8]]
    return want, fits


def test_tcp_output_shape_kat(oracle):
    """util.rs:303-312's two 512-byte fragments of 12 34 behind a 20-byte TCP head fragment
    (field 16 holding garbage), and an odd non-final fragment (util.rs's 0x0807 case)."""
    head = bytes(range(1, 21))
    buf = np.frombuffer(head + bytes([0x12, 0x34]) * 512 + head + bytes([1, 2, 3, 0, 4, 5]), dtype=np.uint8).copy()
    off = [0, 20, 532, 1044, 1064, 1068]
    ln = [20, 512, 512, 20, 3, 2]
    first = np.array([0, 3, 6], dtype=np.uint32)
    want, fits = check(oracle, buf, off, ln, first, [0x1111, 0], [16, 16])
    assert fits.all()


@pytest.mark.parametrize("hint,runs,txp", [(512, False, False), (100, False, False), (512, True, False),
                                           (40, True, False), (512, False, True)])
def test_random_transmit_chains(oracle, hint, runs, txp):
    """Heads of 4-60 bytes back to back in a header region (any start parity), payloads of
    0-5 fragments (odd non-final lengths, empty fragments, back-to-back runs and scattered
    pieces), per-packet fields 2 / 6 / 16 / odd, seeds, rejects (no fragments, heads too
    short for the field)."""
    n = 30_000
    w = O.splitmix64_words(0xCF11 + hint + runs + 2 * txp, 4 * n)
    hl = (w[:n] % np.uint64(57)).astype(np.int64) + 4
    npay = (w[n:2 * n] % np.uint64(6)).astype(np.int64)
    npay[::97] = -1                                         # no fragments at all: rejected
    field = np.array([16, 6, 2, 3, 17, 0], dtype=np.uint16)[(w[2 * n:3 * n] % np.uint64(6)).astype(np.int64)]
    seeds = (w[3 * n:] & np.uint64(0xFFFF)).astype(np.uint16)
    hoff = np.concatenate([[0], np.cumsum(hl[:-1])]) + 3    # header region, odd start
    pos = int(hoff[-1] + hl[-1] + 64)
    off, ln, first = [], [], [0]
    q = O.splitmix64_words(0xCF12 + hint, 12 * n)
    qi = 0
    for i in range(n):
        if npay[i] >= 0:
            off.append(int(hoff[i]))
            ln.append(int(hl[i]))
            adjacent = (i % 3) == 0
            for k in range(npay[i]):
                L = int(q[qi] % np.uint64(2 * hint)) + (0 if k % 4 else 1)
                qi += 1
                if adjacent and k + 1 < npay[i]:
                    L += L & 1                                # even non-final pieces: a run
                pos += 0 if adjacent else int(q[qi] % np.uint64(29))
                qi += 1
                off.append(pos)
                ln.append(L)
                pos += L
        first.append(len(off))
    arena = O.splitmix64_bytes(0xCF13 + hint, pos + 64)
    # (with the transmit hint these scattered chains take the exact per-packet loop)
    check(oracle, arena, np.array(off), np.array(ln), np.array(first, dtype=np.uint32), seeds, field, hint=hint,
          runs=runs, tx_packed=txp)


def tx_blocks(n_blocks, salt):
    """64-packet blocks in the transmit shape RNS_FLAG_CHAIN_TX_PACKED names: heads of 1..64
    bytes back to back in a header region ((start & 15) + length <= 64), then payload runs of
    0-4 pieces (even non-final lengths, empty pieces included) at 16-byte starts with gaps of
    0-3 chunks; some packets rejected (field past the head, no fragments, a piece outside the
    arena).  Every 5th block is broken on purpose (a 70-byte head, an unaligned payload, a
    descending payload, an odd non-final piece, 5 pieces, a 400 KB gap): the exact loop."""
    n = 64 * n_blocks
    w = O.splitmix64_words(0xCF60 + salt, 8 * n)
    field = np.array([16, 6, 2, 3, 17], dtype=np.uint16)[(w[:n] % np.uint64(5)).astype(np.int64)]
    heads, hpos = [], 5
    for i in range(n):
        room = 64 - (hpos & 15)
        hl = 1 + int(w[n + i] % np.uint64(room))
        hl = max(hl, min(room, int(field[i]) + 2)) if i % 11 else hl
        heads.append((hpos, hl))
        hpos += hl
    spare = hpos + 64                                       # own room for the 70-byte heads
    ppos = (hpos + 4096 + 15) & ~15
    off, ln, first = [], [], [0]
    late = []
    for i in range(n):
        b, lane = divmod(i, 64)
        brk = (b // 5) % 6 if b % 5 == 4 else -1
        if i % 97 == 13:                                    # no fragments: rejected
            first.append(len(off))
            continue
        h0, hl = heads[i]
        if brk == 0 and lane == 9:                          # (not overlapping the other heads)
            h0, hl, spare = spare, 70, spare + 80
        off.append(h0)
        ln.append(hl)
        plen = int(w[2 * n + i] % np.uint64(3000)) if i % 7 else 0
        npc = 1 + int(w[3 * n + i] % np.uint64(4)) if plen else int(i % 14 == 0)
        if brk == 4 and lane == 20:
            npc, plen = 5, max(plen, 100)
        cuts = sorted(int(x) & ~1 for x in (w[4 * n + i] % np.uint64(plen + 1), w[5 * n + i] % np.uint64(plen + 1),
                                              w[6 * n + i] % np.uint64(plen + 1), w[7 * n + i] % np.uint64(plen + 1)))
        cuts = [0] + cuts[:npc - 1] + [plen] if npc else []
        ppos += 16 * int(w[4 * n + i] % np.uint64(4))
        if brk == 1 and lane == 30:
            ppos += 8
        if brk == 5 and lane == 40:
            ppos += 400_000
        start = ppos
        if brk == 2 and lane == 5:
            late.append(i)
            start = (24 << 20) + 4096 * len(late)           # this payload lies after every other one
        for k in range(npc):
            L = cuts[k + 1] - cuts[k]
            if brk == 3 and lane == 50 and k == 0 and npc > 1:
                L += 1                                      # odd non-final piece: not a run
            off.append(start + cuts[k] + (1 if brk == 3 and lane == 50 and k > 0 and npc > 1 else 0))
            ln.append(max(L, 0))
        if start == ppos:
            ppos = (ppos + plen + 1 + 15) & ~15
        if i % 89 == 60 and npc:                            # a piece outside the arena: rejected
            off[-1] = 1 << 40
        first.append(len(off))
    end = max(ppos, max(o + l for o, l in zip(off, ln) if o < (1 << 40))) + 256
    arena = O.splitmix64_bytes(0xCF61 + salt, end)
    seeds = (w[:n] >> np.uint64(24) & np.uint64(0xFFFF)).astype(np.uint16)
    return arena, np.array(off, dtype=np.uint64), np.array(ln, dtype=np.uint32), np.array(first, np.uint32), \
        seeds, field


@pytest.mark.parametrize("hint", [512, 100])
def test_tx_packed_blocks(oracle, hint):
    """RNS_FLAG_CHAIN_TX_PACKED on tx_blocks: the fill, every result and every arena byte
    against the oracle; the plain chain checksum of the same chains with the hint == the
    oracle (and == without it)."""
    arena, off, ln, first, seeds, field = tx_blocks(60, hint)
    check(oracle, arena, off, ln, first, seeds, field, hint=hint, tx_packed=True)
    a = torch.from_numpy(arena).to(DEV)
    args = (a, dev(off, np.int64), dev(ln, np.int32), dev(first, np.int32), dev(seeds, np.int16))
    plain = host_u16(csum_chain(*args, complement=True, frag_len_hint=hint))
    txp = host_u16(csum_chain(*args, complement=True, frag_len_hint=hint, tx_packed=True))
    assert np.array_equal(txp, plain)
    inside = np.array([all(int(o) + int(L) <= arena.size for o, L in zip(off[first[i]:first[i + 1]],
                                                                       ln[first[i]:first[i + 1]]))
                       for i in range(first.size - 1)])
    keep = inside & (first[1:] > first[:-1])
    sel = np.flatnonzero(keep)
    cnt = (first[1:] - first[:-1])[sel].astype(np.int64)
    nf = np.concatenate([[0], np.cumsum(cnt)])
    fr = np.repeat(first[:-1][sel].astype(np.int64), cnt) + (np.arange(int(nf[-1])) - np.repeat(nf[:-1], cnt))
    ref = oracle.chain_batch(arena, off[fr], ln[fr], nf.astype(np.uint32), seeds[sel], complement=True)
    assert np.array_equal(txp[sel], ref)


@pytest.mark.parametrize("hint", [512, 100])
def test_runs_with_the_head_in_place(oracle, hint):
    """RNS_FLAG_CHAIN_RUNS's by-packet path: each packet one buffer viewed as [head, payload
    pieces] back to back (even non-final lengths), so every wave sums whole runs; the field
    comes out of the run's sum.  Waves with a scattered packet take the fragment path."""
    n = 64 * 200
    w = O.splitmix64_words(0xCF50 + hint, 3 * n)
    L = (w[:n] % np.uint64(1600)).astype(np.int64) + 20
    off, ln, first, pos = [], [], [0], 0
    for i in range(n):
        cuts = [20] + [2 * int(x) for x in (w[n + i] % np.uint64(200), w[2 * n + i] % np.uint64(300))]
        rest, start = int(L[i]), pos
        for c in cuts:
            c = min(c, rest)
            if c <= 0:
                break
            off.append(start)
            ln.append(c)
            start += c
            rest -= c
        if rest > 0:
            off.append(start)
            ln.append(rest)
        if i % 640 == 5:                                 # one scattered packet in a few waves
            off[-1] += 3
        pos += int(L[i]) + 16
        first.append(len(off))
    arena = O.splitmix64_bytes(0xCF51, pos + 64)
    field = np.array([16, 6, 2, 10], dtype=np.uint16)[np.arange(n) % 4]
    seeds = (w[:n] >> np.uint64(20) & np.uint64(0xFFFF)).astype(np.uint16)
    check(oracle, arena, np.array(off), np.array(ln), np.array(first, dtype=np.uint32), seeds, field, hint=hint,
          runs=True)


def test_single_field_offset_and_no_seeds(oracle):
    """field_off for every packet (d_field NULL), no seeds, and the plain (uncomplemented) sum."""
    lay = tx_chain_layout("c5_imix", n=5000, frag=512)
    arena = O.splitmix64_bytes(0xCF20, lay.arena_bytes + 64)
    for complement in (True, False):
        check(oracle, arena, lay.frag_off, lay.frag_len, lay.first, None, np.full(lay.n, 16, np.uint16),
              per_packet=False, complement=complement)


def test_udp_zero_stored_as_is(oracle):
    """udp.rs:168-171 stores a computed 0 unchanged (no RFC 768 0 -> 0xffff): a chain whose
    sum is 0xffff gets 0 in its field, and an all-zero chain with seed 0 gets 0xffff."""
    head = np.zeros(8, dtype=np.uint8)
    head[0:2] = [0xFF, 0xFF]                                 # one word 0xffff, the rest zero
    buf = np.concatenate([head, np.zeros(8, np.uint8), np.zeros(16, np.uint8)])
    off = [0, 8, 16, 24]
    ln = [8, 8, 8, 8]
    first = np.array([0, 2, 4], dtype=np.uint32)
    want, _ = check(oracle, buf, off, ln, first, [0, 0], [6, 6])
    assert list(want) == [0x0000, 0xFFFF]


def test_field_past_128kib_and_odd_heads(oracle):
    """Head fragments past the no-wrap bound (the exact big-endian path takes the field
    out of the wrapped u32 sum) at odd and even starts, fields at odd offsets, 0xff bytes."""
    sizes = [131_072 - 2, 131_072 + 7, 200_001, 70_000]
    offs, lens, first, pos = [], [], [0], 1
    for s in sizes:
        offs += [pos, pos + s + 5]
        lens += [s, 1001]
        pos += s + 5 + 1001 + (pos & 1)
        first.append(len(offs))
    arena = O.splitmix64_bytes(0xCF30, pos + 64)
    arena[offs[2]:offs[2] + sizes[1]] = 0xFF
    field = np.array([16, 131_000 % 65536, 65_001, 3], dtype=np.uint16)
    seeds = np.array([0xFFFF, 1, 0, 0x8000], dtype=np.uint16)
    for hint in (512, 100):
        check(oracle, arena, offs, lens, np.array(first, dtype=np.uint32), seeds, field, hint=hint)


def test_malformed_ranges_and_out_of_arena(oracle):
    """A range past n_frags, a reversed range and a head outside the arena: rejected,
    counted, nothing stored; their neighbours are filled."""
    arena = O.splitmix64_bytes(0xCF40, 4096)
    off = np.array([0, 40, 100, 140, 8000, 200], dtype=np.uint64)
    ln = np.array([20, 30, 20, 30, 20, 24], dtype=np.uint32)
    first = np.array([0, 2, 4, 5, 6], dtype=np.uint32)       # packet 2 = [8000 ..) outside
    a = torch.from_numpy(arena.copy()).to(DEV)
    out = torch.empty(4, dtype=torch.uint16, device=DEV)
    bad = torch.zeros(1, dtype=torch.int32, device=DEV)
    csum_chain_fill(a, dev(off, np.int64), dev(ln, np.int32), dev(first, np.int32), None, field_off=16, out=out,
                    bad=bad)
    got = host_u16(out)
    assert got[2] == 0 and int(bad.item()) == 1
    want, fits, want_arena = expected(oracle, np.concatenate([arena, np.zeros(8000, np.uint8)]), off, ln,
                                      first, np.zeros(4, np.uint16), np.full(4, 16, np.uint16))
    assert list(got[[0, 1, 3]]) == list(want[[0, 1, 3]])
    assert np.array_equal(a.cpu().numpy(), want_arena[:4096])
    # reversed / past-the-end CSR ranges
    first2 = np.array([0, 2, 1, 9], dtype=np.uint32)
    bad.zero_()
    csum_chain_fill(a, dev(off, np.int64), dev(ln, np.int32), dev(first2, np.int32), None, field_off=16, out=out[:3],
                    bad=bad)
    assert int(bad.item()) == 2


@pytest.mark.parametrize("name,frag", [("c3_1500B", 0), ("c3_1500B", 512), ("c5_imix", 0), ("c5_imix", 512)])
def test_full_size_transmit_chains(oracle, name, frag):
    """Every packet of the c3 / IMIX configs in the transmit shape (20-byte TCP head
    fragments in a header region + the payload as one fragment or 512-byte NetBuffer
    fragments), both hints: the fill, then the receive-side chain checksum of every packet
    is 0 (tcp.rs:838-850 on what was sent), and a sample against the oracle."""
    lay = tx_chain_layout(name, frag=frag)
    a = torch.empty(lay.arena_bytes + 64, dtype=torch.uint8, device=DEV)
    from rustnetworkstack_amd.batch import fill_splitmix64
    fill_splitmix64(a, lay.data_seed)
    d_off, d_len, d_first = dev(lay.frag_off, np.int64), dev(lay.frag_len, np.int32), dev(lay.first, np.int32)
    d_seed = dev(lay.seed, np.int16)
    sample = 20_000
    f_s = int(lay.first[sample])
    host_before = a[:int(lay.frag_off[f_s - 1] + lay.frag_len[f_s - 1]) + 64].cpu().numpy() \
        if name == "c3_1500B" else None
    for runs, txp in ((False, False), (True, False), (False, True)):
        out = torch.empty(lay.n, dtype=torch.uint16, device=DEV)
        bad = torch.zeros(1, dtype=torch.int32, device=DEV)
        csum_chain_fill(a, d_off, d_len, d_first, d_seed, field_off=lay.field, out=out, bad=bad, runs=runs,
                        tx_packed=txp)
        assert int(bad.item()) == 0
        rx = host_u16(csum_chain(a, d_off, d_len, d_first, d_seed, complement=True, runs=runs, tx_packed=txp))
        assert not rx.any()
        if host_before is not None and not runs:
            want, _, _ = expected(oracle, host_before, lay.frag_off[:f_s], lay.frag_len[:f_s],
                                  lay.first[:sample + 1], lay.seed[:sample], np.full(sample, 16, np.uint16))
            assert np.array_equal(host_u16(out)[:sample], want)
    del a
    torch.cuda.empty_cache()
