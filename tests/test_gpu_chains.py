"""GPU fragment chains (rns_csum_chain_dev): util.rs:112-119 compute_buffer_ones_comp
over NetBuffer-style fragment lists, bit-exact against the oracle."""
import numpy as np
import pytest
import torch

from conftest import sweep_arena
from oracle import oracle as O
from rustnetworkstack_amd.batch import csum_batch, csum_chain
from rustnetworkstack_amd.workloads import DeviceBatch, make_layout

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dev(a, view):
    return torch.from_numpy(np.ascontiguousarray(a).view(view)).to(DEV)


def host_u16(t):
    torch.cuda.synchronize()
    return t.view(torch.int16).cpu().numpy().view(np.uint16)


def run_chain(arena_t, offs, lens, first, seeds, complement=False, bad=None, runs=False):
    return host_u16(csum_chain(arena_t, dev(np.asarray(offs, dtype=np.uint64), np.int64),
                               dev(np.asarray(lens, dtype=np.uint32), np.int32),
                               dev(np.asarray(first, dtype=np.uint32), np.int32),
                               None if seeds is None else dev(np.asarray(seeds, dtype=np.uint16), np.int16),
                               complement=complement, bad=bad, runs=runs))


def test_reference_kats():
    # util.rs:303-312: two 512-byte fragments of 12 34 -> 0x6824; odd non-final fragment -> 0x0807
    buf = np.frombuffer(bytes([0x12, 0x34]) * 512 + bytes([1, 2, 3, 0, 4, 5]), dtype=np.uint8).copy()
    a = torch.from_numpy(buf).to(DEV)
    got = run_chain(a, [0, 512, 1024, 1028], [512, 512, 3, 2], [0, 2, 4], [0, 0])
    assert list(got) == [0x6824, 0x0807]


def test_golden_fixture_chains(sweep):
    arena = torch.from_numpy(sweep_arena(sweep)).to(DEV)
    offs, lens, first, seeds = [], [], [0], []
    for ch in sweep["chains"]:
        for o, s in ch["frags"]:
            offs.append(o)
            lens.append(s)
        first.append(len(offs))
        seeds.append(ch["seed"])
    got = run_chain(arena, offs, lens, first, seeds)
    assert np.array_equal(got, np.array([c["expect"] for c in sweep["chains"]], dtype=np.uint16))


def test_random_scattered_chains(oracle):
    """200K chains of 1-8 fragments of 1-700 B (odd sizes, scattered, any alignment)."""
    n = 200_000
    arena_np = O.splitmix64_bytes(0xC4A1, 64 << 20)
    w = O.splitmix64_words(0xC4A2, n)
    nfr = (w % np.uint64(8) + np.uint64(1)).astype(np.int64)
    first = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(nfr, out=first[1:])
    nf = int(first[-1])
    fw = O.splitmix64_words(0xC4A3, nf)
    lens = (fw % np.uint64(700) + np.uint64(1)).astype(np.uint32)
    offs = ((fw >> np.uint64(20)) % np.uint64((64 << 20) - 1024)).astype(np.uint64)
    seeds = (w >> np.uint64(40) & np.uint64(0xFFFF)).astype(np.uint16)
    expect = oracle.chain_batch(arena_np, offs, lens, first, seeds, complement=True)
    got = run_chain(torch.from_numpy(arena_np).to(DEV), offs, lens, first, seeds, complement=True)
    assert np.array_equal(got, expect)


def _c_caller_chains(n, seed):
    """The distribution of tests/c/test_batch_abi.c test_chains, whose run in session r03h
    caught add3326's chain stream kernel (tools/forensics/chain_stream_r03h.py):
    0-6 fragments of 1-700 B per packet; half the packets scattered (gaps of 0-28 B, any
    alignment), half back-to-back views with even non-final lengths (a run)."""
    w = O.splitmix64_words(seed, n)
    nfr = (w % np.uint64(7)).astype(np.int64)
    adjacent = ((w >> np.uint64(8)) & np.uint64(1)).astype(bool)
    first = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(nfr, out=first[1:])
    nf = int(first[-1])
    q = O.splitmix64_words(seed + 1, nf)
    pk = np.repeat(np.arange(n), nfr)
    j = np.arange(nf) - first[pk]
    lens = (np.uint64(1) + (q >> np.uint64(8)) % np.uint64(700)).astype(np.int64)
    run = adjacent[pk] & (j + 1 < nfr[pk])
    lens = np.where(run, np.maximum(lens & ~1, 2), lens)
    gaps = np.where(adjacent[pk], 0, (q % np.uint64(29)).astype(np.int64))
    offs = np.cumsum(gaps + lens) - lens
    seeds = ((w >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.uint16)
    return offs.astype(np.uint64), lens.astype(np.uint32), first, seeds, int(offs[-1] + lens[-1]) + 32


@pytest.mark.parametrize("hint", [0, 40, 350, 512, 1500])
def test_c_caller_chain_distribution(oracle, hint):
    """Every fragment-length hint (each kernel choice) on the C caller's chain mix, including
    the last rows of every 64-fragment group (where the removed kernel lost chunks)."""
    offs, lens, first, seeds, size = _c_caller_chains(20_000, 0xC11A + hint)
    arena_np = O.splitmix64_bytes(0xC11B, size)
    a = torch.from_numpy(arena_np).to(DEV)
    for runs in (False, True):
        expect = oracle.chain_batch(arena_np, offs, lens, first, seeds, complement=True)
        got = host_u16(csum_chain(a, dev(offs, np.int64), dev(lens, np.int32), dev(first.astype(np.uint32), np.int32),
                                  dev(seeds, np.int16), complement=True, frag_len_hint=hint, runs=runs))
        assert np.array_equal(got, expect), (hint, runs, int(np.flatnonzero(got != expect)[0]))


def test_full_size_received_fragments_match_contiguous(oracle):
    """Headline batch (1M x 1500 B) as the stack receives it after the IP trim
    ([492, 512, 476]-byte fragments): chain result == contiguous result == oracle."""
    lay = make_layout("c3_1500B")
    b = DeviceBatch(lay, DEV)
    contiguous = host_u16(csum_batch(b.arena, b.off, b.length, b.seed, complement=True))
    sizes = np.array([492, 512, 496], dtype=np.uint32)
    offs = (lay.off[:, None] + np.array([0, 492, 1004], dtype=np.uint64)[None, :]).reshape(-1)
    lens = np.tile(sizes, lay.n)
    first = np.arange(0, 3 * lay.n + 1, 3, dtype=np.uint32)
    got = run_chain(b.arena, offs, lens, first, lay.seed, complement=True)
    assert np.array_equal(got, contiguous)
    assert np.array_equal(run_chain(b.arena, offs, lens, first, lay.seed, complement=True, runs=True), contiguous)
    sample = slice(0, 20000)
    arena_np = b.arena[:int(lay.off[20000])].cpu().numpy()
    expect = oracle.chain_batch(arena_np, offs[:60000], lens[:60000], first[:20001], lay.seed[sample], complement=True)
    assert np.array_equal(got[sample], expect)
    del b
    torch.cuda.empty_cache()


def test_chain_tail_at_unpadded_arena_end(oracle):
    """Fragments ending on the last byte of an arena whose size is not a multiple of 4."""
    arena_np = O.splitmix64_bytes(3, 1030)
    got = run_chain(torch.from_numpy(arena_np.copy()).to(DEV), [0, 1024, 1028], [1024, 3, 2], [0, 1, 3], [7, 9])
    expect = oracle.chain_batch(arena_np, np.array([0, 1024, 1028]), np.array([1024, 3, 2]), np.array([0, 1, 3]),
                                np.array([7, 9], dtype=np.uint16))
    assert np.array_equal(got, expect)


def test_bad_fragment_rejects_packet():
    a = torch.zeros(4096, dtype=torch.uint8, device=DEV)
    bad = torch.zeros(1, dtype=torch.int32, device=DEV)
    got = run_chain(a, [0, 4000, 10], [16, 200, 4], [0, 2, 3], [5, 6], bad=bad)
    assert got[0] == 0 and got[1] == 6 and int(bad.item()) == 1


def test_many_fragments_no_overflow(oracle):
    """70 000 one-byte 0xff fragments in one packet (each adds the word 0xff00): the
    reference folds after every fragment (util.rs:113-118), so its running sum never
    overflows; a one-fold-at-the-end combine would wrap past 65 537 fragments."""
    arena_np = np.full(70_000 + 64, 0xff, dtype=np.uint8)
    nfr = 70_000
    offs = np.arange(nfr, dtype=np.uint64)
    lens = np.ones(nfr, dtype=np.uint32)
    # packet 0: the 70 000 fragments; packets 1-3: short chains after it (same wave)
    offs = np.concatenate([offs, np.array([70_000, 70_001, 70_010, 70_020], dtype=np.uint64)])
    lens = np.concatenate([lens, np.array([1, 9, 10, 33], dtype=np.uint32)])
    first = np.array([0, nfr, nfr + 2, nfr + 3, nfr + 4], dtype=np.uint32)
    seeds = np.array([0xfffe, 1, 0, 0xffff], dtype=np.uint16)
    for complement in (False, True):
        expect = oracle.chain_batch(arena_np, offs, lens, first, seeds, complement=complement)
        for runs in (False, True):
            got = run_chain(torch.from_numpy(arena_np).to(DEV), offs, lens, first, seeds, complement=complement,
                            runs=runs)
            assert np.array_equal(got, expect)


@pytest.mark.parametrize("fill", [0xff, None])
def test_big_fragment_after_nonzero_running_sum(oracle, fill):
    """A fragment longer than 128 KiB after a fragment that leaves a nonzero running
    sum: the reference's u32 accumulator starts from that sum and wraps (release
    build), which a per-fragment sum from seed 0 cannot reproduce."""
    big = 200_001
    if fill is None:
        arena_np = O.splitmix64_bytes(0xB16, big + 4096)
    else:
        arena_np = np.full(big + 4096, fill, dtype=np.uint8)
    offs = np.array([0, 7, 7 + 1000, 3, 4000, 11, 1], dtype=np.uint64)
    lens = np.array([7, 1000, big, 1, big - 900, 3, big + 11], dtype=np.uint32)
    first = np.array([0, 3, 5, 7], dtype=np.uint32)   # [7 B, 1000 B, big], [1 B, big-900], [3 B, big+11]
    for seeds in (np.array([0xffff, 0x1234, 0], dtype=np.uint16), None):
        expect = oracle.chain_batch(arena_np, offs, lens, first, seeds, complement=True)
        got = run_chain(torch.from_numpy(arena_np).to(DEV), offs, lens, first, seeds, complement=True)
        assert np.array_equal(got, expect)


def test_random_chains_mixed_sizes_and_malformed(oracle):
    """30K chains: 0-12 fragments of 0..3000 B with an occasional jumbo fragment
    (past 128 KiB), empty fragments, and a few malformed CSR ranges (end < start,
    end past n_frags), whose packets must come back 0 and be counted in *bad."""
    n = 30_000
    size = 8 << 20
    arena_np = O.splitmix64_bytes(0xC5A1, size)
    w = O.splitmix64_words(0xC5A2, n)
    nfr = (w % np.uint64(13)).astype(np.int64)
    first = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(nfr, out=first[1:])
    nf = int(first[-1])
    fw = O.splitmix64_words(0xC5A3, nf)
    lens = (fw % np.uint64(3001)).astype(np.uint32)
    jumbo = (fw >> np.uint64(50)) % np.uint64(97) == 0
    lens[jumbo] = (140_000 + (fw[jumbo] >> np.uint64(8)) % np.uint64(300_000)).astype(np.uint32)
    offs = ((fw >> np.uint64(20)) % np.uint64(size - 450_000)).astype(np.uint64)
    seeds = (w >> np.uint64(40) & np.uint64(0xFFFF)).astype(np.uint16)
    first = first.astype(np.uint32)
    first[18] = first[17] + 20 if first[17] + 20 <= nf else nf   # packet 18 starts past where it ends
    first[19] = first[18] - 3                                     # (packet 18: end < start)
    first[4001] = nf + 5                                          # packets 4000/4001: end past n_frags / < start
    first[n] = nf + 1                                             # the last packet: end past n_frags
    lo, hi = first[:-1].astype(np.int64), first[1:].astype(np.int64)
    valid = (lo <= hi) & (hi <= nf)
    # expected: the oracle over each valid packet's own fragment range
    idx = [np.arange(a, b) for a, b in zip(lo[valid], hi[valid])]
    sub_first = np.zeros(int(valid.sum()) + 1, dtype=np.uint32)
    np.cumsum([len(i) for i in idx], out=sub_first[1:])
    cat = np.concatenate(idx) if idx else np.zeros(0, dtype=np.int64)
    expect = oracle.chain_batch(arena_np, offs[cat], lens[cat], sub_first, seeds[valid], complement=True)
    bad = torch.zeros(1, dtype=torch.int32, device=DEV)
    got = run_chain(torch.from_numpy(arena_np).to(DEV), offs, lens, first, seeds, complement=True, bad=bad)
    assert (~valid).sum() >= 4
    assert np.array_equal(got[valid], expect)
    assert (got[~valid] == 0).all()
    assert int(bad.item()) == int((~valid).sum())


def test_packets_without_fragments():
    """Packets with no fragments return their seed (complemented on request); a batch
    with no fragments at all never reads the fragment arrays."""
    a = torch.zeros(64, dtype=torch.uint8, device=DEV)
    got = run_chain(a, [], [], [0] * 101, list(range(100)))
    assert np.array_equal(got, np.arange(100, dtype=np.uint16))
    got = run_chain(a, [], [], [0] * 101, list(range(100)), complement=True)
    assert np.array_equal(got, (0xffff ^ np.arange(100)).astype(np.uint16))


def _adjacent_chains(n, seed, arena_size, max_len, p_odd, p_jump):
    """Chains laid out as runs of adjacent fragments (each fragment starts where the
    previous one ends, across packet boundaries too), with odd lengths, empty
    fragments, long fragments and occasional jumps to a fresh offset."""
    w = O.splitmix64_words(seed, n)
    nfr = (w % np.uint64(9)).astype(np.int64)
    first = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(nfr, out=first[1:])
    nf = int(first[-1])
    fw = O.splitmix64_words(seed + 1, nf)
    lens = ((fw % np.uint64(max_len)) & ~np.uint64(1)).astype(np.int64)       # even ...
    odd = (fw >> np.uint64(32)) % np.uint64(1000) < np.uint64(int(p_odd * 1000))
    lens[odd] += 1                                                              # ... or odd
    lens[(fw >> np.uint64(44)) % np.uint64(50) == 0] = 0                        # empty fragments
    jump = (fw >> np.uint64(52)) % np.uint64(1000) < np.uint64(int(p_jump * 1000))
    offs = np.zeros(nf, dtype=np.int64)
    pos = 0
    for i in range(nf):   # (a few 10K fragments: a Python loop is fine)
        if jump[i]:
            pos = int(fw[i] >> np.uint64(20)) % (arena_size // 2)
        if pos + lens[i] > arena_size:
            pos = 0
        offs[i] = pos
        pos += int(lens[i])
    seeds = (w >> np.uint64(40) & np.uint64(0xFFFF)).astype(np.uint16)
    return offs.astype(np.uint64), lens.astype(np.uint32), first.astype(np.uint32), seeds


@pytest.mark.parametrize("max_len,p_odd", [(1600, 0.1), (600, 0.4), (70_000, 0.05), (300_000, 0.1)])
def test_adjacent_fragment_runs(oracle, max_len, p_odd):
    """Runs of adjacent fragments, with and without RNS_FLAG_CHAIN_RUNS: runs that cross
    packet boundaries, odd lengths mid-run, empty fragments, runs longer than 128 KiB
    and fragments past 128 KiB must all fold exactly as the reference's per-fragment
    loop (util.rs:112-119)."""
    n = 20_000 if max_len <= 1600 else 2_000
    size = 16 << 20
    arena_np = O.splitmix64_bytes(0xAD1 + max_len, size)
    offs, lens, first, seeds = _adjacent_chains(n, 0xAD2 + max_len, size, max_len, p_odd, 0.05)
    expect = oracle.chain_batch(arena_np, offs, lens, first, seeds, complement=True)
    for runs in (False, True):
        got = run_chain(torch.from_numpy(arena_np).to(DEV), offs, lens, first, seeds, complement=True, runs=runs)
        assert np.array_equal(got, expect)


def test_adjacent_runs_all_ones_wrap_edges(oracle):
    """0xff runs whose merged sum sits at the fold edges: 65 536 bytes of 0xff in 64
    adjacent 1 KiB fragments (sum == 0 mod 0xffff, non-zero), a run of exactly 128 KiB,
    one byte past it, and zero runs after a zero seed."""
    arena_np = np.full(3 << 20, 0xff, dtype=np.uint8)
    arena_np[2 << 20:] = 0
    offs, lens, first = [], [], [0]
    pos = 0
    for frag_len, count in ((1024, 64), (2048, 64), (2048, 64), (4096, 33)):
        for _ in range(count):
            offs.append(pos)
            lens.append(frag_len)
            pos += frag_len
        first.append(len(offs))
    lens[-1] = 4095                 # last run: 32*4096 + 4095 bytes (past 128 KiB), odd tail
    for _ in range(64):             # zero bytes, zero seed
        offs.append((2 << 20) + 512 * (len(offs) % 64))
        lens.append(512)
    first.append(len(offs))
    offs, lens = np.array(offs, dtype=np.uint64), np.array(lens, dtype=np.uint32)
    first = np.array(first, dtype=np.uint32)
    for seeds in (np.array([0, 1, 0xffff, 0xfffe, 0], dtype=np.uint16), None):
        for complement in (False, True):
            expect = oracle.chain_batch(arena_np, offs, lens, first, seeds, complement=complement)
            for runs in (False, True):
                got = run_chain(torch.from_numpy(arena_np).to(DEV), offs, lens, first, seeds, complement=complement,
                                runs=runs)
                assert np.array_equal(got, expect)


def test_adjacent_runs_overlapping_ranges(oracle):
    """Malformed CSR whose VALID ranges overlap: a run of adjacent fragments must never
    carry one packet's fragments into another's sum."""
    arena_np = O.splitmix64_bytes(0xAD9, 1 << 20)
    nf = 40
    lens = np.full(nf, 100, dtype=np.uint32)
    offs = np.arange(nf, dtype=np.uint64) * np.uint64(100)          # one long adjacent run
    first = np.array([0, 6, 4, 8, 13, 12, 20, 40], dtype=np.uint32)  # [0,6) [6,4)x [4,8) [8,13) [13,12)x [12,20) [20,40)
    seeds = np.arange(7, dtype=np.uint16) * np.uint16(1000)
    lo, hi = first[:-1].astype(np.int64), first[1:].astype(np.int64)
    valid = (lo <= hi) & (hi <= nf)
    idx = [np.arange(a, b) for a, b in zip(lo[valid], hi[valid])]
    sub_first = np.zeros(int(valid.sum()) + 1, dtype=np.uint32)
    np.cumsum([len(i) for i in idx], out=sub_first[1:])
    cat = np.concatenate(idx)
    expect = oracle.chain_batch(arena_np, offs[cat], lens[cat], sub_first, seeds[valid], complement=True)
    for runs in (False, True):
        got = run_chain(torch.from_numpy(arena_np).to(DEV), offs, lens, first, seeds, complement=True, runs=runs)
        assert np.array_equal(got[valid], expect)
        assert (got[~valid] == 0).all()


@pytest.mark.parametrize("break_every,max_len", [(0, 3000), (997, 3000), (0, 40_000), (0, 64)])
def test_runs_by_packet(oracle, break_every, max_len):
    """Every packet's fragments one run (0-4 adjacent fragments, all but the last of even
    length, at any start parity, empty fragments included): the wave sums each packet as
    one contiguous unit.  break_every: every n-th packet gets a gap or an odd middle
    fragment, so its wave takes the per-fragment path while the others do not."""
    n = 30_000 if max_len <= 3000 else 3_000
    size = 64 << 20
    arena_np = O.splitmix64_bytes(0xB00 + max_len, size)
    w = O.splitmix64_words(0xB01 + break_every, n)
    nfr = (w % np.uint64(5)).astype(np.int64)
    first = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(nfr, out=first[1:])
    nf = int(first[-1])
    fw = O.splitmix64_words(0xB02, nf)
    lens = (fw % np.uint64(max_len + 1)).astype(np.int64)
    last = np.zeros(nf, dtype=bool)
    last[first[1:][nfr > 0] - 1] = True
    lens[~last] &= ~1                                      # even, except each packet's last fragment
    lens[(fw >> np.uint64(40)) % np.uint64(40) == 0] = 0   # empty fragments
    start = ((w >> np.uint64(16)) % np.uint64(size - 5 * max_len - 16)).astype(np.int64)
    offs = np.zeros(nf, dtype=np.int64)
    for p in range(n):
        pos = int(start[p])
        for f in range(int(first[p]), int(first[p + 1])):
            offs[f] = pos
            pos += int(lens[f])
    if break_every:
        for p in range(0, n, break_every):
            f0, f1 = int(first[p]), int(first[p + 1])
            if f1 - f0 >= 2:
                if p % 2:
                    offs[f0 + 1:f1] += 2           # a gap
                else:
                    lens[f0] |= 1                  # an odd fragment before the last
                    offs[f0 + 1:f1] += 1
    seeds = (w >> np.uint64(40) & np.uint64(0xFFFF)).astype(np.uint16)
    offs, lens, first = offs.astype(np.uint64), lens.astype(np.uint32), first.astype(np.uint32)
    for complement in (False, True):
        expect = oracle.chain_batch(arena_np, offs, lens, first, seeds, complement=complement)
        for runs in (False, True):
            got = run_chain(torch.from_numpy(arena_np).to(DEV), offs, lens, first, seeds, complement=complement,
                            runs=runs)
            assert np.array_equal(got, expect)


@pytest.mark.parametrize("max_gap,max_len,align", [(0, 1600, 16), (15, 1600, 16), (48, 700, 16), (0, 20_000, 16),
                                                   (0, 1600, 2), (600, 100, 16)])
def test_runs_tiling_a_region(oracle, max_gap, max_len, align):
    """RNS_FLAG_CHAIN_RUNS with runs that tile the arena (csum_rows_kernel's decomposition
    over 64 runs: 16-byte-aligned starts, ascending, gaps within a quarter of the bytes):
    0-4 adjacent fragments per packet (all but the last even, empty ones included, packets
    without fragments), gaps of 0..max_gap bytes rounded up to `align`.  align 2 / large gaps:
    waves fall back to the class pass.  Both against the oracle, with and without the flag."""
    n = 40_000 if max_len <= 1600 else 4_000
    w = O.splitmix64_words(0x7111 + max_gap + max_len + align, n)
    nfr = (w % np.uint64(5)).astype(np.int64)
    first = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(nfr, out=first[1:])
    nf = int(first[-1])
    fw = O.splitmix64_words(0x7112 + max_len, nf)
    lens = (fw % np.uint64(max_len // 2 + 1)).astype(np.int64)
    last = np.zeros(nf, dtype=bool)
    last[first[1:][nfr > 0] - 1] = True
    lens[~last] &= ~1
    lens[(fw >> np.uint64(40)) % np.uint64(30) == 0] = 0
    offs = np.zeros(nf, dtype=np.int64)
    pos = 64
    gaps = ((w >> np.uint64(20)) % np.uint64(max_gap + 1)).astype(np.int64)
    for p in range(n):
        pos = (pos + int(gaps[p]) + align - 1) // align * align
        for f in range(int(first[p]), int(first[p + 1])):
            offs[f] = pos
            pos += int(lens[f])
    size = pos + 4096
    arena_np = O.splitmix64_bytes(0x7113 + max_len, size)
    seeds = (w >> np.uint64(40) & np.uint64(0xFFFF)).astype(np.uint16)
    offs, lens, first = offs.astype(np.uint64), lens.astype(np.uint32), first.astype(np.uint32)
    a = torch.from_numpy(arena_np).to(DEV)
    for complement in (False, True):
        expect = oracle.chain_batch(arena_np, offs, lens, first, seeds, complement=complement)
        for runs in (False, True):
            for hint in (0, 300):
                got = host_u16(csum_chain(a, dev(offs, np.int64), dev(lens, np.int32), dev(first, np.int32),
                                          dev(seeds, np.int16), complement=complement, frag_len_hint=hint, runs=runs))
                assert np.array_equal(got, expect), (complement, runs, hint, int(np.flatnonzero(got != expect)[0]))
