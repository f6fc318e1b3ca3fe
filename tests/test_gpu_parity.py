"""Parity of the gfx950 HIP path with the oracle (bit-exact), through the C ABI.

Small cases compare every packet with the committed golden fixtures and with
the C oracle; full BASELINE.json sizes compare every packet with the C oracle
(multi-threaded) and check size-independent properties (transmit-fill then
receive-verify gives 0 for every packet).  Runs on one MI355X: one process,
no repeated launches of the runner.
"""
import numpy as np
import pytest
import torch

from conftest import sweep_arena
from oracle import oracle as O
from rustnetworkstack_amd import _lib
from rustnetworkstack_amd.batch import HostBatcher, PinnedBuffer, csum_batch, csum_batch_strided, fill_splitmix64
from rustnetworkstack_amd.workloads import DeviceBatch, make_layout

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
SHAPES = [(var, g, u) for var in (0, 1) for g in (4, 8, 16, 32, 64) for u in (1, 2, 4, 8)]
SHAPES += [(var, 64, 4) for var in (2, 3, 4, 6)]
SHAPES += [(var, 2, u) for var in (1, 3) for u in (1, 2, 4)]  # 2-lane groups: rounds kernel only
SHAPES += [(var, g, u) for var in (9, 11) for g in (2, 4, 8) for u in (1, 2)]  # every round in flight


def host_u16(t: torch.Tensor) -> np.ndarray:
    torch.cuda.synchronize()
    return t.view(torch.int16).cpu().numpy().view(np.uint16)


def to_dev(a: np.ndarray, dtype_view) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(dtype_view)).to(DEV)


def dev_desc(off, ln, sd):
    return to_dev(off.astype(np.uint64), np.int64), to_dev(ln.astype(np.uint32), np.int32), (
        None if sd is None else to_dev(sd.astype(np.uint16), np.int16))


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or _lib.load().rns_device_count() == 0:
        pytest.fail("gpu tests need a GPU (the HIP path has no CPU fallback)")


def test_device_splitmix_fill_matches_oracle():
    for nbytes in (1, 7, 8, 1 << 20, (1 << 20) + 5):
        buf = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
        fill_splitmix64(buf, 0x5EEDC0DE)
        torch.cuda.synchronize()
        assert np.array_equal(buf.cpu().numpy(), O.splitmix64_bytes(0x5EEDC0DE, nbytes))


@pytest.fixture(scope="module")
def sweep_dev(sweep):
    arena = torch.from_numpy(sweep_arena(sweep)).to(DEV)
    off, ln, sd = dev_desc(np.array(sweep["offset"]), np.array(sweep["length"]), np.array(sweep["pkt_seed"]))
    return arena, off, ln, sd, np.array(sweep["expect"], dtype=np.uint16)


@pytest.mark.parametrize("var,g,u", SHAPES)
@pytest.mark.parametrize("max_blocks", [0, 37])
def test_golden_sweep_every_shape(sweep_dev, var, g, u, max_blocks):
    arena, off, ln, sd, expect = sweep_dev
    out = csum_batch(arena, off, ln, sd, shape=(var, g, u, max_blocks))
    assert np.array_equal(host_u16(out), expect)
    outc = csum_batch(arena, off, ln, sd, complement=True, shape=(var, g, u, max_blocks))
    assert np.array_equal(host_u16(outc), expect ^ 0xFFFF)


def test_golden_sweep_default_shapes(sweep_dev):
    arena, off, ln, sd, expect = sweep_dev
    for hint in (0, 40, 64, 576, 1500, 9000, 65535):
        assert np.array_equal(host_u16(csum_batch(arena, off, ln, sd, len_hint=hint)), expect)


def test_length_by_alignment_sweep(oracle):
    """Every length 1..2048 at every start offset mod 16, random seeds, vs the C oracle."""
    arena_np = O.splitmix64_bytes(0xA11A, 4 << 20)
    lens = np.repeat(np.arange(1, 2049, dtype=np.uint32), 16)
    align = np.tile(np.arange(16, dtype=np.uint64), 2048)
    base = (O.splitmix64_words(0xB0B, lens.size) % np.uint64((4 << 20) - 4096)) & ~np.uint64(15)
    off = base + align
    sd = (O.splitmix64_words(0xC0C, lens.size) & np.uint64(0xFFFF)).astype(np.uint16)
    expect = oracle.batch(arena_np, off, lens, sd, complement=True)
    arena = torch.from_numpy(arena_np).to(DEV)
    d_off, d_len, d_sd = dev_desc(off, lens, sd)
    for shape in (None, (0, 4, 1, 0), (0, 64, 2, 512), (1, 4, 1, 0), (1, 16, 2, 0), (1, 64, 4, 0), (1, 8, 8, 3),
                  (1, 64, 2, 512), (3, 16, 8, 0), (4, 0, 0, 0), (6, 0, 0, 0), (6, 0, 0, 7)):
        out = csum_batch(arena, d_off, d_len, d_sd, complement=True, shape=shape, len_hint=1024)
        assert np.array_equal(host_u16(out), expect), shape


def test_edge_patterns_and_zero_handling(oracle):
    zeros = np.zeros(200016, dtype=np.uint8)
    ones = np.full(200016, 0xFF, dtype=np.uint8)
    arena_np = np.concatenate([zeros, ones])
    rows = []
    for base in (0, 200016):
        for L in (1, 2, 3, 64, 1500, 9000, 65535, 131072, 131073, 200001):
            for a in (0, 1, 5):
                for s in (0, 1, 0xFFFE, 0xFFFF):
                    if a + L <= 200016:
                        rows.append((base + a, L, s))
    off = np.array([r[0] for r in rows], dtype=np.uint64)
    ln = np.array([r[1] for r in rows], dtype=np.uint32)
    sd = np.array([r[2] for r in rows], dtype=np.uint16)
    expect = oracle.batch(arena_np, off, ln, sd)
    arena = torch.from_numpy(arena_np).to(DEV)
    d = dev_desc(off, ln, sd)
    for shape in (None, (0, 4, 4, 0), (0, 64, 1, 0), (1, 4, 4, 0), (1, 32, 8, 0), (1, 64, 1, 5), (4, 0, 0, 0),
                  (6, 0, 0, 3)):
        assert np.array_equal(host_u16(csum_batch(arena, *d, shape=shape)), expect), shape
    # all-zero payload with seed 0 is 0 (checksum 0xffff); an even run of 0xff folds to 0xffff (checksum 0)
    assert expect[rows.index((0, 1500, 0))] == 0
    assert expect[rows.index((200016, 1500, 0))] == 0xFFFF


def test_bounds_and_empty_packets():
    arena = torch.zeros(4096, dtype=torch.uint8, device=DEV)
    fill_splitmix64(arena, 3)
    off = np.array([0, 4000, 4096, 4097, 10, 5000, 3, 4000], dtype=np.uint64)
    ln = np.array([16, 97, 0, 0, 0, 1, 4093, 96], dtype=np.uint32)
    sd = np.array([1, 2, 3, 4, 0xABCD, 6, 7, 8], dtype=np.uint16)
    bad = torch.zeros(1, dtype=torch.int32, device=DEV)
    out = host_u16(csum_batch(arena, *dev_desc(off, ln, sd), bad=bad))
    a = arena.cpu().numpy().tobytes()
    assert out[0] == O.ones_comp_py(1, a[0:16])
    assert out[1] == 0                     # 4000+97 > 4096: rejected
    assert out[2] == 3                     # len 0 at the end: seed (reference panics; API-defined)
    assert out[3] == 0                     # offset past the end: rejected
    assert out[4] == 0xABCD                # len 0: seed unchanged
    assert out[5] == 0                     # rejected
    assert out[6] == O.ones_comp_py(7, a[3:4096])
    assert out[7] == O.ones_comp_py(8, a[4000:4096])   # ends exactly at the arena end
    assert int(bad.item()) == 3


def test_unaligned_arena_base(oracle):
    big = torch.empty(1 << 20, dtype=torch.uint8, device=DEV)
    fill_splitmix64(big, 99)
    host = big.cpu().numpy()
    for shift in (1, 3, 8, 15):
        view = big[shift:]
        n = 2000
        ln = (O.splitmix64_words(shift, n) % np.uint64(1600) + np.uint64(1)).astype(np.uint32)
        off = (O.splitmix64_words(shift + 100, n) % np.uint64((1 << 20) - 2000)).astype(np.uint64)
        expect = oracle.batch(host[shift:], off, ln, None, complement=True)
        for shape in (None, (4, 0, 0, 0), (3, 16, 8, 0)):
            out = csum_batch(view, *dev_desc(off, ln, None), complement=True, shape=shape)
            assert np.array_equal(host_u16(out), expect), (shift, shape)


def test_strided_api(oracle):
    for L, stride, first in ((64, 64, 0), (1500, 1504, 0), (1500, 1501, 3), (9000, 9008, 16), (40, 48, 7)):
        n = 5000
        arena = torch.empty(first + stride * n + 64, dtype=torch.uint8, device=DEV)
        fill_splitmix64(arena, L)
        sd_np = (O.splitmix64_words(L, n) & np.uint64(0xFFFF)).astype(np.uint16)
        sd = to_dev(sd_np, np.int16)
        out = csum_batch_strided(arena, n, stride, L, first_off=first, seed=sd, complement=True)
        off = first + np.arange(n, dtype=np.uint64) * np.uint64(stride)
        expect = oracle.batch(arena.cpu().numpy(), off, np.full(n, L, dtype=np.uint32), sd_np, complement=True)
        assert np.array_equal(host_u16(out), expect), (L, stride, first)


def test_strided_tiny_packets(oracle):
    """The strided tiny kernel (len <= 64 at 16-byte-aligned starts and stride): every length
    1..64, strides from the packed one to 2048, packet counts that are not a multiple of 64,
    with and without seeds and the complement, all-0xff bytes, packets past the arena's end
    (rejected and counted), an unaligned arena pointer (the kernel's absolute alignment rule
    then sends the batch to the rounds kernel) and overlapping packets (stride < len)."""
    rng = O.splitmix64_words(0x7A1, 4096)
    k = 0
    for L in list(range(1, 65)) + [64, 48, 17]:
        stride = 2048 if L % 5 == 0 else 16 if L % 3 == 0 else (L + 15) & ~15   # 16: overlapping packets
        n = 64 * (1 + int(rng[k] % np.uint64(40))) + int(rng[k + 1] % np.uint64(64))
        first = 16 * int(rng[k + 2] % np.uint64(8))
        k += 3
        arena_np = O.splitmix64_bytes(L * 7919, first + stride * n + 64)
        if L in (48, 17):
            arena_np[:] = 0xFF
        arena = torch.from_numpy(arena_np.copy()).to(DEV)
        sd_np = (O.splitmix64_words(L + 5, n) & np.uint64(0xFFFF)).astype(np.uint16)
        off = first + np.arange(n, dtype=np.uint64) * np.uint64(stride)
        for seeded, comp in ((True, True), (False, False)):
            out = csum_batch_strided(arena, n, stride, L, first_off=first, seed=to_dev(sd_np, np.int16) if seeded else None,
                                     complement=comp)
            expect = oracle.batch(arena_np, off, np.full(n, L, dtype=np.uint32), sd_np if seeded else None,
                                  complement=comp)
            assert np.array_equal(host_u16(out), expect), (L, stride, first, seeded)
    # past the arena's end: the last packets rejected, counted, 0
    L, stride, n = 64, 64, 1000
    arena_np = O.splitmix64_bytes(3, 64 * 990 + 20)
    arena = torch.from_numpy(arena_np.copy()).to(DEV)
    bad = torch.zeros(1, dtype=torch.int32, device=DEV)
    got = host_u16(csum_batch_strided(arena, n, stride, L, complement=True, bad=bad))
    off = np.arange(990, dtype=np.uint64) * np.uint64(64)
    assert np.array_equal(got[:990], oracle.batch(arena_np, off, np.full(990, L, np.uint32), None, complement=True))
    assert (got[990:] == 0).all() and int(bad.item()) == 10
    # an unaligned arena pointer, and overlapping packets
    base = torch.from_numpy(O.splitmix64_bytes(9, 70_000)).to(DEV)
    for view_off, L, stride in ((8, 64, 64), (0, 64, 32), (0, 40, 16)):
        view = base[view_off:]
        n = 1000
        got = host_u16(csum_batch_strided(view, n, stride, L, complement=True))
        host = view.cpu().numpy()
        off = np.arange(n, dtype=np.uint64) * np.uint64(stride)
        assert np.array_equal(got, oracle.batch(host, off, np.full(n, L, np.uint32), None, complement=True))


@pytest.mark.parametrize("name", ["c2_64B", "c3_1500B", "c4_9000B", "c5_imix"])
def test_full_size_configs_bit_exact(oracle, name):
    """Every packet of every BASELINE.json GPU config, bit-exact against the C oracle."""
    lay = make_layout(name)
    b = DeviceBatch(lay, DEV)
    b.run(complement=False)
    got = b.host_out()
    arena = b.host_arena()
    expect = oracle.batch(arena, lay.off, lay.length, lay.seed, threads=16)
    assert np.array_equal(got, expect)
    del b
    torch.cuda.empty_cache()


def test_full_size_transmit_fill_then_receive_verify():
    """Size-independent property at the headline size: store each packet's complemented
    checksum into its TCP checksum field (tcp.rs:970-973, field zeroed first as
    alloc_header does, buf.rs:286-288), then the receive check (tcp.rs:848) gives 0 for all."""
    lay = make_layout("c3_1500B")
    b = DeviceBatch(lay, DEV)
    arena, off = b.arena, b.off
    field = off.view(-1, 1) + torch.tensor([16, 17], device=DEV)   # header[16..18]
    arena[field.flatten()] = 0
    tx = csum_batch(arena, off, b.length, b.seed, complement=True)
    tx32 = tx.view(torch.int16).to(torch.int32) & 0xFFFF
    arena[field[:, 0]] = (tx32 >> 8).to(torch.uint8)
    arena[field[:, 1]] = (tx32 & 0xFF).to(torch.uint8)
    rx = csum_batch(arena, off, b.length, b.seed, complement=True)
    assert int((rx.view(torch.int16) != 0).sum().item()) == 0
    del b
    torch.cuda.empty_cache()


@pytest.mark.parametrize("pinned", [True, False])
def test_host_resident_pipeline(oracle, pinned):
    lay = make_layout("c5_imix", n=300000)
    nbytes = lay.arena_bytes
    if pinned:
        pb = PinnedBuffer(nbytes)
        arena = pb.array
        arena[:] = O.splitmix64_bytes(lay.data_seed, nbytes)
    else:
        arena = O.splitmix64_bytes(lay.data_seed, nbytes)
    hb = HostBatcher(device=0, chunk_bytes=1 << 20, nstreams=3)
    out = hb.run(arena, lay.off, lay.length, lay.seed, complement=True)
    expect = oracle.batch(arena, lay.off, lay.length, lay.seed, complement=True)
    assert np.array_equal(out, expect)
    # descriptors that violate the host API contract are rejected before any copy
    with pytest.raises(_lib.ChecksumError):
        hb.run(arena, lay.off[::-1].copy(), lay.length, None)
    hb.close()
    if pinned:
        pb.free()


def test_host_toolarge_rejected_before_queueing(oracle):
    """A packet that cannot fit one staging chunk is rejected by the validation
    pass (RNS_E_TOOLARGE) before any chunk is queued, so no slot is left busy: a
    second, smaller call on the same context gets exactly its own results and
    nothing is written past its output (drain skipped on TOOLARGE)."""
    hb = HostBatcher(device=0, chunk_bytes=4096, nstreams=2)
    small = 3000
    ln = np.full(small + 1, 64, dtype=np.uint32)
    ln[-1] = 9000                                 # c4 jumbo frame: > 4096-byte chunks
    off = np.zeros(small + 1, dtype=np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
    arena = O.splitmix64_bytes(0x7001, int(off[-1]) + 9000)
    out = np.full(small + 1, 0xABCD, dtype=np.uint16)
    with pytest.raises(_lib.ChecksumError) as ei:
        hb.run(arena, off, ln, None, complement=True, out=out)
    assert ei.value.status == _lib.RNS_E_TOOLARGE
    assert (out == 0xABCD).all()                 # nothing was queued or drained into it
    # the next, smaller call on the same context: exact results, no stale slot drained into it
    n2 = 100
    guard = np.full(n2 + 64, 0x5A5A, dtype=np.uint16)
    got = hb.run(arena, off[:n2], ln[:n2], None, complement=True, out=guard[:n2])
    assert np.array_equal(got, oracle.batch(arena, off[:n2], ln[:n2], None, complement=True))
    assert (guard[n2:] == 0x5A5A).all()
    hb.close()


def test_arena_beyond_4gib_uses_64bit_path(oracle):
    """Arenas >= 4 GiB cannot use 32-bit buffer offsets: every kernel takes its
    64-bit global-load path.  Packets straddle the 4 GiB line and sit at both ends."""
    nbytes = (4 << 30) + (64 << 20)
    arena = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
    fill_splitmix64(arena, 0xB16)
    four_g = 1 << 32
    rows = []
    for base in (0, four_g - 6000, four_g - 1, four_g + 3, nbytes - 20000):   # every packet inside the arena
        for i, L in enumerate((1, 40, 576, 1500, 9000, 3)):
            rows.append((base + 1700 * i + (i % 3), L))
    off = np.array([r[0] for r in rows], dtype=np.uint64)
    ln = np.array([r[1] for r in rows], dtype=np.uint32)
    sd = (O.splitmix64_words(77, len(rows)) & np.uint64(0xFFFF)).astype(np.uint16)
    assert int((off + ln).max()) <= nbytes
    # expected values from host copies of only the touched windows
    expect = np.array([oracle.compute_ones_comp(int(s), arena[int(o):int(o) + int(L)].cpu().numpy().tobytes())
                       for o, L, s in zip(off, ln, sd)], dtype=np.uint16)
    d = dev_desc(off, ln, sd)
    for shape in (None, (0, 16, 2, 0), (2, 64, 4, 0), (1, 16, 4, 0), (3, 32, 4, 0), (4, 0, 0, 0), (6, 0, 0, 0)):
        assert np.array_equal(host_u16(csum_batch(arena, *d, shape=shape)), expect), shape
    del arena
    torch.cuda.empty_cache()


@pytest.mark.parametrize("total", [4093, 4094, 4095, 4097, 4101, 4111])
def test_packets_ending_at_unpadded_arena_end(oracle, total):
    """Arena lengths that are not a multiple of 4 or 16, packets ending exactly at the
    last byte, at every start parity: no kernel may drop the tail bytes."""
    arena_np = O.splitmix64_bytes(total, total)
    arena = torch.from_numpy(arena_np.copy()).to(DEV)
    lens = np.array([1, 2, 3, 5, 7, 16, 17, 40, 64, 333, 1500], dtype=np.uint32)
    off = (total - lens).astype(np.uint64)
    sd = np.arange(len(lens), dtype=np.uint16) * np.uint16(4099)
    expect = oracle.batch(arena_np, off, lens, sd)
    d = dev_desc(off, lens, sd)
    for shape in [None] + [(v, g, u, 0) for v in range(8) for g, u in ((4, 1), (16, 4), (64, 2))] + \
            [(9, 4, 1, 0), (11, 2, 2, 0), (11, 8, 1, 3)]:
        assert np.array_equal(host_u16(csum_batch(arena, *d, shape=shape)), expect), shape


@pytest.mark.parametrize("name", ["c2_64B", "c3_1500B"])
def test_strided_form_full_size_bit_exact(oracle, name):
    """The fixed-stride form bench.py --desc strided binds (DeviceBatch.launcher(strided=True)),
    every packet of the full config against the C oracle."""
    lay = make_layout(name)
    b = DeviceBatch(lay, DEV)
    assert b.stride() == (0, int(lay.off[1]), int(lay.length[0]))
    b.launcher(complement=True, strided=True)()
    got = b.host_out()
    expect = oracle.batch(b.host_arena(), lay.off, lay.length, lay.seed, complement=True, threads=16)
    assert np.array_equal(got, expect)
    del b
