"""Synthetic batch layouts (rustnetworkstack_amd.workloads) — host logic only."""
import numpy as np

from oracle import oracle as O
from rustnetworkstack_amd import workloads as W


def test_splitmix_matches_oracle_stream():
    assert np.array_equal(W.splitmix64(W.DATA_SEED, 1000), O.splitmix64_words(W.DATA_SEED, 1000))
    assert np.array_equal(W.splitmix64(5, 10, start=7), O.splitmix64_words(5, 17)[7:])


def test_headline_layout():
    L = W.make_layout("c3_1500B")
    assert L.n == 1 << 20 and L.payload_bytes == 1500 << 20
    assert np.all(L.off % 16 == 0) and np.all(np.diff(L.off) == 1504)
    assert L.arena_bytes == 1504 << 20


def test_other_configs():
    assert W.make_layout("c2_64B").payload_bytes == 64 << 20
    c4 = W.make_layout("c4_9000B")
    assert c4.n == 1 << 18 and c4.payload_bytes == 9000 << 18


def test_imix_ratio_and_alignment():
    L = W.make_layout("c5_imix", n=1 << 20)
    counts = {s: int((L.length == s).sum()) for s in W.IMIX_SIZES}
    assert sum(counts.values()) == L.n
    assert abs(counts[40] / L.n - 7 / 12) < 0.01
    assert abs(counts[576] / L.n - 4 / 12) < 0.01
    assert abs(counts[1500] / L.n - 1 / 12) < 0.01
    assert np.all(L.off % 16 == 0)
    assert np.all(L.off[1:] >= L.off[:-1] + L.length[:-1])
    assert L.arena_bytes >= int(L.off[-1]) + int(L.length[-1])


def test_sharding_covers_every_packet_once():
    full = W.make_layout("c5_imix", n=100003)
    for world in (1, 2, 4, 8):
        parts = [W.make_layout("c5_imix", n=100003, shard=(r, world)) for r in range(world)]
        assert sum(p.n for p in parts) == full.n
        assert np.array_equal(np.concatenate([p.length for p in parts]), full.length)
        assert np.array_equal(np.concatenate([p.seed for p in parts]), full.seed)


def test_packed_layout_matches_synthetic_offsets():
    """rns_packed_layout (host C ABI) reproduces every synthetic config's offsets at
    16-byte alignment, and implements align_up(previous end) at any alignment."""
    import numpy as np

    from rustnetworkstack_amd.batch import packed_layout
    from rustnetworkstack_amd.workloads import make_layout
    for name, n in (("c2_64B", 1000), ("c3_1500B", 1000), ("c5_imix", 4099)):
        lay = make_layout(name, n=n)
        blk, off, end = packed_layout(lay.length, 4)
        assert np.array_equal(off, lay.off) and end == lay.arena_bytes
        assert np.array_equal(blk, lay.off[::64])
    rng = np.random.default_rng(3)
    ln = rng.integers(0, 65536, 777)
    for a in (0, 1, 5, 12):
        blk, off, end = packed_layout(ln, a, first_off=9)
        m = (1 << a) - 1
        expect = 9 + np.concatenate([[0], np.cumsum((ln + m) & ~m)])
        assert np.array_equal(off, expect[:-1]) and end == int(expect[-1])
        assert np.array_equal(blk, off[::64])


def test_device_batch_stride_detection():
    """DeviceBatch.stride() (bench.py --desc strided): fixed-size configs are equal-length
    packets at a fixed stride; IMIX is not (no device needed: the check reads the layout)."""
    from rustnetworkstack_amd.workloads import DeviceBatch
    b = object.__new__(DeviceBatch)
    b.layout = W.make_layout("c2_64B", n=1000)
    assert b.stride() == (0, 64, 64)
    b.layout = W.make_layout("c3_1500B", n=1000)
    assert b.stride() == (0, 1504, 1500)
    b.layout = W.make_layout("c5_imix", n=1000)
    assert b.stride() is None
