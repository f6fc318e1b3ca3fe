"""Compact descriptors (rns_csum_batch_dev_off32: 32-bit packet offsets) against the
oracle and against the 64-bit descriptor path, through the C ABI.

Same kernels and same arithmetic as rns_csum_batch_dev (util.rs:88-106); only the
descriptor offset width differs, so every case here must be bit-exact with the
golden fixtures / the C oracle.
"""
import numpy as np
import pytest
import torch

from conftest import sweep_arena
from rustnetworkstack_amd import _lib
from rustnetworkstack_amd.batch import csum_batch
from rustnetworkstack_amd.workloads import DeviceBatch, make_layout

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def host_u16(t: torch.Tensor) -> np.ndarray:
    torch.cuda.synchronize()
    return t.view(torch.int16).cpu().numpy().view(np.uint16)


def off32(off: np.ndarray) -> torch.Tensor:
    assert int(off.max(initial=0)) < 2 ** 32
    return torch.from_numpy(np.ascontiguousarray(off.astype(np.uint32)).view(np.int32)).to(DEV)


def u32(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a.astype(np.uint32)).view(np.int32)).to(DEV)


def u16(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a.astype(np.uint16)).view(np.int16)).to(DEV)


@pytest.fixture(scope="module", autouse=True)
def gpu_present():
    if not torch.cuda.is_available() or _lib.load().rns_device_count() == 0:
        pytest.fail("gpu tests need a GPU (the HIP path has no CPU fallback)")


def test_golden_sweep_compact(sweep):
    arena = torch.from_numpy(sweep_arena(sweep)).to(DEV)
    off = off32(np.array(sweep["offset"]))
    ln, sd = u32(np.array(sweep["length"])), u16(np.array(sweep["pkt_seed"]))
    expect = np.array(sweep["expect"], dtype=np.uint16)
    for hint in (0, 40, 64, 576, 1500, 9000, 65535):
        assert np.array_equal(host_u16(csum_batch(arena, off, ln, sd, len_hint=hint, compact=True)), expect), hint
        got = csum_batch(arena, off, ln, sd, complement=True, len_hint=hint, compact=True)
        assert np.array_equal(host_u16(got), expect ^ 0xFFFF), hint


def test_random_descriptors_and_bounds(oracle):
    """Any start offset, lengths 0..9000, overlapping, some outside the arena."""
    rng = np.random.default_rng(32)
    size = 3 << 20
    arena_np = rng.integers(0, 256, size, dtype=np.uint8)
    n = 50000
    ln = rng.integers(1, 9001, n).astype(np.uint32)
    off = rng.integers(0, size - 9000, n).astype(np.uint64)
    sd = rng.integers(0, 1 << 16, n).astype(np.uint16)
    expect = oracle.batch(arena_np, off, ln, sd)
    # descriptors reaching past the arena: result 0, counted as bad
    bad_rows = rng.choice(n, 100, replace=False)
    off[bad_rows[:50]] = size - 10
    ln[bad_rows[:50]] = 11
    off[bad_rows[50:]] = 0xFFFFFFF0
    expect[bad_rows] = 0
    arena = torch.from_numpy(arena_np).to(DEV)
    d_off, d_len, d_sd = off32(off), u32(ln), u16(sd)
    for hint in (0, 64, 340, 1500, 9000):
        bad = torch.zeros(1, dtype=torch.int32, device=DEV)
        got = host_u16(csum_batch(arena, d_off, d_len, d_sd, len_hint=hint, bad=bad, compact=True))
        assert np.array_equal(got, expect), hint
        assert int(bad.item()) == 100


@pytest.mark.parametrize("name", ["c2_64B", "c3_1500B", "c4_9000B", "c5_imix"])
def test_full_size_compact_equals_64bit(name):
    """Every packet of each BASELINE.json config: compact == 64-bit descriptors (the
    64-bit path is checked packet by packet against the oracle in test_gpu_parity).
    c4's arena is 2.36 GB, so its upper offsets have bit 31 set."""
    lay = make_layout(name)
    b = DeviceBatch(lay, DEV)
    ref = csum_batch(b.arena, b.off, b.length, b.seed, complement=True, len_hint=int(lay.mean_len))
    got = csum_batch(b.arena, off32(lay.off), b.length, b.seed, complement=True, len_hint=int(lay.mean_len),
                     compact=True)
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))
    if name == "c4_9000B":
        assert int(lay.off.max()) >= 2 ** 31
    del b
    torch.cuda.empty_cache()


def test_compact_form_is_explicit():
    """int32 offsets are the compact form only when asked for: without
    compact=True they are a TypeError, and compact=True refuses int64 offsets."""
    arena = torch.zeros(64, dtype=torch.uint8, device=DEV)
    ln = u32(np.array([8]))
    with pytest.raises(TypeError):
        csum_batch(arena, off32(np.array([0])), ln)
    with pytest.raises(TypeError):
        csum_batch(arena, torch.zeros(1, dtype=torch.int64, device=DEV), ln, compact=True)
    assert host_u16(csum_batch(arena, off32(np.array([0])), ln, compact=True))[0] == 0
