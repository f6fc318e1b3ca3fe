"""The oracle is pinned before it is trusted: the C restatement (oracle/csum_oracle.c)
and the pure-Python restatement (oracle/oracle.py) must reproduce every
known-answer vector of the reference's own tests (util.rs:277-317, 436-457),
the RFC 1071 / IPv4 vectors, and the committed sweep fixtures."""
import numpy as np
import pytest

from conftest import expand_fragment, sweep_arena
from oracle import oracle as O


def test_ones_comp_kats(oracle, kats):
    for v in kats["ones_comp"]:
        b = bytes.fromhex(v["bytes"])
        assert oracle.compute_ones_comp(v["seed"], b) == v["expect"], v["source"]
        assert O.ones_comp_py(v["seed"], b) == v["expect"], v["source"]


def test_checksum_kats(oracle, kats):
    for v in kats["checksum"]:
        b = bytes.fromhex(v["bytes"])
        assert oracle.compute_checksum(b) == v["expect"], v["source"]
        assert O.checksum_py(b) == v["expect"], v["source"]


def test_buffer_kats(oracle, kats):
    for v in kats["buffer_ones_comp"]:
        frags = [expand_fragment(f) for f in v["fragments"]]
        assert oracle.compute_buffer_ones_comp(v["seed"], frags) == v["expect"], v["source"]
        assert O.buffer_ones_comp_py(v["seed"], frags) == v["expect"], v["source"]


def test_pseudo_header_kats(oracle, kats):
    for v in kats["pseudo_header"]:
        s, d = bytes.fromhex(v["src"]), bytes.fromhex(v["dst"])
        assert oracle.compute_pseudo_header_checksum(s, d, v["length"], v["protocol"]) == v["expect"], v["source"]
        assert O.pseudo_header_py(s, d, v["length"], v["protocol"]) == v["expect"], v["source"]


def test_reference_panics(oracle):
    with pytest.raises(O.ReferencePanic):
        oracle.compute_ones_comp(0, b"")
    with pytest.raises(O.ReferencePanic):
        O.ones_comp_py(0, b"")
    with pytest.raises(O.ReferencePanic):
        oracle.compute_pseudo_header_checksum(b"\x01" * 16, b"\x02" * 4, 20, 6)
    with pytest.raises(O.ReferencePanic):
        oracle.compute_buffer_ones_comp(0, [b"\x01", b""])


def test_sweep_fixture_matches_c_oracle(oracle, sweep):
    arena = sweep_arena(sweep)
    off = np.array(sweep["offset"], dtype=np.uint64)
    ln = np.array(sweep["length"], dtype=np.uint32)
    sd = np.array(sweep["pkt_seed"], dtype=np.uint16)
    got = oracle.batch(arena, off, ln, sd)
    assert np.array_equal(got, np.array(sweep["expect"], dtype=np.uint16))
    got_c = oracle.batch(arena, off, ln, sd, complement=True)
    assert np.array_equal(got_c, 0xFFFF ^ np.array(sweep["expect"], dtype=np.uint16))


def test_sweep_chains_match_c_oracle(oracle, sweep):
    buf = sweep_arena(sweep).tobytes()
    for ch in sweep["chains"]:
        frags = [buf[o:o + s] for o, s in ch["frags"]]
        assert oracle.compute_buffer_ones_comp(ch["seed"], frags) == ch["expect"]


def test_zero_handling(oracle):
    """SURVEY 7 'hard parts': all-zero data with seed 0 gives 0 (checksum 0xffff);
    a nonzero multiple of 0xffff gives 0xffff (checksum 0)."""
    assert oracle.compute_ones_comp(0, bytes(1500)) == 0
    assert oracle.compute_checksum(bytes(1500)) == 0xFFFF
    assert oracle.compute_ones_comp(0, b"\xff" * 1500) == 0xFFFF
    assert oracle.compute_ones_comp(0xFFFF, bytes(64)) == 0xFFFF


def test_u32_wrap_restated(oracle):
    """Beyond 131072 bytes the reference's u32 accumulator wraps (release build):
    the C and Python restatements agree on it."""
    data = b"\xff" * 131074 + b"\x12\x34" * 3
    assert oracle.compute_ones_comp(0x1234, data) == O.ones_comp_py(0x1234, data)


def test_batch_mt_equals_single(oracle):
    arena = O.splitmix64_bytes(7, 1 << 20)
    n = 3000
    ln = (O.splitmix64_words(9, n) % np.uint64(300) + np.uint64(1)).astype(np.uint32)
    off = (O.splitmix64_words(11, n) % np.uint64((1 << 20) - 400)).astype(np.uint64)
    sd = (O.splitmix64_words(13, n) & np.uint64(0xFFFF)).astype(np.uint16)
    a = oracle.batch(arena, off, ln, sd, complement=True)
    b = oracle.batch(arena, off, ln, sd, complement=True, threads=4)
    assert np.array_equal(a, b)


def test_splitmix64_known_value():
    # splitmix64 with state 0: first output 0xe220a8397b1dcdaf (Vigna's reference generator)
    assert int(O.splitmix64_words(0, 1)[0]) == 0xE220A8397B1DCDAF


def test_chain_batch_matches_per_packet_chains(oracle, sweep):
    """The C batch-of-chains restatement agrees with the single-chain one on the fixtures."""
    arena = sweep_arena(sweep)
    offs, lens, first, seeds = [], [], [0], []
    for ch in sweep["chains"]:
        for o, s in ch["frags"]:
            offs.append(o)
            lens.append(s)
        first.append(len(offs))
        seeds.append(ch["seed"])
    got = oracle.chain_batch(arena, np.array(offs), np.array(lens), np.array(first), np.array(seeds))
    assert np.array_equal(got, np.array([ch["expect"] for ch in sweep["chains"]], dtype=np.uint16))
