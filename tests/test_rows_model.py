"""The decomposition csum_rows_kernel relies on (rns_kernels.hpp), checked on the
CPU against the oracle: in a packed region (packets 16-byte aligned, each followed by its
padding up to the next 2^align boundary), with P(c) the region's inclusive prefix of whole
16-byte chunk sums,

    LE sum of packet p = P(e - 1) - P(c0 - 1) + LE sum of the first ((len - 1) & 15) + 1 bytes of chunk e

(P(-1) = 0; e == c0: the end chunk alone), taken mod 2^32 with u32 prefixes that wrap, and the
result finished as every kernel does (fold, byte swap for an even start, + seed, fold).  The
model works a wave (64 packets) at a time with rows of 64 chunks, as the kernel does, so the
capture rows/lanes are the kernel's — also with the row stream starting at the 128-byte line
below each region (the kernel's default since round 4: the bytes before the region cancel).  Non-zero padding bytes, padding chunks (align 32..4096),
empty packets, maximum lengths and all-0xff bytes (u32 prefix wrap) included."""
import numpy as np
import pytest

from oracle import oracle as O


def fold(x):
    while x > 0xFFFF:
        x = (x & 0xFFFF) + (x >> 16)
    return x


def rows_model(arena, blk_off, length, seed, complement=True, line=0):
    """One 64-packet unit per 'wave'; returns the u16 results.  line = 128: the row stream
    starts at the 128-byte line below the region (RNS_ROWS_LINE_ALIGN), so the prefix also
    holds the bytes before the region — they cancel in every difference."""
    n = len(length)
    out = np.zeros(n, dtype=np.uint16)
    words = arena.view(np.uint16).astype(np.uint64)  # LE words at even offsets
    chunk_sum = words.reshape(-1, 8).sum(axis=1)        # every 16-byte chunk (arena is 16-aligned)
    for u in range((n + 63) // 64):
        r0 = int(blk_off[u])
        ln = np.zeros(64, dtype=np.int64)
        m = min(64, n - 64 * u)
        ln[:m] = length[64 * u:64 * u + m]
        align = ALIGN
        pad = (ln + align - 1) // align * align
        excl = np.concatenate(([0], np.cumsum(pad)[:-1]))
        total = int(pad.sum())
        lead = (r0 % line) if line else 0                  # bytes of the first line before the region
        nch = (total + lead) // 16
        c = chunk_sum[(r0 - lead) // 16:(r0 - lead) // 16 + nch]
        prefix = np.cumsum(c) & 0xFFFFFFFF                 # u32, wraps like the kernel's carry
        excl = excl + lead
        for lane in range(m):
            L = int(ln[lane])
            if L == 0:
                s = 0
            else:
                c0 = int(excl[lane]) // 16
                e = (int(excl[lane]) + L - 1) // 16
                pa = int(prefix[c0 - 1]) if c0 > 0 else 0
                pb = int(prefix[e - 1]) if e > c0 else pa
                nv = ((L - 1) & 15) + 1
                endb = arena[r0 - lead + 16 * e:r0 - lead + 16 * e + nv].astype(np.uint64)
                part = int(endb[0::2].sum() + (endb[1::2].sum() << 8))
                s = (pb - pa + part) & 0xFFFFFFFF
            x = fold(s)
            g = ((x & 0xFF) << 8) | (x >> 8)               # even start: LE -> BE
            acc = int(seed[64 * u + lane]) + g
            acc = (acc & 0xFFFF) + (acc >> 16)
            out[64 * u + lane] = acc ^ 0xFFFF if complement else acc
    return out


ALIGN = 16


@pytest.mark.parametrize("align_log2", [4, 5, 7, 12])
@pytest.mark.parametrize("pattern", ["random", "ff", "zero"])
def test_rows_decomposition_matches_oracle(oracle, align_log2, pattern):
    global ALIGN
    ALIGN = 1 << align_log2
    rng = np.random.default_rng(0x2045 + align_log2)
    n = 64 * 5 + 17
    length = rng.integers(0, 1601, n).astype(np.int64)
    length[rng.random(n) < 0.1] = 0                       # empty packets
    length[3] = 65535                                     # the largest u16 packet
    length[70:74] = [1, 15, 16, 17]
    pad = (length + ALIGN - 1) // ALIGN * ALIGN
    off = np.concatenate(([0], np.cumsum(pad)[:-1])).astype(np.uint64)
    size = int(pad.sum()) + 4096
    if pattern == "random":
        arena = O.splitmix64_bytes(0x5EED + align_log2, size)
    else:
        arena = np.full(size, 0xFF if pattern == "ff" else 0, dtype=np.uint8)
        # non-zero padding between packets must not count: scribble it
        for i in range(n):
            a, b = int(off[i]) + int(length[i]), int(off[i]) + int(pad[i])
            arena[a:b] = 0xA5
    seed = rng.integers(0, 0x10000, n).astype(np.uint16)
    blk_off = off[::64].copy()
    got = rows_model(arena, blk_off, length, seed)
    got_line = rows_model(arena, blk_off, length, seed, line=128)
    # the same packets 48 bytes into the arena (garbage before them): the first region's line
    # starts before its first packet too
    arena48 = np.concatenate((O.splitmix64_bytes(0x48, 48), arena))
    got_line48 = rows_model(arena48, blk_off + 48, length, seed, line=128)
    want = oracle.batch(arena, off, length.astype(np.uint32), seed, complement=True)
    # the oracle panics on empty slices (util.rs:92); the batch kernels return the seed
    empty = length == 0
    want[empty] = (seed[empty] ^ 0xFFFF).astype(np.uint16)
    assert np.array_equal(got, want), np.flatnonzero(got != want)[:5]
    assert np.array_equal(got_line, want), np.flatnonzero(got_line != want)[:5]
    assert np.array_equal(got_line48, want), np.flatnonzero(got_line48 != want)[:5]
