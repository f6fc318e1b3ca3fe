"""Batched datagram I/O (rns_io_recv_batch / rns_io_send_batch) on a SOCK_SEQPACKET
socketpair — the same one-datagram-per-read semantics as the TUN fd the reference
uses (tun.c:84-90).  Host code only: runs without a GPU."""
import socket

import numpy as np

from oracle import oracle as O
from rustnetworkstack_amd.batch import recv_batch, send_batch


def make(n, seed, maxlen=2100):
    w = O.splitmix64_words(seed, n)
    lens = (w % np.uint64(maxlen) + np.uint64(1)).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(lens[:-1].astype(np.uint64), out=off[1:])
    arena = O.splitmix64_bytes(seed + 1, int(lens.sum()))
    return arena, off, lens


def test_roundtrip_and_oversize_dropped():
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 1 << 22)
    b.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 22)
    arena, off, lens = make(300, 5)
    assert send_batch(a.fileno(), arena, off, lens) == 300
    slots = np.zeros(2048 * 512, dtype=np.uint8)
    got_off, got_len = recv_batch(b.fileno(), slots, 2048, timeout_ms=1000)
    # a datagram longer than its 2048-byte slot (the MRU) is dropped, never handed on
    # truncated (recv(MSG_TRUNC) sees its full length); the others arrive in order
    keep = np.nonzero(lens <= 2048)[0]
    assert 0 < keep.shape[0] < 300
    assert got_off.shape[0] == keep.shape[0]
    assert np.array_equal(got_off, np.arange(keep.shape[0], dtype=np.uint64) * 2048)
    assert np.array_equal(got_len, lens[keep])
    for j, i in enumerate(keep):
        k = int(got_len[j])
        assert np.array_equal(slots[2048 * j:2048 * j + k], arena[int(off[i]):int(off[i]) + k])
    a.close()
    b.close()


def test_timeout_and_max_pkts():
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    slots = np.zeros(2048 * 8, dtype=np.uint8)
    o, ln = recv_batch(b.fileno(), slots, 2048, timeout_ms=10)     # nothing queued
    assert o.shape[0] == 0
    arena, off, lens = make(20, 9, maxlen=100)
    send_batch(a.fileno(), arena, off, lens)
    o, ln = recv_batch(b.fileno(), slots, 2048, max_pkts=8)         # capped by max_pkts
    assert o.shape[0] == 8 and np.array_equal(ln, lens[:8])
    o, ln = recv_batch(b.fileno(), slots, 2048)                     # the rest, slots reused
    assert o.shape[0] == 8 and np.array_equal(ln, lens[8:16])
    assert b.getblocking()                                          # fd flags restored
    a.close()
    b.close()
