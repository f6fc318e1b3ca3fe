"""Transmit finalize on the GPU (rns_tx_fill_dev) against the reference's transmit
path restated in oracle.tx_fill_ref (tcp.rs:957-973, udp.rs:151-171, icmp.rs:87-112,
ip.rs:140-160): every byte of the arena after the fill, and the status per datagram."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from rustnetworkstack_amd import _lib
from rustnetworkstack_amd.batch import rx_verify, tx_fill
from rustnetworkstack_amd.workloads import DeviceBatch, make_layout
from test_rx_oracle import L4, L6, R4, R6, icmp4, ipv4, ipv6, tcp_seg

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dev(a, view):
    return torch.from_numpy(np.ascontiguousarray(a).view(view)).to(DEV)


def outgoing(n, seed):
    """Datagrams as the transmit path would hand them over (and some it never would):
    checksum fields holding garbage, every protocol, options, short segments."""
    w = O.splitmix64_words(seed, 4 * n)
    pkts = []
    for i in range(n):
        kind = int(w[4 * i] % np.uint64(12))
        size = int(w[4 * i + 1] % np.uint64(1400))
        body = O.splitmix64_bytes(int(w[4 * i + 2]), size).tobytes()
        if kind == 0:
            p = ipv4(6, tcp_seg(L4, R4, body))
        elif kind == 1:
            p = ipv6(6, tcp_seg(L6, R6, body))
        elif kind == 2:
            p = ipv4(17, tcp_seg(L4, R4, body, proto=17, field=6, hlen=8))
        elif kind == 3:
            p = ipv6(17, tcp_seg(L6, R6, body, proto=17, field=6, hlen=8))
        elif kind == 4:
            p = ipv4(1, icmp4(body))
        elif kind == 5:
            p = ipv6(58, tcp_seg(L6, R6, body, proto=58, field=2, hlen=4))
        elif kind == 6:
            p = ipv4(6, tcp_seg(L4, R4, body), ihl=6 + int(w[4 * i + 3] % np.uint64(10)))
        elif kind == 7:
            p = ipv4(int(w[4 * i + 3] % np.uint64(256)), body)             # any protocol
        elif kind == 8:
            p = ipv4(6, body[: int(w[4 * i + 3] % np.uint64(18))])          # segment too short for its field
        elif kind == 9:
            p = bytes([int(w[4 * i + 3] & np.uint64(0xFF))]) + body[:70]    # garbage / malformed
        elif kind == 10:
            p = ipv6(58, body[:3])
        else:
            p = ipv4(6, b"")
        p = bytearray(p)
        # garbage in the fields the fill computes (they count as zero)
        g = O.splitmix64_bytes(int(w[4 * i + 3]) ^ 0x55, 4).tobytes()
        if len(p) >= 12 and (p[0] >> 4) == 4:
            p[10:12] = g[:2]
        pkts.append(bytes(p))
    return pkts


def pack(pkts, seed, gaps=True):
    w = O.splitmix64_words(seed, len(pkts))
    off, pos = [], 0
    for i, p in enumerate(pkts):
        pos += int(w[i] % np.uint64(16)) if gaps else 0
        off.append(pos)
        pos += len(p)
    arena = O.splitmix64_bytes(seed ^ 0xABC, pos + 64)            # bytes between datagrams must survive
    for o, p in zip(off, pkts):
        arena[o:o + len(p)] = np.frombuffer(p, dtype=np.uint8)
    return arena, np.array(off, dtype=np.uint64), np.array([len(p) for p in pkts], dtype=np.uint32)


@pytest.mark.parametrize("gaps", [True, False])
def test_tx_fill_matches_reference_transmit_path(oracle, gaps):
    pkts = outgoing(12000, 0x7E57 + gaps)
    arena, off, ln = pack(pkts, 0x1234 + gaps, gaps)
    expect_arena = arena.copy()
    expect_st = np.zeros(len(pkts), dtype=np.uint8)
    for i, (o, p) in enumerate(zip(off, pkts)):
        q, st = O.tx_fill_ref(p, ones_comp=oracle.compute_ones_comp)
        expect_arena[int(o):int(o) + len(q)] = np.frombuffer(q, dtype=np.uint8)
        expect_st[i] = st
    assert len(set(expect_st.tolist())) >= 4
    a = torch.from_numpy(arena).to(DEV)
    st = tx_fill(a, dev(off, np.int64), dev(ln, np.int32))
    torch.cuda.synchronize()
    got_st = st.cpu().numpy()
    bad = np.nonzero(got_st != expect_st)[0]
    assert bad.size == 0, [(int(i), int(got_st[i]), int(expect_st[i]), pkts[i][:24].hex()) for i in bad[:5]]
    got = a.cpu().numpy()
    diff = np.nonzero(got != expect_arena)[0]
    assert diff.size == 0, [(int(d), int(got[d]), int(expect_arena[d])) for d in diff[:8]]


def test_tx_fill_then_receive_verify_accepts():
    """Datagrams sent from the remote end to this host: after the fill, the receive
    path (with L4/L6 as the local addresses) accepts every TCP and ICMP datagram."""
    pkts = []
    for k in range(3000):
        body = O.splitmix64_bytes(k, k % 1300).tobytes()
        p = [ipv4(6, tcp_seg(R4, L4, body)), ipv6(6, tcp_seg(R6, L6, body)), ipv4(1, icmp4(body)),
             ipv6(58, tcp_seg(R6, L6, body, proto=58, field=2, hlen=4))][k % 4]
        p = bytearray(p)
        h = 20 if (p[0] >> 4) == 4 else 40
        f = h + (16 if p[h - 40 + 6 if h == 40 else 9] == 6 else 2)
        p[f:f + 2] = b"\x12\x34"                         # wrong L4 checksum before the fill
        if h == 20:
            p[10:12] = b"\x00\x00"
        pkts.append(bytes(p))
    arena, off, ln = pack(pkts, 77)
    a = torch.from_numpy(arena).to(DEV)
    d_off, d_len = dev(off, np.int64), dev(ln, np.int32)
    assert int((rx_verify(a, d_off, d_len, L4, L6) & _lib.RNS_RX_ACCEPT).sum().item() // _lib.RNS_RX_ACCEPT) < len(pkts)
    st = tx_fill(a, d_off, d_len)
    assert int((st == (_lib.RNS_TX_L4_FILLED | _lib.RNS_TX_IP_FILLED)).sum().item()) == len(pkts) // 2
    rx = rx_verify(a, d_off, d_len, L4, L6)
    assert int((rx & _lib.RNS_RX_ACCEPT).ne(0).sum().item()) == len(pkts)


def test_jumbo_datagrams_past_the_u32_wrap(oracle):
    pkts = []
    for k, size in enumerate((131_072 - 60, 131_072 + 5, 200_001)):
        body = O.splitmix64_bytes(0xD0 + k, size).tobytes()
        seg6 = tcp_seg(L6, R6, body)
        pkts.append(bytes(bytearray([0x60, 0, 0, 0, 0, 0, 6, 64]) + L6 + R6) + seg6)
        pkts.append(bytes(bytearray([0x60, 0, 0, 0, 0, 0, 58, 64]) + L6 + R6) + tcp_seg(L6, R6, body, 58, 2, 4))
    arena, off, ln = pack(pkts, 99)
    expect = arena.copy()
    for o, p in zip(off, pkts):
        q, _ = O.tx_fill_ref(p, ones_comp=oracle.compute_ones_comp)
        expect[int(o):int(o) + len(q)] = np.frombuffer(q, dtype=np.uint8)
    a = torch.from_numpy(arena).to(DEV)
    tx_fill(a, dev(off, np.int64), dev(ln, np.int32))
    assert np.array_equal(a.cpu().numpy(), expect)


def test_full_size_batch_tx_then_rx():
    """2^20 x 1500 B IPv4/TCP datagrams (headers written on the GPU, checksum fields
    zero as alloc_header leaves them): one tx_fill, then every datagram is accepted."""
    lay = make_layout("c3_1500B")
    b = DeviceBatch(lay, DEV)
    n = lay.n
    hdr = np.frombuffer(bytes.fromhex("450005dc00004000400600000000000000000000"), dtype=np.uint8).copy()
    hdr[12:16] = np.frombuffer(R4, dtype=np.uint8)
    hdr[16:20] = np.frombuffer(L4, dtype=np.uint8)
    idx = b.off.view(-1, 1) + torch.arange(20, device=DEV)
    b.arena[idx.flatten()] = torch.from_numpy(hdr).to(DEV).repeat(n)
    st = tx_fill(b.arena, b.off, b.length)
    assert int((st != (_lib.RNS_TX_IP_FILLED | _lib.RNS_TX_L4_FILLED)).sum().item()) == 0
    rx = rx_verify(b.arena, b.off, b.length, L4, L6)
    want = _lib.RNS_RX_ACCEPT | _lib.RNS_RX_IP_OK | _lib.RNS_RX_L4_OK
    assert int((rx != want).sum().item()) == 0
    del b
    torch.cuda.empty_cache()
