"""Transmit finalize of a PACKED arena on the GPU (rns_tx_fill_packed_dev: the rows transmit
kernel) against the reference's transmit path restated in oracle.tx_fill_ref (tcp.rs:957-973,
udp.rs:151-171, icmp.rs:87-112, ip.rs:140-160): every byte of the arena after the fill (the
padding between datagrams must survive), and the status per datagram."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from rustnetworkstack_amd import _lib
from rustnetworkstack_amd.batch import packed_layout, rx_verify_packed, tx_fill, tx_fill_packed
from rustnetworkstack_amd.workloads import DeviceBatch, make_layout
from test_gpu_tx import outgoing
from test_rx_oracle import L4, L6, R4, R6, icmp4, ipv4, ipv6, tcp_seg

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dev(a, view):
    return torch.from_numpy(np.ascontiguousarray(a).view(view)).to(DEV)


def run_packed_tx(oracle, pkts, align_log2=4, first_off=0, base_shift=0, len_hint=0):
    """Pack, run the packed finalize, and return (got arena, want arena, got status, want status)."""
    ln = np.array([len(p) for p in pkts], dtype=np.uint32)
    blk, poff, end = packed_layout(ln, align_log2, first_off)
    arena = O.splitmix64_bytes(0xA5A5 + align_log2 + first_off, end + 48 + base_shift)  # padding: any bytes
    want = arena.copy()
    want_st = np.zeros(len(pkts), dtype=np.uint8)
    for i, (o, p) in enumerate(zip(poff.tolist(), pkts)):
        arena[base_shift + o:base_shift + o + len(p)] = np.frombuffer(p, dtype=np.uint8)
        q, s = O.tx_fill_ref(p, ones_comp=oracle.compute_ones_comp)
        want[base_shift + o:base_shift + o + len(q)] = np.frombuffer(q, dtype=np.uint8)
        want_st[i] = s
    big = torch.from_numpy(arena).to(DEV)
    st = tx_fill_packed(big[base_shift:], dev(blk.astype(np.uint64), np.int64), dev(ln.astype(np.uint16), np.int16),
                        align_log2=align_log2, len_hint=len_hint)
    torch.cuda.synchronize()
    return big.cpu().numpy(), want, st.cpu().numpy(), want_st


def assert_same(got, want, got_st, want_st, pkts):
    bad = np.flatnonzero(got_st != want_st)
    assert bad.size == 0, [(int(i), int(got_st[i]), int(want_st[i]), pkts[i][:24].hex()) for i in bad[:5]]
    diff = np.flatnonzero(got != want)
    assert diff.size == 0, [(int(d), int(got[d]), int(want[d])) for d in diff[:8]]


@pytest.mark.parametrize("align_log2,first_off,base_shift,len_hint", [
    (4, 0, 0, 0), (4, 32, 0, 1500), (11, 0, 0, 0), (4, 5, 0, 0), (4, 0, 3, 0), (4, 0, 0, 9000)])
def test_packed_tx_matches_reference_transmit_path(oracle, align_log2, first_off, base_shift, len_hint):
    """Every kind of outgoing datagram (TCP / UDP / ICMP over IPv4 and IPv6, IPv4 options,
    any protocol, segments too short for their field, garbage, empty) with garbage in the
    fields, packed at 16 bytes and in 2048-byte slots; an unaligned first offset and an
    unaligned arena base take the per-datagram path; D = 8 and D = 16 rows."""
    pkts = outgoing(6000, 0x7E58 + align_log2 + first_off + base_shift)
    got, want, got_st, want_st = run_packed_tx(oracle, pkts, align_log2, first_off, base_shift, len_hint)
    assert len(set(want_st.tolist())) >= 4
    assert_same(got, want, got_st, want_st, pkts)


def edge_datagrams():
    pkts = []
    for ihl in range(5, 16):
        for size in (0, 1, 2, 3, 4, 5, 6, 7, 8, 17, 18, 19, 20, 31, 44, 45, 60, 64, 65, 100):
            body = O.splitmix64_bytes(ihl * 1000 + size, size).tobytes()
            pkts.append(ipv4(6, body, ihl=ihl))                       # TCP field at hdr+16 if it fits
            pkts.append(ipv4(17, body, ihl=ihl))                      # UDP at hdr+6
            pkts.append(ipv4(1, body, ihl=ihl))                       # ICMP at hdr+2
    for size in (0, 1, 3, 4, 7, 8, 17, 18, 19, 24, 25, 40, 100, 1000):
        body = O.splitmix64_bytes(size, size).tobytes()
        for proto in (6, 17, 58, 1, 99):
            pkts.append(ipv6(proto, body))
    # maximal sums and the largest packed datagrams
    pkts.append(ipv4(6, b"\xff" * (65535 - 20)))
    pkts.append(ipv6(58, b"\xff" * (65535 - 40)))
    pkts.append(ipv6(6, b"\x00" * 65000))
    pkts += [b"", b"\x45", b"\x45" + b"\x00" * 18, b"\x60" * 39, b"\x4f" * 59, b"\x70" * 80]
    return pkts


@pytest.mark.parametrize("first_off", [0, 16, 7])
def test_packed_tx_edge_datagrams(oracle, first_off):
    """Header-length edges (IHL 5..15) against every field position and segment length
    around it, IPv6 with short segments for each protocol, 65535-byte datagrams with 0xff
    bodies, malformed and empty datagrams."""
    pkts = edge_datagrams()
    got, want, got_st, want_st = run_packed_tx(oracle, pkts, 4, first_off)
    assert_same(got, want, got_st, want_st, pkts)


def test_packed_tx_ack_units_and_mixed_units(oracle):
    """Units of ACK-sized datagrams only (the owners load their datagrams whole) next to
    units where one datagram is longer (the rows), shuffled through one batch."""
    n = 64 * 200
    w = O.splitmix64_words(0xACC, n)
    pkts = []
    for i in range(n):
        size = int(w[i] % np.uint64(25))
        body = bytes([i & 0xFF]) * size
        kind = int(w[i] >> np.uint64(40)) % 4
        p = [ipv4(6, tcp_seg(L4, R4, body)), ipv4(17, body + b"\x00" * 8), ipv4(1, icmp4(body[:20])),
             ipv6(17, body[:16] + b"\x00" * 8)][kind]
        if (i // 64) % 5 == 2 and i % 64 == 33:
            p = ipv4(6, tcp_seg(L4, R4, O.splitmix64_bytes(i, 1400).tobytes()))
        pkts.append(p)
    got, want, got_st, want_st = run_packed_tx(oracle, pkts)
    assert_same(got, want, got_st, want_st, pkts)


def test_packed_tx_equals_explicit_entry_and_round_trips():
    """Datagrams sent to this host (R -> L): the packed finalize stores exactly what
    rns_tx_fill_dev stores, and the receive path then accepts every TCP and ICMP datagram."""
    pkts = []
    for k in range(4000):
        body = O.splitmix64_bytes(k, k % 1450).tobytes()
        p = bytearray([ipv4(6, tcp_seg(R4, L4, body)), ipv6(6, tcp_seg(R6, L6, body)), ipv4(1, icmp4(body)),
                       ipv6(58, tcp_seg(R6, L6, body, proto=58, field=2, hlen=4))][k % 4])
        h = 20 if (p[0] >> 4) == 4 else 40
        f = h + (16 if p[6 if h == 40 else 9] == 6 else 2)
        p[f:f + 2] = b"\x12\x34"
        if h == 20:
            p[10:12] = b"\xab\xcd"
        pkts.append(bytes(p))
    ln = np.array([len(p) for p in pkts], dtype=np.uint32)
    blk, poff, end = packed_layout(ln, 4, 0)
    arena = np.zeros(end + 16, dtype=np.uint8)
    for o, p in zip(poff.tolist(), pkts):
        arena[o:o + len(p)] = np.frombuffer(p, dtype=np.uint8)
    a1 = torch.from_numpy(arena).to(DEV)
    a2 = a1.clone()
    d_blk, d_len16 = dev(blk.astype(np.uint64), np.int64), dev(ln.astype(np.uint16), np.int16)
    st1 = tx_fill_packed(a1, d_blk, d_len16)
    st2 = tx_fill(a2, dev(poff.astype(np.uint64), np.int64), dev(ln, np.int32))
    assert torch.equal(st1, st2) and torch.equal(a1, a2)
    rx = rx_verify_packed(a1, d_blk, d_len16, L4, L6)
    assert int((rx & _lib.RNS_RX_ACCEPT).ne(0).sum().item()) == len(pkts)


@pytest.mark.parametrize("name", ["c3_1500B", "c5_imix"])
def test_packed_tx_full_size_then_receive(name):
    """The bench batches (c3: 2^20 x 1500 B; c5: 2^23 IMIX) as IPv4/TCP datagrams from R to L
    with the checksum fields zero (as alloc_header leaves them): one packed finalize, every
    status is IP + L4 filled, and the packed receive verify then accepts every datagram."""
    lay = make_layout(name)
    b = DeviceBatch(lay, DEV)
    n = lay.n
    hdr = np.frombuffer(bytes.fromhex("4500000000004000400600000000000000000000"), dtype=np.uint8).copy()
    hdr[12:16] = np.frombuffer(R4, dtype=np.uint8)
    hdr[16:20] = np.frombuffer(L4, dtype=np.uint8)
    idx = b.off.view(-1, 1) + torch.arange(20, device=DEV)
    b.arena[idx.flatten()] = torch.from_numpy(hdr).to(DEV).repeat(n)
    del idx
    b.launcher(packed=True)  # uploads blk_off / len16
    st = tx_fill_packed(b.arena, b.blk_off, b.len16, len_hint=int(round(lay.mean_len)))
    assert int((st != (_lib.RNS_TX_IP_FILLED | _lib.RNS_TX_L4_FILLED)).sum().item()) == 0
    rx = rx_verify_packed(b.arena, b.blk_off, b.len16, L4, L6)
    want = _lib.RNS_RX_ACCEPT | _lib.RNS_RX_IP_OK | _lib.RNS_RX_L4_OK
    assert int((rx != want).sum().item()) == 0
    del b
    torch.cuda.empty_cache()


def test_packed_tx_argument_checks():
    arena = torch.zeros(4096, dtype=torch.uint8, device=DEV)
    blk = torch.zeros(1, dtype=torch.int64, device=DEV)
    len16 = torch.full((64,), 40, dtype=torch.int16, device=DEV)
    with pytest.raises(ValueError):
        tx_fill_packed(arena, blk, len16, align_log2=3)
    with pytest.raises(ValueError):
        tx_fill_packed(arena, blk, len16, status=torch.empty(63, dtype=torch.uint8, device=DEV))
    with pytest.raises(ValueError):
        tx_fill_packed(arena, torch.zeros(0, dtype=torch.int64, device=DEV), len16)
    st = tx_fill_packed(arena, blk, len16)  # all-zero datagrams: version 0, malformed, untouched
    assert int((st != _lib.RNS_TX_MALFORMED).sum().item()) == 0
    assert int(arena.sum().item()) == 0
