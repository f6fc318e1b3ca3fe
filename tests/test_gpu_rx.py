"""Receive verify on the GPU (rns_rx_verify_dev) against the reference's receive
path restated in oracle.rx_status_ref (ip.rs:38-128, tcp.rs:838-850, icmp.rs:44-75)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from rustnetworkstack_amd import _lib
from rustnetworkstack_amd.batch import csum_fill, rx_verify
from rustnetworkstack_amd.workloads import DeviceBatch, make_layout
from test_rx_oracle import L4, L6, R4, R6, icmp4, ipv4, ipv6, tcp_seg

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def dev(a, view):
    return torch.from_numpy(np.ascontiguousarray(a).view(view)).to(DEV)


def make_packets(n, seed):
    """Valid and corrupted datagrams of every kind the receive path distinguishes."""
    w = O.splitmix64_words(seed, 4 * n)
    pkts = []
    for i in range(n):
        kind = int(w[4 * i] % np.uint64(10))
        size = int(w[4 * i + 1] % np.uint64(1400))
        body = O.splitmix64_bytes(int(w[4 * i + 2]), size).tobytes()
        if kind == 0:
            p = ipv4(6, tcp_seg(R4, L4, body))
        elif kind == 1:
            p = ipv6(6, tcp_seg(R6, L6, body))
        elif kind == 2:
            p = ipv4(1, icmp4(body))
        elif kind == 3:
            p = ipv6(58, tcp_seg(R6, L6, body, proto=58, field=2, hlen=4))
        elif kind == 4:
            p = ipv4(17, body + b"\x00" * 8)
        elif kind == 5:
            p = ipv4(6, tcp_seg(R4, L4, body), frag=int(w[4 * i + 3] & np.uint64(0x3FFF)) | 1)
        elif kind == 6:
            p = ipv4(6, tcp_seg(R4, L4, body), ihl=6 + int(w[4 * i + 3] % np.uint64(10)))
        elif kind == 7:
            p = bytes([int(w[4 * i + 3] & np.uint64(0xFF))]) + body[:int(w[4 * i + 3] >> np.uint64(8)) % 60]
        else:
            p = ipv4(6, tcp_seg(R4, L4, body)) if kind == 8 else ipv6(6, tcp_seg(R6, L6, body))
        p = bytearray(p)
        if kind >= 8 or (w[4 * i + 3] >> np.uint64(40)) % np.uint64(5) == 0:  # corrupt one byte somewhere
            if len(p):
                k = int(w[4 * i + 2] >> np.uint64(16)) % len(p)
                p[k] ^= 1 << int(w[4 * i + 2] & np.uint64(7))
        pkts.append(bytes(p))
    return pkts


def pack(pkts, shift_seed):
    w = O.splitmix64_words(shift_seed, len(pkts))
    off, pos = [], 0
    for i, p in enumerate(pkts):
        pos += int(w[i] % np.uint64(16))   # any start alignment
        off.append(pos)
        pos += len(p)
    arena = np.zeros(pos + 64, dtype=np.uint8)
    for o, p in zip(off, pkts):
        arena[o:o + len(p)] = np.frombuffer(p, dtype=np.uint8)
    return arena, np.array(off, dtype=np.uint64), np.array([len(p) for p in pkts], dtype=np.uint32)


def test_mixed_datagrams_match_reference_path(oracle):
    pkts = make_packets(20000, 0xF00D)
    arena, off, ln = pack(pkts, 0xBEEF)
    expect = np.array([O.rx_status_ref(p, L4, L6, ones_comp=oracle.compute_ones_comp) for p in pkts], dtype=np.uint8)
    assert len(set(expect.tolist())) >= 6          # every kind of verdict is exercised
    l4 = torch.empty(len(pkts), dtype=torch.uint16, device=DEV)
    st = rx_verify(torch.from_numpy(arena).to(DEV), dev(off, np.int64), dev(ln, np.int32), L4, L6, l4_sum=l4)
    torch.cuda.synchronize()
    got = st.cpu().numpy()
    bad = np.nonzero(got != expect)[0]
    assert bad.size == 0, [(int(i), int(got[i]), int(expect[i]), pkts[i][:24].hex()) for i in bad[:5]]
    want_l4 = np.array([O.rx_verify_ref(p, L4, L6, ones_comp=oracle.compute_ones_comp)[1] for p in pkts],
                       dtype=np.uint16)
    got_l4 = l4.view(torch.int16).cpu().numpy().view(np.uint16)
    bad = np.nonzero(got_l4 != want_l4)[0]
    assert bad.size == 0, [(int(i), int(got_l4[i]), int(want_l4[i])) for i in bad[:5]]


def jumbo_v4(proto, seg):
    """IPv4 datagram longer than 64 KiB (the total-length field wraps; the stack uses
    the buffer length, ip.rs:94-96)."""
    h = bytearray(20)
    h[0] = 0x45
    h[2:4] = ((20 + len(seg)) & 0xFFFF).to_bytes(2, "big")
    h[8], h[9] = 64, proto
    h[12:16], h[16:20] = R4, L4
    h[10:12] = O.checksum_py(bytes(h)).to_bytes(2, "big")
    return bytes(h) + seg


def test_edge_datagrams_match_reference_path(oracle):
    """Datagrams the split header/L4 pass must get right: L4 segments past the
    128 KiB no-wrap bound (exact big-endian path, the IP header still split off),
    headers with options whose end falls anywhere in a 16-byte chunk, empty L4
    segments, header-only UDP, and 0xff-filled bodies (maximal sums)."""
    pkts = []
    for k, size in enumerate((131_072 - 20, 131_072 + 7, 200_001, 262_144 + 3)):
        body = O.splitmix64_bytes(0xB16 + k, size).tobytes()
        seg = bytearray(tcp_seg(R4, L4, body))
        pkts.append(jumbo_v4(6, bytes(seg)))
        seg6 = tcp_seg(R6, L6, body)
        pkts.append(ipv6(6, seg6) if len(seg6) < 65536 else
                    bytes(bytearray([0x60, 0, 0, 0, 0, 0, 6, 64]) + R6 + L6) + seg6)
        bad = bytearray(pkts[-2])
        bad[len(bad) // 2] ^= 0x80
        pkts.append(bytes(bad))
    ff = b"\xff" * 70_000
    pkts.append(jumbo_v4(1, icmp4(ff)))
    for ihl in range(5, 16):
        for size in (0, 1, 2, 3, 17, 31, 64):
            pkts.append(ipv4(6, tcp_seg(R4, L4, b"\xa5" * size), ihl=ihl))
        pkts.append(ipv4(6, b"", ihl=ihl))                 # empty TCP segment: L4 sum = seed
        pkts.append(ipv4(17, b"", ihl=ihl))                # header-only UDP
        pkts.append(ipv4(1, b"\x00", ihl=ihl))             # 1-byte ICMP
    pkts.append(ipv6(6, b""))
    pkts.append(ipv6(58, b"\x01"))
    expect = [O.rx_verify_ref(p, L4, L6, ones_comp=oracle.compute_ones_comp) for p in pkts]
    for shift in (0, 1, 0x11):
        arena, off, ln = pack(pkts, 0x5A17 + shift)
        off = off + shift
        arena = np.concatenate([np.zeros(shift, dtype=np.uint8), arena])
        l4 = torch.empty(len(pkts), dtype=torch.uint16, device=DEV)
        st = rx_verify(torch.from_numpy(arena).to(DEV), dev(off, np.int64), dev(ln, np.int32), L4, L6, l4_sum=l4)
        got = list(zip(st.cpu().numpy().tolist(), l4.view(torch.int16).cpu().numpy().view(np.uint16).tolist()))
        bad = [(i, len(pkts[i]), got[i], expect[i]) for i in range(len(pkts)) if got[i] != tuple(expect[i])]
        assert not bad, bad[:5]


def test_full_size_tcp_batch_verifies_and_catches_corruption():
    """1M x 1500 B IPv4/TCP datagrams built on the GPU: IPv4 header + TCP checksum
    filled by rns_csum_fill_dev, then every packet is accepted; corrupting chosen
    packets flips exactly their verdicts."""
    lay = make_layout("c3_1500B")
    b = DeviceBatch(lay, DEV)
    n = lay.n
    hdr = np.frombuffer(bytes.fromhex("450005dc00004000400600000000000000000000"), dtype=np.uint8).copy()
    hdr[12:16] = np.frombuffer(R4, dtype=np.uint8)
    hdr[16:20] = np.frombuffer(L4, dtype=np.uint8)
    idx = b.off.view(-1, 1) + torch.arange(20, device=DEV)
    b.arena[idx.flatten()] = torch.from_numpy(hdr).to(DEV).repeat(n)
    ip_len = torch.full((n,), 20, dtype=torch.int32, device=DEV)
    csum_fill(b.arena, b.off, ip_len, None, field_off=10)                   # ip.rs:158-159
    seg_off = b.off + 20
    seg_len = b.length - 20
    ph = O.pseudo_header_py(R4, L4, 1480, 6)
    seeds = torch.full((n,), ph if ph < 0x8000 else ph - 0x10000, dtype=torch.int16, device=DEV)
    csum_fill(b.arena, seg_off, seg_len, seeds, field_off=16)               # tcp.rs:957-973
    st = rx_verify(b.arena, b.off, b.length, L4, L6)
    want = _lib.RNS_RX_ACCEPT | _lib.RNS_RX_IP_OK | _lib.RNS_RX_L4_OK
    assert int((st != want).sum().item()) == 0
    # corrupt: payload bytes of packets 7, 1000, ...; the TTL of others
    pay = torch.arange(7, n, 997, device=DEV)
    ttl = torch.arange(11, n, 1009, device=DEV)
    b.arena[b.off[pay] + 700] ^= 0x10
    b.arena[b.off[ttl] + 8] ^= 0x01
    st = rx_verify(b.arena, b.off, b.length, L4, L6).cpu().numpy()
    exp = np.full(n, want, dtype=np.uint8)
    exp[pay.cpu().numpy()] = _lib.RNS_RX_IP_OK
    exp[ttl.cpu().numpy()] &= ~np.uint8(_lib.RNS_RX_IP_OK | _lib.RNS_RX_ACCEPT)
    assert np.array_equal(st, exp)
    del b
    torch.cuda.empty_cache()


def test_tiny_datagrams_capped_grid_every_status():
    """ACK-sized datagrams (arena bytes per datagram <= 128) run on a capped grid whose
    waves loop over several 64-datagram batches: every status must still be exact —
    accepted, or (the planted corruptions, one TCP byte flipped) IP-only."""
    from rustnetworkstack_amd.workloads import LOCAL4, LOCAL6, corrupt_mask, make_verify_batch
    n = 4096 * 64 * 2 + 123            # > 2 batches per wave of the 4096-wave cap, ragged tail
    lay = make_layout("d40B", n=n)
    b = DeviceBatch(lay, DEV)
    make_verify_batch(b)
    assert lay.arena_bytes // n <= 128
    st = rx_verify(b.arena, b.off, b.length, LOCAL4, LOCAL6).cpu().numpy()
    want = np.full(n, _lib.RNS_RX_ACCEPT | _lib.RNS_RX_IP_OK | _lib.RNS_RX_L4_OK, dtype=np.uint8)
    want[corrupt_mask(n)] = _lib.RNS_RX_IP_OK
    assert np.array_equal(st, want)


# --- packed receive arenas (rns_rx_verify_packed_dev: the rows receive kernel) ---------
def run_packed_rx(pkts, align_log2, first_off, base_shift=0):
    from rustnetworkstack_amd.batch import packed_layout, rx_verify_packed
    ln = np.array([len(p) for p in pkts], dtype=np.uint32)
    blk, poff, end = packed_layout(ln, align_log2, first_off)
    arena = np.full(end + 16 + base_shift, 0xA5, dtype=np.uint8)   # padding never counts
    for o, p in zip(poff.tolist(), pkts):
        arena[base_shift + o:base_shift + o + len(p)] = np.frombuffer(p, dtype=np.uint8)
    big = torch.from_numpy(arena).to(DEV)
    l4 = torch.empty(len(pkts), dtype=torch.uint16, device=DEV)
    st = rx_verify_packed(big[base_shift:], dev(blk.astype(np.uint64), np.int64), dev(ln.astype(np.uint16), np.int16),
                          L4, L6, align_log2=align_log2, l4_sum=l4)
    return st.cpu().numpy(), l4.view(torch.int16).cpu().numpy().view(np.uint16)


@pytest.mark.parametrize("align_log2,first_off,base_shift", [(4, 0, 0), (4, 32, 0), (11, 0, 0), (4, 5, 0), (4, 0, 3)])
def test_packed_mixed_datagrams_match_reference_path(oracle, align_log2, first_off, base_shift):
    """Every kind of datagram (valid, corrupted, fragments, options, UDP, ICMP, garbage)
    packed at 16 bytes and in 2048-byte slots; an unaligned first offset and an unaligned
    arena base take the kernel's per-datagram path.  Status and L4 sum per datagram
    against the reference's receive path."""
    pkts = make_packets(6000, 0xF00D + align_log2 + first_off)
    expect = [O.rx_verify_ref(p, L4, L6, ones_comp=oracle.compute_ones_comp) for p in pkts]
    st, l4 = run_packed_rx(pkts, align_log2, first_off, base_shift)
    got = list(zip(st.tolist(), l4.tolist()))
    bad = [(i, len(pkts[i]), got[i], expect[i]) for i in range(len(pkts)) if got[i] != tuple(expect[i])]
    assert not bad, bad[:5]


def test_packed_edge_datagrams_match_reference_path(oracle):
    """Header-length edges (IHL 5..15 with short and empty segments), header-only UDP,
    one-byte ICMP, IPv6 with empty segments and 0xff bodies up to 65535 bytes."""
    pkts = []
    for ihl in range(5, 16):
        for size in (0, 1, 2, 3, 17, 31, 64, 65):
            pkts.append(ipv4(6, tcp_seg(R4, L4, b"\xa5" * size), ihl=ihl))
        pkts.append(ipv4(6, b"", ihl=ihl))
        pkts.append(ipv4(17, b"", ihl=ihl))
        pkts.append(ipv4(1, b"\x00", ihl=ihl))
    pkts += [ipv6(6, b""), ipv6(58, b"\x01"), ipv4(1, icmp4(b"\xff" * 65000)), ipv6(6, tcp_seg(R6, L6, b"\xff" * 65400))]
    pkts += [b"", b"\x45", b"\x60" * 39]
    expect = [O.rx_verify_ref(p, L4, L6, ones_comp=oracle.compute_ones_comp) for p in pkts]
    for first_off in (0, 16, 7):
        st, l4 = run_packed_rx(pkts, 4, first_off)
        got = list(zip(st.tolist(), l4.tolist()))
        bad = [(i, len(pkts[i]), got[i], expect[i]) for i in range(len(pkts)) if got[i] != tuple(expect[i])]
        assert not bad, (first_off, bad[:5])


def test_packed_ack_arena_with_longer_datagrams(oracle):
    """An arena of ACK-sized datagrams (at most 128 arena bytes per datagram: the receive
    kernel's instantiation without the rows) in which a few units hold longer datagrams
    (every 37th unit one of 1400 B, one of 65): those units take the per-datagram wave loop;
    every status and L4 sum against the reference's receive path."""
    n = 64 * 300
    w = O.splitmix64_words(0xAC4, n)
    pkts = []
    for i in range(n):
        size = int(w[i] % np.uint64(25))
        p = bytearray(ipv4(6, tcp_seg(R4, L4, bytes([i & 0xFF]) * size)))
        if (i // 64) % 37 == 3 and i % 64 == 17:
            p = bytearray(ipv4(6, tcp_seg(R4, L4, O.splitmix64_bytes(i, 1360).tobytes())))
        if (i // 64) % 37 == 5 and i % 64 == 40:
            p = bytearray(ipv6(58, tcp_seg(R6, L6, b"\x11" * 21, proto=58, field=2, hlen=4)))
        if (w[i] >> np.uint64(32)) % np.uint64(11) == 0:
            p[int(w[i] >> np.uint64(8)) % len(p)] ^= 0x10
        pkts.append(bytes(p))
    ln = np.array([len(p) for p in pkts])
    assert ((ln + 15) // 16 * 16).sum() // n <= 128 and ln.max() > 64
    expect = [O.rx_verify_ref(p, L4, L6, ones_comp=oracle.compute_ones_comp) for p in pkts]
    st, l4 = run_packed_rx(pkts, 4, 0)
    got = list(zip(st.tolist(), l4.tolist()))
    bad = [(i, len(pkts[i]), got[i], expect[i]) for i in range(len(pkts)) if got[i] != tuple(expect[i])]
    assert not bad, bad[:5]


@pytest.mark.parametrize("name", ["c2_64B", "c5_imix"])
def test_packed_full_size_equals_descriptor_entry(name):
    """bench.py --op verify's batches (headers and checksums written on the device, every
    1009th datagram corrupted): the packed entry's statuses equal rns_rx_verify_dev's, and
    exactly the planted corruptions are rejected."""
    from rustnetworkstack_amd.batch import rx_verify_packed
    from rustnetworkstack_amd.workloads import LOCAL4, LOCAL6, make_verify_batch
    lay = make_layout(name)
    b = DeviceBatch(lay, DEV)
    make_verify_batch(b)
    b.launcher(packed=True)  # uploads blk_off / len16
    ref = rx_verify(b.arena, b.off, b.length, LOCAL4, LOCAL6).clone()
    got = rx_verify_packed(b.arena, b.blk_off, b.len16, LOCAL4, LOCAL6)
    assert torch.equal(got, ref)
    assert int(((got & _lib.RNS_RX_ACCEPT) == 0).sum().item()) == b.expected_bad
    del b
    torch.cuda.empty_cache()


def test_output_buffers_are_checked():
    """The kernels write one status (and L4 sum) per datagram: an undersized or wrongly typed
    output buffer, or descriptors on another device, is refused before any launch."""
    from rustnetworkstack_amd.batch import rx_verify_packed
    arena = torch.zeros(4096, dtype=torch.uint8, device=DEV)
    off = torch.arange(0, 4096, 64, dtype=torch.int64, device=DEV)
    ln = torch.full((64,), 64, dtype=torch.int32, device=DEV)
    with pytest.raises(ValueError):
        rx_verify(arena, off, ln, L4, L6, status=torch.empty(63, dtype=torch.uint8, device=DEV))
    with pytest.raises(ValueError):
        rx_verify(arena, off, ln, L4, L6, l4_sum=torch.empty(10, dtype=torch.int16, device=DEV))
    with pytest.raises(TypeError):
        rx_verify(arena, off, ln, L4, L6, status=torch.empty(64, dtype=torch.int16, device=DEV))
    blk = torch.zeros(1, dtype=torch.int64, device=DEV)
    len16 = torch.full((64,), 64, dtype=torch.int16, device=DEV)
    with pytest.raises(ValueError):
        rx_verify_packed(arena, blk, len16, L4, L6, status=torch.empty(1, dtype=torch.uint8, device=DEV))
    with pytest.raises(ValueError):
        rx_verify_packed(arena, blk, len16, L4, L6, l4_sum=torch.empty(63, dtype=torch.uint16, device=DEV))
    st = rx_verify_packed(arena, blk, len16, L4, L6, status=torch.empty(64, dtype=torch.uint8, device=DEV))
    assert st.numel() == 64


# --- receive rings of fixed-size slots (rns_rx_verify_strided_dev) -------------------------
def run_strided_rx(pkts, stride, first_off, base_shift=0):
    from rustnetworkstack_amd.batch import rx_verify_strided
    n = len(pkts)
    ln = np.array([len(p) for p in pkts], dtype=np.uint16)
    arena = np.full(first_off + n * stride + 64 + base_shift, 0xA5, dtype=np.uint8)  # slot tails never count
    for i, p in enumerate(pkts):
        o = base_shift + first_off + i * stride
        arena[o:o + len(p)] = np.frombuffer(p, dtype=np.uint8)
    big = torch.from_numpy(arena).to(DEV)
    l4 = torch.empty(n, dtype=torch.uint16, device=DEV)
    st = rx_verify_strided(big[base_shift:], stride, dev(ln, np.int16), L4, L6, first_off=first_off, l4_sum=l4)
    return st.cpu().numpy(), l4.view(torch.int16).cpu().numpy().view(np.uint16)


@pytest.mark.parametrize("stride,first_off,base_shift", [(2048, 0, 0), (2048, 48, 0), (2051, 0, 0), (2048, 5, 0),
                                                         (2048, 0, 7), (1504, 16, 0)])
def test_strided_mixed_datagrams_match_reference_path(oracle, stride, first_off, base_shift):
    """Every kind of datagram in MRU-sized receive slots (netif.rs:66): 16-byte-aligned slots
    (ACK-sized datagrams from the owners' loads, longer ones summed by the wave), and
    unaligned strides, first offsets and arena bases (every datagram through the wave loop,
    header chunks from the boundary below).  Status and L4 sum against the reference."""
    pkts = make_packets(5000, 0x57D + stride + first_off + base_shift)
    expect = [O.rx_verify_ref(p, L4, L6, ones_comp=oracle.compute_ones_comp) for p in pkts]
    st, l4 = run_strided_rx(pkts, stride, first_off, base_shift)
    got = list(zip(st.tolist(), l4.tolist()))
    bad = [(i, len(pkts[i]), got[i], expect[i]) for i in range(len(pkts)) if got[i] != tuple(expect[i])]
    assert not bad, bad[:5]


@pytest.mark.parametrize("stride", [64, 80, 128])
def test_strided_ack_slots_edge_datagrams(oracle, stride):
    """ACK-sized slots: every IHL with short and empty segments, header-only UDP, one-byte
    ICMP, short IPv6, garbage and empty datagrams; each slot's bytes past its datagram hold
    0xA5 (never counted).  Datagrams longer than the slot overlap the next slot (read only)."""
    pkts = []
    for ihl in range(5, 16):
        for size in (0, 1, 2, 3, 17, 31):
            p = ipv4(6, tcp_seg(R4, L4, b"\x5a" * size), ihl=ihl)
            pkts.append(p[:stride])
        pkts.append(ipv4(6, b"", ihl=ihl))
        pkts.append(ipv4(17, b"", ihl=ihl))
        pkts.append(ipv4(1, b"\x00", ihl=ihl))
    pkts += [ipv6(6, b""), ipv6(58, b"\x01"), ipv6(6, tcp_seg(R6, L6, b"\xff" * 4)), b"", b"\x45", b"\x60" * 39]
    pkts += [ipv4(1, icmp4(b"\xff" * (stride - 28)))] * 70
    bad_l4 = bytearray(ipv4(6, tcp_seg(R4, L4, b"ack!")))
    bad_l4[-1] ^= 4
    pkts += [bytes(bad_l4)] * 65
    expect = [O.rx_verify_ref(p, L4, L6, ones_comp=oracle.compute_ones_comp) for p in pkts]
    st, l4 = run_strided_rx(pkts, stride, 0)
    got = list(zip(st.tolist(), l4.tolist()))
    bad = [(i, len(pkts[i]), got[i], expect[i]) for i in range(len(pkts)) if got[i] != tuple(expect[i])]
    assert not bad, bad[:5]


def test_strided_full_size_64B_equals_packed_entry():
    """bench.py --op verify's c2 batch (2^20 x 64 B IPv4/TCP, every 1009th corrupted) read as
    64-byte slots: the strided entry's statuses and L4 sums equal the packed entry's, and
    exactly the planted corruptions are rejected."""
    from rustnetworkstack_amd.batch import rx_verify_packed, rx_verify_strided
    from rustnetworkstack_amd.workloads import LOCAL4, LOCAL6, make_verify_batch
    lay = make_layout("c2_64B")
    b = DeviceBatch(lay, DEV)
    make_verify_batch(b)
    b.launcher(packed=True)
    assert np.all(lay.off == np.arange(lay.n, dtype=np.uint64) * np.uint64(64))
    l4a = torch.empty(lay.n, dtype=torch.uint16, device=DEV)
    l4b = torch.empty(lay.n, dtype=torch.uint16, device=DEV)
    ref = rx_verify_packed(b.arena, b.blk_off, b.len16, LOCAL4, LOCAL6, l4_sum=l4a).clone()
    got = rx_verify_strided(b.arena, 64, b.len16, LOCAL4, LOCAL6, l4_sum=l4b)
    assert torch.equal(got, ref) and torch.equal(l4a, l4b)
    assert int(((got & _lib.RNS_RX_ACCEPT) == 0).sum().item()) == b.expected_bad
    del b
    torch.cuda.empty_cache()
