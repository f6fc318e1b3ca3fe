"""The receive-path restatement (oracle.rx_status_ref) on hand-built datagrams:
valid IPv4/IPv6 TCP, ICMP, UDP packets are accepted; each corruption is caught by
the check the reference applies (ip.rs:76-87, tcp.rs:838-850, icmp.rs:46-75)."""
from oracle import oracle as O

L4 = bytes([192, 168, 1, 2])
L6 = bytes.fromhex("fe800000000000000000000000000002")
R4 = bytes([192, 168, 1, 1])
R6 = bytes.fromhex("fe800000000000000000000000000001")


def ipv4(proto, payload, frag=0, ihl=5):
    h = bytearray(ihl * 4)
    h[0] = 0x40 | ihl
    h[2:4] = (len(h) + len(payload)).to_bytes(2, "big")
    h[6:8] = frag.to_bytes(2, "big")
    h[8], h[9] = 64, proto
    h[12:16], h[16:20] = R4, L4
    h[10:12] = O.checksum_py(bytes(h)).to_bytes(2, "big")
    return bytes(h) + payload


def ipv6(proto, payload):
    h = bytearray(40)
    h[0] = 0x60
    h[4:6] = len(payload).to_bytes(2, "big")
    h[6], h[7] = proto, 64
    h[8:24], h[24:40] = R6, L6
    return bytes(h) + payload


def tcp_seg(src, dst, body=b"hello, world", proto=6, field=16, hlen=20):
    seg = bytearray(hlen) + bytearray(body)
    ph = O.pseudo_header_py(src, dst, len(seg), proto)
    c = O.ones_comp_py(ph, bytes(seg)) ^ 0xFFFF
    seg[field:field + 2] = c.to_bytes(2, "big")
    return bytes(seg)


def icmp4(body=b"ping" * 10):
    seg = bytearray([8, 0, 0, 0]) + bytearray(body)
    seg[2:4] = (O.ones_comp_py(0, bytes(seg)) ^ 0xFFFF).to_bytes(2, "big")
    return bytes(seg)


def test_valid_packets_accepted():
    acc = O.RX_ACCEPT | O.RX_IP_OK
    assert O.rx_status_ref(ipv4(6, tcp_seg(R4, L4)), L4, L6) == acc | O.RX_L4_OK
    assert O.rx_status_ref(ipv6(6, tcp_seg(R6, L6)), L4, L6) == acc | O.RX_L4_OK
    assert O.rx_status_ref(ipv4(1, icmp4()), L4, L6) == acc | O.RX_L4_OK
    assert O.rx_status_ref(ipv6(58, tcp_seg(R6, L6, proto=58, field=2, hlen=4)), L4, L6) == acc | O.RX_L4_OK
    assert O.rx_status_ref(ipv4(17, b"\x00" * 30), L4, L6) == acc | O.RX_L4_UNCHECKED


def test_corruptions_caught():
    good = ipv4(6, tcp_seg(R4, L4))
    bad_hdr = bytearray(good)
    bad_hdr[8] ^= 1                                        # TTL: IP header checksum fails
    assert O.rx_status_ref(bytes(bad_hdr), L4, L6) & O.RX_IP_OK == 0
    bad_l4 = bytearray(good)
    bad_l4[-1] ^= 0x40                                     # payload byte: TCP checksum fails
    st = O.rx_status_ref(bytes(bad_l4), L4, L6)
    assert st & O.RX_IP_OK and not st & O.RX_L4_OK and not st & O.RX_ACCEPT
    # the pseudo-header uses the LOCAL address, not the header's destination (tcp.rs:839-843)
    assert not O.rx_status_ref(ipv4(6, tcp_seg(R4, bytes([10, 0, 0, 9]))), L4, L6) & O.RX_L4_OK
    assert O.rx_status_ref(ipv4(6, tcp_seg(R4, L4), frag=0x2000), L4, L6) & O.RX_FRAGMENT
    assert O.rx_status_ref(ipv4(99, b"x" * 8), L4, L6) == O.RX_IP_OK | O.RX_UNKNOWN


def test_malformed():
    assert O.rx_status_ref(b"", L4, L6) == O.RX_MALFORMED
    assert O.rx_status_ref(bytes([0x50]) + b"\x00" * 40, L4, L6) == O.RX_MALFORMED      # version 5
    assert O.rx_status_ref(bytes([0x40]) + b"\x00" * 40, L4, L6) == O.RX_MALFORMED      # IHL 0
    assert O.rx_status_ref(bytes([0x4F]) + b"\x00" * 40, L4, L6) == O.RX_MALFORMED      # IHL*4 > len
    assert O.rx_status_ref(ipv6(6, b"")[:39], L4, L6) == O.RX_MALFORMED                 # short IPv6
    assert O.rx_status_ref(ipv4(58, b"x" * 8), L4, L6) == O.RX_MALFORMED               # V4 src, V6 pseudo-header
