"""The transmit-path restatement (oracle.tx_fill_ref) on hand-built datagrams: what
tcp_output / udp_output / icmp_output_v4 / icmp_output_v6 / ip_output_v4 store
(tcp.rs:957-973, udp.rs:151-171, icmp.rs:87-112, ip.rs:140-160)."""
from oracle import oracle as O
from test_rx_oracle import L4, L6, R4, R6, icmp4, ipv4, ipv6, tcp_seg


def zero(p, *fields):
    q = bytearray(p)
    for f in fields:
        q[f:f + 2] = b"\x00\x00"
    return bytes(q)


def test_fill_reproduces_correct_checksums():
    # the builders in test_rx_oracle compute the same fields with the pinned util.rs restatement
    cases = [
        (ipv4(6, tcp_seg(L4, R4, b"abc")), (10, 36), O.TX_IP_FILLED | O.TX_L4_FILLED),
        (ipv4(17, tcp_seg(L4, R4, b"datagram", proto=17, field=6, hlen=8)), (10, 26), O.TX_IP_FILLED | O.TX_L4_FILLED),
        (ipv4(1, icmp4()), (10, 22), O.TX_IP_FILLED | O.TX_L4_FILLED),
        (ipv6(6, tcp_seg(L6, R6, b"xyz" * 7)), (56,), O.TX_L4_FILLED),
        (ipv6(58, tcp_seg(L6, R6, b"echo", proto=58, field=2, hlen=4)), (42,), O.TX_L4_FILLED),
    ]
    for pkt, fields, status in cases:
        out, st = O.tx_fill_ref(zero(pkt, *fields))
        assert (out, st) == (pkt, status)
        # garbage in the fields counts as zero (alloc_header zero-fills them, buf.rs:286-288)
        junk = bytearray(pkt)
        for f in fields:
            junk[f:f + 2] = b"\xde\xad"
        assert O.tx_fill_ref(bytes(junk)) == (pkt, status)


def sent_by_local(pkt):
    """The builders address datagrams R -> L; swap to L -> R (what this host sends)."""
    q = bytearray(pkt)
    if q[0] >> 4 == 4:
        q[12:16], q[16:20] = q[16:20], q[12:16]
    else:
        q[8:24], q[24:40] = q[24:40], q[8:24]
    return bytes(q)


def test_received_by_the_other_end():
    """A datagram this host sends (source L, destination R) and fills verifies at R:
    the receive path there uses R as the local address (tcp.rs:839-843)."""
    out, _ = O.tx_fill_ref(zero(sent_by_local(ipv4(6, tcp_seg(R4, L4, b"payload" * 9))), 10, 36))
    assert O.rx_status_ref(out, R4, R6) & O.RX_ACCEPT
    assert not O.rx_status_ref(out, L4, L6) & O.RX_L4_OK      # ... and not at an address it was not sent to
    out, _ = O.tx_fill_ref(zero(sent_by_local(ipv6(58, tcp_seg(R6, L6, b"p", proto=58, field=2, hlen=4))), 42))
    assert O.rx_status_ref(out, R4, R6) & O.RX_ACCEPT


def test_udp_zero_stored_as_is_and_length_as_u16():
    # udp.rs:168-171: no RFC 768 0 -> 0xffff substitution; find a payload whose sum is 0
    base = bytearray(ipv4(17, tcp_seg(L4, R4, b"\x00\x00", proto=17, field=6, hlen=8)))
    out, _ = O.tx_fill_ref(bytes(base))
    c = int.from_bytes(out[26:28], "big")
    fix = bytearray(base)
    fix[28:30] = c.to_bytes(2, "big")          # payload word = the old checksum: the new sum folds to 0xffff
    out2, _ = O.tx_fill_ref(bytes(fix))
    assert out2[26:28] == b"\x00\x00"


def test_not_produced_by_the_stack_left_alone():
    assert O.tx_fill_ref(b"") == (b"", O.TX_MALFORMED)
    bad = bytes([0x50]) + b"\x00" * 40
    assert O.tx_fill_ref(bad) == (bad, O.TX_MALFORMED)
    short6 = ipv6(6, b"")[:39]
    assert O.tx_fill_ref(short6) == (short6, O.TX_MALFORMED)
    unknown = ipv4(99, b"x" * 30)
    out, st = O.tx_fill_ref(unknown)
    assert st == O.TX_IP_FILLED and out == unknown     # header filled (already correct), no L4 field
    tiny = zero(ipv4(6, b"x" * 17), 10)
    out, st = O.tx_fill_ref(tiny)
    assert st == O.TX_IP_FILLED                         # segment too short for [16..18]
