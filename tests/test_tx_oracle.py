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


def chain(pkt, cuts):
    """pkt cut at the given offsets: [pkt[:c0], pkt[c0:c1], ...]."""
    b = [0] + list(cuts) + [len(pkt)]
    return [pkt[b[i]:b[i + 1]] for i in range(len(b) - 1)]


def test_chain_fill_equals_whole_datagram_fill_for_even_pieces():
    """A head holding the IP and L4 headers, then payload pieces of even length (the
    reference's 512-byte NetBuffer fragments): the same bytes tx_fill_ref stores in the
    contiguous datagram, in the head, and the same status."""
    cases = [
        (ipv4(6, tcp_seg(L4, R4, b"p" * 1460)), 40),
        (ipv6(6, tcp_seg(L6, R6, b"q" * 1000)), 60),
        (ipv4(17, tcp_seg(L4, R4, b"r" * 777, proto=17, field=6, hlen=8)), 28),
        (ipv4(1, icmp4(b"s" * 600)), 28),
        (ipv6(58, tcp_seg(L6, R6, b"t" * 333, proto=58, field=2, hlen=4)), 48),
        (ipv4(6, tcp_seg(L4, R4, b"u" * 100), ihl=15), 80),
    ]
    for pkt, hl in cases:
        pkt = zero(pkt, 10) if pkt[0] >> 4 == 4 else pkt
        want, st = O.tx_fill_ref(pkt)
        for step in (512, 2, 1000):
            cuts = list(range(hl, len(pkt), step))
            frags = chain(pkt, cuts)
            head, st2 = O.tx_chain_fill_ref(frags)
            assert st2 == st and head == want[:hl]
        # the whole datagram as one head fragment
        assert O.tx_chain_fill_ref([pkt]) == (want, st)


def test_chain_fill_folds_odd_pieces_per_fragment():
    """An odd-length L4 header part or payload piece pairs its bytes from its own start
    (util.rs:112-119 folds every fragment on its own): the L4 value is the per-fragment fold,
    not the contiguous sum."""
    pkt = ipv4(6, tcp_seg(L4, R4, bytes(range(1, 200))))
    frags = chain(pkt, [41, 100, 151])                     # head with 21 L4 bytes, odd pieces
    head, st = O.tx_chain_fill_ref(frags)
    assert st == O.TX_IP_FILLED | O.TX_L4_FILLED
    l4 = bytearray(frags[0][20:])
    l4[16:18] = b"\x00\x00"
    ph = O.pseudo_header_py(pkt[12:16], pkt[16:20], len(pkt) - 20, 6)
    want = O.buffer_ones_comp_py(ph, [bytes(l4)] + frags[1:]) ^ 0xFFFF
    assert int.from_bytes(head[36:38], "big") == want
    assert want != int.from_bytes(O.tx_fill_ref(pkt)[0][36:38], "big")
    assert O.checksum_py(head[:20]) == 0                  # the IP header verifies


def test_chain_fill_rejects_and_partial_fills():
    pkt = ipv4(6, tcp_seg(L4, R4, b"x" * 64))
    assert O.tx_chain_fill_ref([]) == (b"", O.TX_MALFORMED)
    assert O.tx_chain_fill_ref([b"", pkt]) == (b"", O.TX_MALFORMED)
    assert O.tx_chain_fill_ref([pkt[:19], pkt[19:]]) == (pkt[:19], O.TX_MALFORMED)   # IP header split
    v6 = ipv6(6, tcp_seg(L6, R6, b"y" * 10))
    assert O.tx_chain_fill_ref([v6[:39], v6[39:]])[1] == O.TX_MALFORMED
    head, st = O.tx_chain_fill_ref([pkt[:30], pkt[30:]])                               # field past the head
    assert st == O.TX_IP_FILLED and head[20:30] == pkt[20:30] and O.checksum_py(head[:20]) == 0
    head, st = O.tx_chain_fill_ref([v6[:40], v6[40:]])                                 # IPv6: no IP field
    assert st == 0 and head == v6[:40]
    head, st = O.tx_chain_fill_ref([pkt[:38], b"", pkt[38:]])                          # empty piece: nothing
    assert st == O.TX_IP_FILLED | O.TX_L4_FILLED and head == O.tx_fill_ref(pkt)[0][:38]


def test_chain_fill_c_restatement_equals_python(oracle):
    """oracle_tx_chain_fill (C: bench.py --op finalize's CPU baseline) == tx_chain_fill_ref on
    random chains of every datagram kind: heads cut anywhere, odd pieces, empty pieces, no
    fragments, fragments outside the arena; 1 thread and 4."""
    import numpy as np
    from test_gpu_tx import outgoing
    pkts = outgoing(1500, 0xC0C0)
    w = O.splitmix64_words(0xC0C1, 4 * len(pkts))
    arena = bytearray()
    off, ln, first, chains = [], [], [0], []
    for i, p in enumerate(pkts):
        if i % 97 == 5:
            first.append(len(off))
            chains.append(None)
            continue
        cuts = sorted({int(w[4 * i + k]) % (len(p) + 1) for k in range(1 + int(w[4 * i + 3] % np.uint64(3)))})
        hl = min(len(p), 20 + int(w[4 * i] % np.uint64(50))) if i % 3 else cuts[0]
        b = [0, hl] + [c for c in cuts if c > hl] + [len(p)]
        frags = [p[b[k]:b[k + 1]] for k in range(len(b) - 1)]
        if not frags[-1] and len(frags) > 1:
            frags = frags[:-1]
        for f in frags:
            arena += bytes(int(w[4 * i + 1] % np.uint64(5)))
            off.append(len(arena))
            ln.append(len(f))
            arena += f
        first.append(len(off))
        chains.append(frags)
    off.append(1 << 40)                       # a chain with a fragment outside the arena
    ln.append(4)
    first.append(len(off))
    chains.append(None)
    arena_np = np.frombuffer(bytes(arena), dtype=np.uint8)
    for threads in (1, 4):
        a = arena_np.copy()
        st = oracle.tx_chain_fill(a, np.array(off, np.uint64), np.array(ln, np.uint32), np.array(first, np.uint32),
                                  threads=threads)
        for i, frags in enumerate(chains):
            if frags is None:
                assert st[i] == O.TX_MALFORMED
                continue
            h, s = O.tx_chain_fill_ref(frags)
            o = off[first[i]]
            assert st[i] == s and bytes(a[o:o + len(h)]) == h, i
