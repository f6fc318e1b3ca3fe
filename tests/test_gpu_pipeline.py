"""End-to-end batched receive: SOCK_SEQPACKET socketpair (TUN-like datagram fd) ->
rns_io_recv_batch into pinned MRU slots -> H2D -> fused rns_rx_verify_dev -> verdicts,
compared with the reference receive path restated in the oracle."""
import socket
import threading

import numpy as np
import pytest

from oracle import oracle as O
from rustnetworkstack_amd.batch import send_batch
from rustnetworkstack_amd.pipeline import RxPipeline
from test_gpu_rx import make_packets
from test_rx_oracle import L4, L6

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("packed", [True, False])
def test_socket_to_verdicts(oracle, packed):
    """Every kind of datagram through the synchronous receive: packed (rns_io_recv_batch_packed
    -> the used bytes only -> rns_rx_verify_packed_dev) and in MRU slots (rns_rx_verify_dev);
    verdicts, lengths and bytes against the reference's receive path."""
    pkts = make_packets(6000, 0xD1CE)
    lens = np.array([len(p) for p in pkts], dtype=np.uint32)
    off = np.zeros(len(pkts), dtype=np.uint64)
    np.cumsum(lens[:-1].astype(np.uint64), out=off[1:])
    arena = np.frombuffer(b"".join(pkts), dtype=np.uint8).copy()
    nonempty = lens > 0                      # a zero-length datagram cannot be told from EOF
    expect = np.array([O.rx_status_ref(p, L4, L6, ones_comp=oracle.compute_ones_comp) for p in pkts],
                      dtype=np.uint8)[nonempty]
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    t = threading.Thread(target=send_batch, args=(a.fileno(), arena, off[nonempty], lens[nonempty]))
    t.start()
    pipe = RxPipeline(L4, L6, device=0, max_pkts=1024, packed=packed)
    want = [p for p in pkts if len(p)]
    got_st, got_len, bad_bytes = [], [], 0
    while sum(x.shape[0] for x in got_st) < int(nonempty.sum()):
        st, ln = pipe.receive(b.fileno(), timeout_ms=2000)
        assert st.shape[0] > 0, "receive timed out"
        i0 = sum(x.shape[0] for x in got_st)
        bad_bytes += sum(pipe.last[k].tobytes() != want[i0 + k] for k in range(ln.shape[0]))
        got_st.append(st)
        got_len.append(ln.copy())
    t.join()
    h2d, n = pipe.h2d_bytes, pipe.datagrams
    pipe.close()
    a.close()
    b.close()
    assert bad_bytes == 0
    assert np.array_equal(np.concatenate(got_len), lens[nonempty])
    assert np.array_equal(np.concatenate(got_st), expect)
    pad = int(((lens[nonempty].astype(np.int64) + 15) // 16 * 16).sum())
    assert h2d == (pad if packed else n * 2048)  # packed: the datagrams' padded bytes cross PCIe, not slots


def test_tx_pipeline_to_socket(oracle):
    """Datagrams with unset checksum fields in pinned slots -> TxPipeline -> socket; the
    other end receives exactly what the reference's transmit path would send."""
    from rustnetworkstack_amd.batch import recv_batch
    from rustnetworkstack_amd.pipeline import TxPipeline
    from test_gpu_tx import outgoing
    pkts = [p for p in outgoing(5000, 0x5E4D) if 0 < len(p) <= 2048]
    want = [O.tx_fill_ref(p, ones_comp=oracle.compute_ones_comp) for p in pkts]
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    for s_, opt in ((a, socket.SO_SNDBUF), (b, socket.SO_RCVBUF)):
        s_.setsockopt(socket.SOL_SOCKET, opt, 32 << 20)
    received = []

    def drain():
        buf = np.empty(2048 * 1024, dtype=np.uint8)
        while len(received) < len(pkts):
            off, ln = recv_batch(b.fileno(), buf, 2048, 1024, timeout_ms=5000)
            if ln.shape[0] == 0:
                return
            received.extend(buf[int(o):int(o) + int(n)].tobytes() for o, n in zip(off, ln))

    t = threading.Thread(target=drain)
    t.start()
    pipe = TxPipeline(device=0, max_pkts=1024)
    statuses = []
    for i0 in range(0, len(pkts), 1024):
        chunk = pkts[i0:i0 + 1024]
        slots = pipe.slots()
        for k, p in enumerate(chunk):
            slots[k, :len(p)] = np.frombuffer(p, dtype=np.uint8)
        statuses.append(pipe.send(a.fileno(), np.array([len(p) for p in chunk], dtype=np.uint32)))
    t.join(timeout=60)
    pipe.close()
    a.close()
    b.close()
    assert np.array_equal(np.concatenate(statuses), np.array([w[1] for w in want], dtype=np.uint8))
    assert len(received) == len(pkts)
    bad = [i for i in range(len(pkts)) if received[i] != want[i][0]]
    assert not bad, bad[:5]


@pytest.mark.parametrize("packed", [True, False])
def test_stream_overlapped(oracle, packed):
    """RxPipeline.stream: the host reads batch k+1 while batch k is verified; verdicts,
    lengths and slot bytes as the synchronous path would give them."""
    pkts = [p for p in make_packets(6000, 0x0BE1) if len(p) > 0]
    lens = np.array([len(p) for p in pkts], dtype=np.uint32)
    off = np.zeros(len(pkts), dtype=np.uint64)
    np.cumsum(lens[:-1].astype(np.uint64), out=off[1:])
    arena = np.frombuffer(b"".join(pkts), dtype=np.uint8).copy()
    expect = np.array([O.rx_status_ref(p, L4, L6, ones_comp=oracle.compute_ones_comp) for p in pkts], dtype=np.uint8)
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    t = threading.Thread(target=send_batch, args=(a.fileno(), arena, off, lens))
    t.start()
    pipe = RxPipeline(L4, L6, device=0, max_pkts=512, packed=packed)
    got_st, got_len, bad_bytes, i = [], [], 0, 0
    for st, ln, dg in pipe.stream(b.fileno(), timeout_ms=2000):
        got_st.append(st.copy())
        got_len.append(ln.copy())
        for k in range(ln.shape[0]):
            bad_bytes += dg[k].tobytes() != pkts[i + k]
        i += ln.shape[0]
        if i >= len(pkts):
            break
    t.join()
    pipe.close()
    a.close()
    b.close()
    assert len(got_st) >= 2 and bad_bytes == 0
    assert np.array_equal(np.concatenate(got_len), lens)
    assert np.array_equal(np.concatenate(got_st), expect)


def test_tx_overlapped_to_socket(oracle):
    """TxPipeline.submit/complete: two buffer sets in flight; the far end receives
    exactly what the reference's transmit path would send, in order."""
    from rustnetworkstack_amd.batch import recv_batch
    from rustnetworkstack_amd.pipeline import TxPipeline
    from test_gpu_tx import outgoing
    pkts = [p for p in outgoing(5000, 0x7A11) if 0 < len(p) <= 2048]
    want = [O.tx_fill_ref(p, ones_comp=oracle.compute_ones_comp) for p in pkts]
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    for s_, opt in ((a, socket.SO_SNDBUF), (b, socket.SO_RCVBUF)):
        s_.setsockopt(socket.SOL_SOCKET, opt, 32 << 20)
    received = []

    def drain():
        buf = np.empty(2048 * 1024, dtype=np.uint8)
        while len(received) < len(pkts):
            off, ln = recv_batch(b.fileno(), buf, 2048, 1024, timeout_ms=5000)
            if ln.shape[0] == 0:
                return
            received.extend(buf[int(o):int(o) + int(n)].tobytes() for o, n in zip(off, ln))

    t = threading.Thread(target=drain)
    t.start()
    pipe = TxPipeline(device=0, max_pkts=700)
    statuses = []
    with pytest.raises(RuntimeError):
        pipe.complete(a.fileno())
    for i0 in range(0, len(pkts), 700):
        if pipe.pending() == pipe.DEPTH:
            statuses.append(pipe.complete(a.fileno()))
        chunk = pkts[i0:i0 + 700]
        slots = pipe.slots()
        for k, p in enumerate(chunk):
            slots[k, :len(p)] = np.frombuffer(p, dtype=np.uint8)
        pipe.submit(np.array([len(p) for p in chunk], dtype=np.uint32))
        if pipe.pending() == pipe.DEPTH:
            with pytest.raises(RuntimeError):
                pipe.slots()
    while pipe.pending():
        statuses.append(pipe.complete(a.fileno()))
    t.join(timeout=60)
    pipe.close()
    a.close()
    b.close()
    assert np.array_equal(np.concatenate(statuses), np.array([w[1] for w in want], dtype=np.uint8))
    assert len(received) == len(pkts)
    bad = [i for i in range(len(pkts)) if received[i] != want[i][0]]
    assert not bad, bad[:5]


@pytest.mark.parametrize("overlap", [False, True])
def test_tx_chain_pipeline_to_socket(oracle, overlap):
    """TxChainPipeline: every kind of outgoing datagram as the reference builds it — a head
    fragment (IP + L4 headers, alloc_header) in the header region and its payload in the payload
    region — finalized on the GPU and sent gathered from its two fragments (send_packet's
    writev); the far end receives exactly the contiguous datagram the reference's transmit path
    would send (oracle.tx_chain_fill_ref == tx_fill_ref for an even L4 header part), in order."""
    from rustnetworkstack_amd.batch import recv_batch
    from rustnetworkstack_amd.pipeline import TxChainPipeline
    from test_gpu_tx import outgoing
    from test_gpu_tx_chain import l4_header_len
    pkts = [p for p in outgoing(4000, 0x7C4A + overlap) if 0 < len(p) <= 2048]
    heads = [p[:min(len(p), max(1, l4_header_len(p)), TxChainPipeline.HEAD_MAX)] for p in pkts]  # (garbage: IHL 0)
    want = []
    for p, h in zip(pkts, heads):
        frags = [h] + ([p[len(h):]] if len(p) > len(h) else [])
        hh, st = O.tx_chain_fill_ref(frags, ones_comp=oracle.compute_ones_comp)
        want.append((hh + p[len(h):], st))
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    for s_, opt in ((a, socket.SO_SNDBUF), (b, socket.SO_RCVBUF)):
        s_.setsockopt(socket.SOL_SOCKET, opt, 32 << 20)
    received = []

    def drain():
        buf = np.empty(2048 * 1024, dtype=np.uint8)
        while len(received) < len(pkts):
            off, ln = recv_batch(b.fileno(), buf, 2048, 1024, timeout_ms=5000)
            if ln.shape[0] == 0:
                return
            received.extend(buf[int(o):int(o) + int(n)].tobytes() for o, n in zip(off, ln))

    t = threading.Thread(target=drain)
    t.start()
    pipe = TxChainPipeline(device=0, max_pkts=600)
    statuses = []
    for i0 in range(0, len(pkts), 600):
        if overlap and pipe.pending() == pipe.DEPTH:
            statuses.append(pipe.complete(a.fileno()))
        chunk = range(i0, min(i0 + 600, len(pkts)))
        hreg, preg = pipe.heads(), pipe.payloads()
        hl, po, pl = [], [], []
        hpos = ppos = 0
        for i in chunk:
            h, body = heads[i], pkts[i][len(heads[i]):]
            hreg[hpos:hpos + len(h)] = np.frombuffer(h, dtype=np.uint8)
            preg[ppos:ppos + len(body)] = np.frombuffer(body, dtype=np.uint8)
            hl.append(len(h))
            po.append(ppos)
            pl.append(len(body))
            hpos += len(h)
            ppos = (ppos + len(body) + 15) & ~15
        if overlap:
            pipe.submit(np.array(hl), np.array(po), np.array(pl))
        else:
            statuses.append(pipe.send(a.fileno(), np.array(hl), np.array(po), np.array(pl)))
    while pipe.pending():
        statuses.append(pipe.complete(a.fileno()))
    t.join(timeout=60)
    pipe.close()
    a.close()
    b.close()
    assert np.array_equal(np.concatenate(statuses), np.array([w[1] for w in want], dtype=np.uint8))
    assert len(received) == len(pkts)
    bad = [i for i in range(len(pkts)) if received[i] != want[i][0]]
    assert not bad, bad[:5]
