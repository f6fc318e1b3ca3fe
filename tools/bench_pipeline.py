"""End-to-end batched receive / transmit rates over a SOCK_SEQPACKET socketpair
(TUN-like: one datagram per read / write).

Receive (default): a sender thread writes N valid IPv4/TCP datagrams (1500 B, or 64 B
with --config c2_64B; sendmmsg); the receiver runs RxPipeline until all arrived — packed
(rns_io_recv_batch_packed: recvmmsg into a packed pinned arena -> H2D of the used bytes ->
rns_rx_verify_packed_dev -> verdicts D2H), or with --slots the round-5 form (2048-B slots ->
H2D of whole slots -> rns_rx_verify_dev).
Transmit (--tx): the same datagrams with their checksum fields zeroed are placed in
TxPipeline's pinned slots and sent (H2D -> rns_tx_fill_dev -> header bytes D2H ->
rns_io_send_batch); a drain thread reads them and the result is spot-checked.
Transmit chains (--tx --chain): each datagram as the reference builds it — a 40-byte head
fragment (IPv4 + TCP headers) in TxChainPipeline's header region, its 1460-byte payload in the
payload region (H2D of the used bytes -> rns_tx_fill_chain_dev -> the header region D2H ->
rns_io_send_batch_chain, each datagram gathered from its two fragments).

    python tools/bench_pipeline.py [--packets 262144] [--batch 8192] [--tx] [--overlap]

--overlap runs the two-buffer-set forms (RxPipeline.stream, TxPipeline.submit/complete):
the GPU work of one batch is queued on its own stream while the host reads or writes
the datagrams of the other.
"""
import argparse
import json
import os
import socket
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rustnetworkstack_amd.batch import send_batch  # noqa: E402
from rustnetworkstack_amd.batch import recv_batch  # noqa: E402
from rustnetworkstack_amd.pipeline import RxPipeline, TxChainPipeline, TxPipeline  # noqa: E402
from rustnetworkstack_amd.workloads import DeviceBatch, make_layout  # noqa: E402
from bench_ops import L4, L6, write_ipv4_tcp_headers  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 18)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--out", default="")
    ap.add_argument("--tx", action="store_true")
    ap.add_argument("--overlap", action="store_true")
    ap.add_argument("--chain", action="store_true", help="with --tx: TxChainPipeline (head + payload fragments)")
    ap.add_argument("--slots", action="store_true", help="receive into 2048-B slots (round-5 form)")
    ap.add_argument("--config", default="c3_1500B", help="datagram sizes: c3_1500B or c2_64B")
    args = ap.parse_args()
    if args.tx:
        return main_tx(args)
    dev = torch.device("cuda:0")
    lay = make_layout(args.config, n=args.packets)
    b = DeviceBatch(lay, dev)
    write_ipv4_tcp_headers(b, lay, dev)          # valid datagrams, built on the GPU
    arena = b.arena[:lay.arena_bytes].cpu().numpy()
    del b
    a, r = socket.socketpair(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    for s_, opt in ((a, socket.SO_SNDBUF), (r, socket.SO_RCVBUF)):
        s_.setsockopt(socket.SOL_SOCKET, opt, 64 << 20)
    pipe = RxPipeline(L4, L6, device=0, max_pkts=args.batch, packed=not args.slots)
    sender = threading.Thread(target=send_batch, args=(a.fileno(), arena, lay.off, lay.length))
    t0 = time.perf_counter()
    sender.start()
    got = accepted = batches = 0
    if args.overlap:
        for st, ln, _ in pipe.stream(r.fileno(), timeout_ms=5000):
            got += st.shape[0]
            accepted += int((st == 0x43).sum())
            batches += 1
            if got >= lay.n:
                break
    while got < lay.n:
        st, ln = pipe.receive(r.fileno(), timeout_ms=5000)
        if st.shape[0] == 0:
            break
        got += st.shape[0]
        accepted += int((st == 0x43).sum())
        batches += 1
    dt = time.perf_counter() - t0
    sender.join()
    size = int(lay.length[0])
    res = {"packets": lay.n, "datagram_bytes": size, "received": got, "accepted": accepted, "batches": batches,
           "seconds": round(dt, 3), "packets_per_s": round(got / dt), "GBps": round(got * size / dt / 1e9, 3),
           "h2d_bytes_per_datagram": round(pipe.h2d_bytes / max(pipe.datagrams, 1), 1),
           "overlap": args.overlap, "packed": not args.slots,
           "path": ("AF_UNIX SOCK_SEQPACKET socketpair (TUN-like; sendmmsg) -> " +
                    ("rns_io_recv_batch (recvmmsg into 2048-B slots, pinned) -> H2D of whole slots -> rns_rx_verify_dev"
                     if args.slots else
                     "rns_io_recv_batch_packed (recvmmsg, 16-byte packing, pinned) -> H2D of the used bytes -> "
                     "rns_rx_verify_packed_dev") + " -> status D2H; sender on another host thread")}
    print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    pipe.close()


def main_tx(args):
    dev = torch.device("cuda:0")
    lay = make_layout("c3_1500B", n=args.packets)
    b = DeviceBatch(lay, dev)
    write_ipv4_tcp_headers(b, lay, dev)          # valid datagrams, built on the GPU
    good = b.arena[:lay.arena_bytes].cpu().numpy()
    del b
    n = lay.n
    dgrams = good[(lay.off.reshape(-1, 1) + np.arange(1500, dtype=np.uint64)).reshape(-1)].reshape(n, 1500)
    unfilled = dgrams.copy()
    unfilled[:, 10:12] = 0                       # what ip_output_v4 / tcp_output see before their checksums
    unfilled[:, 36:38] = 0
    a, r = socket.socketpair(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    for s_, opt in ((a, socket.SO_SNDBUF), (r, socket.SO_RCVBUF)):
        s_.setsockopt(socket.SOL_SOCKET, opt, 64 << 20)
    pipe = TxChainPipeline(device=0, max_pkts=args.batch) if args.chain else TxPipeline(device=0, max_pkts=args.batch)
    got = [0]
    sample = {}

    def drain():
        buf = np.empty(2048 * 4096, dtype=np.uint8)
        while got[0] < n:
            off, ln = recv_batch(r.fileno(), buf, 2048, 4096, timeout_ms=5000)
            if ln.shape[0] == 0:
                return
            for k in range(0, ln.shape[0], 997):   # spot-check every 997th datagram
                sample[got[0] + k] = buf[int(off[k]):int(off[k]) + int(ln[k])].copy()
            got[0] += ln.shape[0]

    t = threading.Thread(target=drain)
    t0 = time.perf_counter()
    t.start()
    filled = 0
    for i0 in range(0, n, args.batch):
        k = min(args.batch, n - i0)
        if args.overlap and pipe.pending() == pipe.DEPTH:
            filled += int((pipe.complete(a.fileno()) == 3).sum())
        if args.chain:  # heads back to back, payloads at 16-byte steps (1472 B)
            pipe.heads()[:40 * k] = unfilled[i0:i0 + k, :40].reshape(-1)
            pipe.payloads()[:1472 * k].reshape(k, 1472)[:, :1460] = unfilled[i0:i0 + k, 40:]
            desc = (np.full(k, 40), np.arange(k) * 1472, np.full(k, 1460))
        else:
            pipe.slots()[:k, :1500] = unfilled[i0:i0 + k]
            desc = (np.full(k, 1500, dtype=np.uint32),)
        if args.overlap:
            pipe.submit(*desc)
        else:
            filled += int((pipe.send(a.fileno(), *desc) == 3).sum())
    while pipe.pending():
        filled += int((pipe.complete(a.fileno()) == 3).sum())
    t.join()
    dt = time.perf_counter() - t0
    exact = all(np.array_equal(v, dgrams[i]) for i, v in sample.items())
    res = {"direction": "transmit", "chain": args.chain, "overlap": args.overlap, "packets": n, "received": got[0], "filled": filled,
           "sample_exact": exact, "sampled": len(sample), "seconds": round(dt, 3),
           "packets_per_s": round(got[0] / dt), "GBps": round(got[0] * 1500 / dt / 1e9, 3),
           "path": ("host chains [40 B head, 1460 B payload] -> pinned header / payload regions -> H2D of the used "
                    "bytes -> rns_tx_fill_chain_dev -> header region D2H -> rns_io_send_batch_chain (sendmmsg, "
                    "two iovecs per datagram)" if args.chain else
                    "host datagrams -> pinned 2048-B slots -> H2D -> rns_tx_fill_dev -> 128 B/slot D2H -> "
                    "rns_io_send_batch") + " -> AF_UNIX SOCK_SEQPACKET socketpair; drain on another host thread"}
    print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    pipe.close()


if __name__ == "__main__":
    main()
