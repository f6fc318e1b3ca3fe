"""End-to-end batched receive rate: a sender thread writes N valid IPv4/TCP datagrams
(1500 B) into a SOCK_SEQPACKET socketpair (TUN-like: one datagram per read); the
receiver runs RxPipeline (rns_io_recv_batch into pinned 2048-B slots -> H2D ->
fused rns_rx_verify_dev -> verdicts D2H) until all arrived.  Reports packets/s and
GB/s of datagram bytes, and the share of time in each stage.

    python tools/bench_pipeline.py [--packets 262144] [--batch 8192]
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
from rustnetworkstack_amd.pipeline import RxPipeline  # noqa: E402
from rustnetworkstack_amd.workloads import DeviceBatch, make_layout  # noqa: E402
from bench_ops import L4, L6, write_ipv4_tcp_headers  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 18)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lay = make_layout("c3_1500B", n=args.packets)
    b = DeviceBatch(lay, dev)
    write_ipv4_tcp_headers(b, lay, dev)          # valid datagrams, built on the GPU
    arena = b.arena[:lay.arena_bytes].cpu().numpy()
    del b
    a, r = socket.socketpair(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    for s_, opt in ((a, socket.SO_SNDBUF), (r, socket.SO_RCVBUF)):
        s_.setsockopt(socket.SOL_SOCKET, opt, 64 << 20)
    pipe = RxPipeline(L4, L6, device=0, max_pkts=args.batch)
    sender = threading.Thread(target=send_batch, args=(a.fileno(), arena, lay.off, lay.length))
    t0 = time.perf_counter()
    sender.start()
    got = accepted = batches = 0
    while got < lay.n:
        st, ln = pipe.receive(r.fileno(), timeout_ms=5000)
        if st.shape[0] == 0:
            break
        got += st.shape[0]
        accepted += int((st == 0x43).sum())
        batches += 1
    dt = time.perf_counter() - t0
    sender.join()
    res = {"packets": lay.n, "received": got, "accepted": accepted, "batches": batches,
           "seconds": round(dt, 3), "packets_per_s": round(got / dt), "GBps": round(got * 1500 / dt / 1e9, 3),
           "path": "AF_UNIX SOCK_SEQPACKET socketpair (TUN-like) -> rns_io_recv_batch (2048-B slots, pinned) -> "
                   "H2D -> rns_rx_verify_dev -> status D2H; sender on another host thread"}
    print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    pipe.close()


if __name__ == "__main__":
    main()
