"""Device time of the widened §8f operations on MI355X (one GPU), next to the plain
batch checksum, on the headline batch (2^20 x 1500 B) and on IMIX:

* csum     — rns_csum_batch_dev (the hot path itself)
* chain    — rns_csum_chain_dev: every packet as the stack receives it after the
             IP trim, three fragments [492, 512, 496]
* fill     — rns_csum_fill_dev: transmit fill of the TCP checksum field [16..18]
* fill_packed — rns_csum_fill_packed_dev: the same fill with the packed descriptors
* verify   — rns_rx_verify_dev: IPv4 header + TCP checks of whole datagrams
* tx       — rns_tx_fill_dev: IPv4 header + TCP checksums of whole datagrams stored in
             place, pseudo-headers formed on the device
* tx_packed — rns_tx_fill_packed_dev: the same finalize over the packed form (the rows transmit
             kernel; round 6)
* verify_packed — rns_rx_verify_packed_dev: receive verify over the packed form
* chain_fill — rns_csum_chain_fill_dev on the transmit shape (workloads.tx_chain_layout:
             20-byte TCP head fragments back to back in a header region, the payload as one
             fragment or as 512-byte NetBuffer fragments), next to the plain chain checksum
             of the same chains (chain_tx)
* tx_chain — rns_tx_fill_chain_dev: whole-datagram finalize of the same transmit shape with
             40-byte IPv4 + TCP head fragments (the layout alloc_header builds, buf.rs:262-291),
             payload as one fragment or 512-byte NetBuffer fragments (round 6)

Timing: one pair of HIP events around K back-to-back launches on the launch stream,
median of R rounds.  GB/s counts algorithmic bytes (payload read + result bytes
written); descriptor and workspace traffic is not credited.

    python tools/bench_ops.py [--steps 20] [--rounds 5] [--out profiles/archive/r01/r01_ops.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rustnetworkstack_amd.batch import (PreparedBatch, csum_chain, csum_fill, csum_fill_packed,  # noqa: E402
                                        packed_layout, rx_verify, rx_verify_packed, tx_fill, tx_fill_packed)
from rustnetworkstack_amd.workloads import DeviceBatch, make_layout  # noqa: E402

L4 = bytes([192, 168, 1, 2])
L6 = bytes.fromhex("fe800000000000000000000000000002")


def write_ipv4_tcp_headers(b, lay, dev):
    """IPv4 header (src R4, dst L4, proto 6) in each packet's first 20 bytes, header
    checksum filled (ip.rs:158-159), TCP checksum filled with the per-packet
    pseudo-header seed (tcp.rs:957-973)."""
    from oracle.oracle import pseudo_header_py  # test infrastructure: builds inputs only
    n = lay.n
    hdr = np.frombuffer(bytes.fromhex("4500000000004000400600000000000000000000"), dtype=np.uint8).copy()
    hdr[12:16] = [192, 168, 1, 1]
    hdr[16:20] = np.frombuffer(L4, dtype=np.uint8)
    hdrs = np.tile(hdr, (n, 1))
    hdrs[:, 2] = (lay.length >> 8) & 0xFF
    hdrs[:, 3] = lay.length & 0xFF
    idx = b.off.view(-1, 1) + torch.arange(20, device=dev)
    b.arena[idx.flatten()] = torch.from_numpy(hdrs.reshape(-1)).to(dev)
    del idx
    csum_fill(b.arena, b.off, torch.full((n,), 20, dtype=torch.int32, device=dev), None, field_off=10)
    l4 = lay.length.astype(np.int64) - 20
    uniq = {int(x): pseudo_header_py(bytes([192, 168, 1, 1]), L4, int(x), 6) for x in np.unique(l4)}
    seeds = np.array([uniq[int(x)] for x in l4], dtype=np.uint16) if len(uniq) > 1 else \
        np.full(n, next(iter(uniq.values())), dtype=np.uint16)
    csum_fill(b.arena, b.off + 20, b.length - 20, torch.from_numpy(seeds.view(np.int16)).to(dev), field_off=16)
    torch.cuda.synchronize()


def timed(fn, steps, rounds):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    fn()
    res = []
    for _ in range(rounds):
        e0.record()
        for _ in range(steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / steps)
    res.sort()
    return res[len(res) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--configs", default="c3_1500B,c5_imix")
    ap.add_argument("--ops", default="csum,chain,fill,verify,tx")
    ap.add_argument("--out", default="")
    ap.add_argument("--chain-layouts", default="packed,netbuf,netbuf_shuffled",
                    help="packed: [492, 512, rest] fragments back to back inside each packet; netbuf: every "
                         "fragment in its own 512-byte buffer (NetBuffer, buf.rs:50), ceil(L/512) per packet, "
                         "the buffers in order (a packet's fragments adjacent); netbuf_shuffled: the same "
                         "buffers in a random order (no two fragments adjacent)")
    ap.add_argument("--tx-frags", default="0,512", help="chain_fill: payload fragment sizes (0 = one fragment)")
    ap.add_argument("--tx-modes", default="plain,runs,txpacked", help="chain_fill: hint flags to time")
    args = ap.parse_args()
    ops = set(args.ops.split(","))
    dev = torch.device("cuda:0")
    results = {}
    for cfg in args.configs.split(","):
        lay = make_layout(cfg)
        b = DeviceBatch(lay, dev)
        n, pay = lay.n, lay.payload_bytes
        r = {}
        pb = PreparedBatch(b.arena, b.off, b.length, b.seed, complement=True, out=b.out,
                           len_hint=int(round(lay.mean_len)))
        if "csum" in ops:
            ms = timed(pb, args.steps, args.rounds)
            r["csum"] = {"us": round(ms * 1e3, 1), "GBps": round((pay + 2 * n) / ms / 1e6, 1)}
        if "chain" in ops:
            for cl in args.chain_layouts.split(","):
                key = "chain" if cl == "packed" else f"chain_{cl}"
                for runs in (False, True):  # without / with RNS_FLAG_CHAIN_RUNS
                    r[key + ("_runs" if runs else "")] = bench_chain(b, lay, dev, args, runs) if cl == "packed" else \
                        bench_chain_netbuf(lay, dev, args, shuffled=cl == "netbuf_shuffled", runs=runs)
        if "chain_fill" in ops:
            for frag in (int(x) for x in args.tx_frags.split(",")):
                r.update(bench_chain_fill(cfg, dev, args, frag))
        if "tx_chain" in ops:
            for frag in (int(x) for x in args.tx_frags.split(",")):
                r.update(bench_tx_chain(cfg, dev, args, frag))
        if "fill" in ops:
            ms = timed(lambda: csum_fill(b.arena, b.off, b.length, b.seed, field_off=16), args.steps, args.rounds)
            r["fill"] = {"us": round(ms * 1e3, 1), "GBps": round((pay + 2 * n) / ms / 1e6, 1)}
        if "fill_packed" in ops:
            blk, _, _ = packed_layout(lay.length, align_log2=4)
            blk_t = torch.from_numpy(blk.view(np.int64)).to(dev)
            len16 = torch.from_numpy(lay.length.astype(np.uint16).view(np.int16)).to(dev)
            hint = int(round(lay.mean_len))
            ms = timed(lambda: csum_fill_packed(b.arena, blk_t, len16, b.seed, align_log2=4, field_off=16,
                                                len_hint=hint), args.steps, args.rounds)
            r["fill_packed"] = {"us": round(ms * 1e3, 1), "GBps": round((pay + 2 * n) / ms / 1e6, 1)}
        if "tx" in ops:
            write_ipv4_tcp_headers(b, lay, dev)
            st = torch.empty(n, dtype=torch.uint8, device=dev)
            ms = timed(lambda: tx_fill(b.arena, b.off, b.length, status=st), args.steps, args.rounds)
            filled = int((st == 3).sum().item())
            r["tx"] = {"us": round(ms * 1e3, 1), "GBps": round((pay + n) / ms / 1e6, 1), "filled": filled,
                       "packets": n}
        if "tx_packed" in ops:
            write_ipv4_tcp_headers(b, lay, dev)
            b.launcher(packed=True)  # uploads blk_off / len16
            st = torch.empty(n, dtype=torch.uint8, device=dev)
            hint = int(round(lay.mean_len))
            ms = timed(lambda: tx_fill_packed(b.arena, b.blk_off, b.len16, status=st, len_hint=hint),
                       args.steps, args.rounds)
            filled = int((st == 3).sum().item())
            r["tx_packed"] = {"us": round(ms * 1e3, 1), "GBps": round((pay + n) / ms / 1e6, 1), "filled": filled,
                              "packets": n}
        if "verify_packed" in ops:
            write_ipv4_tcp_headers(b, lay, dev)
            b.launcher(packed=True)
            st = torch.empty(n, dtype=torch.uint8, device=dev)
            ms = timed(lambda: rx_verify_packed(b.arena, b.blk_off, b.len16, L4, L6, status=st),
                       args.steps, args.rounds)
            accepted = int((st == 0x43).sum().item())
            r["verify_packed"] = {"us": round(ms * 1e3, 1), "GBps": round((pay + n) / ms / 1e6, 1),
                                  "accepted": accepted, "packets": n}
        if "verify" in ops:
            # turn every packet into a valid IPv4/TCP datagram first (header written
            # on the GPU, IPv4 and TCP checksums filled), so every byte is checked
            write_ipv4_tcp_headers(b, lay, dev)
            st = torch.empty(n, dtype=torch.uint8, device=dev)
            ms = timed(lambda: rx_verify(b.arena, b.off, b.length, L4, L6, status=st),
                       args.steps, args.rounds)
            accepted = int((st == 0x43).sum().item())
            r["verify"] = {"us": round(ms * 1e3, 1), "GBps": round((pay + n) / ms / 1e6, 1),
                           "accepted": accepted, "packets": n}
        results[cfg] = r
        print(cfg, json.dumps(r), flush=True)
        del b
        torch.cuda.empty_cache()
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"tool": "tools/bench_ops.py", "steps": args.steps, "rounds": args.rounds,
                       "results": results}, f, indent=1)
    print(json.dumps(results))


def bench_chain(b, lay, dev, args, runs=False):
    n, pay = lay.n, lay.payload_bytes
    # chain: three fragments per packet where the packet is long enough, else one
    L = lay.length.astype(np.int64)
    nfr = np.where(L > 1004, 3, 1)
    first = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(nfr, out=first[1:])
    nf = int(first[-1])
    frag_off = np.empty(nf, dtype=np.uint64)
    frag_len = np.empty(nf, dtype=np.uint32)
    three = nfr == 3
    i3 = first[:-1][three]
    frag_off[i3] = lay.off[three]
    frag_off[i3 + 1] = lay.off[three] + 492
    frag_off[i3 + 2] = lay.off[three] + 1004
    frag_len[i3] = 492
    frag_len[i3 + 1] = 512
    frag_len[i3 + 2] = (L[three] - 1004).astype(np.uint32)
    i1 = first[:-1][~three]
    frag_off[i1] = lay.off[~three]
    frag_len[i1] = lay.length[~three]
    d_fo = torch.from_numpy(frag_off.view(np.int64)).to(dev)
    d_fl = torch.from_numpy(frag_len.view(np.int32)).to(dev)
    d_first = torch.from_numpy(first.astype(np.uint32).view(np.int32)).to(dev)
    sums = torch.empty(nf, dtype=torch.uint16, device=dev)
    out = torch.empty(n, dtype=torch.uint16, device=dev)
    ms = timed(lambda: csum_chain(b.arena, d_fo, d_fl, d_first, b.seed, complement=True, out=out,
                                  frag_sums=sums, frag_len_hint=int(round(pay / nf)), runs=runs),
               args.steps, args.rounds)
    return {"us": round(ms * 1e3, 1), "GBps": round((pay + 2 * n) / ms / 1e6, 1), "fragments": nf}


def bench_chain_fill(cfg, dev, args, frag):
    """The head-fragment fill and the plain chain checksum over the transmit shape."""
    from rustnetworkstack_amd.batch import csum_chain_fill, fill_splitmix64
    from rustnetworkstack_amd.workloads import tx_chain_layout
    t = tx_chain_layout(cfg, frag=frag)
    n, pay, nf = t.n, t.payload_bytes, int(t.frag_off.shape[0])
    arena = torch.empty(t.arena_bytes + 64, dtype=torch.uint8, device=dev)
    fill_splitmix64(arena, t.data_seed)
    d_fo = torch.from_numpy(t.frag_off.view(np.int64)).to(dev)
    d_fl = torch.from_numpy(t.frag_len.view(np.int32)).to(dev)
    d_first = torch.from_numpy(t.first.view(np.int32)).to(dev)
    seed = torch.from_numpy(t.seed.view(np.int16)).to(dev)
    out = torch.empty(n, dtype=torch.uint16, device=dev)
    hint = int(round(pay / nf))
    tag = "tx" if frag == 0 else f"tx{frag}"
    res = {}
    modes = {"plain": (False, False), "runs": (True, False), "txpacked": (False, True)}
    for runs, txp in (modes[m] for m in args.tx_modes.split(",")):
        sfx = "_runs" if runs else "_txpacked" if txp else ""
        ms = timed(lambda: csum_chain_fill(arena, d_fo, d_fl, d_first, seed, field_off=t.field, out=out,
                                           frag_len_hint=hint, runs=runs, tx_packed=txp), args.steps, args.rounds)
        res[f"chain_fill_{tag}{sfx}"] = {"us": round(ms * 1e3, 1), "GBps": round((pay + 2 * n) / ms / 1e6, 1),
                                        "fragments": nf, "hint": hint}
        ms = timed(lambda: csum_chain(arena, d_fo, d_fl, d_first, seed, complement=True, out=out,
                                      frag_len_hint=hint, runs=runs, tx_packed=txp), args.steps, args.rounds)
        res[f"chain_{tag}{sfx}"] = {"us": round(ms * 1e3, 1), "GBps": round((pay + 2 * n) / ms / 1e6, 1)}
    del arena
    torch.cuda.empty_cache()
    return res


def bench_tx_chain(cfg, dev, args, frag):
    """Whole-datagram transmit finalize over NetBuffer chains: 40-byte IPv4 + TCP heads back to
    back in a header region, payloads packed at 16-byte starts (one fragment, or 512-byte ones)."""
    from rustnetworkstack_amd.batch import fill_splitmix64, tx_fill_chain
    from rustnetworkstack_amd.workloads import tx_chain_layout
    t = tx_chain_layout(cfg, head=40, frag=frag)
    n, pay, nf = t.n, t.payload_bytes, int(t.frag_off.shape[0])
    arena = torch.empty(t.arena_bytes + 64, dtype=torch.uint8, device=dev)
    fill_splitmix64(arena, t.data_seed)
    hoff = torch.from_numpy(t.frag_off[t.first[:-1].astype(np.int64)].view(np.int64)).to(dev)
    hdr = np.frombuffer(bytes.fromhex("4500000000004000400600000000000000000000"), dtype=np.uint8).copy()
    hdr[12:16] = [192, 168, 1, 1]
    hdr[16:20] = np.frombuffer(L4, dtype=np.uint8)
    idx = hoff.view(-1, 1) + torch.arange(20, device=dev)
    arena[idx.flatten()] = torch.from_numpy(hdr).to(dev).repeat(n)
    del idx
    d_fo = torch.from_numpy(t.frag_off.view(np.int64)).to(dev)
    d_fl = torch.from_numpy(t.frag_len.view(np.int32)).to(dev)
    d_first = torch.from_numpy(t.first.view(np.int32)).to(dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    ms = timed(lambda: tx_fill_chain(arena, d_fo, d_fl, d_first, status=st), args.steps, args.rounds)
    filled = int((st == 3).sum().item())
    tag = "tx_chain" if frag == 0 else f"tx_chain{frag}"
    del arena
    torch.cuda.empty_cache()
    return {tag: {"us": round(ms * 1e3, 1), "GBps": round((pay + n) / ms / 1e6, 1), "filled": filled,
                  "packets": n, "fragments": nf}}


def bench_chain_netbuf(lay, dev, args, shuffled=False, runs=False):
    """Fragments as NetBuffer holds them: packet i of L bytes is ceil(L/512) fragments,
    each in its own 512-byte buffer (buf.rs:50; the fragment arena is those buffers
    back to back, filled with splitmix64 bytes).  shuffled: fragment f lives in buffer
    perm[f] (a random permutation), as buffers from a free list are."""
    from rustnetworkstack_amd.batch import fill_splitmix64
    n, pay = lay.n, lay.payload_bytes
    L = lay.length.astype(np.int64)
    nfr = (L + 511) // 512
    first = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(nfr, out=first[1:])
    nf = int(first[-1])
    pkt = np.repeat(np.arange(n), nfr)
    k = np.arange(nf) - first[:-1][pkt]
    slot = np.random.default_rng(0x5B0F).permutation(nf) if shuffled else np.arange(nf)
    frag_off = slot.astype(np.uint64) * np.uint64(512)
    frag_len = np.minimum(L[pkt] - 512 * k, 512).astype(np.uint32)
    arena = torch.empty(nf * 512 + 16, dtype=torch.uint8, device=dev)
    fill_splitmix64(arena, 0xF4A6)
    d_fo = torch.from_numpy(frag_off.view(np.int64)).to(dev)
    d_fl = torch.from_numpy(frag_len.view(np.int32)).to(dev)
    d_first = torch.from_numpy(first.astype(np.uint32).view(np.int32)).to(dev)
    seed = torch.from_numpy(lay.seed.view(np.int16)).to(dev)
    out = torch.empty(n, dtype=torch.uint16, device=dev)
    ms = timed(lambda: csum_chain(arena, d_fo, d_fl, d_first, seed, complement=True, out=out,
                                  frag_len_hint=int(round(pay / nf)), runs=runs),
               args.steps, args.rounds)
    del arena
    torch.cuda.empty_cache()
    return {"us": round(ms * 1e3, 1), "GBps": round((pay + 2 * n) / ms / 1e6, 1), "fragments": nf,
            "layout": "netbuf: 512-byte fragment buffers" + (", shuffled" if shuffled else ", in order")}


if __name__ == "__main__":
    main()
