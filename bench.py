#!/usr/bin/env python3
"""Device-resident batched Internet checksum throughput on MI355X.

Metric (BASELINE.json): GiB/s device-resident Internet checksum, 1500 B-packet
batches, 1/2/4/8 GPUs.  One STEP = one pass of the hot path — one launch of the
gfx950 checksum kernel — over one batch (config c3_1500B: 2^20 packets x 1500 B
per GPU, already resident in HBM).  value = payload bytes checksummed by all
ranks / max-over-ranks wall time of the K timed steps / 2^30.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3_1500B]
        (N > 1 without a launcher: bench.py starts N ranks under torch.distributed.run itself,
         as a child process, and exits with its code)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Packets shard trivially: every rank checksums its own batch with
no data-path collective ("scaling": "weak"), so `value` is the compute-only
aggregate.  At N>1 the line also carries the §8(e) collective leg measured
separately: `value_gather` = the same steps with one RCCL all-gather of every
rank's u16 results (as uint8, 2 B per packet) per step, and `gather_ms` = the
all-gather alone.  Rank 0 prints one JSON line.

Descriptors (--desc auto): the packed form (rns_csum_batch_packed_dev: u16 length and
u16 seed per packet, one u64 offset per 64 packets; the synthetic batches are packed at
16-byte alignment, and the rows kernel streams them), except the tiny fixed-size c2
batch, which takes the strided form (seeds only; no offsets or lengths at all).

Kernel time: one event pair around the K back-to-back timed launches gives the
per-launch mean (`kernel_avg_us`) from which `roofline.frac` is computed.  A
rocprofv3 --kernel-trace of the same command reproduces it (tools/profile_bench.py
reports the trace's per-dispatch mean and median of the same K launches).  Event
pairs around single launches are NOT used for the figure: each pair measured
≈5 µs above the dispatch rocprof records (profiles/archive/r02/r02_evpair_vs_rocprof_c3_1500B.json);
`--median-launches N` still reports their median as a diagnostic.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip-level table)
METRIC = "GiB/s device-resident Internet checksum, 1500B-packet batches, 1/2/4/8 GPUs"
# --op verify (not the headline): receive verify of IPv4/TCP datagrams (rns_rx_verify_dev)
METRIC_VERIFY = "GiB/s device-resident receive verify (ip.rs:76 + tcp.rs:838-850), IPv4/TCP datagrams"
# --op finalize (not the headline): transmit finalize of NetBuffer chains (rns_tx_fill_chain_dev)
METRIC_FINALIZE = ("GiB/s device-resident transmit finalize (tcp.rs:957-973 + ip.rs:140-160) of NetBuffer chains, "
                   "IPv4/TCP datagrams")


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="c3_1500B")
    p.add_argument("--op", choices=("csum", "verify", "finalize"), default="csum",
                   help="csum (the headline): the batch checksum, per-packet seed, complemented result; verify: "
                        "every packet is an IPv4/TCP datagram (checksums filled by rns_tx_fill_dev, every 1009th "
                        "corrupted) and a step is one rns_rx_verify_dev launch; at N>1 the SURVEY §8(e) leg is an "
                        "all-reduce(sum) of the per-rank rejected-datagram counts instead of the result all-gather; "
                        "finalize: every packet is an outgoing IPv4/TCP datagram held as a NetBuffer chain [40-byte "
                        "head fragment, payload] (heads in a header region) and a step is one rns_tx_fill_chain_dev "
                        "launch (both checksums stored into every head); nothing is exchanged between ranks")
    p.add_argument("--desc", choices=("auto", "64", "32", "packed", "strided"), default="auto",
                   help="descriptor form: 64 = u64 offsets (rns_csum_batch_dev); 32 = u32 offsets "
                        "(rns_csum_batch_dev_off32); packed = u16 lengths + one offset per 64 packets "
                        "(rns_csum_batch_packed_dev); strided = equal-length packets at a fixed stride, no "
                        "offset or length descriptors (rns_csum_batch_strided_dev; fixed-size configs only); "
                        "auto = strided for tiny equal-length packets (c2), packed otherwise (u16 lengths: packets "
                        "above 65535 B take 32 below 4 GiB, else 64)")
    p.add_argument("--shape", default="", help="variant,G,U,max_blocks kernel shape override (tuning)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample duration (single thread)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-host-pipeline", action="store_true", help="skip the PCIe-inclusive extra measurement")
    p.add_argument("--no-gather", action="store_true",
                   help="N>1: skip the compute+all-gather and gather-only legs (value is compute-only either way)")
    p.add_argument("--median-launches", type=int, default=0,
                   help="diagnostic: N extra launches each inside its own event pair, median reported "
                        "(pairs add ~5 us per launch; 0 = skip)")
    p.add_argument("--ramp-s", type=float, default=0.5,
                   help="before the W warmup steps, repeat the step (untimed) for this many seconds so the "
                        "GPU leaves its idle clock state: a 2.9 GB IMIX launch takes 505-550 us in the first "
                        "~0.1 s of load and 493-496 us after it (profiles/archive/r02/r02_clock_ramp.json); 0 = off")
    p.add_argument("--graph", choices=("auto", "on", "off"), default="auto",
                   help="launch the K timed steps (and the warmup) as one HIP graph of K kernel launches "
                        "(torch.cuda.CUDAGraph) alternating over --graph-streams streams: no host launch cost "
                        "between steps, and consecutive (independent) batches overlap one kernel's drain with the "
                        "next one's ramp (c2 13.5 -> 11.8 us per step, c3 -4 %%, c5 -1.5 %%, c4 -1.2 %%: "
                        "profiles/archive/r02/r02_graph_overlap.json); auto = on (every rank, so N=1 and N>1 are timed alike)")
    p.add_argument("--graph-streams", type=int, default=0,
                   help="graph mode: steps alternate over this many streams (independent batches may overlap); "
                        "0 = auto: 3 for tiny packets (mean < 128 B: c2 11.15-11.19 us with 3, 11.2-11.5 with 2 or 4), "
                        "4 for small mixed packets (mean < 1000 B), 2 otherwise (c3 and c4 equal for 2-6; "
                        "profiles/archive/r02/r02_graph_overlap.json, r02_graph_streams.json).  Every stream reads its own batch "
                        "(cache-honest); with that, IMIX gains nothing from 2-4 streams (r03a: 491-498 us per step "
                        "either way; round 2's 405-424 us with 4 streams over ONE arena was partly cache-served)")
    p.add_argument("--shard", default="",
                   help="r/N: one GPU runs rank r's packet-index shard of the config's batch as an N-rank strong-scaling "
                        "run would cut it (make_layout(config, shard=(r, N))) — the per-rank workload of the N-GPU "
                        "point measured on one GPU; the line adds the shard's all-gather payload as a separate leg")
    p.add_argument("--scaling", choices=("auto", "weak", "strong"), default="auto",
                   help="weak: every rank checksums a full batch of the config; strong: the config's batch is "
                        "sharded by packet index across ranks (auto: strong for c5_imix, whose BASELINE.json "
                        "config is one 8M-packet batch over 8 GPUs; weak otherwise)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_{config}.json"))
    args = p.parse_args(argv)
    if args.shape and args.desc in ("32", "packed"):
        p.error("--shape overrides take 64-bit descriptors (--desc 64 or auto)")
    if args.op == "verify" and (args.shape or args.desc not in ("auto", "64", "packed", "strided")):
        p.error("--op verify takes the packed form (rns_rx_verify_packed_dev), the strided form "
                "(rns_rx_verify_strided_dev; auto for tiny datagrams in fixed-size slots) or 64-bit descriptors "
                "(rns_rx_verify_dev) and the receive kernel's own shape")
    if args.op == "finalize" and (args.shape or args.desc != "auto"):
        p.error("--op finalize takes the chain form (rns_tx_fill_chain_dev) and its kernel's own shape")
    args.shard_rw = None
    if args.shard:
        try:
            r_, n_ = (int(x) for x in args.shard.split("/"))
        except ValueError:
            p.error("--shard takes r/N, e.g. 7/8")
        if not (n_ >= 1 and 0 <= r_ < n_):
            p.error("--shard r/N needs 0 <= r < N")
        args.shard_rw = (r_, n_)
    return args


def auto_graph_streams(mean_len: float, step_bytes: float = 0.0) -> int:
    """Streams the graph-mode timed steps alternate over (profiles/archive/r02/r02_graph_streams.json, and
    r03/r04 with every concurrently running step reading its own batch): 3 for tiny packets, 2 for
    MTU and jumbo batches and for small mixed ones, 1 for a small-mixed step of a GiB or more
    (session r04h, rows kernel: 2^23 IMIX 452.5 / 462.0 / 468.6 / 469.7 us per step at 1 / 2 / 3 / 4
    streams, its 2^20 shard 58.8 / 58.3 / - / 60.4; c3 229.6 / 224.4 / 228.0)."""
    if mean_len < 128:
        return 3
    if mean_len < 1000 and step_bytes >= (1 << 30):
        return 1
    return 2


# ---------------------------------------------------------------------------
# distributed plumbing (one process per GPU; gloo when run on CPU in tests)
# ---------------------------------------------------------------------------
class Dist:
    def __init__(self, backend: str | None = None):
        import torch
        import torch.distributed as dist
        self.dist = dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        # Rehearsal knobs (never set by the driver): RNS_BENCH_BACKEND=gloo and
        # RNS_BENCH_DEVICE=0 run N ranks on ONE GPU to exercise the N>1 path.
        if os.environ.get("RNS_BENCH_DEVICE") is not None:
            self.local_rank = int(os.environ["RNS_BENCH_DEVICE"])
        backend = backend or os.environ.get("RNS_BENCH_BACKEND") or None
        self.enabled = self.world > 1
        if self.enabled:
            backend = backend or ("nccl" if torch.cuda.is_available() else "gloo")
            if backend == "nccl":
                torch.cuda.set_device(self.local_rank)  # before RCCL binds its communicator
        if self.enabled and not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group(backend=backend)
        self.backend = dist.get_backend() if self.enabled else None
        self.torch = torch

    def barrier(self):
        if self.enabled:
            if self.backend == "nccl":
                self.dist.barrier(device_ids=[self.local_rank])
            else:
                self.dist.barrier()

    def _reduce(self, x: float, op) -> float:
        if not self.enabled:
            return x
        dev = f"cuda:{self.local_rank}" if self.backend == "nccl" else "cpu"
        t = self.torch.tensor([x], dtype=self.torch.float64, device=dev)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.MAX)

    def sum(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.SUM)

    def close(self):
        if self.enabled and self.dist.is_initialized():
            self.dist.destroy_process_group()


def clock_ramp(engine, seconds: float, step=None, graph=None) -> int:
    """Untimed load for `seconds` of wall time before the warmup steps (DVFS: the chip
    runs its first ~0.1 s of load at lower clocks).  Returns the steps run."""
    step = step or engine.step
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(8):
            if graph is not None:
                graph.replay()
            else:
                step()
        engine.sync()
        n += 8
    return n


def timed_loop(engine, dist: Dist, steps: int, warmup: int, step=None, graph=None) -> dict:
    """W untimed steps, then exactly K steps bracketed by sync + barrier on both
    sides; wall time is the max over ranks.  Device time per launch = one pair of
    events on the launch stream around the K back-to-back launches, / K (events
    between launches would insert ~10 µs gaps: see DESIGN.md, measurement).
    `step` (default engine.step) is what one step runs; `graph` (optional) = a
    captured graph of exactly K steps, replayed once for the timed region (and
    once untimed as warmup when W > 0)."""
    step = step or engine.step
    if graph is not None:
        if warmup:
            graph.replay()
    else:
        for _ in range(warmup):
            step()
    engine.sync()
    dist.barrier()
    engine.sync()
    t0 = time.perf_counter()
    engine.begin_timing()
    if graph is not None:
        graph.replay()
    else:
        for _ in range(steps):
            step()
    engine.end_timing(steps)
    engine.sync()
    dist.barrier()
    engine.sync()
    elapsed = time.perf_counter() - t0
    return {"elapsed_s": dist.max(elapsed), "local_elapsed_s": elapsed,
            "kernel_ms": engine.kernel_ms()}


class ResultGather:
    """SURVEY §8(e)'s collective: every rank's per-packet u16 results all-gathered
    to every rank, sent as uint8 (RCCL has no 16-bit unsigned type: ncclUint8 with
    2·n bytes per rank; gloo has no int16 either).  Ranks with fewer packets (strong
    scaling of a batch that does not divide evenly) pad to the largest shard; the
    counts are all-gathered once so `results()` rebuilds the global order."""

    def __init__(self, dist: Dist, n_local: int, device):
        import torch
        self.dist, self.torch = dist, torch
        self.n_local = int(n_local)
        self.n_max = int(dist.max(float(n_local)))
        self.counts = [int(c) for c in self._counts()]
        # gloo (CPU tests, one-GPU rehearsals) moves host tensors: stage through CPU there
        self.host_staged = dist.enabled and dist.backend != "nccl" and torch.device(device).type == "cuda"
        bufdev = "cpu" if self.host_staged else device
        self.send = torch.zeros(2 * self.n_max, dtype=torch.uint8, device=bufdev)
        self.recv = torch.empty(2 * self.n_max * dist.world, dtype=torch.uint8, device=bufdev)

    def _counts(self):
        if not self.dist.enabled:
            return [self.n_local]
        t = self.torch.tensor([self.n_local], dtype=self.torch.int64,
                              device=self.send_device() if self.dist.backend == "nccl" else "cpu")
        out = [self.torch.zeros_like(t) for _ in range(self.dist.world)]
        self.dist.dist.all_gather(out, t)
        return [int(x.item()) for x in out]

    def send_device(self):
        return f"cuda:{self.dist.local_rank}"

    @property
    def bytes_per_rank(self) -> int:
        return 2 * self.n_max

    def __call__(self, out_u16):
        src = out_u16.view(self.torch.uint8)
        if self.host_staged:
            src = src.cpu()
        if self.n_local == self.n_max:
            send = src
        else:
            self.send[:src.numel()].copy_(src)
            send = self.send
        if self.dist.enabled:
            self.dist.dist.all_gather_into_tensor(self.recv, send)
        else:
            self.recv.copy_(send)
        return self.recv

    def results(self):
        """The gathered u16 results of all ranks, rank order, padding removed (numpy)."""
        import numpy as np
        raw = self.recv.cpu().numpy().view(np.uint16).reshape(self.dist.world, self.n_max)
        return np.concatenate([raw[r, :c] for r, c in enumerate(self.counts)])


class BadCountReduce:
    """SURVEY §8(e) in verify mode: the per-rank count of rejected datagrams (status
    without RNS_RX_ACCEPT), summed over ranks with one all-reduce (RCCL on the device
    under nccl; gloo moves a host tensor).  The count is reduced on the device first,
    so the collective moves 8 bytes per rank."""

    ACCEPT = 0x40  # RNS_RX_ACCEPT

    def __init__(self, dist: Dist, device):
        import torch
        self.dist, self.torch = dist, torch
        self.host_staged = dist.enabled and dist.backend != "nccl"
        self.device = "cpu" if self.host_staged else device
        self.total = torch.zeros(1, dtype=torch.int64, device=self.device)

    def __call__(self, status):
        torch = self.torch
        cnt = ((status & self.ACCEPT) == 0).sum(dtype=torch.int64).view(1)
        if self.host_staged:
            cnt = cnt.cpu()
        self.total.copy_(cnt)
        if self.dist.enabled:
            self.dist.dist.all_reduce(self.total)
        return self.total


class OverlappedGather:
    """The §8(e) all-gather of step i's results overlapped with step i+1's compute:
    the kernel of step i goes to the launch stream, its all-gather to a side stream that waits
    only for that kernel; the next step's kernel (an independent batch) starts at once.  Before
    a kernel rewrites a batch's results it waits for the gather that still reads them (batches
    rotate, so with two or more batches one gather is always in flight under the next kernel).
    Under gloo (CPU tests, host-staged) the gather is synchronous: the same steps, no overlap."""

    def __init__(self, engine):
        torch = engine.torch
        self.engine, self.torch = engine, torch
        dev = getattr(engine, "device", None)
        self.side = torch.cuda.Stream(device=dev) if dev is not None and dev.type == "cuda" else None
        self.pending = {}  # batch index -> event: its last gather has finished reading its results

    def __call__(self):
        eng, torch = self.engine, self.torch
        i = eng.k % len(eng.batches)
        if self.side is None:
            eng.step()
            eng.gather()
            return
        ev = self.pending.get(i)
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)
        eng.step()
        ready = torch.cuda.Event()
        ready.record()
        with torch.cuda.stream(self.side):
            self.side.wait_event(ready)
            eng.gather()
            done = torch.cuda.Event()
            done.record(self.side)
        self.pending[i] = done


def rank_parity(engine, threads: int = 8) -> dict:
    """This rank's own check of the GPU results: every packet of its first batch (the batch
    the timed steps, and the gather legs after them, left results in) against the oracle's
    restatement of util.rs:88-106, on the host.  Test infrastructure, after all timing."""
    import numpy as np

    from oracle.oracle import get_oracle
    b = engine.batches[0]
    lay = b.layout
    arena = b.arena[:lay.arena_bytes].cpu().numpy()
    want = get_oracle().batch(arena, lay.off, lay.length, lay.seed, complement=True, threads=threads, check=False)
    got = b.out.view(engine.torch.int16).cpu().numpy().view(np.uint16)
    return {"bit_exact": bool(np.array_equal(got[:lay.n], want)), "packets": int(lay.n)}


# ---------------------------------------------------------------------------
# GPU engine: the product path
# ---------------------------------------------------------------------------
class GpuEngine:
    def __init__(self, config: str, rank: int, local_rank: int, shape=None, steps: int = 0, world: int = 1,
                 strong: bool = False, compact="64", op: str = "csum", min_batches: int = 1, shard=None):
        import torch

        from rustnetworkstack_amd.workloads import DATA_SEED, DeviceBatch, make_layout
        self.torch = torch
        self.device = torch.device(f"cuda:{local_rank}")
        torch.cuda.set_device(self.device)

        if shard is not None:  # --shard r/N on one process: rank r of an N-rank strong-scaling run
            rank, world, strong = shard[0], shard[1], True

        def layout(r):
            if strong:  # this rank's packet-index shard of the one batch (same sizes and seeds on every rank)
                lay = make_layout(config, shard=(rank, world))
                lay.data_seed = DATA_SEED + 0x1000 * rank + r
                return lay
            # weak scaling: every rank owns a full batch of the config, with its own bytes
            return make_layout(config, data_seed=DATA_SEED + 0x1000 * rank + r)

        self.op = op
        if op == "finalize":
            self._init_finalize(config, rank, world, strong, min_batches)
            return
        self.layout = layout(0)
        small = self.layout.arena_bytes < (512 << 20)
        # Rotating batches, each with its own bytes (cache honesty):
        #  * batches that fit the 256 MiB Infinity Cache rotate so each step reads cold bytes
        #    (>= 768 MiB between two reads of one batch);
        #  * at least one batch per graph stream (min_batches), so no two steps that may run
        #    at the same time read the same arena — a follower dispatch a few tens of us
        #    behind another over the SAME bytes would be served from the Infinity Cache.
        nrot = max(1, -(-(768 << 20) // max(self.layout.arena_bytes, 1))) if small else 1
        nrot = max(nrot, int(min_batches))
        self.batches = [DeviceBatch(self.layout if r == 0 else layout(r), self.device) for r in range(nrot)]
        self.shape = shape
        form = {True: "32", False: "64"}.get(compact, compact)
        if form == "auto":
            small = self.layout.arena_bytes + 16 < 2 ** 32
            # the packed form takes u16 lengths (an IP datagram's length field)
            packable = self.layout.n == 0 or int(self.layout.length.max()) <= 0xFFFF
            # tiny equal-length packets at a fixed stride (c2): the strided form, whose offsets need no
            # descriptor load before a wave's first data load (isolated 13.68 -> 12.98 us, r03h)
            tiny_fixed = op == "csum" and self.layout.mean_len < 128 and self.batches[0].stride() is not None
            form = "64" if shape is not None else ("strided" if tiny_fixed else "packed" if packable else
                                                   ("32" if small else "64"))
        if op == "verify":  # packed receive arena (16-byte-aligned datagrams): the stream kernel; else 64-bit
            from rustnetworkstack_amd.workloads import make_verify_batch
            aligned = self.layout.n == 0 or int(self.layout.off[0]) % 16 == 0
            # datagrams in fixed-size slots (c2's 64-byte ACKs): the strided receive entry, whose
            # lanes load their datagrams beside their lengths (no block offset, no scan)
            slots = self.layout.mean_len < 128 and self.batches[0].stride() is not None
            form = ("strided" if (compact == "auto" and slots) or compact == "strided" else
                    "packed" if compact in ("auto", "packed") and aligned else "64")
            for b in self.batches:
                make_verify_batch(b)
                if form in ("packed", "strided"):
                    b.launcher(packed=True)  # uploads blk_off / len16
        self.form = form
        self.compact = form == "32"
        self.packed = form == "packed"
        self.strided = form == "strided"
        self.verify_packed = op == "verify" and self.packed
        self.verify_strided = op == "verify" and self.strided
        for b in self.batches:  # bind every rotating batch (and upload its descriptors) before any timing
            if op == "csum":
                b.launcher(complement=True, shape=shape, compact=self.compact, packed=self.packed,
                     strided=self.strided)
        self.k = 0
        self.used = set()  # indices of the rotating batches some step has run on
        self.last = self.batches[0]
        self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        self.timed = 0
        self.gatherer = None
        torch.cuda.synchronize()

    def _init_finalize(self, config, rank, world, strong, min_batches):
        """--op finalize: rotating transmit batches held as NetBuffer chains (workloads.TxChainBatch)."""
        torch = self.torch
        from rustnetworkstack_amd.workloads import DATA_SEED, TxChainBatch

        def batch(r):
            seed = DATA_SEED + 0x1000 * rank + r
            return TxChainBatch(config, self.device, data_seed=seed, shard=(rank, world) if strong else (0, 1))

        b0 = batch(0)
        self.layout = b0.layout
        # Cache honesty for the transmit side: a finalize reads and rewrites its header region (40 B per
        # datagram, 42 MB for c3), small enough to stay in the 256 MB Infinity Cache from one launch to
        # the next on the same arena (c3: 254.8 us per launch on one arena, 275.8-277.6 over two, r06o /
        # r06p).  Batches rotate until their header regions add up to >= 768 MiB, so every launch meets
        # cold heads as well as cold payloads (HBM for the rotation capped at 48 GB).
        head_bytes = TxChainBatch.HEAD * max(self.layout.n, 1)
        nrot = max(1, -(-(768 << 20) // head_bytes))
        nrot = min(nrot, max(1, (48 << 30) // max(self.layout.arena_bytes, 1)))
        nrot = max(nrot, int(min_batches))
        self.batches = [b0] + [batch(r) for r in range(1, nrot)]
        self.shape = None
        self.form = "chain"
        self.compact = self.packed = self.strided = False
        self.verify_packed = self.verify_strided = False
        self.k = 0
        self.used = set()
        self.last = self.batches[0]
        self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        self.timed = 0
        self.gatherer = None
        torch.cuda.synchronize()

    @property
    def n(self):
        return self.layout.n

    @property
    def payload_bytes(self):
        return self.layout.payload_bytes

    def _verify_call(self, b):
        from rustnetworkstack_amd.batch import rx_verify, rx_verify_packed, rx_verify_strided
        from rustnetworkstack_amd.workloads import LOCAL4, LOCAL6
        if self.verify_strided:
            if not hasattr(b, "slot_stride"):
                b.slot_stride = b.stride()[:2]  # (first_off, stride), computed once per batch
            first, stride = b.slot_stride
            return lambda: rx_verify_strided(b.arena, stride, b.len16, LOCAL4, LOCAL6, first_off=first, status=b.status)
        if self.verify_packed:
            return lambda: rx_verify_packed(b.arena, b.blk_off, b.len16, LOCAL4, LOCAL6, status=b.status)
        return lambda: rx_verify(b.arena, b.off, b.length, LOCAL4, LOCAL6, status=b.status)  # current stream

    def _finalize_call(self, b):
        from rustnetworkstack_amd.batch import tx_fill_chain
        return lambda: tx_fill_chain(b.arena, b.d_off, b.d_len, b.d_first, status=b.status)  # current stream

    def step(self):
        b = self.batches[self.k % len(self.batches)]
        self.used.add(self.k % len(self.batches))
        self.k += 1
        if self.op == "finalize":
            self._finalize_call(b)()
        elif self.op == "verify":
            self._verify_call(b)()
        else:
            b.launcher(complement=True, shape=self.shape, compact=self.compact, packed=self.packed,
                     strided=self.strided)()  # one ctypes call
        self.last = b

    def capture(self, steps: int, streams: int = 1):
        """K steps captured as one HIP graph (K kernel launches, rotating batches in
        step order), each launcher re-bound to its capture stream.  streams > 1: step
        i goes to stream i % streams (forked from and joined back to the capture
        stream), so consecutive steps — independent batches — may overlap on the
        device: one kernel's ramp-up under the previous one's drain."""
        torch = self.torch
        if self.op == "csum":
            fns = [b.rebind(complement=True, shape=self.shape, compact=self.compact, packed=self.packed,
                     strided=self.strided)
                   for b in self.batches]
            del fns  # (bound once outside the capture: descriptor uploads happen here, not inside it)
        side = [torch.cuda.Stream(device=self.device) for _ in range(max(streams, 1) - 1)]
        self.sync()
        g = torch.cuda.CUDAGraph()
        # thread_local: a process group's watchdog thread may query events while this thread captures
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            cap = torch.cuda.current_stream()
            for s_ in side:
                s_.wait_stream(cap)
            lanes = [cap] + side
            for i in range(steps):
                b = self.batches[i % len(self.batches)]
                self.used.add(i % len(self.batches))
                with torch.cuda.stream(lanes[i % len(lanes)]):
                    if self.op == "finalize":
                        self._finalize_call(b)()
                    elif self.op == "verify":
                        self._verify_call(b)()
                    else:
                        b.rebind(complement=True, shape=self.shape, compact=self.compact, packed=self.packed,
                     strided=self.strided)()
            for s_ in side:
                cap.wait_stream(s_)
        self.sync()
        self.last = self.batches[(steps - 1) % len(self.batches)]
        return g

    def gather(self):
        """The all-gather of the results of the batch the last step checksummed."""
        return self.gatherer(self.last.out)

    def step_and_gather(self):
        self.step()
        self.gather()

    def reduce_bad(self):
        """Verify mode: the all-reduce of the rejected-datagram counts of the last step's batch."""
        return self.reducer(self.last.status)

    def step_and_reduce(self):
        self.step()
        self.reduce_bad()

    def verified_batches(self):
        """The rotating batches some step has verified (K < the rotation leaves some untouched)."""
        return [self.batches[i] for i in sorted(self.used)]

    def bad_count(self) -> int:
        """Rejected datagrams in the verified batches after the timed steps."""
        return sum(int(((b.status & BadCountReduce.ACCEPT) == 0).sum().item()) for b in self.verified_batches())

    def expected_bad(self) -> int:
        return sum(b.expected_bad for b in self.verified_batches())

    def per_launch_us(self, count: int) -> list:
        """`count` launches, each bracketed by its own event pair on the launch stream
        (the rocprof-style per-dispatch duration; the gaps these events put BETWEEN
        launches are outside every pair)."""
        torch = self.torch
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(count)]
        self.sync()
        for a, b in evs:
            a.record()
            self.step()
            b.record()
        self.sync()
        return [1e3 * a.elapsed_time(b) for a, b in evs]

    def sync(self):
        self.torch.cuda.synchronize()

    def begin_timing(self):
        self.ev[0].record()  # current stream = the stream every launch goes to

    def end_timing(self, steps: int):
        self.ev[1].record()
        self.timed = steps

    def kernel_ms(self) -> float:
        if not self.timed:
            return float("nan")
        return self.ev[0].elapsed_time(self.ev[1]) / self.timed

    def kernel_name(self) -> str:
        from rustnetworkstack_amd import _lib
        if self.op == "finalize":
            return ("csum_txrows_kernel FIN (rns_tx_fill_chain_dev: one wave per 64 chains streams the packed "
                    "payloads as 1 KiB rows, each owner parses its head, and the wave writes its back-to-back heads "
                    "back as whole chunks from LDS)")
        if self.op == "verify":
            if self.verify_strided:
                return ("csum_strided_rx_kernel (rns_rx_verify_strided_dev: datagrams in fixed-size slots; a lane "
                        "quad per datagram loads its first 64 bytes beside the lengths, one 64-datagram batch per wave)")
            if self.verify_packed:
                b = self.batches[0]
                if (b.arena.numel() // max(self.layout.n, 1)) <= 128:
                    return ("csum_stream_kernel (rns_rx_verify_packed_dev, an arena of ACK-sized datagrams: "
                            "owners load their datagrams whole)")
                return ("csum_rows_rx_kernel (rns_rx_verify_packed_dev: 1 KiB rows; owners load their headers "
                        "a group of rows ahead)")
            return "csum_mixed_kernel<RX> (rns_rx_verify_dev: class-sorted data pass + header stash)"
        mean = self.layout.mean_len
        if getattr(self, "strided", False):
            st = self.batches[0].stride()
            if st is not None and 0 < st[2] <= 64 and st[0] % 16 == 0 and st[1] % 16 == 0:
                return ("csum_strided_tiny_kernel (rns_csum_batch_strided_dev, packets <= 64 B at 16-byte-aligned "
                        "starts: 4 rows of 16 packets x 4 chunks per 64-packet batch, two batches per wave)")
        if self.packed and self.layout.n and int(self.layout.off[0]) % 16 == 0 and mean > 112:
            return ("csum_rows_kernel (packed form, 16-byte-aligned packets: one wave streams each 64-packet "
                    "block as 1 KiB rows; owners capture two region prefixes and sum their own end chunk)")
        return _lib.load().rns_csum_shape_name(int(round(self.layout.mean_len))).decode()

    def out_sample(self, count: int):
        import numpy as np
        return self.batches[0].out[:count].view(self.torch.int16).cpu().numpy().view(np.uint16)


# ---------------------------------------------------------------------------
# CPU baseline: the reference's algorithm (oracle/ restatement), host cores
# ---------------------------------------------------------------------------
def cpu_grant() -> dict:
    """CPUs this process may actually use: the affinity mask, capped by a cgroup CPU
    quota when one is set (a gpurun box shows the whole machine in its mask but
    grants a share of it through cpu.max)."""
    visible = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                parts = f.read().split()
        except OSError:
            continue
        if path.endswith("cpu.max"):
            if parts and parts[0] != "max":
                quota = float(parts[0]) / float(parts[1] if len(parts) > 1 else 100000)
        else:
            try:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    period = float(f.read().strip())
                q = float(parts[0])
                if q > 0:
                    quota = q / period
            except (OSError, ValueError, IndexError):
                pass
        break
    threads = visible if quota is None else max(1, min(visible, int(quota + 0.5)))
    return {"visible": visible, "quota_cpus": quota, "threads": threads}


def cpu_baseline(engine: GpuEngine, seconds: float, sample_min_bytes: int = 512 << 20,
                 sample_max_bytes: int = 3 << 30) -> dict:
    """Times the literal C restatement of util.rs:88-106 (oracle/csum_oracle.c,
    gcc -O3, baseline x86-64 — gcc auto-vectorises its loop; it is not the Rust
    build, which this image cannot compile) on the same batches the GPU reads:
    whole batches, at least `sample_min_bytes` (larger than the host's L3, so the
    CPU reads DRAM like the GPU reads HBM) and at most `sample_max_bytes`.  Run on
    every CPU the process is granted (`value`) and on one thread (`value_1_thread`).
    Also checks the GPU results of every sampled packet against it."""
    import numpy as np

    from oracle.oracle import get_oracle
    orc = get_oracle()
    grant = cpu_grant()
    samples, total = [], 0
    for b in engine.batches:  # rotating batches (c2) each bring their own bytes
        lay = b.layout
        if samples and total + lay.arena_bytes > sample_max_bytes:
            break
        arena = b.arena[:lay.arena_bytes].cpu().numpy()
        samples.append((b, arena, lay))
        total += lay.payload_bytes
        if total >= sample_min_bytes:
            break
    sample_bytes = sum(lay.payload_bytes for _, _, lay in samples)
    arena_bytes = sum(lay.arena_bytes for _, _, lay in samples)

    def one_pass(threads: int):
        return [orc.batch(arena, lay.off, lay.length, lay.seed, complement=True, threads=threads, check=False)
                for _, arena, lay in samples]

    def rate(threads: int, budget: float):
        passes, t0 = 0, time.perf_counter()
        while True:
            res = one_pass(threads)
            passes += 1
            dt = time.perf_counter() - t0
            if dt >= budget:
                return sample_bytes * passes / dt / 2 ** 30, res, passes, dt

    vmt, res, passes_mt, dt_mt = rate(grant["threads"], max(seconds / 2, 1.0))
    v1, res1, passes1, dt1 = rate(1, seconds)
    exact = all(np.array_equal(b.out.view(engine.torch.int16).cpu().numpy().view(np.uint16), r)
                for (b, _, _), r in zip(samples, res))
    exact = exact and all(np.array_equal(a, c) for a, c in zip(res, res1))
    ns_zero = orc.time_ones_comp(bytes(512), 2_000_000)
    ns_ff = orc.time_ones_comp(b"\xff" * 512, 2_000_000)
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((ln_.split(":", 1)[1].strip() for ln_ in f if ln_.startswith("model name")), "")
    except OSError:
        pass
    n_pk = sum(lay.n for _, _, lay in samples)
    return {
        "value": round(vmt, 3), "unit": "GiB/s", "cores": grant["threads"], "kind": "port",
        "sample": f"{len(samples)} whole {engine.layout.name} batch(es): {n_pk} packets, {sample_bytes} B of payload "
                  f"in {arena_bytes} B of arena (> host L3: read from DRAM); {grant['threads']} threads x "
                  f"{passes_mt} passes in {dt_mt:.1f} s, 1 thread x {passes1} passes in {dt1:.1f} s",
        "what": "gcc -O3 restatement of util.rs:88-106 (oracle/csum_oracle.c, baseline x86-64; gcc auto-vectorises "
                "the loop), not the Rust build (no cargo/rustc in the image); packets partitioned by index over threads",
        "value_1_thread": round(v1, 3),
        "threads_granted": grant["threads"], "host_cpus_visible": grant["visible"],
        "cgroup_cpu_quota": grant["quota_cpus"],
        "util_bench_ns_per_iter": {"compute_ones_comp_512B_zeros": round(ns_zero, 2),
                                   "compute_ones_comp_512B_0xff": round(ns_ff, 2)},
        "host_cpu": cpu_model,
        "gpu_sample_bit_exact": bool(exact),
    }


def finalize_parity(engine: GpuEngine, threads: int = 8) -> dict:
    """--op finalize: the GPU's finalized heads against the C restatement of the reference's transmit
    path (oracle_tx_chain_fill: tcp.rs:957-973 + ip.rs:140-160 over [head[20..], payload]) run on a
    host copy of the same arena.  Both fields count as zero, so finalizing the GPU's output again
    must reproduce it byte for byte; statuses must agree."""
    import numpy as np

    from oracle.oracle import get_oracle
    b = engine.batches[0]
    lay = b.layout
    host = b.arena.cpu().numpy()
    gpu_st = b.status.cpu().numpy()
    cpu = host.copy()
    st = get_oracle().tx_chain_fill(cpu, lay.frag_off, lay.frag_len, lay.first, threads=threads)
    return {"bit_exact": bool(np.array_equal(cpu, host) and np.array_equal(st, gpu_st)),
            "packets": int(lay.n), "arena": cpu, "layout": lay}


def cpu_baseline_finalize(engine: GpuEngine, seconds: float) -> dict:
    """--op finalize's CPU baseline: oracle_tx_chain_fill (gcc -O3; the reference's per-datagram
    transmit path: compute_pseudo_header_checksum + compute_buffer_ones_comp over the chain + the
    IPv4 header's compute_checksum + two set_be16) over rank 0's first batch, on every granted
    thread and on one; the GPU's heads are checked against it in the same pass."""
    grant = cpu_grant()
    par = finalize_parity(engine, threads=grant["threads"])
    cpu, lay = par.pop("arena"), par.pop("layout")
    from oracle.oracle import get_oracle
    orc = get_oracle()

    def rate(threads: int, budget: float):
        passes, t0 = 0, time.perf_counter()
        while True:
            orc.tx_chain_fill(cpu, lay.frag_off, lay.frag_len, lay.first, threads=threads)
            passes += 1
            dt = time.perf_counter() - t0
            if dt >= budget:
                return lay.payload_bytes * passes / dt / 2 ** 30, passes, dt

    vmt, passes_mt, dt_mt = rate(grant["threads"], max(seconds / 2, 1.0))
    v1, passes1, dt1 = rate(1, seconds)
    return {
        "value": round(vmt, 3), "unit": "GiB/s", "cores": grant["threads"], "kind": "port",
        "sample": f"rank 0's first {engine.layout.name} chain batch: {lay.n} datagrams, {lay.payload_bytes} B in "
                  f"{lay.arena_bytes} B of arena (> host L3); {grant['threads']} threads x {passes_mt} passes in "
                  f"{dt_mt:.1f} s, 1 thread x {passes1} passes in {dt1:.1f} s",
        "what": "gcc -O3 restatement of the transmit path (oracle/csum_oracle.c oracle_tx_chain_fill: tcp.rs:957-973, "
                "udp.rs:151-171, icmp.rs:87-112, ip.rs:140-160 over buf.rs's head fragment), not the Rust build; "
                "datagrams partitioned by index over threads",
        "value_1_thread": round(v1, 3),
        "threads_granted": grant["threads"], "host_cpus_visible": grant["visible"],
        "cgroup_cpu_quota": grant["quota_cpus"],
        "gpu_sample_bit_exact": par["bit_exact"],
    }


def host_pipeline_rate(engine: GpuEngine) -> dict:
    """PCIe-inclusive rate: the same batch from pinned host memory through
    rns_csum_batch_host (chunked H2D + kernel + D2H of results on 3 streams).
    Reported beside `value`, never as it."""
    from rustnetworkstack_amd.batch import HostBatcher, PinnedBuffer
    lay = engine.layout
    pb = PinnedBuffer(lay.arena_bytes)
    pb.array[:] = engine.batches[0].arena[:lay.arena_bytes].cpu().numpy()
    hb = HostBatcher(device=engine.device.index or 0, chunk_bytes=64 << 20, nstreams=3)
    hb.run(pb.array, lay.off, lay.length, lay.seed, complement=True)  # warm-up
    reps, t0 = 3, time.perf_counter()
    for _ in range(reps):
        out = hb.run(pb.array, lay.off, lay.length, lay.seed, complement=True)
    dt = (time.perf_counter() - t0) / reps
    import numpy as np
    exact = bool(np.array_equal(out, engine.out_sample(lay.n)))
    hb.close()
    pb.free()
    return {"value": round(lay.payload_bytes / dt / 2 ** 30, 2), "unit": "GiB/s", "ms_per_batch": round(dt * 1e3, 3),
            "path": "pinned host arena -> 64 MiB chunks H2D -> kernel -> D2H of 2 B results, 3 streams",
            "matches_device_resident": exact}


def shard_leg(engine, args) -> dict:
    """--shard r/N: what the N-rank strong-scaling run adds to this rank's compute — the
    SURVEY §8(e) all-gather of the u16 results (2 B per packet of the WHOLE batch land on
    every rank).  A one-GPU box has no peer for the RCCL all-gather itself, so this leg
    reports its payload and the time of a local HBM copy of the same bytes (a floor for
    writing them; the xGMI collective is what the driver's N-GPU run times as gather_ms)."""
    import torch

    from rustnetworkstack_amd.workloads import make_layout
    r_, n_ = args.shard_rw
    whole = make_layout(args.config)
    recv_bytes = 2 * whole.n
    per_rank = 2 * (-(-whole.n // n_))
    src = torch.empty(recv_bytes, dtype=torch.uint8, device=engine.device)
    dst = torch.empty_like(src)
    dst.copy_(src)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize()
    copy_us = 1e3 * e0.elapsed_time(e1) / reps
    return {"rank": r_, "world": n_, "packets": engine.n, "payload_bytes": engine.payload_bytes,
            "batch_packets": whole.n, "batch_payload_bytes": whole.payload_bytes,
            "share_of_batch_bytes": round(engine.payload_bytes / whole.payload_bytes, 5),
            "gather": {"collective": "all_gather of uint8 results (2 B per packet), run by the N-GPU driver bench",
                       "bytes_sent_per_rank": per_rank, "bytes_received_per_rank": per_rank * (n_ - 1),
                       "bytes_resident_after_per_rank": recv_bytes,
                       "local_copy_us": round(copy_us, 2),
                       "local_copy_what": f"device-to-device copy of {recv_bytes} B in this GPU's HBM "
                                          "(no peer GPU on a 1-GPU box), mean of 20"}}


class _NoDist:
    """Single-process stand-in for Dist (the isolated re-measurement needs no barrier)."""
    enabled = False

    def barrier(self):
        pass

    def max(self, x):
        return x


def load_traffic(path: str, config: str):
    path = path.format(config=config)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        t = json.load(f)
    return t


def load_traffic_finalize(config: str):
    """HBM bytes per finalize launch from the PMC passes over the same kernel and layout
    (profiles/r06_pmc_write_tx_chain.json: FETCH_SIZE (gfx950-corrected) + WRITE_SIZE)."""
    path = os.path.join(ROOT, "profiles", "r06_pmc_write_tx_chain.json")
    try:
        with open(path) as f:
            d = json.load(f)
        k = d[config]["per_kernel"]["tx_chain"]
        v = next(iter(k.values()))
        return {"hbm_bytes_per_launch": int(v["fetch_bytes_corrected"] + v["write_bytes"]),
                "source": f"{os.path.relpath(path, ROOT)} (session {d.get('session')}: rocprofv3 --pmc FETCH_SIZE / "
                          "WRITE_SIZE / TCC_EA0_WRREQ, separate passes)"}
    except (OSError, KeyError, ValueError, StopIteration):
        return None


def launch_ranks(args, argv) -> int:
    """`--gpus N` (N > 1) without a torch.distributed launcher: start N ranks of this
    same script under `torch.distributed.run` as a CHILD process (never an exec: no
    GPU has been touched yet, but the child must own the ranks, not this process),
    relay its output and return its exit code.  The child sees WORLD_SIZE == N, so
    its main() runs the ranks' path."""
    import subprocess
    script = os.path.abspath(sys.argv[0]) if sys.argv and sys.argv[0].endswith(".py") else os.path.abspath(__file__)
    # the c10d rendezvous on port 0: the launcher's own store picks a free port (no probe-then-
    # release race with another process), on 127.0.0.1 (the hostname may not resolve)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--rdzv-backend=c10d", "--rdzv-endpoint=127.0.0.1:0", "--local-addr=127.0.0.1", script] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    print(f"bench.py: --gpus {args.gpus} without WORLD_SIZE: launching {args.gpus} ranks via torch.distributed.run",
          file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def check_world(args) -> None:
    """--gpus must agree with the launcher's WORLD_SIZE (a silent N=1 line for an N-GPU
    request would be a wrong measurement)."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None and int(world) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: the launcher and --gpus disagree")


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and os.environ.get("WORLD_SIZE") is None:
        rc = launch_ranks(args, argv)  # before any torch.cuda / HIP call in this process
        if rc != 0:
            raise SystemExit(rc)
        return None
    check_world(args)
    dist = Dist()
    shape = tuple(int(x) for x in args.shape.split(",")) if args.shape else None
    strong = args.scaling == "strong" or (args.scaling == "auto" and args.config == "c5_imix")
    verify = args.op == "verify"
    finalize = args.op == "finalize"
    if verify:
        args.no_cpu_baseline = args.no_host_pipeline = True  # the headline's CPU legs; not this mode's
    if finalize:
        args.no_host_pipeline = args.no_gather = True  # nothing crosses ranks; the pipeline is TxChainPipeline
    if args.shard_rw is not None and dist.world > 1:
        raise SystemExit("--shard r/N is a one-process measurement of one rank's shard (use --scaling strong at N>1)")
    if args.shard_rw is not None:
        strong = True
    if args.graph_streams <= 0 and args.op == "finalize":
        # two finalizes at once slow each other (c3: 285.9 us per step over 2 streams against 277.6
        # one after another, both on cold arenas, r06o): the transmit kernels run on one stream
        args.graph_streams = 1
    if args.graph_streams <= 0:
        from rustnetworkstack_amd.workloads import make_layout
        from rustnetworkstack_amd.workloads import CONFIGS
        mean = make_layout(args.config, n=4096).mean_len
        per_rank = CONFIGS[args.config]["n"] if args.config in CONFIGS else 0
        if strong:  # the rank's shard of the config's one batch
            per_rank = -(-per_rank // (args.shard_rw[1] if args.shard_rw is not None else dist.world))
        args.graph_streams = auto_graph_streams(mean, per_rank * mean)
    # min_batches is a hint for the graph path (one batch per graph stream); an engine
    # that is not on a GPU ignores it, and the graph decision follows the engine's device
    engine = GpuEngine(args.config, dist.rank, dist.local_rank, shape=shape, steps=args.steps, world=dist.world,
                       strong=strong, compact=args.desc, op=args.op,
                       min_batches=args.graph_streams if args.graph != "off" else 1, shard=args.shard_rw)
    on_gpu = getattr(engine, "device", None) is not None and engine.device.type == "cuda"
    if args.graph == "on" and not on_gpu:
        raise SystemExit("bench.py: --graph on needs the GPU engine")
    use_graph = args.graph == "on" or (args.graph == "auto" and on_gpu)
    graph = engine.capture(args.steps, args.graph_streams) if use_graph else None
    ramp_steps = clock_ramp(engine, args.ramp_s, graph=graph) if args.ramp_s > 0 else 0
    r = timed_loop(engine, dist, args.steps, args.warmup, graph=graph)
    elapsed = r["elapsed_s"]
    # all ranks' payload (strong: the shards add up to the config's one batch)
    step_bytes = int(dist.sum(engine.payload_bytes))
    total_bytes = step_bytes * args.steps
    value = total_bytes / elapsed / 2 ** 30
    kernel_ms = r["kernel_ms"]
    isolated = None
    if use_graph and args.graph_streams > 1:
        # the same K launches one after another on ONE stream, as a graph too (no host launch cost;
        # untimed for `value`): the per-dispatch duration rocprof reports, next to the pipelined
        # per-step time above
        ri = timed_loop(engine, _NoDist(), args.steps, 0, graph=engine.capture(args.steps, 1))
        isolated = ri["kernel_ms"] * 1e3
    per = engine.per_launch_us(args.median_launches) if args.median_launches > 0 else []
    # payload read + the result written: u16 sum (csum), u8 status (verify), or the two 2-byte fields
    # and the u8 status (finalize)
    algo_bytes = engine.payload_bytes + (5 if finalize else 1 if verify else 2) * engine.n
    # descriptor bytes a launch reads (seeds included): packed 2 B length + 8 B per 64 packets
    desc_bytes = (12 * engine.batches[0].n_frags + 4 * (engine.n + 1) if finalize  # u64 off + u32 len, u32 first
                  else engine.n * (2 + (0 if verify else 2)) + 8 * ((engine.n + 63) // 64) if engine.packed
                  else 2 * engine.n if getattr(engine, "strided", False)  # the seeds (verify: the u16 lengths)
                  else engine.n * ((4 if engine.compact else 8) + 4 + (0 if verify else 2)))
    kernel_us = kernel_ms * 1e3
    achieved = algo_bytes / (kernel_us * 1e-6) / 1e9
    traffic = load_traffic_finalize(args.config) if finalize else load_traffic(args.traffic_json, args.config)
    line = {
        "metric": METRIC_FINALIZE if finalize else METRIC_VERIFY if verify else METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": dist.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "clock_ramp": {"seconds": args.ramp_s, "untimed_launches": ramp_steps * (args.steps if graph else 1)},
        # kernel launches before the first timed one (ramp + warmup; a graph warmup is one replay of K)
        "launches_before_timed": ramp_steps * (args.steps if graph else 1)
        + ((args.steps if args.warmup else 0) if graph else args.warmup),
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": ("synthetic: IPv4/TCP datagrams from 10.0.0.2 to 10.0.0.1 as NetBuffer chains (IPv4 header written, "
                 "TCP header and payload splitmix64 bytes, seed 0x5EEDC0DE + per-rank offset; checksum fields hold "
                 "whatever is there and count as zero)" if finalize else
                 "synthetic: IPv4/TCP datagrams to 10.0.0.2 (splitmix64 payload, seed 0x5EEDC0DE + per-rank "
                 "offset; checksums filled by rns_tx_fill_dev; every 1009th datagram corrupted)" if verify else
                 "synthetic: splitmix64 packet bytes (seed 0x5EEDC0DE + per-rank offset), per-packet u16 seeds"),
        "config": {
            "workload": (f"{args.config} finalize: {engine.n} IPv4/TCP datagrams x "
                         f"{engine.payload_bytes // max(engine.n, 1)} B per GPU as [40 B head fragment, payload] chains "
                         "(heads back to back in a header region, payloads packed at 16 B), IPv4 header + TCP "
                         "checksums computed and stored into the heads, u8 status out" if finalize else
                         f"{args.config} verify: {engine.n} IPv4/TCP datagrams x "
                         f"{engine.payload_bytes // max(engine.n, 1)} B per GPU, 16 B-aligned arena in HBM, "
                         "IPv4 header + TCP checksum checked, u8 status out" if verify else
                         f"{args.config}: {engine.n} packets x {engine.payload_bytes // max(engine.n, 1)} B per GPU, "
                         "16 B-aligned arena in HBM, per-packet seed, complemented result (tcp.rs:970 form)"),
            "packets_per_gpu": engine.n,
            "payload_bytes_per_gpu": engine.payload_bytes,
            "batch": "one batch sharded by packet index across ranks" if strong else "a full batch per rank",
            "parallelism": f"packet shards x{dist.world}, no data-path collective in `value`",
            "kernel_shape": list(shape) if shape else "auto",
            "descriptors": ({"chain": "u64 offset + u32 length per fragment, u32 first fragment per datagram "
                                      "(rns_tx_fill_chain_dev)"} if finalize else
                            {"64": "u64 offset + u32 length per datagram (rns_rx_verify_dev)",
                             "packed": "packed: u16 length per datagram, u64 offset per 64 datagrams "
                                       "(rns_rx_verify_packed_dev)",
                             "strided": "strided: u16 length per datagram, offsets implied by the slot stride "
                                        "(rns_rx_verify_strided_dev)"} if verify else
                            {"32": "u32 offset + u32 length + u16 seed (rns_csum_batch_dev_off32)",
                             "64": "u64 offset + u32 length + u16 seed (rns_csum_batch_dev)",
                             "packed": "packed: u16 length + u16 seed per packet, u64 offset per 64 packets "
                                       "(rns_csum_batch_packed_dev)",
                             "strided": "strided: u16 seed per packet; offsets and the one length implied "
                                        "(rns_csum_batch_strided_dev)"})[engine.form],
            "rotating_batches": len(engine.batches),
            "rotation": ("one batch per graph stream at least, each with its own bytes: steps that may run at the same "
                         "time never read the same arena" if use_graph and args.graph_streams > 1 else
                         "batches below 512 MiB rotate over >= 768 MiB of arenas"),
            "launch": (f"one HIP graph of the {args.steps} step launches (torch.cuda.CUDAGraph) over "
                       f"{args.graph_streams} stream(s), replayed once" if use_graph else "one C-ABI call per step"),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": (traffic or {}).get("hbm_bytes_per_launch"),
            "kernel": engine.kernel_name() if shape is None else f"shape {list(shape)}",
            "kernel_avg_us": round(kernel_us, 2),
            "frac_from": ("kernel_avg_us: one event pair (capture stream) around the graph replay of the K timed "
                          "launches / K — consecutive steps overlap on " + str(args.graph_streams) + " streams, so "
                          "this is the per-step time, shorter than one dispatch (isolated below)"
                          if isolated is not None else
                          "kernel_avg_us: one event pair (launch stream) around the K back-to-back timed launches / K"),
            "algorithmic_bytes_per_launch": algo_bytes,
            "descriptor_bytes_per_launch": desc_bytes,
            "frac_incl_descriptors": round((algo_bytes + desc_bytes) / (kernel_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic_source": (traffic or {}).get("source"),
        },
        "cpu_baseline": None,
    }
    if args.shard_rw is not None:
        line["shard"] = shard_leg(engine, args)
        line["config"]["workload"] = (f"{args.config} shard {args.shard_rw[0]}/{args.shard_rw[1]} (one rank's packet-index "
                                      f"range of the config's batch, measured alone on one GPU): "
                                      + line["config"]["workload"].split(": ", 1)[1])
        line["config"]["batch"] = (f"rank {args.shard_rw[0]}'s shard of one batch sharded by packet index across "
                                   f"{args.shard_rw[1]} ranks")
    if isolated is not None:
        line["roofline"]["isolated"] = {
            "kernel_avg_us": round(isolated, 2),
            "frac": round(algo_bytes / (isolated * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "launches": args.steps,
            "how": "after the timed region: the same K launches as a graph on ONE stream (no overlap), one event "
                   "pair / K (what rocprof's per-dispatch durations measure)"}
    if per:
        srt = sorted(per)
        line["roofline"]["evpair_median_us"] = round(srt[len(srt) // 2], 2)
        line["roofline"]["evpair_launches"] = len(per)
    if verify:
        # every rotating batch was verified at least once (ramp / warmup / timed steps)
        line["verify"] = {"rejected_total": int(dist.sum(float(engine.bad_count()))),
                          "rejected_expected": int(dist.sum(float(engine.expected_bad()))),
                          "datagrams_total": int(dist.sum(float(sum(b.layout.n for b in engine.verified_batches()))))}
    if dist.world > 1 and not args.no_gather and verify:
        # SURVEY §8(e), verify mode: the same steps plus one all-reduce(sum) of the per-rank rejected counts
        engine.reducer = BadCountReduce(dist, engine.device)
        rr = timed_loop(engine, dist, args.steps, args.warmup, step=engine.step_and_reduce)
        rro = timed_loop(engine, dist, args.steps, args.warmup, step=engine.reduce_bad)
        line["value_compute"] = line["value"]
        line["value_allreduce"] = round(total_bytes / rr["elapsed_s"] / 2 ** 30, 2)
        line["ms_per_step_allreduce"] = round(rr["elapsed_s"] * 1e3 / args.steps, 4)
        line["allreduce_ms"] = round(rro["elapsed_s"] * 1e3 / args.steps, 4)
        line["allreduce"] = {"collective": f"all_reduce sum ({dist.backend}) of the int64 rejected-datagram count",
                             "bytes_per_rank": 8,
                             "rejected_total_last_step": int(engine.reducer.total.item())}
    elif dist.world > 1 and not args.no_gather:
        # the same steps plus one all-gather of every rank's results, and the gather alone
        engine.gatherer = ResultGather(dist, engine.n, engine.device)
        # every collective leg runs eagerly (one C-ABI call and one collective call per step); the
        # compute-only leg is re-timed the same way so the two compare like for like
        re_ = timed_loop(engine, dist, args.steps, args.warmup)
        rg = timed_loop(engine, dist, args.steps, args.warmup, step=engine.step_and_gather)
        rgo = timed_loop(engine, dist, args.steps, args.warmup, step=engine.gather)
        # (last: the gathered results the run leaves behind are the overlapped leg's)
        ro = timed_loop(engine, dist, args.steps, args.warmup, step=OverlappedGather(engine))
        line["value_compute"] = line["value"]
        line["value_compute_eager"] = round(total_bytes / re_["elapsed_s"] / 2 ** 30, 2)
        line["value_gather"] = round(total_bytes / rg["elapsed_s"] / 2 ** 30, 2)
        line["ms_per_step_gather"] = round(rg["elapsed_s"] * 1e3 / args.steps, 4)
        line["value_gather_overlap"] = round(total_bytes / ro["elapsed_s"] / 2 ** 30, 2)
        line["ms_per_step_gather_overlap"] = round(ro["elapsed_s"] * 1e3 / args.steps, 4)
        line["gather_ms"] = round(rgo["elapsed_s"] * 1e3 / args.steps, 4)
        line["gather"] = {"collective": f"all_gather_into_tensor ({dist.backend}) of uint8 results",
                          "bytes_per_rank": engine.gatherer.bytes_per_rank,
                          "bytes_received_per_rank": engine.gatherer.bytes_per_rank * (dist.world - 1)}
        line["legs"] = {
            "value / value_compute": "compute only; the K steps as one HIP graph replay (the N=1 timing)",
            "value_compute_eager": "compute only; one C-ABI launch per step from the host (the gather legs' mode)",
            "value_gather": "eager; each step's kernel, then its all-gather, in order on one stream",
            "value_gather_overlap": "eager; step i's all-gather on a side stream under step i+1's kernel "
                                    "(OverlappedGather, DESIGN §6)",
            "gather_ms": "eager; the all-gather alone, per step"}
    if finalize:
        # every rank: its first batch's heads against the CPU restatement; rank 0 then times it
        par = finalize_parity(engine, threads=max(1, min(8, cpu_grant()["threads"])))
        par.pop("arena", None)
        par.pop("layout", None)
        ranks_exact = int(dist.sum(1.0 if par["bit_exact"] else 0.0))
        line["parity"] = {"ranks_bit_exact": ranks_exact, "ranks": dist.world,
                          "packets_checked": int(dist.sum(float(par["packets"]))),
                          "bit_exact_all_ranks": ranks_exact == dist.world,
                          "how": "every rank: every byte of its first batch's arena and every status after the timed "
                                 "legs vs oracle_tx_chain_fill run on a host copy (both fields count as zero, so the "
                                 "CPU must reproduce the GPU's heads); the counts are all-reduced"}
        dist.barrier()
        if dist.rank == 0 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline_finalize(engine, args.cpu_seconds)
        dist.barrier()
    if dist.world > 1 and not verify and not finalize:
        # after every rank's GPU legs: each rank checks its own results; rank 0 times the CPU
        # baseline on its own batch while the others wait (benches/util_bench.rs:20-45 beside
        # the N-GPU figure, on the same box's host cores, in the same run)
        par = rank_parity(engine, threads=max(1, min(8, cpu_grant()["threads"])))
        ranks_exact = int(dist.sum(1.0 if par["bit_exact"] else 0.0))
        checked = int(dist.sum(float(par["packets"])))
        dist.barrier()
        if dist.rank == 0 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(engine, args.cpu_seconds)
            line["cpu_baseline"]["sample"] = "rank 0's batch: " + line["cpu_baseline"]["sample"]
            line["cpu_baseline"]["gpu_sample_bit_exact_rank0"] = line["cpu_baseline"]["gpu_sample_bit_exact"]
            line["cpu_baseline"]["gpu_sample_bit_exact"] = ranks_exact == dist.world
        dist.barrier()
        line["parity"] = {"ranks_bit_exact": ranks_exact, "ranks": dist.world, "packets_checked": checked,
                          "bit_exact_all_ranks": ranks_exact == dist.world,
                          "how": "every rank: every packet of its first batch vs the oracle (util.rs:88-106 "
                                 "restated), after the timed legs; the counts are all-reduced"}
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline and not finalize:
        line["cpu_baseline"] = cpu_baseline(engine, args.cpu_seconds)
    if dist.rank == 0 and dist.world == 1 and not args.no_host_pipeline:
        line["host_inclusive"] = host_pipeline_rate(engine)
    if dist.rank == 0:
        print(json.dumps(line), flush=True)
    dist.close()
    return line


if __name__ == "__main__":
    main()
