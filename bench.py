#!/usr/bin/env python3
"""Device-resident batched Internet checksum throughput on MI355X.

Metric (BASELINE.json): GiB/s device-resident Internet checksum, 1500 B-packet
batches, 1/2/4/8 GPUs.  One STEP = one pass of the hot path — one launch of the
gfx950 checksum kernel — over one batch (config c3_1500B: 2^20 packets x 1500 B
per GPU, already resident in HBM).  value = payload bytes checksummed by all
ranks / max-over-ranks wall time of the K timed steps / 2^30.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3_1500B]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Packets shard trivially: every rank checksums its own batch with
no data-path collective ("scaling": "weak").  Rank 0 prints one JSON line.
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


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="c3_1500B")
    p.add_argument("--desc", choices=("auto", "64", "32"), default="auto",
                   help="descriptor offset width: 32 = compact form (rns_csum_batch_dev_off32); "
                        "auto = 32 when the arena is below 4 GiB")
    p.add_argument("--shape", default="", help="variant,G,U,max_blocks kernel shape override (tuning)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample duration (single thread)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-host-pipeline", action="store_true", help="skip the PCIe-inclusive extra measurement")
    p.add_argument("--gather", action="store_true",
                   help="add an RCCL all_gather of every rank's results to each step (not the default: "
                        "the stack consumes results where they are produced)")
    p.add_argument("--scaling", choices=("auto", "weak", "strong"), default="auto",
                   help="weak: every rank checksums a full batch of the config; strong: the config's batch is "
                        "sharded by packet index across ranks (auto: strong for c5_imix, whose BASELINE.json "
                        "config is one 8M-packet batch over 8 GPUs; weak otherwise)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_{config}.json"))
    return p.parse_args(argv)


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
        if self.enabled and torch.cuda.is_available():
            torch.cuda.set_device(self.local_rank)  # before RCCL binds its communicator
        if self.enabled and not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group(backend=backend or ("nccl" if torch.cuda.is_available() else "gloo"))
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


def timed_loop(engine, dist: Dist, steps: int, warmup: int) -> dict:
    """W untimed steps, then exactly K steps bracketed by sync + barrier on both
    sides; wall time is the max over ranks.  Device time per launch = one pair of
    events on the launch stream around the K back-to-back launches, / K (events
    between launches would insert ~10 µs gaps: see DESIGN.md, measurement)."""
    for _ in range(warmup):
        engine.step()
    engine.sync()
    dist.barrier()
    engine.sync()
    t0 = time.perf_counter()
    engine.begin_timing()
    for _ in range(steps):
        engine.step()
    engine.end_timing(steps)
    engine.sync()
    dist.barrier()
    engine.sync()
    elapsed = time.perf_counter() - t0
    return {"elapsed_s": dist.max(elapsed), "local_elapsed_s": elapsed,
            "kernel_ms": engine.kernel_ms()}


# ---------------------------------------------------------------------------
# GPU engine: the product path
# ---------------------------------------------------------------------------
class GpuEngine:
    def __init__(self, config: str, rank: int, local_rank: int, shape=None, gather_dist: Dist | None = None,
                 steps: int = 0, world: int = 1, strong: bool = False, compact="64"):
        import torch

        from rustnetworkstack_amd.workloads import DATA_SEED, DeviceBatch, make_layout
        self.torch = torch
        self.device = torch.device(f"cuda:{local_rank}")
        torch.cuda.set_device(self.device)

        def layout(r):
            if strong:  # this rank's packet-index shard of the one batch (same sizes and seeds on every rank)
                lay = make_layout(config, shard=(rank, world))
                lay.data_seed = DATA_SEED + 0x1000 * rank + r
                return lay
            # weak scaling: every rank owns a full batch of the config, with its own bytes
            return make_layout(config, data_seed=DATA_SEED + 0x1000 * rank + r)

        self.layout = layout(0)
        small = self.layout.arena_bytes < (512 << 20)
        # batches that fit the 256 MiB Infinity Cache are rotated so each step reads cold bytes
        nrot = max(1, -(-(768 << 20) // max(self.layout.arena_bytes, 1))) if small else 1
        self.batches = [DeviceBatch(self.layout if r == 0 else layout(r), self.device) for r in range(nrot)]
        self.shape = shape
        if compact == "auto":
            compact = shape is None and self.layout.arena_bytes + 16 < 2 ** 32
        self.compact = compact in (True, "32")
        for b in self.batches:  # bind every rotating batch (and upload compact offsets) before any timing
            b.launcher(complement=True, shape=shape, compact=self.compact)
        self.gather = gather_dist
        self.k = 0
        self.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        self.timed = 0
        if gather_dist is not None and gather_dist.enabled:
            n = self.layout.n
            self.gathered = torch.empty(n * gather_dist.world, dtype=torch.int16, device=self.device)
        torch.cuda.synchronize()

    @property
    def n(self):
        return self.layout.n

    @property
    def payload_bytes(self):
        return self.layout.payload_bytes

    def step(self):
        b = self.batches[self.k % len(self.batches)]
        self.k += 1
        b.launcher(complement=True, shape=self.shape, compact=self.compact)()  # pre-bound: one ctypes call
        if self.gather is not None and self.gather.enabled:
            self.gather.dist.all_gather_into_tensor(self.gathered, b.out.view(self.torch.int16))

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
        return _lib.load().rns_csum_shape_name(int(round(self.layout.mean_len))).decode()

    def out_sample(self, count: int):
        import numpy as np
        return self.batches[0].out[:count].view(self.torch.int16).cpu().numpy().view(np.uint16)


# ---------------------------------------------------------------------------
# CPU baseline: the reference's algorithm (oracle/ restatement), host cores
# ---------------------------------------------------------------------------
def cpu_baseline(engine: GpuEngine, seconds: float) -> dict:
    """Times the literal C restatement of util.rs:88-106 (oracle/csum_oracle.c,
    gcc -O3, baseline x86-64) on a bounded sample of the same batch: single
    thread for `seconds`, all host cores for a quarter of that.  Also checks
    the GPU results of the sample packets against it."""
    import numpy as np

    from oracle.oracle import get_oracle
    orc = get_oracle()
    lay = engine.layout
    # sample: the first packets of the batch, ~64 MiB of payload
    count = int(min(lay.n, max(1, (64 << 20) // max(int(lay.mean_len), 1))))
    end = int(lay.off[count - 1] + lay.length[count - 1])
    arena = engine.batches[0].arena[:end].cpu().numpy()
    off, ln, sd = lay.off[:count], lay.length[:count], lay.seed[:count]
    sample_bytes = int(ln.astype(np.uint64).sum())

    def rate(threads: int, budget: float):
        passes, t0 = 0, time.perf_counter()
        while True:
            res = orc.batch(arena, off, ln, sd, complement=True, threads=threads)
            passes += 1
            dt = time.perf_counter() - t0
            if dt >= budget:
                return sample_bytes * passes / dt / 2 ** 30, res, passes, dt

    v1, res, passes, dt = rate(1, seconds)
    box_cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    mt = int(min(16, box_cores))   # gpurun boxes grant 16 CPUs; cpu_count() shows the whole machine
    vmt, _, _, _ = rate(mt, max(seconds / 4, 1.0))
    gpu = engine.out_sample(count)
    ns_zero = orc.time_ones_comp(bytes(512), 2_000_000)
    ns_ff = orc.time_ones_comp(b"\xff" * 512, 2_000_000)
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((ln_.split(":", 1)[1].strip() for ln_ in f if ln_.startswith("model name")), "")
    except OSError:
        pass
    return {
        "value": round(v1, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
        "sample": f"first {count} packets ({sample_bytes} B) of the {lay.name} batch, "
                  f"{passes} passes in {dt:.1f} s; oracle/csum_oracle.c literal util.rs:88-106 loop, gcc -O3",
        "value_all_cores": round(vmt, 3), "all_cores_threads": mt,
        "util_bench_ns_per_iter": {"compute_ones_comp_512B_zeros": round(ns_zero, 2),
                                   "compute_ones_comp_512B_0xff": round(ns_ff, 2)},
        "host_cpu": cpu_model, "host_cpus_visible": box_cores,
        "gpu_sample_bit_exact": bool(np.array_equal(gpu, res)),
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


def load_traffic(path: str, config: str):
    path = path.format(config=config)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        t = json.load(f)
    return t


def main(argv=None):
    args = parse_args(argv)
    dist = Dist()
    shape = tuple(int(x) for x in args.shape.split(",")) if args.shape else None
    strong = args.scaling == "strong" or (args.scaling == "auto" and args.config == "c5_imix")
    engine = GpuEngine(args.config, dist.rank, dist.local_rank, shape=shape,
                       gather_dist=dist if args.gather else None, steps=args.steps, world=dist.world, strong=strong,
                       compact=args.desc)
    r = timed_loop(engine, dist, args.steps, args.warmup)
    elapsed = r["elapsed_s"]
    # all ranks' payload (strong: the shards add up to the config's one batch)
    total_bytes = int(dist.sum(engine.payload_bytes)) * args.steps
    value = total_bytes / elapsed / 2 ** 30
    kernel_ms = r["kernel_ms"]
    algo_bytes = engine.payload_bytes + 2 * engine.n
    achieved = algo_bytes / (kernel_ms * 1e-3) / 1e9
    traffic = load_traffic(args.traffic_json, args.config)
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": dist.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: splitmix64 packet bytes (seed 0x5EEDC0DE + per-rank offset), per-packet u16 seeds",
        "config": {
            "workload": f"{args.config}: {engine.n} packets x {engine.payload_bytes // max(engine.n, 1)} B per GPU, "
                        "16 B-aligned arena in HBM, per-packet seed, complemented result (tcp.rs:970 form)",
            "packets_per_gpu": engine.n,
            "payload_bytes_per_gpu": engine.payload_bytes,
            "batch": "one batch sharded by packet index across ranks" if strong else "a full batch per rank",
            "parallelism": f"packet shards x{dist.world}, no data-path collective"
                           + (" + RCCL all_gather of results" if args.gather else ""),
            "kernel_shape": list(shape) if shape else "auto",
            "descriptors": ("u32 offset + u32 length + u16 seed (rns_csum_batch_dev_off32)" if engine.compact
                            else "u64 offset + u32 length + u16 seed (rns_csum_batch_dev)"),
            "rotating_batches": len(engine.batches),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": (traffic or {}).get("hbm_bytes_per_launch"),
            "kernel": engine.kernel_name() if shape is None else f"shape {list(shape)}",
            "kernel_avg_us": round(kernel_ms * 1e3, 2),
            "algorithmic_bytes_per_launch": algo_bytes,
            "traffic_source": (traffic or {}).get("source"),
        },
        "cpu_baseline": None,
    }
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(engine, args.cpu_seconds)
    if dist.rank == 0 and dist.world == 1 and not args.no_host_pipeline:
        line["host_inclusive"] = host_pipeline_rate(engine)
    if dist.rank == 0:
        print(json.dumps(line), flush=True)
    dist.close()
    return line


if __name__ == "__main__":
    main()
