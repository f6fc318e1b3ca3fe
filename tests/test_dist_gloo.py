"""The N>1 bench path (bench.py's Dist + timed_loop: barriers, max-over-ranks wall
time, weak-scaling aggregation) with world_size 2 over gloo on CPU.  The GPU
engine is replaced by a CPU engine that checksums each rank's shard with the
oracle (tests may use the oracle); the harness code is bench.py's own."""
import json
import os
import socket
import subprocess
import sys

from conftest import ROOT

WORKER = r'''
import json, os, sys, time
sys.path.insert(0, {root!r})
import numpy as np
import bench
from oracle.oracle import get_oracle, splitmix64_bytes
from rustnetworkstack_amd.workloads import make_layout

class CpuEngine:
    """Stand-in for bench.GpuEngine: same interface, oracle compute."""
    def __init__(self, rank, world):
        self.layout = make_layout("c5_imix", n=40000, shard=(rank, world))
        self.arena = splitmix64_bytes(self.layout.data_seed, self.layout.arena_bytes)
        self.orc = get_oracle()
        self.times = []
        self.out = None
    n = property(lambda s: s.layout.n)
    payload_bytes = property(lambda s: s.layout.payload_bytes)
    def step(self):
        self.out = self.orc.batch(self.arena, self.layout.off, self.layout.length, self.layout.seed, complement=True)
    def sync(self):
        pass
    def begin_timing(self):
        self.t0 = time.perf_counter()
    def end_timing(self, steps):
        self.ms = 1e3 * (time.perf_counter() - self.t0) / steps
    def kernel_ms(self):
        return self.ms

d = bench.Dist(backend="gloo")
eng = CpuEngine(d.rank, d.world)
r = bench.timed_loop(eng, d, steps=3, warmup=1)
# ranks' results, gathered to check the shards tile the whole batch
import torch, torch.distributed as dist
outs = [torch.zeros(0) for _ in range(d.world)]
obj = [None] * d.world
dist.all_gather_object(obj, (d.rank, eng.n, eng.out.tolist(), r["local_elapsed_s"], r["elapsed_s"],
                             d.sum(eng.payload_bytes)))
if d.rank == 0:
    print(json.dumps(obj))
d.close()
'''


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo_harness(tmp_path, oracle):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(script)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("[[")][-1]
    ranks = json.loads(line)
    # the max-over-ranks time every rank reports is the same and >= each local time
    assert len({round(x[4], 9) for x in ranks}) == 1
    assert all(x[4] >= x[3] - 1e-9 for x in ranks)
    # shards by packet index tile the full batch, and each rank's results are the oracle's
    import numpy as np

    from oracle.oracle import splitmix64_bytes
    from rustnetworkstack_amd.workloads import make_layout
    total = sum(x[1] for x in ranks)
    assert total == 40000
    # strong scaling's aggregate: the shards' payload adds up to the one batch's, on every rank
    assert {x[5] for x in ranks} == {make_layout("c5_imix", n=40000).payload_bytes}
    for rank, n, out, _, _, _ in ranks:
        lay = make_layout("c5_imix", n=40000, shard=(rank, 2))
        arena = splitmix64_bytes(lay.data_seed, lay.arena_bytes)
        assert np.array_equal(np.array(out, dtype=np.uint16),
                              oracle.batch(arena, lay.off, lay.length, lay.seed, complement=True))
