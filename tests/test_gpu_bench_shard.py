"""bench.py's cache-honest rotation and the one-GPU shard measurement.

* Every graph stream reads its own batch: concurrently running steps never share an arena,
  so no dispatch is served from bytes another dispatch just pulled into the Infinity Cache.
* `--shard r/N` times rank r's packet-index shard of c5 IMIX (the per-GPU work of the
  N-GPU point), and the CPU-baseline leg re-checks the shard's results against the oracle.
"""
import numpy as np
import pytest

import bench

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shard", ["0/8", "7/8"])
def test_bench_c5_shard_of_8(shard):
    line = bench.main(["--config", "c5_imix", "--shard", shard, "--steps", "4", "--warmup", "1", "--ramp-s", "0",
                       "--cpu-seconds", "1", "--no-host-pipeline", "--traffic-json", "/nonexistent/{config}.json"])
    from rustnetworkstack_amd.workloads import make_layout
    r, n = (int(x) for x in shard.split("/"))
    lay = make_layout("c5_imix", shard=(r, n))
    sh = line["shard"]
    assert (sh["rank"], sh["world"]) == (r, n)
    assert sh["packets"] == lay.n == line["config"]["packets_per_gpu"] == (1 << 23) // 8
    assert sh["payload_bytes"] == lay.payload_bytes
    assert sh["gather"]["bytes_resident_after_per_rank"] == 2 * (1 << 23)
    assert line["scaling"] == "strong" and line["n_gpus"] == 1
    # value = this shard's bytes over the timed steps
    assert abs(line["value"] - lay.payload_bytes * 4 / (line["ms_per_step"] * 4e-3) / 2 ** 30) <= 0.01 * line["value"]
    assert line["config"]["rotating_batches"] >= 2      # one batch per graph stream (2 for the IMIX shard)
    assert line["cpu_baseline"]["gpu_sample_bit_exact"] is True


def test_every_graph_stream_reads_its_own_batch():
    """GpuEngine(min_batches=S): S batches with pairwise different bytes, steps i..i+S-1 on
    different batches (the capture assigns step i to batch i % nrot and stream i % S)."""
    import torch
    eng = bench.GpuEngine("c3_1500B", 0, 0, compact="auto", min_batches=3)
    assert len(eng.batches) == 3
    heads = [b.arena[:4096].cpu().numpy() for b in eng.batches]
    for i in range(3):
        for j in range(i + 1, 3):
            assert not np.array_equal(heads[i], heads[j])
    g = eng.capture(6, streams=3)
    g.replay()
    torch.cuda.synchronize()
    assert eng.used == {0, 1, 2}


def test_bench_c2_strided_form():
    """--desc strided (rns_csum_batch_strided_dev: no offset/length descriptors) on the c2
    config: the CPU-baseline leg re-checks the rotating batches' results against the oracle."""
    line = bench.main(["--config", "c2_64B", "--desc", "strided", "--steps", "24", "--warmup", "1", "--ramp-s", "0",
                       "--cpu-seconds", "1", "--no-host-pipeline", "--traffic-json", "/nonexistent/{config}.json"])
    assert line["config"]["descriptors"].startswith("strided")
    assert line["roofline"]["descriptor_bytes_per_launch"] == 2 * (1 << 20)
    assert line["cpu_baseline"]["gpu_sample_bit_exact"] is True
