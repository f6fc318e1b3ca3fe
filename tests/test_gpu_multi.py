"""Multi-GPU batch entry points: rns_csum_batch_multi_host
and rns_csum_batch_multi_dev against the oracle.  The box has one GPU, so the
sharding logic is exercised with several contexts / shards on device 0 (a device
may repeat in the device list); each range still runs through its own staging
context, streams and thread exactly as it would on separate GPUs."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from rustnetworkstack_amd import _lib
from rustnetworkstack_amd.batch import MultiHostBatcher, csum_batch_multi_dev
from rustnetworkstack_amd.workloads import make_layout

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0, 0]])
def test_multi_host_matches_oracle(oracle, devices):
    lay = make_layout("c5_imix", n=200000)
    arena = O.splitmix64_bytes(lay.data_seed, lay.arena_bytes)
    mb = MultiHostBatcher(devices, chunk_bytes=1 << 20, nstreams=2)
    out = mb.run(arena, lay.off, lay.length, lay.seed, complement=True)
    expect = oracle.batch(arena, lay.off, lay.length, lay.seed, complement=True)
    assert np.array_equal(out, expect)
    # fewer packets than devices: the empty ranges are skipped
    few = mb.run(arena, lay.off[:2], lay.length[:2], None)
    assert np.array_equal(few, oracle.batch(arena, lay.off[:2], lay.length[:2], None))
    # a descriptor outside the arena in the LAST range is reported, not ignored
    bad_len = lay.length.copy()
    bad_len[-1] = np.uint32(lay.arena_bytes)
    with pytest.raises(_lib.ChecksumError):
        mb.run(arena, lay.off, bad_len, None)
    mb.close()


def test_multi_dev_shards(oracle):
    """Three device-resident shards (different layouts and arenas), launched by one
    call; each shard's results land in its own output."""
    shards, expects = [], []
    for k, (cfg, n) in enumerate((("c3_1500B", 20000), ("c5_imix", 50000), ("c2_64B", 30000))):
        lay = make_layout(cfg, n=n, data_seed=0x5EEDC0DE + k)
        arena_np = O.splitmix64_bytes(lay.data_seed, lay.arena_bytes)
        expects.append(oracle.batch(arena_np, lay.off, lay.length, lay.seed, complement=True))
        shards.append(dict(arena=torch.from_numpy(arena_np).to(DEV),
                           off=torch.from_numpy(lay.off.view(np.int64)).to(DEV),
                           length=torch.from_numpy(lay.length.view(np.int32)).to(DEV),
                           seed=torch.from_numpy(lay.seed.view(np.int16)).to(DEV),
                           out=torch.empty(lay.n, dtype=torch.uint16, device=DEV)))
    csum_batch_multi_dev(shards, complement=True)
    torch.cuda.synchronize()
    for sh, exp in zip(shards, expects):
        assert np.array_equal(sh["out"].view(torch.int16).cpu().numpy().view(np.uint16), exp)
