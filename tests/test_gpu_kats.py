"""The reference's own single-slice known-answer tests, run as batches through the HIP
entries.  The vectors are the values util.rs asserts —
compute_ones_comp (util.rs:277-285, 315-317) and compute_checksum (util.rs:288-293) —
plus the RFC 1071 / IPv4 vectors of tests/golden/reference_kats.json, transcribed as
data.  Every KAT runs at every start offset mod 16 through rns_csum_batch_dev (64-bit
descriptors) under each kernel family's length hint, and through
rns_csum_batch_packed_dev at byte, 16-byte (the stream kernels) and 64-byte alignment,
with non-zero padding bytes between the packets."""
import numpy as np
import pytest
import torch

from rustnetworkstack_amd.batch import csum_batch, csum_batch_packed, packed_layout

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
HINTS = (0, 40, 64, 576, 1500, 9000)  # stream / tiny rounds / class / group kernels


def host_u16(t):
    torch.cuda.synchronize()
    return t.view(torch.int16).cpu().numpy().view(np.uint16)


def dev(a, view):
    return torch.from_numpy(np.ascontiguousarray(a).view(view)).to(DEV)


def kat_cases(kats):
    """(bytes, seed, complement, expect) for every single-slice KAT."""
    out = []
    for k in kats["ones_comp"]:
        out.append((bytes.fromhex(k["bytes"]), k["seed"], False, k["expect"]))
    for k in kats["checksum"]:
        out.append((bytes.fromhex(k["bytes"]), 0, True, k["expect"]))
    return out


def test_kat_values_are_the_references(kats):
    """The fixture holds util.rs's asserted values (guards against an edited fixture)."""
    got = {k["source"].split(" ")[1]: k["expect"] for k in kats["ones_comp"] + kats["checksum"]
           if k["source"].startswith("reference")}
    assert got["util.rs:278"] == 0 and got["util.rs:279"] == 1 and got["util.rs:280"] == 0xFF
    assert got["util.rs:281-284"] == 0xEE79 and got["util.rs:316"] == 0x6834
    assert got["util.rs:289"] == 0xFFFF and got["util.rs:290"] == 0xFFFE
    assert got["util.rs:291"] == 0xFF00 and got["util.rs:292"] == 0x1186


@pytest.mark.parametrize("complement", [False, True])
def test_kats_batch_dev_every_offset(kats, complement):
    cases = [c for c in kat_cases(kats) if c[2] == complement]
    arena = np.full(64 * 16 * len(cases) + 64, 0xC3, dtype=np.uint8)  # non-zero filler around every slice
    off, ln, sd, expect = [], [], [], []
    pos = 16
    for data, seed, _, exp in cases:
        for s in range(16):
            o = pos + s
            arena[o:o + len(data)] = np.frombuffer(data, dtype=np.uint8)
            off.append(o)
            ln.append(len(data))
            sd.append(seed)
            expect.append(exp)
            pos += 64
    a = torch.from_numpy(arena).to(DEV)
    expect = np.array(expect, dtype=np.uint16)
    for hint in HINTS:
        got = host_u16(csum_batch(a, dev(np.array(off, dtype=np.uint64), np.int64),
                                  dev(np.array(ln, dtype=np.uint32), np.int32),
                                  dev(np.array(sd, dtype=np.uint16), np.int16), complement=complement,
                                  len_hint=hint))
        assert np.array_equal(got, expect), (hint, np.nonzero(got != expect)[0][:8])


@pytest.mark.parametrize("align_log2", [0, 4, 6])
@pytest.mark.parametrize("complement", [False, True])
def test_kats_packed(kats, align_log2, complement):
    """Each KAT repeated 67 times (more than one 64-packet block, a partial last block)
    in one packed arena, padding bytes 0xA5."""
    cases = [c for c in kat_cases(kats) if c[2] == complement]
    reps = 67
    datas = [c[0] for c in cases for _ in range(reps)]
    ln = np.array([len(d) for d in datas], dtype=np.uint32)
    sd = np.array([c[1] for c in cases for _ in range(reps)], dtype=np.uint16)
    expect = np.array([c[3] for c in cases for _ in range(reps)], dtype=np.uint16)
    blk, poff, end = packed_layout(ln, align_log2, 0)
    arena = np.full(end + 32, 0xA5, dtype=np.uint8)
    for d, o in zip(datas, poff.tolist()):
        arena[o:o + len(d)] = np.frombuffer(d, dtype=np.uint8)
    a = torch.from_numpy(arena).to(DEV)
    for hint in HINTS:
        got = host_u16(csum_batch_packed(a, dev(blk.astype(np.uint64), np.int64), dev(ln.astype(np.uint16), np.int16),
                                         dev(sd, np.int16), align_log2=align_log2, complement=complement,
                                         len_hint=hint))
        assert np.array_equal(got, expect), (hint, np.nonzero(got != expect)[0][:8])
