"""Synthetic packet batches for the configurations BASELINE.json names.

SURVEY §8d: packet bytes from splitmix64 (seed 0x5EED_C0DE), per-packet 16-bit
seeds from the same generator family, packet starts 16-byte aligned in the
arena (padding bytes are not counted as payload).

========  =====================  ============================================
name      packets                BASELINE.json config
========  =====================  ============================================
c1_512B   1 x 512 B (host)       cargo bench util_bench (CPU, single buffer)
c2_64B    2^20 x 64 B            1 GPU minimum-size packets
c3_1500B  2^20 x 1500 B          1 GPU MTU packets — the headline metric
c4_9000B  2^18 x 9000 B          1 GPU jumbo frames
c5_imix   2^23 IMIX 40/576/1500  8 GPU mixed sizes, sharded by packet index
          in a 7:4:1 ratio
========  =====================  ============================================
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

DATA_SEED = 0x5EEDC0DE
SEED_STREAM = 0x5EED5EED  # xor-ed into DATA_SEED for the per-packet seed stream
ALIGN = 16

CONFIGS = {
    "c2_64B": dict(n=1 << 20, kind="fixed", length=64),
    "c3_1500B": dict(n=1 << 20, kind="fixed", length=1500),
    "c4_9000B": dict(n=1 << 18, kind="fixed", length=9000),
    "c5_imix": dict(n=1 << 23, kind="imix"),
}
HEADLINE = "c3_1500B"
# Diagnostic batches (not BASELINE.json configs): one IMIX size each, for per-class tuning.
DIAG_CONFIGS = {
    "d40B": dict(n=1 << 22, kind="fixed", length=40),
    "d576B": dict(n=1 << 21, kind="fixed", length=576),
    "d1000B": dict(n=1 << 20, kind="fixed", length=1000),
    # past 4 GiB (the kernels' 64-bit-address forms): 3 x c3 and 2 x IMIX in one batch
    "d1500B_big": dict(n=3 << 20, kind="fixed", length=1500),
    "dimix_big": dict(n=1 << 24, kind="imix"),
}
IMIX_SIZES = (40, 576, 1500)  # 7:4:1


def splitmix64(seed: int, count: int, start: int = 0) -> np.ndarray:
    """z_i = mix(seed + (start+i+1) * 0x9E3779B97F4A7C15) — the stream
    rns_fill_splitmix64_dev writes on the device."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + np.arange(start + 1, start + count + 1, dtype=np.uint64) * np.uint64(
            0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


@dataclass
class Layout:
    """Host-side description of a batch: where each packet sits in the arena."""
    name: str
    off: np.ndarray      # uint64
    length: np.ndarray   # uint32
    seed: np.ndarray     # uint16
    arena_bytes: int
    data_seed: int
    payload_bytes: int = field(init=False)

    def __post_init__(self):
        self.payload_bytes = int(self.length.astype(np.uint64).sum())

    @property
    def n(self) -> int:
        return int(self.off.shape[0])

    @property
    def mean_len(self) -> float:
        return self.payload_bytes / max(self.n, 1)


def imix_lengths(n: int, seed: int) -> np.ndarray:
    r = splitmix64(seed ^ 0x1A1A1A1A, n) % np.uint64(12)
    out = np.full(n, IMIX_SIZES[2], dtype=np.uint32)
    out[r < 11] = IMIX_SIZES[1]
    out[r < 7] = IMIX_SIZES[0]
    return out


def make_layout(name: str, n: int | None = None, data_seed: int = DATA_SEED, shard: tuple[int, int] = (0, 1),
                align: int = ALIGN) -> Layout:
    """Packets of config `name`; `shard=(rank, world)` keeps the contiguous
    packet-index range ceil(n/world) of that rank."""
    cfg = CONFIGS[name] if name in CONFIGS else DIAG_CONFIGS[name]
    total = cfg["n"] if n is None else n
    if cfg["kind"] == "fixed":
        length_all = None
    else:
        length_all = imix_lengths(total, data_seed)
    rank, world = shard
    per = -(-total // world)
    lo, hi = min(rank * per, total), min((rank + 1) * per, total)
    count = hi - lo
    if length_all is None:
        length = np.full(count, cfg["length"], dtype=np.uint32)
    else:
        length = length_all[lo:hi].copy()
    padded = (length.astype(np.uint64) + np.uint64(align - 1)) & ~np.uint64(align - 1)
    off = np.zeros(count, dtype=np.uint64)
    if count > 1:
        np.cumsum(padded[:-1], out=off[1:])
    arena_bytes = int(off[-1] + padded[-1]) if count else 0
    seed = (splitmix64(data_seed ^ SEED_STREAM, count, start=lo) & np.uint64(0xFFFF)).astype(np.uint16)
    return Layout(name=name, off=off, length=length, seed=seed, arena_bytes=arena_bytes,
                  data_seed=(data_seed + rank) & 0xFFFFFFFFFFFFFFFF)


class DeviceBatch:
    """A Layout materialised in HBM: arena filled with splitmix64 bytes on the
    device, descriptors uploaded once (inputs resident before any timing)."""

    def __init__(self, layout: Layout, device):
        import torch

        from .batch import fill_splitmix64

        self.layout = layout
        self.device = torch.device(device)
        # +16 slack keeps the arena a whole number of 16-byte chunks
        self.arena = torch.empty(layout.arena_bytes + 16, dtype=torch.uint8, device=self.device)
        fill_splitmix64(self.arena, layout.data_seed)
        self.off = torch.from_numpy(layout.off.view(np.int64)).to(self.device)
        self.length = torch.from_numpy(layout.length.view(np.int32)).to(self.device)
        self.seed = torch.from_numpy(layout.seed.view(np.int16)).to(self.device)
        self.out = torch.empty(layout.n, dtype=torch.uint16, device=self.device)
        self._prepared = {}

    def stride(self):
        """(first_off, stride, length) if every packet has one length and the packets lie at
        a fixed stride (c2-c4: fixed-size configs), else None."""
        lay = self.layout
        if lay.n == 0 or not np.all(lay.length == lay.length[0]):
            return None
        step = int(lay.off[1] - lay.off[0]) if lay.n > 1 else ALIGN
        if lay.n > 1 and not np.array_equal(np.diff(lay.off), np.full(lay.n - 1, step, dtype=np.uint64)):
            return None
        return int(lay.off[0]), step, int(lay.length[0])

    def launcher(self, complement: bool = False, shape=None, compact: bool = False, packed: bool = False,
                 strided: bool = False):
        """Pre-bound launch (one ctypes call per launch) on the current stream.
        ``compact`` binds 32-bit offsets (rns_csum_batch_dev_off32; arenas < 4 GiB);
        ``packed`` binds the packed form (rns_csum_batch_packed_dev: u16 lengths + one
        offset per 64 packets; the synthetic layouts ARE packed at 16-byte alignment);
        ``strided`` binds the fixed-stride form (rns_csum_batch_strided_dev: equal-length
        packets, no offset or length descriptors)."""
        import torch

        from .batch import PackedBatch, PreparedBatch, StridedBatch, packed_layout
        key = (complement, shape, compact, packed, strided)
        if key not in self._prepared:
            if strided:
                if shape is not None or compact or packed:
                    raise ValueError("the strided form takes no shape override, compact or packed descriptors")
                st = self.stride()
                if st is None:
                    raise ValueError("layout is not equal-length packets at a fixed stride")
                self._prepared[key] = StridedBatch(self.arena, self.layout.n, st[1], st[2], first_off=st[0],
                                                   seed=self.seed, complement=complement, out=self.out)
                return self._prepared[key]
            if packed:
                if shape is not None or compact:
                    raise ValueError("the packed form takes no shape override and no compact offsets")
                blk, off, _ = packed_layout(self.layout.length, align_log2=ALIGN.bit_length() - 1,
                                            first_off=int(self.layout.off[0]) if self.layout.n else 0)
                if not np.array_equal(off, self.layout.off):
                    raise ValueError("layout is not packed at the default alignment")
                self.blk_off = torch.from_numpy(blk.view(np.int64)).to(self.device)
                self.len16 = torch.from_numpy(self.layout.length.astype(np.uint16).view(np.int16)).to(self.device)
                self._prepared[key] = PackedBatch(self.arena, self.blk_off, self.len16, self.seed,
                                                  align_log2=ALIGN.bit_length() - 1, complement=complement,
                                                  out=self.out, len_hint=int(round(self.layout.mean_len)))
                return self._prepared[key]
            off = self.off
            if compact:
                if self.layout.arena_bytes + 16 >= 2 ** 32:
                    raise ValueError("compact descriptors need an arena below 4 GiB")
                off = torch.from_numpy(self.layout.off.astype(np.uint32).view(np.int32)).to(self.device)
            self._prepared[key] = PreparedBatch(self.arena, off, self.length, self.seed, complement=complement,
                                                out=self.out, len_hint=int(round(self.layout.mean_len)), shape=shape,
                                                compact=compact)
        return self._prepared[key]

    def rebind(self, complement: bool = False, shape=None, compact: bool = False, packed: bool = False,
               strided: bool = False):
        """A fresh launcher bound to the CURRENT stream (e.g. a graph-capture stream),
        from the descriptors launcher() already uploaded (no copies: safe inside a
        capture).  Not cached."""
        from .batch import PackedBatch, PreparedBatch, StridedBatch
        bound = self.launcher(complement, shape, compact, packed, strided)  # uploads once, outside any capture
        if strided:
            st = self.stride()
            return StridedBatch(self.arena, self.layout.n, st[1], st[2], first_off=st[0], seed=self.seed,
                                complement=complement, out=self.out)
        if packed:
            return PackedBatch(self.arena, self.blk_off, self.len16, self.seed, align_log2=ALIGN.bit_length() - 1,
                               complement=complement, out=self.out, len_hint=int(round(self.layout.mean_len)))
        off = bound._keep[1]
        return PreparedBatch(self.arena, off, self.length, self.seed, complement=complement, out=self.out,
                             len_hint=int(round(self.layout.mean_len)), shape=shape, compact=compact)

    def run(self, complement: bool = False, shape=None):
        return self.launcher(complement, shape)()

    def host_arena(self) -> np.ndarray:
        return self.arena.cpu().numpy()

    def host_out(self) -> np.ndarray:
        return self.out.view(__import__("torch").int16).cpu().numpy().view(np.uint16)


# ---------------------------------------------------------------------------
# Receive-verify batches (bench.py --op verify): every packet becomes an IPv4/TCP
# datagram addressed to LOCAL4, its checksums filled by the product's own transmit
# finalize (rns_tx_fill_dev), then every CORRUPT_EVERY-th datagram gets one payload
# byte flipped so a known number fail (tcp.rs:544-547 drops them).
# ---------------------------------------------------------------------------
LOCAL4 = bytes([10, 0, 0, 2])
REMOTE4 = bytes([10, 0, 0, 1])
LOCAL6 = bytes.fromhex("fd000000000000000000000000000002")
CORRUPT_EVERY, CORRUPT_FIRST = 1009, 7
MIN_DATAGRAM = 40  # IPv4 header + TCP header


def ipv4_tcp_headers(length: np.ndarray, src4: bytes = REMOTE4, dst4: bytes = LOCAL4) -> np.ndarray:
    """[n, 20] IPv4 headers (IHL 5, DF, TTL 64, protocol 6, total length = the
    datagram's length, checksum field zero) for datagrams of `length` bytes."""
    n = int(length.shape[0])
    h = np.zeros((n, 20), dtype=np.uint8)
    h[:, 0] = 0x45
    h[:, 2] = (length >> 8) & 0xFF
    h[:, 3] = length & 0xFF
    h[:, 6] = 0x40
    h[:, 8] = 64
    h[:, 9] = 6
    h[:, 12:16] = np.frombuffer(src4, dtype=np.uint8)
    h[:, 16:20] = np.frombuffer(dst4, dtype=np.uint8)
    return h


def corrupt_mask(n: int) -> np.ndarray:
    """Datagrams whose payload byte is flipped (local packet index)."""
    return (np.arange(n) % CORRUPT_EVERY) == CORRUPT_FIRST


def corrupt_pos(length: np.ndarray) -> np.ndarray:
    """Byte (from the datagram start) that corruption flips: the middle of the TCP segment."""
    return 20 + (length.astype(np.int64) - 20) // 2


def make_verify_batch(b: "DeviceBatch") -> None:
    """Turn a DeviceBatch into received datagrams in place (headers written, checksums
    filled by rns_tx_fill_dev, known corruptions applied) and give it a status array."""
    import torch

    from . import _lib
    from .batch import tx_fill
    lay = b.layout
    if lay.n and int(lay.length.min()) < MIN_DATAGRAM:
        raise ValueError(f"verify batches need datagrams of at least {MIN_DATAGRAM} B")
    dev = b.device
    hdr = torch.from_numpy(ipv4_tcp_headers(lay.length)).to(dev)
    step = 1 << 20  # packets per scatter (bounds the index tensor)
    for i in range(0, lay.n, step):
        idx = b.off[i:i + step].view(-1, 1) + torch.arange(20, device=dev)
        b.arena[idx.flatten()] = hdr[i:i + step].flatten()
    st = tx_fill(b.arena, b.off, b.length)
    want = _lib.RNS_TX_IP_FILLED | _lib.RNS_TX_L4_FILLED
    if int((st != want).sum().item()):
        raise RuntimeError("transmit finalize did not fill every synthetic datagram")
    mask = corrupt_mask(lay.n)
    sel = np.nonzero(mask)[0]
    if sel.size:
        pos = lay.off[sel].astype(np.int64) + corrupt_pos(lay.length[sel])
        p = torch.from_numpy(pos).to(dev)
        b.arena[p] ^= 0x5A
    b.status = torch.empty(lay.n, dtype=torch.uint8, device=dev)
    b.expected_bad = int(sel.size)


# ---------------------------------------------------------------------------
# Transmit chains (rns_csum_chain_fill_dev): the shape tcp_output checksums
# (tcp.rs:938-973).  alloc_header prepends a head fragment holding the TCP header
# (buf.rs:262-291); the payload follows as the NetBuffer's data fragments.  A batching
# transmit path keeps the head fragments of consecutive packets back to back in a
# header region, so a wave's field stores share cache lines, and the payloads in a
# payload region.
# ---------------------------------------------------------------------------
@dataclass
class TxChainLayout:
    """Fragment chains of a transmit batch: packet i = fragments first[i] .. first[i+1]
    (the head fragment first), its checksum field at byte `field` of the head."""
    name: str
    frag_off: np.ndarray   # uint64
    frag_len: np.ndarray   # uint32
    first: np.ndarray      # uint32 [n + 1]
    seed: np.ndarray       # uint16
    field: int
    head: int
    arena_bytes: int
    data_seed: int
    payload_bytes: int     # sum of the packets' lengths (head + payload), the metric's bytes

    @property
    def n(self) -> int:
        return int(self.first.shape[0] - 1)


def tx_chain_layout(name: str, n: int | None = None, head: int = 20, frag: int = 0, field: int = 16,
                    data_seed: int = DATA_SEED, shard: tuple[int, int] = (0, 1)) -> TxChainLayout:
    """Packet i of config `name` (length L_i) as [a `head`-byte head fragment, L_i - head
    payload bytes].  Heads lie back to back in packet order from offset 0 (a header region
    of n * head bytes, padded to 4 KiB); payloads follow, 16-byte aligned and back to back,
    as one fragment (frag = 0) or as fragments of `frag` bytes, the last shorter (NetBuffer
    data fragments: frag = 512, buf.rs:50).  Seeds as make_layout's (the pseudo-header sums
    the caller passes)."""
    lay = make_layout(name, n=n, data_seed=data_seed, shard=shard)
    L = lay.length.astype(np.int64)
    h = np.minimum(L, head)
    pay = L - h
    nh = lay.n
    hoff = np.zeros(nh, dtype=np.int64)
    if nh > 1:
        np.cumsum(h[:-1], out=hoff[1:])
    base = (int(h.sum()) + 4095) & ~4095
    padded = (pay + ALIGN - 1) & ~(ALIGN - 1)
    poff = np.zeros(nh, dtype=np.int64)
    if nh > 1:
        np.cumsum(padded[:-1], out=poff[1:])
    poff += base
    if frag <= 0:
        nfp = (pay > 0).astype(np.int64)
    else:
        nfp = (pay + frag - 1) // frag
    nfr = 1 + nfp
    first = np.zeros(nh + 1, dtype=np.int64)
    np.cumsum(nfr, out=first[1:])
    nf = int(first[-1])
    off = np.zeros(nf, dtype=np.int64)
    ln = np.zeros(nf, dtype=np.int64)
    off[first[:-1]] = hoff
    ln[first[:-1]] = h
    pk = np.repeat(np.arange(nh), nfp)                 # packet of every payload fragment
    is_pay = np.ones(nf, dtype=bool)
    is_pay[first[:-1]] = False
    pidx = np.flatnonzero(is_pay)                       # fragment indices of the payload fragments
    k = pidx - first[pk] - 1                            # fragment number within the payload
    step = frag if frag > 0 else 0
    off[pidx] = poff[pk] + k * step
    ln[pidx] = pay[pk] if step == 0 else np.minimum(pay[pk] - k * step, step)
    arena_bytes = int(poff[-1] + padded[-1]) if nh else base
    return TxChainLayout(name=name, frag_off=off.astype(np.uint64), frag_len=ln.astype(np.uint32),
                         first=first.astype(np.uint32), seed=lay.seed, field=field, head=head,
                         arena_bytes=arena_bytes, data_seed=lay.data_seed, payload_bytes=lay.payload_bytes)


class TxChainBatch:
    """A transmit batch as NetBuffer chains in HBM (bench.py --op finalize): the chains of
    tx_chain_layout(config, head=40) — 40-byte head fragments (an IPv4 header from LOCAL4 to
    REMOTE4, then the TCP header alloc_header left: splitmix64 bytes, the checksum fields counting
    as zero) back to back in a header region, the payloads packed at 16-byte starts — with the
    fragment descriptors and a status array on the device.  A finalize of it stores the two
    checksums into every head (rns_tx_fill_chain_dev); finalizing again stores the same bytes."""

    HEAD = 40  # IPv4 header + TCP header

    def __init__(self, config: str, device, data_seed: int = DATA_SEED, frag: int = 0,
                 shard: tuple[int, int] = (0, 1)):
        import torch

        from .batch import fill_splitmix64
        lay = tx_chain_layout(config, head=self.HEAD, frag=frag, data_seed=data_seed, shard=shard)
        self.layout = lay
        self.device = device
        n = lay.n
        first = lay.first.astype(np.int64)
        self.length = (np.add.reduceat(lay.frag_len.astype(np.int64), first[:-1]) if n
                       else np.zeros(0, dtype=np.int64))
        if n and int(self.length.min()) < MIN_DATAGRAM:
            raise ValueError(f"finalize batches need datagrams of at least {MIN_DATAGRAM} B")
        self.hoff = lay.frag_off[first[:-1]].astype(np.int64) if n else np.zeros(0, dtype=np.int64)
        self.arena = torch.empty(lay.arena_bytes + 64, dtype=torch.uint8, device=device)
        fill_splitmix64(self.arena, lay.data_seed)
        hdr = torch.from_numpy(ipv4_tcp_headers(self.length, LOCAL4, REMOTE4)).to(device)
        d_hoff = torch.from_numpy(self.hoff).to(device)
        step = 1 << 20  # datagrams per scatter (bounds the index tensor)
        for i in range(0, n, step):
            idx = d_hoff[i:i + step].view(-1, 1) + torch.arange(20, device=device)
            self.arena[idx.flatten()] = hdr[i:i + step].flatten()
        self.d_off = torch.from_numpy(lay.frag_off.view(np.int64)).to(device)
        self.d_len = torch.from_numpy(lay.frag_len.view(np.int32)).to(device)
        self.d_first = torch.from_numpy(lay.first.view(np.int32)).to(device)
        self.status = torch.empty(n, dtype=torch.uint8, device=device)

    @property
    def n_frags(self) -> int:
        return int(self.layout.frag_off.shape[0])
