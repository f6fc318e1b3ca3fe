"""Batched checksums on the GPU (device-resident and host-resident), over the C ABI.

The reference has no batch API: every packet's checksum is one
util::compute_ones_comp call on the thread handling it.  A batch
here is a packet ARENA (one uint8 buffer) plus per-packet descriptors:

* ``off``  — int64 byte offset of each packet in the arena (any alignment);
* ``length`` — int32 length in bytes;
* ``seed`` — optional 16-bit seed per packet (the pseudo-header sum callers
  pass as in_checksum / initial_sum: tcp.rs:845-848, udp.rs:158-168, icmp.rs:63-71);
* ``complement`` — store ``0xffff ^ sum`` (what every call site stores or tests).

PyTorch only provides device memory and the stream; the compute is the
hand-written gfx950 kernel in csrc/rns_checksum.hip.  There is no CPU fallback:
a missing library or device raises.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib


def _require_cuda(t: torch.Tensor, name: str, dtypes) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must be on a GPU device (got {t.device}); there is no CPU fallback")
    if t.dtype not in dtypes:
        raise TypeError(f"{name} dtype {t.dtype} not in {dtypes}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


_U16 = (torch.uint16, torch.int16)


def _rx_outputs(dev: torch.device, n: int, status, l4_sum, inputs):
    """Receive verify's outputs (caller-supplied or new) and its inputs' device: the kernel
    writes n entries to each output, so an undersized or misplaced buffer is refused."""
    for name, t in inputs:
        if t.device != dev:
            raise ValueError(f"{name} is on {t.device}, the arena on {dev}")
    if status is None:
        status = torch.empty(n, dtype=torch.uint8, device=dev)
    else:
        _require_cuda(status, "status", (torch.uint8,))
        if status.numel() != n or status.device != dev:
            raise ValueError(f"status must be {n} uint8 entries on {dev}")
    if l4_sum is not None:
        _require_cuda(l4_sum, "l4_sum", _U16)
        if l4_sum.numel() != n or l4_sum.device != dev:
            raise ValueError(f"l4_sum must be {n} 16-bit entries on {dev}")
    return status, (l4_sum.data_ptr() if l4_sum is not None else None)


def _bad_ptr(bad: torch.Tensor | None, dev: torch.device):
    """The rejected-descriptor counter the kernels atomically add to: an int32 tensor of at
    least one entry on the arena's device, or None."""
    if bad is None:
        return None
    _require_cuda(bad, "bad", (torch.int32,))
    if bad.numel() < 1 or bad.device != dev:
        raise ValueError(f"bad must be an int32 counter (at least 1 entry) on {dev}")
    return bad.data_ptr()


def _stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


class PreparedBatch:
    """A device-resident batch bound to the C ABI once: validation and argument
    marshalling happen here, so each launch is a single ctypes call (a few µs of
    host time).  Launches go to the stream that was current at construction.

    ``shape`` = (variant, lanes_per_packet, unroll, max_blocks) overrides the
    automatic kernel shape (tuning); see rns_csum_batch_dev_cfg.

    ``compact=True`` selects the compact descriptor form explicitly
    (rns_csum_batch_dev_off32): ``off`` is then an int32 tensor whose bits are
    UNSIGNED 32-bit offsets (arenas below 4 GiB; 10 B of descriptors per packet
    instead of 14).  Otherwise ``off`` must be int64; an int32 ``off`` without
    ``compact=True`` is a TypeError, never a silent switch of the descriptor form.
    """

    def __init__(self, arena: torch.Tensor, off: torch.Tensor, length: torch.Tensor,
                 seed: torch.Tensor | None = None, *, complement: bool = False, out: torch.Tensor | None = None,
                 len_hint: int = 0, bad: torch.Tensor | None = None,
                 shape: tuple[int, int, int, int] | None = None, compact: bool = False):
        _require_cuda(arena, "arena", (torch.uint8,))
        _require_cuda(off, "off", (torch.int32,) if compact else (torch.int64,))
        _require_cuda(length, "length", (torch.int32,))
        if compact and shape is not None:
            raise ValueError("shape overrides take 64-bit offsets")
        n = off.numel()
        if length.numel() != n:
            raise ValueError("off and length must have the same number of packets")
        if n >= 2 ** 32:
            raise ValueError("at most 2^32-1 packets per call")
        dev = arena.device
        for name, t in (("off", off), ("length", length)):
            if t.device != dev:
                raise ValueError(f"{name} is on {t.device}, arena on {dev}")
        seed_ptr = None
        if seed is not None:
            _require_cuda(seed, "seed", _U16)
            if seed.numel() != n or seed.device != dev:
                raise ValueError("seed must have one entry per packet on the arena's device")
            seed_ptr = seed.data_ptr()
        if out is None:
            out = torch.empty(n, dtype=torch.uint16, device=dev)
        else:
            _require_cuda(out, "out", _U16)
            if out.numel() != n or out.device != dev:
                raise ValueError("out must have one entry per packet on the arena's device")
        bad_ptr = _bad_ptr(bad, arena.device)
        lib = _lib.load()
        flags = _lib.RNS_FLAG_COMPLEMENT if complement else 0
        stream = _stream_handle(dev)
        # keep the tensors alive as long as the bound pointers
        self._keep = (arena, off, length, seed, out, bad)
        self.out = out
        self.n = n
        self.device = dev
        self._name = "rns_csum_batch_dev_off32" if compact else "rns_csum_batch_dev"
        if shape is None:
            self._fn = getattr(lib, self._name)
            self._args = (arena.data_ptr(), arena.numel(), off.data_ptr(), length.data_ptr(), seed_ptr,
                          out.data_ptr(), n, flags, int(len_hint), bad_ptr, stream)
        else:
            var, g, u, mb = shape
            self._fn = lib.rns_csum_batch_dev_cfg
            self._args = (arena.data_ptr(), arena.numel(), off.data_ptr(), length.data_ptr(), seed_ptr,
                          out.data_ptr(), n, flags, var, g, u, mb, bad_ptr, stream)

    def __call__(self) -> torch.Tensor:
        if self.n:
            # The bound stream handle belongs to self.device (the null stream is 0): launch
            # with that device current even if the caller has switched devices since.
            if torch.cuda.current_device() != self.device.index:
                with torch.cuda.device(self.device):
                    st = self._fn(*self._args)
            else:
                st = self._fn(*self._args)
            if st != _lib.RNS_OK:
                raise _lib.ChecksumError(st, self._name)
        return self.out


def packed_layout(length, align_log2: int = 4, first_off: int = 0):
    """Offsets of the packed form (rns_packed_layout): packets back to back in index
    order, each starting at the next multiple of 2**align_log2.  ``length``: lengths
    (< 65536).  Returns (blk_off uint64 [ceil(n/64)], off uint64 [n], end)."""
    import numpy as np
    ln = np.asarray(length)
    if ln.size and (int(ln.max()) > 0xFFFF or int(ln.min()) < 0):
        raise ValueError("packed descriptors hold u16 lengths (< 65536)")
    len16 = np.ascontiguousarray(ln, dtype=np.uint16)
    n = int(len16.size)
    blk = np.zeros(max((n + 63) // 64, 1), dtype=np.uint64)
    off = np.zeros(max(n, 1), dtype=np.uint64)
    end = ctypes.c_uint64(0)
    st = _lib.load().rns_packed_layout(len16.ctypes.data, n, int(align_log2), int(first_off), blk.ctypes.data,
                                       off.ctypes.data, ctypes.byref(end))
    _lib.check(st, "rns_packed_layout")
    return blk[:(n + 63) // 64], off[:n], int(end.value)


class PackedBatch:
    """A device-resident batch in the packed form (rns_csum_batch_packed_dev), bound
    once like PreparedBatch: ``blk_off`` int64 [ceil(n/64)] (the offset of every 64th
    packet), ``len16`` int16/uint16 [n] (lengths as unsigned 16-bit), packets back to
    back at 2**align_log2 boundaries (see packed_layout)."""

    def __init__(self, arena: torch.Tensor, blk_off: torch.Tensor, len16: torch.Tensor,
                 seed: torch.Tensor | None = None, *, align_log2: int = 4, complement: bool = False,
                 out: torch.Tensor | None = None, len_hint: int = 0, bad: torch.Tensor | None = None):
        _require_cuda(arena, "arena", (torch.uint8,))
        _require_cuda(blk_off, "blk_off", (torch.int64,))
        _require_cuda(len16, "len16", _U16)
        n = len16.numel()
        if blk_off.numel() != (n + 63) // 64:
            raise ValueError("blk_off must have one entry per 64 packets")
        if not 0 <= align_log2 <= 12:
            raise ValueError("align_log2 must be in 0..12")
        dev = arena.device
        for name, t in (("blk_off", blk_off), ("len16", len16)):
            if t.device != dev:
                raise ValueError(f"{name} is on {t.device}, arena on {dev}")
        seed_ptr = None
        if seed is not None:
            _require_cuda(seed, "seed", _U16)
            if seed.numel() != n or seed.device != dev:
                raise ValueError("seed must have one entry per packet on the arena's device")
            seed_ptr = seed.data_ptr()
        if out is None:
            out = torch.empty(n, dtype=torch.uint16, device=dev)
        else:
            _require_cuda(out, "out", _U16)
            if out.numel() != n or out.device != dev:
                raise ValueError("out must have one entry per packet on the arena's device")
        bad_ptr = _bad_ptr(bad, arena.device)
        lib = _lib.load()
        self._keep = (arena, blk_off, len16, seed, out, bad)
        self.out, self.n, self.device = out, n, dev
        self._fn = lib.rns_csum_batch_packed_dev
        self._args = (arena.data_ptr(), arena.numel(), blk_off.data_ptr(), len16.data_ptr(), int(align_log2),
                      seed_ptr, out.data_ptr(), n, _lib.RNS_FLAG_COMPLEMENT if complement else 0, int(len_hint),
                      bad_ptr, _stream_handle(dev))

    def __call__(self) -> torch.Tensor:
        if self.n:
            if torch.cuda.current_device() != self.device.index:
                with torch.cuda.device(self.device):
                    st = self._fn(*self._args)
            else:
                st = self._fn(*self._args)
            if st != _lib.RNS_OK:
                raise _lib.ChecksumError(st, "rns_csum_batch_packed_dev")
        return self.out


def csum_batch_packed(arena: torch.Tensor, blk_off: torch.Tensor, len16: torch.Tensor,
                      seed: torch.Tensor | None = None, *, align_log2: int = 4, complement: bool = False,
                      out: torch.Tensor | None = None, len_hint: int = 0,
                      bad: torch.Tensor | None = None) -> torch.Tensor:
    """Checksum a batch in the packed form (offsets implied by lengths; see PackedBatch)."""
    _require_cuda(arena, "arena", (torch.uint8,))
    with torch.cuda.device(arena.device):
        return PackedBatch(arena, blk_off, len16, seed, align_log2=align_log2, complement=complement, out=out,
                           len_hint=len_hint, bad=bad)()


def csum_batch(arena: torch.Tensor, off: torch.Tensor, length: torch.Tensor, seed: torch.Tensor | None = None,
               *, complement: bool = False, out: torch.Tensor | None = None, len_hint: int = 0,
               bad: torch.Tensor | None = None, shape: tuple[int, int, int, int] | None = None,
               compact: bool = False) -> torch.Tensor:
    """Checksum every packet of a device-resident batch; returns uint16 [n] on the same device.

    Launches on the current torch stream of ``arena``'s device and returns
    without synchronising.  A packet outside the arena yields 0 and increments
    ``bad`` (int32 [1] device tensor) if given.  ``shape`` = (variant,
    lanes_per_packet, unroll, max_blocks) overrides the kernel shape (tuning).
    ``compact=True``: ``off`` holds unsigned 32-bit offsets in an int32 tensor.
    """
    _require_cuda(arena, "arena", (torch.uint8,))
    with torch.cuda.device(arena.device):
        return PreparedBatch(arena, off, length, seed, complement=complement, out=out, len_hint=len_hint, bad=bad,
                             shape=shape, compact=compact)()


class StridedBatch:
    """A device-resident batch of equal-length packets at a fixed stride
    (rns_csum_batch_strided_dev), bound once like PreparedBatch: packet i =
    arena[first_off + i*stride : + length].  No offset or length descriptors travel."""

    def __init__(self, arena: torch.Tensor, n: int, stride: int, length: int, *, first_off: int = 0,
                 seed: torch.Tensor | None = None, complement: bool = False,
                 out: torch.Tensor | None = None, bad: torch.Tensor | None = None):
        _require_cuda(arena, "arena", (torch.uint8,))
        dev = arena.device
        if n < 0 or n >= 2 ** 32 or stride < 0 or not 0 <= length < 2 ** 32 or first_off < 0:
            raise ValueError("n, stride, length and first_off must be non-negative (n, length < 2^32)")
        seed_ptr = None
        if seed is not None:
            _require_cuda(seed, "seed", _U16)
            if seed.numel() != n or seed.device != dev:
                raise ValueError("seed must have one entry per packet on the arena's device")
            seed_ptr = seed.data_ptr()
        if out is None:
            out = torch.empty(n, dtype=torch.uint16, device=dev)
        else:
            _require_cuda(out, "out", _U16)
            if out.numel() != n or out.device != dev:
                raise ValueError("out must have one entry per packet on the arena's device")
        bad_ptr = _bad_ptr(bad, arena.device)
        lib = _lib.load()
        self._keep = (arena, seed, out, bad)
        self.out, self.n, self.device = out, int(n), dev
        self._fn = lib.rns_csum_batch_strided_dev
        self._args = (arena.data_ptr(), arena.numel(), int(first_off), int(stride), int(length), seed_ptr,
                      out.data_ptr(), int(n), _lib.RNS_FLAG_COMPLEMENT if complement else 0, bad_ptr,
                      _stream_handle(dev))

    def __call__(self) -> torch.Tensor:
        if self.n:
            if torch.cuda.current_device() != self.device.index:
                with torch.cuda.device(self.device):
                    st = self._fn(*self._args)
            else:
                st = self._fn(*self._args)
            if st != _lib.RNS_OK:
                raise _lib.ChecksumError(st, "rns_csum_batch_strided_dev")
        return self.out


def csum_batch_strided(arena: torch.Tensor, n: int, stride: int, length: int, *, first_off: int = 0,
                       seed: torch.Tensor | None = None, complement: bool = False,
                       out: torch.Tensor | None = None, bad: torch.Tensor | None = None) -> torch.Tensor:
    """Packets at a fixed stride: packet i = arena[first_off + i*stride : + length]."""
    _require_cuda(arena, "arena", (torch.uint8,))
    with torch.cuda.device(arena.device):
        return StridedBatch(arena, n, stride, length, first_off=first_off, seed=seed, complement=complement,
                            out=out, bad=bad)()


def csum_chain(arena: torch.Tensor, frag_off: torch.Tensor, frag_len: torch.Tensor, first: torch.Tensor,
               seed: torch.Tensor | None = None, *, complement: bool = False, out: torch.Tensor | None = None,
               frag_sums: torch.Tensor | None = None, bad: torch.Tensor | None = None,
               frag_len_hint: int = 512, runs: bool = False, tx_packed: bool = False) -> torch.Tensor:
    """util.rs:112 ``compute_buffer_ones_comp`` for a batch of fragment chains.

    Packet i = fragments ``first[i] .. first[i+1]`` (``first``: int32 [n+1]) of
    ``(frag_off, frag_len)``; each fragment is folded on its own like the reference,
    in one pass (``frag_sums`` is accepted for compatibility and unused).
    ``runs``: RNS_FLAG_CHAIN_RUNS, the hint that fragments are often back-to-back
    views of one buffer (same results either way).  ``tx_packed``: RNS_FLAG_CHAIN_TX_PACKED
    (see csum_chain_fill).
    """
    _require_cuda(arena, "arena", (torch.uint8,))
    _require_cuda(frag_off, "frag_off", (torch.int64,))
    _require_cuda(frag_len, "frag_len", (torch.int32,))
    _require_cuda(first, "first", (torch.int32,))
    nf = frag_off.numel()
    n = first.numel() - 1
    if frag_len.numel() != nf or n < 0:
        raise ValueError("frag_off/frag_len sizes differ or first is empty")
    if n > _lib.RNS_CHAIN_MAX_PACKETS or nf >= 2 ** 32:
        raise ValueError(f"at most {_lib.RNS_CHAIN_MAX_PACKETS} packets and 2^32-1 fragments per chain call")
    dev = arena.device
    seed_ptr = None
    if seed is not None:
        _require_cuda(seed, "seed", _U16)
        if seed.numel() != n:
            raise ValueError("seed must have one entry per packet")
        seed_ptr = seed.data_ptr()
    if out is None:
        out = torch.empty(max(n, 0), dtype=torch.uint16, device=dev)
    bad_ptr = _bad_ptr(bad, arena.device)
    lib = _lib.load()
    with torch.cuda.device(dev):
        st = lib.rns_csum_chain_dev(arena.data_ptr(), arena.numel(), frag_off.data_ptr(), frag_len.data_ptr(), nf,
                                    first.data_ptr(), seed_ptr, out.data_ptr(), n,
                                    (_lib.RNS_FLAG_COMPLEMENT if complement else 0) |
                                    (_lib.RNS_FLAG_CHAIN_RUNS if runs else 0) |
                                    (_lib.RNS_FLAG_CHAIN_TX_PACKED if tx_packed else 0), frag_len_hint,
                                    frag_sums.data_ptr() if frag_sums is not None else None, bad_ptr,
                                    _stream_handle(dev))
    _lib.check(st, "rns_csum_chain_dev")
    return out


def csum_chain_fill(arena: torch.Tensor, frag_off: torch.Tensor, frag_len: torch.Tensor, first: torch.Tensor,
                    seed: torch.Tensor | None = None, *, field: torch.Tensor | None = None, field_off: int = 16,
                    complement: bool = True, out: torch.Tensor | None = None, bad: torch.Tensor | None = None,
                    frag_len_hint: int = 512, runs: bool = False, tx_packed: bool = False) -> torch.Tensor | None:
    """Transmit fill over fragment chains (rns_csum_chain_fill_dev): packet i = fragments
    ``first[i] .. first[i+1]`` as for ``csum_chain``; its checksum field is at byte
    ``field[i]`` (or ``field_off``) of its FIRST fragment (the head fragment
    alloc_header prepended, buf.rs:262-291), counts as zero, and receives
    ``compute_buffer_ones_comp(seed, chain) ^ 0xffff`` big-endian (tcp.rs:957-973).
    ``tx_packed``: RNS_FLAG_CHAIN_TX_PACKED, the hint that packets are [head <= 4 chunks,
    payload run] with the payloads packed at 16-byte starts (same results either way).
    Returns ``out`` if given."""
    _require_cuda(arena, "arena", (torch.uint8,))
    _require_cuda(frag_off, "frag_off", (torch.int64,))
    _require_cuda(frag_len, "frag_len", (torch.int32,))
    _require_cuda(first, "first", (torch.int32,))
    nf = frag_off.numel()
    n = first.numel() - 1
    if frag_len.numel() != nf or n < 0:
        raise ValueError("frag_off/frag_len sizes differ or first is empty")
    if n > _lib.RNS_CHAIN_MAX_PACKETS or nf >= 2 ** 32:
        raise ValueError(f"at most {_lib.RNS_CHAIN_MAX_PACKETS} packets and 2^32-1 fragments per chain call")
    dev = arena.device
    for name, t in (("frag_off", frag_off), ("frag_len", frag_len), ("first", first)):
        if t.device != dev:
            raise ValueError(f"{name} is on {t.device}, arena on {dev}")
    ptrs = []
    for name, t in (("seed", seed), ("field", field), ("out", out)):
        if t is None:
            ptrs.append(None)
            continue
        _require_cuda(t, name, _U16)
        if t.numel() != n or t.device != dev:
            raise ValueError(f"{name} must have one entry per packet on the arena's device")
        ptrs.append(t.data_ptr())
    if field is None and not 0 <= int(field_off) < 2 ** 32:
        raise ValueError("field_off must be a u32")
    bad_ptr = _bad_ptr(bad, arena.device)
    flags = (_lib.RNS_FLAG_COMPLEMENT if complement else 0) | (_lib.RNS_FLAG_CHAIN_RUNS if runs else 0) | \
        (_lib.RNS_FLAG_CHAIN_TX_PACKED if tx_packed else 0)
    with torch.cuda.device(dev):
        st = _lib.load().rns_csum_chain_fill_dev(arena.data_ptr(), arena.numel(), frag_off.data_ptr(),
                                                 frag_len.data_ptr(), nf, first.data_ptr(), ptrs[0], ptrs[1],
                                                 int(field_off), ptrs[2], n, flags, int(frag_len_hint), bad_ptr,
                                                 _stream_handle(dev))
    _lib.check(st, "rns_csum_chain_fill_dev")
    return out


def csum_fill(arena: torch.Tensor, off: torch.Tensor, length: torch.Tensor, seed: torch.Tensor | None = None, *,
              field: torch.Tensor | None = None, field_off: int = 16, complement: bool = True,
              out: torch.Tensor | None = None, bad: torch.Tensor | None = None) -> torch.Tensor | None:
    """Transmit in-place fill: each packet's checksum, computed with its 2-byte field
    counted as zero, is stored big-endian into the field (tcp.rs:970-973 ``set_be16``).

    ``field`` (int16/uint16 [n]) gives per-packet field offsets, else ``field_off``
    for all (TCP 16, UDP 6, ICMP 2, IPv4 header 10).  Returns ``out`` if given.
    """
    _require_cuda(arena, "arena", (torch.uint8,))
    _require_cuda(off, "off", (torch.int64,))
    _require_cuda(length, "length", (torch.int32,))
    n = off.numel()
    if length.numel() != n:
        raise ValueError("off and length must have the same number of packets")
    dev = arena.device
    ptrs = []
    for name, t in (("seed", seed), ("field", field), ("out", out)):
        if t is None:
            ptrs.append(None)
            continue
        _require_cuda(t, name, _U16)
        if t.numel() != n or t.device != dev:
            raise ValueError(f"{name} must have one entry per packet on the arena's device")
        ptrs.append(t.data_ptr())
    bad_ptr = _bad_ptr(bad, arena.device)
    lib = _lib.load()
    with torch.cuda.device(dev):
        st = lib.rns_csum_fill_dev(arena.data_ptr(), arena.numel(), off.data_ptr(), length.data_ptr(), ptrs[0],
                                   ptrs[1], int(field_off), ptrs[2], n,
                                   _lib.RNS_FLAG_COMPLEMENT if complement else 0, bad_ptr, _stream_handle(dev))
    _lib.check(st, "rns_csum_fill_dev")
    return out


def csum_fill_packed(arena: torch.Tensor, blk_off: torch.Tensor, len16: torch.Tensor,
                     seed: torch.Tensor | None = None, *, align_log2: int = 4, field: torch.Tensor | None = None,
                     field_off: int = 16, complement: bool = True, out: torch.Tensor | None = None,
                     len_hint: int = 0, bad: torch.Tensor | None = None) -> torch.Tensor | None:
    """Transmit in-place fill of a packed arena (rns_csum_fill_packed_dev): ``csum_fill``'s
    result and stores, with the packed form's descriptors (see PackedBatch; align_log2 >= 4)."""
    _require_cuda(arena, "arena", (torch.uint8,))
    _require_cuda(blk_off, "blk_off", (torch.int64,))
    _require_cuda(len16, "len16", _U16)
    n = len16.numel()
    if blk_off.numel() != (n + 63) // 64:
        raise ValueError("blk_off must have one entry per 64 packets")
    if not 4 <= align_log2 <= 12:
        raise ValueError("the packed fill needs align_log2 in 4..12")
    if field is None and not 0 <= int(field_off) <= 0xFFFD:
        # packed lengths are u16: no packet can hold a field past byte 65533 (the C ABI itself
        # rejects every packet of such a call and leaves the arena unchanged)
        raise ValueError("field_off must be in 0..65533 for the packed form")
    dev = arena.device
    ptrs = []
    for name, t in (("blk_off", blk_off), ("len16", len16)):
        if t.device != dev:
            raise ValueError(f"{name} is on {t.device}, arena on {dev}")
    for name, t in (("seed", seed), ("field", field), ("out", out)):
        if t is None:
            ptrs.append(None)
            continue
        _require_cuda(t, name, _U16)
        if t.numel() != n or t.device != dev:
            raise ValueError(f"{name} must have one entry per packet on the arena's device")
        ptrs.append(t.data_ptr())
    bad_ptr = _bad_ptr(bad, arena.device)
    lib = _lib.load()
    with torch.cuda.device(dev):
        st = lib.rns_csum_fill_packed_dev(arena.data_ptr(), arena.numel(), blk_off.data_ptr(), len16.data_ptr(),
                                          int(align_log2), ptrs[0], ptrs[1], int(field_off), ptrs[2], n,
                                          _lib.RNS_FLAG_COMPLEMENT if complement else 0, int(len_hint), bad_ptr,
                                          _stream_handle(dev))
    _lib.check(st, "rns_csum_fill_packed_dev")
    return out


def rx_verify(arena: torch.Tensor, off: torch.Tensor, length: torch.Tensor, local_ipv4: bytes, local_ipv6: bytes,
              *, status: torch.Tensor | None = None, l4_sum: torch.Tensor | None = None) -> torch.Tensor:
    """Receive verify of a batch of IP datagrams (rns_rx_verify_dev): returns a uint8
    status per packet (RNS_RX_* bits; RNS_RX_ACCEPT = the stack would deliver it)."""
    _require_cuda(arena, "arena", (torch.uint8,))
    _require_cuda(off, "off", (torch.int64,))
    _require_cuda(length, "length", (torch.int32,))
    if len(local_ipv4) != 4 or len(local_ipv6) != 16:
        raise ValueError("local_ipv4 must be 4 bytes and local_ipv6 16 bytes")
    n = off.numel()
    if length.numel() != n:
        raise ValueError("off and length must have the same number of datagrams")
    dev = arena.device
    lib = _lib.load()
    status, l4_ptr = _rx_outputs(dev, n, status, l4_sum, (("off", off), ("length", length)))
    with torch.cuda.device(dev):
        st = lib.rns_rx_verify_dev(arena.data_ptr(), arena.numel(), off.data_ptr(), length.data_ptr(), n,
                                   bytes(local_ipv4), bytes(local_ipv6), status.data_ptr(), l4_ptr,
                                   _stream_handle(dev))
    _lib.check(st, "rns_rx_verify_dev")
    return status


def rx_verify_packed(arena: torch.Tensor, blk_off: torch.Tensor, len16: torch.Tensor, local_ipv4: bytes,
                     local_ipv6: bytes, *, align_log2: int = 4, status: torch.Tensor | None = None,
                     l4_sum: torch.Tensor | None = None) -> torch.Tensor:
    """Receive verify of a PACKED arena of datagrams (rns_rx_verify_packed_dev: u16 lengths,
    one offset per 64 datagrams, 16-byte-aligned starts): the same uint8 status per datagram
    as rx_verify."""
    _require_cuda(arena, "arena", (torch.uint8,))
    _require_cuda(blk_off, "blk_off", (torch.int64,))
    _require_cuda(len16, "len16", _U16)
    if len(local_ipv4) != 4 or len(local_ipv6) != 16:
        raise ValueError("local_ipv4 must be 4 bytes and local_ipv6 16 bytes")
    n = len16.numel()
    if blk_off.numel() < (n + 63) // 64:
        raise ValueError("blk_off needs one offset per 64 datagrams")
    dev = arena.device
    lib = _lib.load()
    status, l4_ptr = _rx_outputs(dev, n, status, l4_sum, (("blk_off", blk_off), ("len16", len16)))
    with torch.cuda.device(dev):
        st = lib.rns_rx_verify_packed_dev(arena.data_ptr(), arena.numel(), blk_off.data_ptr(), len16.data_ptr(),
                                          int(align_log2), n, bytes(local_ipv4), bytes(local_ipv6),
                                          status.data_ptr(), l4_ptr, _stream_handle(dev))
    _lib.check(st, "rns_rx_verify_packed_dev")
    return status


def rx_verify_strided(arena: torch.Tensor, stride: int, len16: torch.Tensor, local_ipv4: bytes, local_ipv6: bytes,
                      *, first_off: int = 0, status: torch.Tensor | None = None,
                      l4_sum: torch.Tensor | None = None) -> torch.Tensor:
    """Receive verify of datagrams at a fixed stride (rns_rx_verify_strided_dev): datagram i
    = ``arena[first_off + i*stride : + len16[i]]``, a ring of fixed-size receive slots.  The
    same uint8 status per datagram as rx_verify."""
    _require_cuda(arena, "arena", (torch.uint8,))
    _require_cuda(len16, "len16", _U16)
    if len(local_ipv4) != 4 or len(local_ipv6) != 16:
        raise ValueError("local_ipv4 must be 4 bytes and local_ipv6 16 bytes")
    if not (0 <= int(first_off) < 2 ** 64 and 0 <= int(stride) < 2 ** 64):
        raise ValueError("first_off and stride must be u64")
    n = len16.numel()
    if n >= 2 ** 32:
        raise ValueError("at most 2^32-1 datagrams per call")
    dev = arena.device
    lib = _lib.load()
    status, l4_ptr = _rx_outputs(dev, n, status, l4_sum, (("len16", len16),))
    with torch.cuda.device(dev):
        st = lib.rns_rx_verify_strided_dev(arena.data_ptr(), arena.numel(), int(first_off), int(stride),
                                           len16.data_ptr(), n, bytes(local_ipv4), bytes(local_ipv6),
                                           status.data_ptr(), l4_ptr, _stream_handle(dev))
    _lib.check(st, "rns_rx_verify_strided_dev")
    return status


def tx_fill_packed(arena: torch.Tensor, blk_off: torch.Tensor, len16: torch.Tensor, *, align_log2: int = 4,
                   status: torch.Tensor | None = None, len_hint: int = 0) -> torch.Tensor:
    """Transmit finalize of a PACKED arena of outgoing datagrams (rns_tx_fill_packed_dev: u16
    lengths, one offset per 64 datagrams, starts at 2^align_log2 boundaries, align_log2 >= 4):
    the bytes and the uint8 status per datagram of ``tx_fill``."""
    _require_cuda(arena, "arena", (torch.uint8,))
    _require_cuda(blk_off, "blk_off", (torch.int64,))
    _require_cuda(len16, "len16", _U16)
    n = len16.numel()
    if blk_off.numel() < (n + 63) // 64:
        raise ValueError("blk_off needs one offset per 64 datagrams")
    if not 4 <= align_log2 <= 12:
        raise ValueError("the packed transmit finalize needs align_log2 in 4..12")
    if n >= 2 ** 32:
        raise ValueError("at most 2^32-1 datagrams per call")
    dev = arena.device
    for name, t in (("blk_off", blk_off), ("len16", len16)):
        if t.device != dev:
            raise ValueError(f"{name} is on {t.device}, arena on {dev}")
    if status is None:
        status = torch.empty(n, dtype=torch.uint8, device=dev)
    else:
        _require_cuda(status, "status", (torch.uint8,))
        if status.numel() != n or status.device != dev:
            raise ValueError(f"status must be {n} uint8 entries on {dev}")
    with torch.cuda.device(dev):
        st = _lib.load().rns_tx_fill_packed_dev(arena.data_ptr(), arena.numel(), blk_off.data_ptr(),
                                               len16.data_ptr(), int(align_log2), n, status.data_ptr(),
                                               int(len_hint), _stream_handle(dev))
    _lib.check(st, "rns_tx_fill_packed_dev")
    return status


def tx_fill_chain(arena: torch.Tensor, frag_off: torch.Tensor, frag_len: torch.Tensor, first: torch.Tensor, *,
                  status: torch.Tensor | None = None) -> torch.Tensor:
    """Transmit finalize of datagrams held as NetBuffer chains (rns_tx_fill_chain_dev):
    datagram i = fragments ``first[i] .. first[i+1]`` as for ``csum_chain``, its FIRST
    fragment the head alloc_header built (the IP header, then the L4 header: buf.rs:262-291),
    the rest its payload.  The L4 checksum over [head[hdr:], payload...] (folded per fragment,
    tcp.rs:957-973, udp.rs:151-171, icmp.rs:87-112) and the IPv4 header checksum
    (ip.rs:140-160) are stored into the head.  Returns a uint8 status per datagram (RNS_TX_*)."""
    _require_cuda(arena, "arena", (torch.uint8,))
    _require_cuda(frag_off, "frag_off", (torch.int64,))
    _require_cuda(frag_len, "frag_len", (torch.int32,))
    _require_cuda(first, "first", (torch.int32,))
    nf = frag_off.numel()
    n = first.numel() - 1
    if frag_len.numel() != nf or n < 0:
        raise ValueError("frag_off/frag_len sizes differ or first is empty")
    if n > _lib.RNS_CHAIN_MAX_PACKETS or nf >= 2 ** 32:
        raise ValueError(f"at most {_lib.RNS_CHAIN_MAX_PACKETS} datagrams and 2^32-1 fragments per chain call")
    dev = arena.device
    for name, t in (("frag_off", frag_off), ("frag_len", frag_len), ("first", first)):
        if t.device != dev:
            raise ValueError(f"{name} is on {t.device}, arena on {dev}")
    if status is None:
        status = torch.empty(n, dtype=torch.uint8, device=dev)
    else:
        _require_cuda(status, "status", (torch.uint8,))
        if status.numel() != n or status.device != dev:
            raise ValueError(f"status must be {n} uint8 entries on {dev}")
    with torch.cuda.device(dev):
        st = _lib.load().rns_tx_fill_chain_dev(arena.data_ptr(), arena.numel(), frag_off.data_ptr(),
                                              frag_len.data_ptr(), nf, first.data_ptr(), n, status.data_ptr(),
                                              _stream_handle(dev))
    _lib.check(st, "rns_tx_fill_chain_dev")
    return status


def tx_fill(arena: torch.Tensor, off: torch.Tensor, length: torch.Tensor, *,
            status: torch.Tensor | None = None) -> torch.Tensor:
    """Transmit finalize of a batch of outgoing IP datagrams (rns_tx_fill_dev): the
    IPv4 header checksum and the TCP / UDP / ICMP checksum of every datagram stored in
    place, pseudo-headers formed on the device (tcp.rs:957-973, udp.rs:151-171,
    icmp.rs:87-112, ip.rs:140-160).  Returns a uint8 status per datagram (RNS_TX_*)."""
    _require_cuda(arena, "arena", (torch.uint8,))
    _require_cuda(off, "off", (torch.int64,))
    _require_cuda(length, "length", (torch.int32,))
    n = off.numel()
    if length.numel() != n:
        raise ValueError("off and length must have the same number of datagrams")
    dev = arena.device
    if status is None:
        status = torch.empty(n, dtype=torch.uint8, device=dev)
    else:
        _require_cuda(status, "status", (torch.uint8,))
        if status.numel() != n:
            raise ValueError("status must have one entry per datagram")
    with torch.cuda.device(dev):
        st = _lib.load().rns_tx_fill_dev(arena.data_ptr(), arena.numel(), off.data_ptr(), length.data_ptr(), n,
                                        status.data_ptr(), _stream_handle(dev))
    _lib.check(st, "rns_tx_fill_dev")
    return status


def fill_splitmix64(buf: torch.Tensor, seed: int) -> torch.Tensor:
    """Fill a device uint8 buffer with the splitmix64 byte stream (same bytes as
    oracle.splitmix64_bytes(seed, n))."""
    _require_cuda(buf, "buf", (torch.uint8,))
    lib = _lib.load()
    with torch.cuda.device(buf.device):
        st = lib.rns_fill_splitmix64_dev(buf.data_ptr(), buf.numel(), seed & 0xFFFFFFFFFFFFFFFF,
                                         _stream_handle(buf.device))
    _lib.check(st, "rns_fill_splitmix64_dev")
    return buf


def recv_batch(fd: int, arena: np.ndarray, slot_bytes: int = 2048, max_pkts: int | None = None,
               timeout_ms: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """Read every queued datagram (after waiting up to ``timeout_ms`` for the first)
    into consecutive ``slot_bytes`` slots of ``arena`` (rns_io_recv_batch; the batched
    form of recv_packet, netif.rs:65-83).  Returns (offsets uint64, lengths uint32)."""
    if arena.dtype != np.uint8 or not arena.flags["C_CONTIGUOUS"]:
        raise ValueError("arena must be a contiguous uint8 array")
    cap = arena.shape[0] // slot_bytes
    max_pkts = cap if max_pkts is None else min(max_pkts, cap)
    off = np.empty(max(max_pkts, 1), dtype=np.uint64)
    ln = np.empty(max(max_pkts, 1), dtype=np.uint32)
    r = _lib.load().rns_io_recv_batch(int(fd), arena.ctypes.data, slot_bytes, max_pkts, off.ctypes.data,
                                      ln.ctypes.data, int(timeout_ms))
    if r < 0:
        raise _lib.ChecksumError(r, "rns_io_recv_batch")
    return off[:r], ln[:r]


def recv_batch_packed(fd: int, arena: np.ndarray, mru: int = 2048, max_pkts: int | None = None,
                      timeout_ms: int = 0) -> tuple[np.ndarray, np.ndarray, int]:
    """Read every queued datagram (after waiting up to ``timeout_ms`` for the first) into
    ``arena`` PACKED: each at the next 16-byte boundary while a datagram of ``mru`` bytes
    still fits (rns_io_recv_batch_packed).  Returns (lengths uint16 [n], blk_off uint64
    [ceil(n/64)], end) — the packed form's descriptors (rx_verify_packed) and the bytes used."""
    if arena.dtype != np.uint8 or not arena.flags["C_CONTIGUOUS"]:
        raise ValueError("arena must be a contiguous uint8 array")
    if not 0 < int(mru) <= 0xFFFF:
        raise ValueError("mru must be in 1..65535 (the packed form's lengths are u16)")
    cap = arena.shape[0] // 16  # no more datagrams than 16-byte slots
    max_pkts = cap if max_pkts is None else min(int(max_pkts), cap)
    max_pkts = min(max_pkts, 2 ** 31 - 1)
    ln = np.empty(max(max_pkts, 1), dtype=np.uint16)
    blk = np.empty(max((max_pkts + 63) // 64, 1), dtype=np.uint64)
    end = ctypes.c_uint64(0)
    if max_pkts <= 0:
        return ln[:0], blk[:0], 0
    r = _lib.load().rns_io_recv_batch_packed(int(fd), arena.ctypes.data, arena.shape[0], int(mru), max_pkts,
                                             ln.ctypes.data, blk.ctypes.data, ctypes.byref(end), int(timeout_ms))
    if r < 0:
        raise _lib.ChecksumError(r, "rns_io_recv_batch_packed")
    return ln[:r], blk[:(r + 63) // 64], int(end.value)


def send_batch(fd: int, arena: np.ndarray, off: np.ndarray, length: np.ndarray) -> int:
    """Write one datagram per packet (rns_io_send_batch; batched send_packet, netif.rs:85-98)."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    r = _lib.load().rns_io_send_batch(int(fd), arena.ctypes.data, off.ctypes.data, length.ctypes.data,
                                      off.shape[0])
    if r < 0:
        raise _lib.ChecksumError(r, "rns_io_send_batch")
    return r


def send_batch_chain(fd: int, arena: np.ndarray, frag_off: np.ndarray, frag_len: np.ndarray,
                     first: np.ndarray) -> int:
    """Send NetBuffer chains (rns_io_send_batch_chain; batched send_packet, netif.rs:85-98):
    datagram i = fragments ``first[i] .. first[i+1]`` of ``arena`` gathered into one datagram,
    as to_iovec + tun_send's writev do.  Returns the number of datagrams sent."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    frag_off = np.ascontiguousarray(frag_off, dtype=np.uint64)
    frag_len = np.ascontiguousarray(frag_len, dtype=np.uint32)
    first = np.ascontiguousarray(first, dtype=np.uint32)
    n = first.shape[0] - 1
    if n < 0 or frag_off.shape[0] != frag_len.shape[0]:
        raise ValueError("first needs n+1 entries; frag_off and frag_len one per fragment")
    if n and int(first[-1]) > frag_off.shape[0]:
        raise ValueError("first points past the fragment arrays")
    if frag_off.shape[0] and int((frag_off + frag_len.astype(np.uint64)).max()) > arena.shape[0]:
        raise ValueError("a fragment lies outside the arena")
    r = _lib.load().rns_io_send_batch_chain(int(fd), arena.ctypes.data, frag_off.ctypes.data, frag_len.ctypes.data,
                                            first.ctypes.data, n)
    if r < 0:
        raise _lib.ChecksumError(r, "rns_io_send_batch_chain")
    return r


class PinnedBuffer:
    """Page-locked host memory (rns_host_alloc) viewed as a numpy uint8 array."""

    def __init__(self, nbytes: int):
        lib = _lib.load()
        p = ctypes.c_void_p()
        _lib.check(lib.rns_host_alloc(max(nbytes, 1), ctypes.byref(p)), "rns_host_alloc")
        self.ptr = p.value
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * max(nbytes, 1)).from_address(self.ptr))[:nbytes]

    def free(self) -> None:
        if self.ptr:
            self.array = None
            _lib.load().rns_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class HostBatcher:
    """Host-resident batches: chunked H2D, kernel, D2H of results overlapped on
    ``nstreams`` streams (rns_csum_batch_host).  Offsets must be ascending."""

    def __init__(self, device: int = 0, chunk_bytes: int = 64 << 20, nstreams: int = 3):
        lib = _lib.load()
        ctx = ctypes.c_void_p()
        _lib.check(lib.rns_host_ctx_create(device, chunk_bytes, nstreams, ctypes.byref(ctx)), "rns_host_ctx_create")
        self.ctx = ctx.value

    def run(self, arena: np.ndarray, off: np.ndarray, length: np.ndarray, seed: np.ndarray | None = None,
            complement: bool = False, out: np.ndarray | None = None) -> np.ndarray:
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        n = off.shape[0]
        if out is None:
            out = np.empty(n, dtype=np.uint16)
        sp = None
        if seed is not None:
            seed = np.ascontiguousarray(seed, dtype=np.uint16)
            sp = seed.ctypes.data
        st = _lib.load().rns_csum_batch_host(self.ctx, arena.ctypes.data, arena.shape[0], off.ctypes.data,
                                             length.ctypes.data, sp, out.ctypes.data, n,
                                             _lib.RNS_FLAG_COMPLEMENT if complement else 0)
        _lib.check(st, "rns_csum_batch_host")
        return out

    def close(self) -> None:
        if self.ctx:
            _lib.load().rns_host_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiHostBatcher(HostBatcher):
    """Host-resident batches over several GPUs (rns_csum_batch_multi_host): the
    batch is cut into contiguous packet ranges of about equal bytes, one per entry
    of ``devices`` (a device may repeat), each through its own staging context."""

    def __init__(self, devices, chunk_bytes: int = 64 << 20, nstreams: int = 3):
        lib = _lib.load()
        devs = (ctypes.c_int * len(devices))(*devices)
        ctx = ctypes.c_void_p()
        _lib.check(lib.rns_multi_ctx_create(devs, len(devices), chunk_bytes, nstreams, ctypes.byref(ctx)),
                   "rns_multi_ctx_create")
        self.ctx = ctx.value
        self.devices = list(devices)

    def run(self, arena: np.ndarray, off: np.ndarray, length: np.ndarray, seed: np.ndarray | None = None,
            complement: bool = False, out: np.ndarray | None = None) -> np.ndarray:
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        n = off.shape[0]
        if out is None:
            out = np.empty(n, dtype=np.uint16)
        sp = None
        if seed is not None:
            seed = np.ascontiguousarray(seed, dtype=np.uint16)
            sp = seed.ctypes.data
        st = _lib.load().rns_csum_batch_multi_host(self.ctx, arena.ctypes.data, arena.shape[0], off.ctypes.data,
                                                   length.ctypes.data, sp, out.ctypes.data, n,
                                                   _lib.RNS_FLAG_COMPLEMENT if complement else 0)
        _lib.check(st, "rns_csum_batch_multi_host")
        return out

    def close(self) -> None:
        if self.ctx:
            _lib.load().rns_multi_ctx_destroy(self.ctx)
            self.ctx = None


def csum_batch_multi_dev(shards, *, complement: bool = False) -> None:
    """Launch every GPU's shard (rns_csum_batch_multi_dev).  ``shards``: a sequence of
    dicts with keys arena, off, length, out (torch tensors on that shard's device)
    and optional seed, len_hint, stream.  Asynchronous on each device's stream."""
    arr = (_lib.RnsDevBatch * len(shards))()
    keep = []
    for k, sh in enumerate(shards):
        arena, off, length, out = sh["arena"], sh["off"], sh["length"], sh["out"]
        seed = sh.get("seed")
        for t, name, dt in ((arena, "arena", (torch.uint8,)), (off, "off", (torch.int64,)),
                            (length, "length", (torch.int32,)), (out, "out", _U16)):
            _require_cuda(t, name, dt)
        if seed is not None:
            _require_cuda(seed, "seed", _U16)
        n = off.shape[0]
        if length.shape[0] != n or out.shape[0] < n or (seed is not None and seed.shape[0] < n):
            raise ValueError(f"shard {k}: descriptor arrays disagree in length")
        dev = arena.device.index
        if any(t.device != arena.device for t in (off, length, out)):
            raise ValueError(f"shard {k}: tensors on different devices")
        stream = sh.get("stream")
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        hint = sh.get("len_hint")
        if hint is None:
            hint = int(length.float().mean().item()) if n else 0
        arr[k] = _lib.RnsDevBatch(dev, arena.data_ptr(), arena.numel(), off.data_ptr(), length.data_ptr(),
                                  seed.data_ptr() if seed is not None else None, out.data_ptr(), n, hint, None,
                                  stream.cuda_stream)
        keep.append(sh)
    flags = _lib.RNS_FLAG_COMPLEMENT if complement else 0
    _lib.check(_lib.load().rns_csum_batch_multi_dev(arr, len(shards), flags), "rns_csum_batch_multi_dev")
