"""Python mirror of the reference's checksum surface, `netstack::util`
(jbush001/RustNetworkStack src/stack/util.rs), over the C ABI.

Same names, argument meaning and error behaviour as the Rust functions:

==================================  =====================================
reference (util.rs)                 here
==================================  =====================================
``compute_ones_comp`` :88-106       ``compute_ones_comp(in_checksum, slice)``
``compute_checksum`` :108-110       ``compute_checksum(slice)``
``compute_buffer_ones_comp`` :112   ``compute_buffer_ones_comp(initial_sum, buffer)``
``compute_pseudo_header_checksum``  ``compute_pseudo_header_checksum(src, dst, length, protocol)``
  :180-207
``IPAddr`` :22-57                   ``IPAddr`` (``V4`` / ``V6`` / ``new_from`` / ``copy_to``)
``set_be16`` / ``get_be16`` ...     same names (the checksum store convention)
==================================  =====================================

Where the reference panics (empty slice, util.rs:92; IPAddr length mismatch,
util.rs:47, 51-56) these raise ``ReferencePanic``.  Per-packet calls run the
library's host path (rns_compute_*); batches go to the GPU (``batch.py``).
"""
from __future__ import annotations

import ctypes
from typing import Iterable

from . import _lib


class ReferencePanic(RuntimeError):
    """Raised where the Rust reference would panic."""


def _bytes(data) -> bytes:
    if isinstance(data, bytes):
        return data
    return data.tobytes() if hasattr(data, "tobytes") else bytes(data)


def _buf(data) -> tuple[bytes, int]:
    b = _bytes(data)
    return b, len(b)


def _result(r: int, what: str) -> int:
    if r == _lib.RNS_E_EMPTY:
        raise ReferencePanic(f"{what}: empty slice (util.rs:92 would panic)")
    if r == _lib.RNS_E_INVALID:
        raise ReferencePanic(f"{what}: invalid argument (the reference panics)")
    if r < 0:
        raise _lib.ChecksumError(r, what)
    return r


def compute_ones_comp(in_checksum: int, slice) -> int:
    """util.rs:88 — one's complement sum of `slice` seeded with `in_checksum` (not complemented)."""
    b, n = _buf(slice)
    return _result(_lib.load().rns_compute_ones_comp(in_checksum & 0xFFFF, b, n), "compute_ones_comp")


def compute_checksum(slice) -> int:
    """util.rs:108 — 0xffff ^ compute_ones_comp(0, slice)."""
    b, n = _buf(slice)
    return _result(_lib.load().rns_compute_checksum(b, n), "compute_checksum")


def compute_buffer_ones_comp(initial_sum: int, buffer: Iterable) -> int:
    """util.rs:112 — fold each fragment of `buffer` in turn (buf.rs:466-487 order).

    `buffer` is anything that yields the fragment slices (a list of bytes, or an
    object with ``iter()`` like NetBuffer's).
    """
    frags = list(buffer.iter()) if hasattr(buffer, "iter") else list(buffer)
    keep = [_bytes(f) for f in frags]
    arr = (_lib.RnsIovec * max(len(keep), 1))()
    for i, f in enumerate(keep):
        arr[i].base = ctypes.cast(ctypes.c_char_p(f), ctypes.c_void_p).value if f else None
        arr[i].len = len(f)
    return _result(_lib.load().rns_compute_buffer_ones_comp(initial_sum & 0xFFFF, arr, len(keep)),
                   "compute_buffer_ones_comp")


class IPAddr:
    """`enum IPAddr { V4([u8;4]), V6([u8;16]) }` (util.rs:22-57)."""

    __slots__ = ("addr",)

    def __init__(self, addr: bytes):
        self.addr = bytes(addr)

    @classmethod
    def V4(cls, addr) -> "IPAddr":
        a = bytes(addr)
        if len(a) != 4:
            raise ReferencePanic("V4 address must be 4 bytes")
        return cls(a)

    @classmethod
    def V6(cls, addr) -> "IPAddr":
        a = bytes(addr)
        if len(a) != 16:
            raise ReferencePanic("V6 address must be 16 bytes")
        return cls(a)

    @classmethod
    def new_from(cls, addr) -> "IPAddr":
        a = bytes(addr)
        if len(a) not in (4, 16):
            raise ReferencePanic("Invalid IP address length")  # util.rs:47
        return cls(a)

    @property
    def is_v4(self) -> bool:
        return len(self.addr) == 4

    def copy_to(self, buffer: bytearray) -> None:
        if len(buffer) != len(self.addr):
            raise ReferencePanic("copy_from_slice length mismatch (util.rs:51-56)")
        buffer[:] = self.addr

    def _c(self) -> _lib.RnsIpAddr:
        c = _lib.RnsIpAddr()
        c.version = 4 if self.is_v4 else 6
        for i, v in enumerate(self.addr):
            c.bytes[i] = v
        return c

    def __eq__(self, other):
        return isinstance(other, IPAddr) and other.addr == self.addr

    def __hash__(self):
        return hash(self.addr)

    def __repr__(self):
        return f"IPAddr.{'V4' if self.is_v4 else 'V6'}({self.addr.hex()})"


def compute_pseudo_header_checksum(source_ip: IPAddr, dest_ip: IPAddr, length: int, protocol: int) -> int:
    """util.rs:180 — one's complement sum of the v4 (12 B) / v6 (40 B) pseudo-header."""
    if source_ip.is_v4 != dest_ip.is_v4:
        raise ReferencePanic("source/dest IPAddr variants differ (copy_to would panic)")
    s, d = source_ip._c(), dest_ip._c()
    return _result(_lib.load().rns_compute_pseudo_header_checksum(
        ctypes.byref(s), ctypes.byref(d), length & 0xFFFFFFFFFFFFFFFF, protocol & 0xFF),
        "compute_pseudo_header_checksum")


# util.rs:121-142 — big-endian helpers; set_be16 is how every call site stores a checksum.
def get_be16(buffer) -> int:
    return (buffer[0] << 8) | buffer[1]


def get_be32(buffer) -> int:
    return (buffer[0] << 24) | (buffer[1] << 16) | (buffer[2] << 8) | buffer[3]


def set_be16(buffer, value: int) -> None:
    buffer[0] = (value >> 8) & 0xFF
    buffer[1] = value & 0xFF


def set_be32(buffer, value: int) -> None:
    buffer[0] = (value >> 24) & 0xFF
    buffer[1] = (value >> 16) & 0xFF
    buffer[2] = (value >> 8) & 0xFF
    buffer[3] = value & 0xFF
