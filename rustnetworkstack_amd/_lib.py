"""ctypes binding of librns_checksum.so (include/rns_checksum.h).

The product path has no CPU fallback for batches: if the library is missing,
``load()`` raises ``ChecksumLibraryMissing``; if no gfx950 device is usable the
batch entry points return RNS_E_NODEVICE and the Python layer raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# RNS_CHECKSUM_LIB overrides the library path (A/B builds in tools/ experiments only).
LIB_PATH = os.environ.get("RNS_CHECKSUM_LIB") or os.path.join(PKG_DIR, "librns_checksum.so")

RNS_OK = 0
RNS_E_INVALID = -1
RNS_E_EMPTY = -2
RNS_E_BOUNDS = -3
RNS_E_NODEVICE = -4
RNS_E_ORDER = -5
RNS_E_TOOLARGE = -6
RNS_E_IO = -7
RNS_E_HIP_BASE = -1000
RNS_FLAG_COMPLEMENT = 0x1
RNS_FLAG_CHAIN_RUNS = 0x2
RNS_FLAG_CHAIN_TX_PACKED = 0x4
RNS_CHAIN_MAX_PACKETS = 0xFFFFFFFF - 512  # packets per chain call (rns_checksum.h)
RNS_IO_MAX_FRAGS = 8  # fragments per datagram of rns_io_send_batch_chain (netif.rs:22 MAX_VECS)
RNS_RX_IP_OK = 0x01
RNS_RX_L4_OK = 0x02
RNS_RX_L4_UNCHECKED = 0x04
RNS_RX_FRAGMENT = 0x08
RNS_RX_UNKNOWN_PROTO = 0x10
RNS_RX_ACCEPT = 0x40
RNS_RX_MALFORMED = 0x80
RNS_TX_IP_FILLED = 0x01
RNS_TX_L4_FILLED = 0x02
RNS_TX_MALFORMED = 0x80

# Every symbol include/rns_checksum.h declares (tests/test_abi.py checks the header,
# this list and the library's dynamic symbol table agree).
EXPORTED_SYMBOLS = (
    "rns_compute_ones_comp",
    "rns_compute_checksum",
    "rns_compute_buffer_ones_comp",
    "rns_compute_pseudo_header_checksum",
    "rns_csum_batch_dev",
    "rns_csum_batch_dev_off32",
    "rns_csum_batch_packed_dev",
    "rns_packed_layout",
    "rns_csum_batch_strided_dev",
    "rns_csum_batch_dev_cfg",
    "rns_csum_chain_dev",
    "rns_csum_chain_fill_dev",
    "rns_csum_fill_dev",
    "rns_csum_fill_packed_dev",
    "rns_rx_verify_dev",
    "rns_rx_verify_packed_dev",
    "rns_rx_verify_strided_dev",
    "rns_tx_fill_dev",
    "rns_tx_fill_packed_dev",
    "rns_tx_fill_chain_dev",
    "rns_host_ctx_create",
    "rns_host_ctx_destroy",
    "rns_csum_batch_host",
    "rns_multi_ctx_create",
    "rns_multi_ctx_destroy",
    "rns_csum_batch_multi_host",
    "rns_csum_batch_multi_dev",
    "rns_io_recv_batch",
    "rns_io_send_batch",
    "rns_io_send_batch_chain",
    "rns_io_recv_batch_packed",
    "rns_host_alloc",
    "rns_host_free",
    "rns_fill_splitmix64_dev",
    "rns_abi_version",
    "rns_strerror",
    "rns_build_info",
    "rns_csum_shape_name",
    "rns_device_count",
)


class ChecksumLibraryMissing(RuntimeError):
    """librns_checksum.so is not built: run __graft_entry__.build() (or `make`)."""


class ChecksumError(RuntimeError):
    def __init__(self, status: int, what: str):
        self.status = status
        super().__init__(f"{what}: {strerror(status)} (status {status})")


class RnsIovec(ctypes.Structure):
    """`#[repr(C)] struct IOVec { base: *const u8, len: usize }` (netif.rs:24-29)."""
    _fields_ = [("base", ctypes.c_void_p), ("len", ctypes.c_size_t)]


class RnsIpAddr(ctypes.Structure):
    """C form of `enum IPAddr { V4([u8;4]), V6([u8;16]) }` (util.rs:22-26)."""
    _fields_ = [("version", ctypes.c_uint32), ("bytes", ctypes.c_uint8 * 16)]


class RnsDevBatch(ctypes.Structure):
    """`rns_dev_batch`: one GPU's shard for rns_csum_batch_multi_dev."""
    _fields_ = [("device", ctypes.c_int), ("d_arena", ctypes.c_void_p), ("arena_bytes", ctypes.c_uint64),
                ("d_off", ctypes.c_void_p), ("d_len", ctypes.c_void_p), ("d_seed", ctypes.c_void_p),
                ("d_out", ctypes.c_void_p), ("n", ctypes.c_uint32), ("len_hint", ctypes.c_uint32),
                ("d_bad", ctypes.c_void_p), ("stream", ctypes.c_void_p)]


_LIB = None
_LOCK = threading.Lock()

_vp, _u8, _u16, _u32, _u64, _i32, _int, _sz = (
    ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64,
    ctypes.c_int32, ctypes.c_int, ctypes.c_size_t)

_SIGNATURES = {
    "rns_compute_ones_comp": (_i32, [_u16, _vp, _sz]),
    "rns_compute_checksum": (_i32, [_vp, _sz]),
    "rns_compute_buffer_ones_comp": (_i32, [_u16, ctypes.POINTER(RnsIovec), _sz]),
    "rns_compute_pseudo_header_checksum": (_i32, [ctypes.POINTER(RnsIpAddr), ctypes.POINTER(RnsIpAddr), _u64, _u8]),
    "rns_csum_batch_dev": (_int, [_vp, _u64, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp]),
    "rns_csum_batch_dev_off32": (_int, [_vp, _u64, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp]),
    "rns_csum_batch_packed_dev": (_int, [_vp, _u64, _vp, _vp, _u32, _vp, _vp, _u32, _u32, _u32, _vp, _vp]),
    "rns_packed_layout": (_int, [_vp, _u64, _u32, _u64, _vp, _vp, ctypes.POINTER(_u64)]),
    "rns_csum_batch_strided_dev": (_int, [_vp, _u64, _u64, _u64, _u32, _vp, _vp, _u32, _u32, _vp, _vp]),
    "rns_csum_batch_dev_cfg": (_int, [_vp, _u64, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _u32, _u32, _u32, _vp, _vp]),
    "rns_csum_chain_dev": (_int, [_vp, _u64, _vp, _vp, _u32, _vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp, _vp]),
    "rns_csum_chain_fill_dev": (_int, [_vp, _u64, _vp, _vp, _u32, _vp, _vp, _vp, _u32, _vp, _u32, _u32, _u32, _vp,
                                       _vp]),
    "rns_csum_fill_dev": (_int, [_vp, _u64, _vp, _vp, _vp, _vp, _u32, _vp, _u32, _u32, _vp, _vp]),
    "rns_csum_fill_packed_dev": (_int, [_vp, _u64, _vp, _vp, _u32, _vp, _vp, _u32, _vp, _u32, _u32, _u32, _vp, _vp]),
    "rns_rx_verify_dev": (_int, [_vp, _u64, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp]),
    "rns_rx_verify_packed_dev": (_int, [_vp, _u64, _vp, _vp, _u32, _u32, _vp, _vp, _vp, _vp, _vp]),
    "rns_rx_verify_strided_dev": (_int, [_vp, _u64, _u64, _u64, _vp, _u32, _vp, _vp, _vp, _vp, _vp]),
    "rns_tx_fill_dev": (_int, [_vp, _u64, _vp, _vp, _u32, _vp, _vp]),
    "rns_tx_fill_packed_dev": (_int, [_vp, _u64, _vp, _vp, _u32, _u32, _vp, _u32, _vp]),
    "rns_tx_fill_chain_dev": (_int, [_vp, _u64, _vp, _vp, _u32, _vp, _u32, _vp, _vp]),
    "rns_host_ctx_create": (_int, [_int, _u64, _u32, ctypes.POINTER(_vp)]),
    "rns_host_ctx_destroy": (_int, [_vp]),
    "rns_csum_batch_host": (_int, [_vp, _vp, _u64, _vp, _vp, _vp, _vp, _u32, _u32]),
    "rns_multi_ctx_create": (_int, [ctypes.POINTER(ctypes.c_int), _u32, _u64, _u32, ctypes.POINTER(_vp)]),
    "rns_multi_ctx_destroy": (_int, [_vp]),
    "rns_csum_batch_multi_host": (_int, [_vp, _vp, _u64, _vp, _vp, _vp, _vp, _u32, _u32]),
    "rns_csum_batch_multi_dev": (_int, [ctypes.POINTER(RnsDevBatch), _u32, _u32]),
    "rns_io_recv_batch": (_int, [_int, _vp, _u64, _u32, _vp, _vp, _int]),
    "rns_io_send_batch": (_int, [_int, _vp, _vp, _vp, _u32]),
    "rns_io_send_batch_chain": (_int, [_int, _vp, _vp, _vp, _vp, _u32]),
    "rns_io_recv_batch_packed": (_int, [_int, _vp, _u64, _u32, _u32, _vp, _vp, ctypes.POINTER(_u64), _int]),
    "rns_host_alloc": (_int, [_u64, ctypes.POINTER(_vp)]),
    "rns_host_free": (_int, [_vp]),
    "rns_fill_splitmix64_dev": (_int, [_vp, _u64, _u64, _vp]),
    "rns_abi_version": (_int, []),
    "rns_strerror": (ctypes.c_char_p, [_int]),
    "rns_build_info": (ctypes.c_char_p, []),
    "rns_csum_shape_name": (ctypes.c_char_p, [_u32]),
    "rns_device_count": (_int, []),
}


def load() -> ctypes.CDLL:
    """Load the in-tree library (raises ChecksumLibraryMissing if it was not built)."""
    global _LIB
    with _LOCK:
        if _LIB is None:
            # PyTorch-ROCm bundles its own libamdhip64 (SONAME libamdhip64.so.7).  Importing
            # torch first makes the dynamic linker bind this library to that same runtime, so
            # the process has ONE HIP runtime and torch's streams / events / allocations are
            # valid here.  (Loading ours first would pull /opt/rocm's runtime under torch.)
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            if not os.path.exists(LIB_PATH):
                raise ChecksumLibraryMissing(f"{LIB_PATH} not found; run __graft_entry__.build()")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _LIB = lib
    return _LIB


def strerror(status: int) -> str:
    try:
        return load().rns_strerror(status).decode()
    except ChecksumLibraryMissing:
        return f"status {status}"


def check(status: int, what: str) -> None:
    if status != RNS_OK:
        raise ChecksumError(status, what)
