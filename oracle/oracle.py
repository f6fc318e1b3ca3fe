"""ORACLE — test infrastructure only.

Python access to the CPU restatement of jbush001/RustNetworkStack's checksum
path (src/stack/util.rs:88-119, 180-207):

* ``ones_comp_py`` etc. — pure-Python literal loops, for tiny inputs and for
  cross-checking the C restatement;
* ``Oracle`` — ctypes binding of ``oracle/build/libcsum_oracle.so`` (the C
  restatement in csum_oracle.c), fast enough for full-size batches.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
Panics of the reference are raised as ``ReferencePanic``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libcsum_oracle.so")


class ReferencePanic(Exception):
    """The reference would panic here (e.g. util.rs:92 on an empty slice)."""


# --------------------------------------------------------------------------
# pure-Python literal restatement (small inputs only)
# --------------------------------------------------------------------------
def ones_comp_py(in_checksum: int, data: bytes) -> int:
    """util.rs:88-106, literally (u32 accumulator, BE words, odd byte << 8)."""
    if len(data) == 0:
        raise ReferencePanic("compute_ones_comp on empty slice (util.rs:92)")
    checksum = in_checksum & 0xFFFF
    i = 0
    while i < len(data) - 1:
        checksum = (checksum + ((data[i] << 8) | data[i + 1])) & 0xFFFFFFFF
        i += 2
    if i < len(data):
        checksum = (checksum + (data[i] << 8)) & 0xFFFFFFFF
    while checksum > 0xFFFF:
        checksum = (checksum & 0xFFFF) + (checksum >> 16)
    return checksum


def checksum_py(data: bytes) -> int:
    """util.rs:108-110."""
    return 0xFFFF ^ ones_comp_py(0, data)


def buffer_ones_comp_py(initial_sum: int, fragments) -> int:
    """util.rs:112-119 over the fragment slices buf.rs:466-487 yields."""
    s = initial_sum
    for frag in fragments:
        s = ones_comp_py(s, bytes(frag))
    return s


def pseudo_header_py(src: bytes, dst: bytes, length: int, protocol: int) -> int:
    """util.rs:180-207 (layout chosen by the dest variant, util.rs:186)."""
    if len(src) not in (4, 16) or len(dst) not in (4, 16) or len(src) != len(dst):
        raise ReferencePanic("IPAddr variant/length mismatch (util.rs:41-56)")
    if len(dst) == 4:
        ph = bytearray(12)
        ph[0:4] = src
        ph[4:8] = dst
        ph[9] = protocol & 0xFF
        ph[10:12] = (length & 0xFFFF).to_bytes(2, "big")
    else:
        ph = bytearray(40)
        ph[0:16] = src
        ph[16:32] = dst
        ph[32:36] = (length & 0xFFFFFFFF).to_bytes(4, "big")
        ph[39] = protocol & 0xFF
    return ones_comp_py(0, bytes(ph))


# receive path restated (status bits of include/rns_checksum.h RNS_RX_*)
RX_IP_OK, RX_L4_OK, RX_L4_UNCHECKED, RX_FRAGMENT, RX_UNKNOWN, RX_ACCEPT, RX_MALFORMED = (
    0x01, 0x02, 0x04, 0x08, 0x10, 0x40, 0x80)


def rx_status_ref(pkt: bytes, local4: bytes, local6: bytes, ones_comp=None) -> int:
    """What the reference's receive path decides for one datagram, as status bits
    (see rx_verify_ref)."""
    return rx_verify_ref(pkt, local4, local6, ones_comp)[0]


def rx_verify_ref(pkt: bytes, local4: bytes, local6: bytes, ones_comp=None) -> tuple:
    """(status bits, complemented L4 sum) the reference's receive path computes for
    one datagram; the L4 value is 0 where the stack checks no L4 checksum (UDP,
    unknown protocols, malformed datagrams).

    ip_input (ip.rs:38-48) -> ip_input_v4 (ip.rs:65-92: header checksum over
    header[..IHL*4], fragment drop, protocol header[9], source header[12..16],
    trim_head(IHL*4)) / ip_input_v6 (ip.rs:114-121: protocol header[6], source
    header[8..24], trim_head(40)) -> ip_input_common (ip.rs:123-131) -> tcp_input's
    validate_checksum (tcp.rs:838-850: pseudo-header with dest = local address of
    the source's family, length = remaining buffer length), icmp_input_v4
    (icmp.rs:44-50: no pseudo-header), icmp_input_v6 (icmp.rs:62-75: dest = local
    IPv6), udp_input (udp.rs:126-148: no check).  Where the Rust code would panic
    (empty header slice, short buffers, trim past the end, V4 source in a V6
    pseudo-header) or rejects the version, the result is RX_MALFORMED.
    """
    oc = ones_comp or ones_comp_py
    L = len(pkt)
    if L == 0:
        return RX_MALFORMED, 0
    version = pkt[0] >> 4
    if version == 4:
        hdr = (pkt[0] & 0xF) * 4
        if hdr == 0 or L < 16 or hdr > L:
            return RX_MALFORMED, 0
        st = RX_IP_OK if (0xFFFF ^ oc(0, pkt[:hdr])) == 0 else 0
        if ((pkt[6] << 8 | pkt[7]) & 0x3FFF) != 0:
            st |= RX_FRAGMENT
        proto, src = pkt[9], pkt[12:16]
    elif version == 6:
        hdr = 40
        if L < 40:
            return RX_MALFORMED, 0
        st = RX_IP_OK
        proto, src = pkt[6], pkt[8:24]
    else:
        return RX_MALFORMED, 0
    seg = pkt[hdr:]

    def buf_sum(seed):  # compute_buffer_ones_comp over a one-fragment buffer; empty buffer -> seed
        return oc(seed, seg) if len(seg) else seed

    l4 = 0
    if proto == 6:
        dst = local4 if len(src) == 4 else local6
        l4 = buf_sum(pseudo_header_py(src, dst, len(seg), 6)) ^ 0xFFFF
        st |= RX_L4_OK if l4 == 0 else 0
    elif proto == 1:
        l4 = buf_sum(0) ^ 0xFFFF
        st |= RX_L4_OK if l4 == 0 else 0
    elif proto == 58:
        if len(src) == 4:
            return RX_MALFORMED, 0
        l4 = buf_sum(pseudo_header_py(src, local6, len(seg), 58)) ^ 0xFFFF
        st |= RX_L4_OK if l4 == 0 else 0
    elif proto == 17:
        st |= RX_L4_UNCHECKED
    else:
        st |= RX_UNKNOWN
    if (st & RX_IP_OK) and not (st & RX_FRAGMENT) and (st & (RX_L4_OK | RX_L4_UNCHECKED)):
        st |= RX_ACCEPT
    return st, l4


TX_IP_FILLED = 0x01
TX_L4_FILLED = 0x02
TX_MALFORMED = 0x80


def tx_fill_ref(pkt: bytes, ones_comp=None) -> tuple:
    """(datagram bytes, status bits) after the reference's transmit path has filled the
    checksums of one finished datagram — the fields are computed as zero, as
    alloc_header leaves them (buf.rs:286-288), whatever they hold on input:

    tcp_output (tcp.rs:957-973): pseudo-header (source = the local address = the
    header's source, dest, length = segment length as u16, 6), then
    compute_buffer_ones_comp(ph, segment) ^ 0xffff at segment[16..18];
    udp_output (udp.rs:151-171): the same with protocol 17 at [6..8] (a result of 0 is
    stored as is); icmp_output_v4 (icmp.rs:87-95): compute_buffer_ones_comp(0, segment)
    ^ 0xffff at [2..4]; icmp_output_v6 (icmp.rs:97-112): pseudo-header with the full
    segment length, protocol 58, at [2..4]; ip_output_v4 (ip.rs:140-160):
    compute_checksum(header) at header[10..12] (the reference always sends IHL 5; IHL*4
    bytes here).  Datagrams the reference cannot produce (bad version, IHL < 5, short
    buffers) are TX_MALFORMED and left unchanged; protocols it does not checksum, or a
    segment too short for its field, get no L4 fill.
    """
    oc = ones_comp or ones_comp_py
    p = bytearray(pkt)
    L = len(p)
    if L == 0:
        return bytes(p), TX_MALFORMED
    version = p[0] >> 4
    if version == 4:
        hdr = (p[0] & 0xF) * 4
        if hdr < 20 or hdr > L:
            return bytes(p), TX_MALFORMED
        proto, src, dst = p[9], bytes(p[12:16]), bytes(p[16:20])
    elif version == 6:
        hdr = 40
        if L < 40:
            return bytes(p), TX_MALFORMED
        proto, src, dst = p[6], bytes(p[8:24]), bytes(p[24:40])
    else:
        return bytes(p), TX_MALFORMED
    seg_len = L - hdr
    field, seed = None, 0
    if proto == 6:
        field, seed = 16, pseudo_header_py(src, dst, seg_len & 0xFFFF, 6)
    elif proto == 17:
        field, seed = 6, pseudo_header_py(src, dst, seg_len & 0xFFFF, 17)
    elif proto == 1 and version == 4:
        field = 2
    elif proto == 58 and version == 6:
        field, seed = 2, pseudo_header_py(src, dst, seg_len, 58)
    st = 0
    if field is not None and seg_len >= field + 2:
        f = hdr + field
        p[f:f + 2] = b"\x00\x00"
        c = oc(seed, bytes(p[hdr:])) ^ 0xFFFF
        p[f:f + 2] = c.to_bytes(2, "big")
        st |= TX_L4_FILLED
    if version == 4:
        p[10:12] = b"\x00\x00"
        c = oc(0, bytes(p[:hdr])) ^ 0xFFFF
        p[10:12] = c.to_bytes(2, "big")
        st |= TX_IP_FILLED
    return bytes(p), st


def tx_chain_fill_ref(frags, ones_comp=None) -> tuple:
    """(head fragment bytes, status bits) after the reference's transmit path has filled the
    checksums of one datagram held as a NetBuffer chain: frags[0] is the head fragment, where
    alloc_header leaves the L4 header and then, prepended into the same fragment's headroom,
    the IP header (buf.rs:262-291: a header is always contiguous); frags[1:] are the payload
    fragments.  The L4 checksum is compute_buffer_ones_comp(pseudo-header, packet) taken when
    the packet was [head[hdr:], payload...] (tcp.rs:957-973, udp.rs:150-171,
    icmp.rs:87-112): folded per fragment (util.rs:112-119), so an odd-length fragment pairs
    its bytes from its own start; the IPv4 header checksum covers head[:IHL*4] (ip.rs:140-160).
    Fields count as zero, as alloc_header leaves them.  Only head bytes change.  A chain whose
    head cannot hold its IP header (or no fragments / bad version) is TX_MALFORMED and left
    unchanged; an L4 field outside the head fragment, or a protocol the stack does not
    checksum, gets no L4 fill.  Empty payload fragments add nothing (the reference would
    panic, util.rs:92)."""
    oc = ones_comp or ones_comp_py
    if not frags or len(frags[0]) == 0:
        return (bytes(frags[0]) if frags else b""), TX_MALFORMED
    head = bytearray(frags[0])
    hl = len(head)
    L = sum(len(f) for f in frags)
    version = head[0] >> 4
    if version == 4:
        hdr = (head[0] & 0xF) * 4
        if hdr < 20 or hdr > hl:
            return bytes(head), TX_MALFORMED
        proto, src, dst = head[9], bytes(head[12:16]), bytes(head[16:20])
    elif version == 6:
        hdr = 40
        if hl < 40:
            return bytes(head), TX_MALFORMED
        proto, src, dst = head[6], bytes(head[8:24]), bytes(head[24:40])
    else:
        return bytes(head), TX_MALFORMED
    seg_len = L - hdr
    field, seed = None, 0
    if proto == 6:
        field, seed = 16, pseudo_header_py(src, dst, seg_len & 0xFFFF, 6)
    elif proto == 17:
        field, seed = 6, pseudo_header_py(src, dst, seg_len & 0xFFFF, 17)
    elif proto == 1 and version == 4:
        field = 2
    elif proto == 58 and version == 6:
        field, seed = 2, pseudo_header_py(src, dst, seg_len, 58)
    st = 0
    if field is not None and seg_len >= field + 2 and hdr + field + 2 <= hl:
        f = hdr + field
        head[f:f + 2] = b"\x00\x00"
        acc = seed
        for piece in [bytes(head[hdr:])] + [bytes(x) for x in frags[1:]]:
            if len(piece):
                acc = oc(acc, piece)
        head[f:f + 2] = (acc ^ 0xFFFF).to_bytes(2, "big")
        st |= TX_L4_FILLED
    if version == 4:
        head[10:12] = b"\x00\x00"
        head[10:12] = (oc(0, bytes(head[:hdr])) ^ 0xFFFF).to_bytes(2, "big")
        st |= TX_IP_FILLED
    return bytes(head), st


# --------------------------------------------------------------------------
# deterministic synthetic bytes: splitmix64 (seed 0x5EED_C0DE)
# --------------------------------------------------------------------------
GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def splitmix64_words(seed: int, count: int, start: int = 0) -> np.ndarray:
    """Words z_i = mix(seed + (start+i+1)*GOLDEN), i in [0, count)."""
    with np.errstate(over="ignore"):
        idx = np.arange(start + 1, start + count + 1, dtype=np.uint64)
        z = np.uint64(seed) + idx * GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def splitmix64_bytes(seed: int, nbytes: int) -> np.ndarray:
    """Little-endian byte stream of splitmix64 words (uint8 array of nbytes)."""
    words = splitmix64_words(seed, (nbytes + 7) // 8)
    return words.view(np.uint8)[:nbytes].copy()


# --------------------------------------------------------------------------
# ctypes binding of the C restatement
# --------------------------------------------------------------------------
def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


_u8p = ctypes.POINTER(ctypes.c_uint8)


def _ptr(a: np.ndarray, ctype=ctypes.c_uint8):
    return a.ctypes.data_as(ctypes.POINTER(ctype))


class Oracle:
    """ctypes view of oracle/csum_oracle.c."""

    def __init__(self, path: str | None = None):
        self.lib = ctypes.CDLL(path or build())
        L = self.lib
        L.oracle_compute_ones_comp.restype = ctypes.c_int32
        L.oracle_compute_ones_comp.argtypes = [ctypes.c_uint16, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_compute_checksum.restype = ctypes.c_int32
        L.oracle_compute_checksum.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_compute_buffer_ones_comp.restype = ctypes.c_int32
        L.oracle_compute_buffer_ones_comp.argtypes = [
            ctypes.c_uint16, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t]
        L.oracle_compute_pseudo_header_checksum.restype = ctypes.c_int32
        L.oracle_compute_pseudo_header_checksum.argtypes = [
            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint8]
        L.oracle_batch.restype = None
        L.oracle_batch.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_int]
        L.oracle_batch_mt.restype = ctypes.c_int
        L.oracle_batch_mt.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
        L.oracle_chain_batch.restype = None
        L.oracle_chain_batch.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_size_t, ctypes.c_int]
        L.oracle_tx_chain_fill.restype = None
        L.oracle_tx_chain_fill.argtypes = [ctypes.c_void_p, ctypes.c_uint64] + [ctypes.c_void_p] * 3 + [
            ctypes.c_uint32, ctypes.c_size_t, ctypes.c_void_p]
        L.oracle_tx_chain_fill_mt.restype = ctypes.c_int
        L.oracle_tx_chain_fill_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint64] + [ctypes.c_void_p] * 3 + [
            ctypes.c_uint32, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
        L.oracle_time_ones_comp.restype = ctypes.c_double
        L.oracle_time_ones_comp.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]

    @staticmethod
    def _check(r: int) -> int:
        if r < 0:
            raise ReferencePanic("reference would panic")
        return r

    def compute_ones_comp(self, in_checksum: int, data) -> int:
        b = bytes(data)
        return self._check(self.lib.oracle_compute_ones_comp(in_checksum & 0xFFFF, b, len(b)))

    def compute_checksum(self, data) -> int:
        b = bytes(data)
        return self._check(self.lib.oracle_compute_checksum(b, len(b)))

    def compute_buffer_ones_comp(self, initial_sum: int, fragments) -> int:
        frags = [bytes(f) for f in fragments]
        n = len(frags)
        bufs = [ctypes.create_string_buffer(f, len(f) or 1) for f in frags]
        bases = (ctypes.c_void_p * max(n, 1))(*[ctypes.cast(b, ctypes.c_void_p).value for b in bufs])
        lens = (ctypes.c_size_t * max(n, 1))(*[len(f) for f in frags])
        return self._check(self.lib.oracle_compute_buffer_ones_comp(initial_sum & 0xFFFF, bases, lens, n))

    def compute_pseudo_header_checksum(self, src: bytes, dst: bytes, length: int, protocol: int) -> int:
        return self._check(self.lib.oracle_compute_pseudo_header_checksum(
            bytes(src), len(src), bytes(dst), len(dst), length & 0xFFFFFFFFFFFFFFFF, protocol & 0xFF))

    def batch(self, arena: np.ndarray, off: np.ndarray, length: np.ndarray, seed: np.ndarray | None,
              complement: bool = False, threads: int = 1, check: bool = True) -> np.ndarray:
        """One compute_ones_comp per packet (optionally complemented).  ``check=False``
        skips the bounds pass (the CPU baseline times the loop alone, on descriptors it
        already checked)."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        n = off.shape[0]
        if check and n and int((off + length.astype(np.uint64)).max()) > arena.shape[0]:
            raise ValueError("descriptor out of arena bounds")
        out = np.empty(n, dtype=np.uint16)
        sp = None
        if seed is not None:
            seed = np.ascontiguousarray(seed, dtype=np.uint16)
            sp = seed.ctypes.data
        if threads <= 1:
            self.lib.oracle_batch(arena.ctypes.data, off.ctypes.data, length.ctypes.data, sp,
                                  out.ctypes.data, n, int(complement))
        else:
            rc = self.lib.oracle_batch_mt(arena.ctypes.data, off.ctypes.data, length.ctypes.data, sp,
                                          out.ctypes.data, n, int(complement), int(threads))
            if rc != 0:
                raise RuntimeError("oracle_batch_mt: thread creation failed")
        return out


    def chain_batch(self, arena: np.ndarray, frag_off: np.ndarray, frag_len: np.ndarray, first: np.ndarray,
                    seed: np.ndarray | None, complement: bool = False) -> np.ndarray:
        """compute_buffer_ones_comp per packet over fragment chains (CSR `first`)."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        frag_off = np.ascontiguousarray(frag_off, dtype=np.uint64)
        frag_len = np.ascontiguousarray(frag_len, dtype=np.uint32)
        first = np.ascontiguousarray(first, dtype=np.uint32)
        n = first.shape[0] - 1
        if frag_off.shape[0] and int((frag_off + frag_len.astype(np.uint64)).max()) > arena.shape[0]:
            raise ValueError("fragment out of arena bounds")
        out = np.empty(n, dtype=np.uint16)
        sp = None
        if seed is not None:
            seed = np.ascontiguousarray(seed, dtype=np.uint16)
            sp = seed.ctypes.data
        self.lib.oracle_chain_batch(arena.ctypes.data, frag_off.ctypes.data, frag_len.ctypes.data, first.ctypes.data,
                                    sp, out.ctypes.data, n, int(complement))
        return out

    def tx_chain_fill(self, arena: np.ndarray, frag_off: np.ndarray, frag_len: np.ndarray, first: np.ndarray,
                      threads: int = 1) -> np.ndarray:
        """tx_chain_fill_ref for a batch of chains, IN PLACE on ``arena`` (a writable uint8 array):
        the heads get their checksums; returns the status per datagram."""
        if arena.dtype != np.uint8 or not arena.flags.c_contiguous or not arena.flags.writeable:
            raise ValueError("arena must be a writable contiguous uint8 array (filled in place)")
        frag_off = np.ascontiguousarray(frag_off, dtype=np.uint64)
        frag_len = np.ascontiguousarray(frag_len, dtype=np.uint32)
        first = np.ascontiguousarray(first, dtype=np.uint32)
        n = first.shape[0] - 1
        st = np.empty(max(n, 0), dtype=np.uint8)
        args = (arena.ctypes.data, arena.shape[0], frag_off.ctypes.data, frag_len.ctypes.data, first.ctypes.data,
                frag_off.shape[0], n, st.ctypes.data)
        if threads <= 1:
            self.lib.oracle_tx_chain_fill(*args)
        elif self.lib.oracle_tx_chain_fill_mt(*args, int(threads)) != 0:
            raise RuntimeError("oracle_tx_chain_fill_mt: thread creation failed")
        return st

    def time_ones_comp(self, data: bytes, iters: int) -> float:
        """ns per compute_ones_comp(0, data) call (benches/util_bench.rs:20-45 equivalent)."""
        b = bytes(data)
        return float(self.lib.oracle_time_ones_comp(b, len(b), iters))


_ORACLE: Oracle | None = None


def get_oracle() -> Oracle:
    global _ORACLE
    if _ORACLE is None:
        _ORACLE = Oracle()
    return _ORACLE
