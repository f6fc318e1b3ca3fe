"""End-to-end batched receive and transmit.

Receive (RxPipeline): datagram fd -> pinned host arena -> HBM -> fused receive verify
-> per-packet verdicts.  By default the datagrams are received PACKED (each at the next
16-byte boundary, rns_io_recv_batch_packed), so the copy to the GPU carries their bytes
only — not whole 2048-byte slots — and the verify is the rows receive kernel
(rns_rx_verify_packed_dev); ``packed=False`` keeps MRU slots and rns_rx_verify_dev.  Transmit (TxPipeline): pinned slots -> HBM -> transmit
finalize -> the changed header bytes back -> datagram fd.  TxChainPipeline does the same for
datagrams built as the reference builds them — NetBuffer chains of a head fragment (IP + L4
headers) and a payload — with the heads in a header region and the payloads in a payload region:
only used bytes cross PCIe to the GPU, only the header region comes back, and each datagram leaves
gathered from its two fragments (rns_io_send_batch_chain, like send_packet's writev).

The reference handles one packet per loop iteration on its receive thread
(packet_receive_thread lib.rs:26-31 -> recv_packet netif.rs:65-83 -> ip_input
ip.rs:38 -> checks ip.rs:76, tcp.rs:544).  Here one call moves every queued datagram
(rns_io_recv_batch into 2048-byte MRU slots, netif.rs:66), copies the used slots to
the GPU in one transfer and verifies them with one kernel (rns_rx_verify_dev).

Both directions also run overlapped (``RxPipeline.stream``, ``TxPipeline.submit`` /
``complete``): two buffer sets, the GPU work of one batch (H2D, kernel, D2H into
pinned memory) queued on a private stream while the host reads or writes the
datagrams of the other.
"""
from __future__ import annotations

from collections import deque
from typing import Iterator

import numpy as np
import torch

from .batch import (PinnedBuffer, recv_batch, recv_batch_packed, rx_verify, rx_verify_packed, send_batch,
                    send_batch_chain, tx_fill, tx_fill_chain)

MRU = 2048  # netif.rs:66


class _Slots:
    """One buffer set: pinned host slots + lengths + per-slot results, and their HBM twins
    (packed: u16 lengths and one block offset per 64 datagrams instead of u32 lengths)."""

    def __init__(self, dev: torch.device, max_pkts: int, slot_bytes: int, head: int = 0, packed: bool = False):
        self.host = PinnedBuffer(slot_bytes * max_pkts)
        self.h_len = PinnedBuffer(4 * max_pkts)
        self.h_status = PinnedBuffer(max_pkts)
        self.h_head = PinnedBuffer(head * max_pkts) if head else None
        self.d_arena = torch.empty(slot_bytes * max_pkts, dtype=torch.uint8, device=dev)
        self.d_len = torch.empty(max_pkts, dtype=torch.int32, device=dev)
        self.d_status = torch.empty(max_pkts, dtype=torch.uint8, device=dev)
        nblk = (max_pkts + 63) // 64
        self.h_blk = PinnedBuffer(8 * nblk) if packed else None
        self.d_blk = torch.empty(nblk, dtype=torch.int64, device=dev) if packed else None
        self.done = torch.cuda.Event()

    def close(self):
        for b in (self.host, self.h_len, self.h_status, self.h_head, self.h_blk):
            if b is not None:
                b.free()


class Datagrams:
    """The datagrams of one received batch: ``d[i]`` is datagram i's bytes (a view of the
    pinned arena, valid until the buffer set is reused)."""

    def __init__(self, arena: np.ndarray, off: np.ndarray, length: np.ndarray):
        self.arena, self.off, self.length = arena, off, length

    def __len__(self) -> int:
        return int(self.length.shape[0])

    def __getitem__(self, i: int) -> np.ndarray:
        o = int(self.off[i])
        return self.arena[o:o + int(self.length[i])]


class RxPipeline:
    def __init__(self, local_ipv4: bytes, local_ipv6: bytes, device: int = 0, max_pkts: int = 65536,
                 slot_bytes: int = MRU, packed: bool = True):
        self.local_ipv4, self.local_ipv6 = bytes(local_ipv4), bytes(local_ipv6)
        self.slot = slot_bytes  # the MRU: the arena holds max_pkts datagrams of this size
        self.max_pkts = max_pkts
        self.packed = packed
        self.dev = torch.device(f"cuda:{device}")
        self._sets = [_Slots(self.dev, max_pkts, slot_bytes, packed=packed)]
        self.d_off = (torch.arange(max_pkts, dtype=torch.int64, device=self.dev) * slot_bytes).contiguous()
        self._stream = None
        self.h2d_bytes = 0  # arena bytes copied to the GPU so far (packed: the datagrams' 16-byte-padded bytes)
        self.datagrams = 0
        self.last: Datagrams | None = None  # the datagrams of the last batch ``receive`` returned

    @property
    def host(self) -> PinnedBuffer:
        """Set 0's pinned arena: where ``receive`` leaves its datagrams (``last``)."""
        return self._sets[0].host

    def _read(self, s: _Slots, fd: int, timeout_ms: int):
        """One batched read into set ``s``: (lengths, Datagrams, arena bytes used)."""
        if self.packed:
            ln16, blk, end = recv_batch_packed(fd, s.host.array, self.slot, self.max_pkts, timeout_ms)
            n = ln16.shape[0]
            if n:
                s.h_blk.array.view(np.uint64)[: blk.shape[0]] = blk
            pad = (ln16.astype(np.uint64) + np.uint64(15)) & ~np.uint64(15)
            off = np.zeros(n, dtype=np.uint64)
            if n > 1:
                np.cumsum(pad[:-1], out=off[1:])
            return ln16.astype(np.uint32), Datagrams(s.host.array, off, ln16), end
        off, ln = recv_batch(fd, s.host.array, self.slot, self.max_pkts, timeout_ms)
        return ln, Datagrams(s.host.array, off, ln), ln.shape[0] * self.slot

    def _submit(self, s: _Slots, ln: np.ndarray, used: int) -> None:
        """Queue H2D + verify + status D2H of the batch in ``s`` (len(ln) datagrams in its
        first ``used`` arena bytes) on the current stream; ``s.done`` marks the status
        landing in pinned memory."""
        n = ln.shape[0]
        # pinned host memory (rns_host_alloc): every copy is a DMA transfer
        s.d_arena[:used].copy_(torch.from_numpy(s.host.array[:used]), non_blocking=True)
        self.h2d_bytes += used
        self.datagrams += n
        if self.packed:
            h16 = s.h_len.array.view(np.uint16)[:n]
            h16[:] = ln
            nb = (n + 63) // 64
            d16 = s.d_len.view(torch.int16)[:n]
            d16.copy_(torch.from_numpy(h16.view(np.int16)), non_blocking=True)
            s.d_blk[:nb].copy_(torch.from_numpy(s.h_blk.array.view(np.int64)[:nb]), non_blocking=True)
            rx_verify_packed(s.d_arena[:max(used, 1)], s.d_blk[:nb], d16, self.local_ipv4, self.local_ipv6,
                             status=s.d_status[:n])
        else:
            hl = s.h_len.array.view(np.uint32)[:n]
            hl[:] = ln
            s.d_len[:n].copy_(torch.from_numpy(hl.view(np.int32)), non_blocking=True)
            rx_verify(s.d_arena, self.d_off[:n], s.d_len[:n], self.local_ipv4, self.local_ipv6,
                      status=s.d_status[:n])
        torch.from_numpy(s.h_status.array[:n]).copy_(s.d_status[:n], non_blocking=True)
        s.done.record()

    def receive(self, fd: int, timeout_ms: int = 0) -> tuple[np.ndarray, np.ndarray]:
        """One batch: returns (status uint8 [n], lengths uint32 [n]); ``self.last[i]`` is
        datagram i's bytes in the pinned arena."""
        s = self._sets[0]
        ln, dg, used = self._read(s, fd, timeout_ms)
        self.last = dg
        n = ln.shape[0]
        if n == 0:
            return np.empty(0, dtype=np.uint8), ln
        with torch.cuda.device(self.dev):
            self._submit(s, ln, used)
            s.done.synchronize()
        return s.h_status.array[:n].copy(), ln

    def stream(self, fd: int, timeout_ms: int = 0) -> Iterator[tuple[np.ndarray, np.ndarray, Datagrams]]:
        """Overlapped receive: yields (status [n], lengths [n], Datagrams) per batch until a
        read finds nothing within ``timeout_ms``.  While batch k is on the GPU the host reads
        batch k+1 into the other buffer set; the yielded arrays stay valid until the
        generator is resumed."""
        if len(self._sets) == 1:
            self._sets.append(_Slots(self.dev, self.max_pkts, self.slot, packed=self.packed))
        if self._stream is None:
            self._stream = torch.cuda.Stream(self.dev)
        pending = None  # (set, lengths, datagrams) on the GPU
        k = 0
        while True:
            s = self._sets[k]
            if pending is None:
                ln, dg, used = self._read(s, fd, timeout_ms)
            else:
                # take what is queued now (no wait), hand the finished batch over, and
                # only then block for more: the last batch is not held back by the timeout
                ln, dg, used = self._read(s, fd, 0)
                p, pln, pdg = pending
                p.done.synchronize()
                yield p.h_status.array[: pln.shape[0]], pln, pdg
                pending = None
                if ln.shape[0] == 0:
                    ln, dg, used = self._read(s, fd, timeout_ms)
            if ln.shape[0] == 0:
                return
            with torch.cuda.device(self.dev), torch.cuda.stream(self._stream):
                self._submit(s, ln, used)
            pending = (s, ln, dg)
            k ^= 1

    def close(self):
        for s in self._sets:
            s.close()


class TxPipeline:
    """End-to-end batched transmit (transmit side): the caller builds
    datagrams in pinned MRU slots with their checksum fields unset (what tcp_output /
    udp_output / icmp_output_* and ip_output_v4 hand over before their checksum step)
    -> one H2D copy -> rns_tx_fill_dev (IPv4 header + L4 checksums, pseudo-headers on the
    device) -> D2H of each slot's first HEAD bytes (every byte the fill can change)
    -> rns_io_send_batch (one writev per datagram, like tun_send via send_packet,
    netif.rs:85-98).

    ``send`` does one batch synchronously.  ``submit`` / ``complete`` overlap: submit
    queues a batch's GPU work and returns; complete waits for the oldest submitted
    batch and writes it to the fd.  With two buffer sets, the caller fills the next
    batch's ``slots()`` and the host sends one batch while the GPU finalizes the other:

        for lengths in batches:
            if pipe.pending() == pipe.DEPTH:
                statuses.append(pipe.complete(fd))
            fill(pipe.slots(), ...)
            pipe.submit(lengths)
        while pipe.pending():
            statuses.append(pipe.complete(fd))
    """

    HEAD = 128  # the fill writes only below byte 96 of a slot-aligned datagram
    DEPTH = 2

    def __init__(self, device: int = 0, max_pkts: int = 65536, slot_bytes: int = MRU):
        self.slot = slot_bytes
        self.max_pkts = max_pkts
        self.dev = torch.device(f"cuda:{device}")
        self._sets = [_Slots(self.dev, max_pkts, slot_bytes, head=self.HEAD) for _ in range(self.DEPTH)]
        self.d_off = (torch.arange(max_pkts, dtype=torch.int64, device=self.dev) * slot_bytes).contiguous()
        self.off = np.arange(max_pkts, dtype=np.uint64) * np.uint64(slot_bytes)
        self._next = 0                    # the set slots() hands out
        self._inflight: deque = deque()   # (set, lengths), oldest first
        self._stream = None

    def slots(self) -> np.ndarray:
        """The free set's pinned slots, shape (max_pkts, slot_bytes): datagram i goes in row i."""
        if len(self._inflight) == self.DEPTH:
            raise RuntimeError("every buffer set is in flight: complete() one first")
        return self._sets[self._next].host.array[: self.slot * self.max_pkts].reshape(self.max_pkts, self.slot)

    def pending(self) -> int:
        return len(self._inflight)

    def _check(self, lengths: np.ndarray) -> np.ndarray:
        n = int(lengths.shape[0])
        if n > self.max_pkts:
            raise ValueError("more datagrams than slots")
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        if n and int(ln.max()) > self.slot:
            raise ValueError("datagram longer than its slot")
        return ln

    def _queue(self, s: _Slots, ln: np.ndarray) -> None:
        n = ln.shape[0]
        hl = s.h_len.array.view(np.uint32)[:n]
        hl[:] = ln
        head = s.h_head.array[: self.HEAD * n].reshape(n, self.HEAD)
        s.d_arena[: n * self.slot].copy_(torch.from_numpy(s.host.array[: n * self.slot]), non_blocking=True)
        s.d_len[:n].copy_(torch.from_numpy(hl.view(np.int32)), non_blocking=True)
        tx_fill(s.d_arena, self.d_off[:n], s.d_len[:n], status=s.d_status[:n])
        heads = s.d_arena[: n * self.slot].view(n, self.slot)[:, : self.HEAD].contiguous()
        torch.from_numpy(head).copy_(heads, non_blocking=True)
        torch.from_numpy(s.h_status.array[:n]).copy_(s.d_status[:n], non_blocking=True)
        s.done.record()

    def _finish(self, fd: int, s: _Slots, ln: np.ndarray) -> np.ndarray:
        n = ln.shape[0]
        s.done.synchronize()
        slots = s.host.array[: self.slot * n].reshape(n, self.slot)
        slots[:, : self.HEAD] = s.h_head.array[: self.HEAD * n].reshape(n, self.HEAD)
        sent = send_batch(fd, s.host.array, self.off[:n], ln)
        if sent != n:
            raise OSError(f"sent {sent} of {n} datagrams")
        return s.h_status.array[:n].copy()

    def send(self, fd: int, lengths: np.ndarray) -> np.ndarray:
        """Fill and send the datagrams in slots [0, n) of ``slots()``; returns their
        RNS_TX_* status."""
        if self._inflight:
            raise RuntimeError("submitted batches pending: complete() them first")
        ln = self._check(lengths)
        if ln.shape[0] == 0:
            return np.empty(0, dtype=np.uint8)
        s = self._sets[self._next]
        with torch.cuda.device(self.dev):
            self._queue(s, ln)
        return self._finish(fd, s, ln)

    def submit(self, lengths: np.ndarray) -> None:
        """Queue the GPU work for slots [0, n) of ``slots()`` and hand out the other set."""
        if len(self._inflight) == self.DEPTH:
            raise RuntimeError("every buffer set is in flight: complete() one first")
        ln = self._check(lengths)
        s = self._sets[self._next]
        with torch.cuda.device(self.dev):
            if self._stream is None:
                self._stream = torch.cuda.Stream(self.dev)
            with torch.cuda.stream(self._stream):
                if ln.shape[0]:
                    self._queue(s, ln)
                else:
                    s.done.record()
        self._inflight.append((s, ln))
        self._next = (self._next + 1) % self.DEPTH

    def complete(self, fd: int) -> np.ndarray:
        """Wait for the oldest submitted batch, send it; returns its RNS_TX_* status."""
        if not self._inflight:
            raise RuntimeError("nothing submitted")
        s, ln = self._inflight.popleft()
        if ln.shape[0] == 0:
            return np.empty(0, dtype=np.uint8)
        return self._finish(fd, s, ln)

    def close(self):
        for s in self._sets:
            s.close()


class _ChainSet:
    """One buffer set of TxChainPipeline: a pinned arena [header region | payload region], its
    chain descriptors and statuses, and their HBM twins (the same offsets on both sides)."""

    def __init__(self, dev: torch.device, max_pkts: int, head_region: int, payload_bytes: int):
        self.host = PinnedBuffer(head_region + payload_bytes)
        self.h_off = PinnedBuffer(8 * 2 * max_pkts)
        self.h_len = PinnedBuffer(4 * 2 * max_pkts)
        self.h_first = PinnedBuffer(4 * (max_pkts + 1))
        self.h_status = PinnedBuffer(max_pkts)
        self.d_arena = torch.empty(head_region + payload_bytes, dtype=torch.uint8, device=dev)
        self.d_off = torch.empty(2 * max_pkts, dtype=torch.int64, device=dev)
        self.d_len = torch.empty(2 * max_pkts, dtype=torch.int32, device=dev)
        self.d_first = torch.empty(max_pkts + 1, dtype=torch.int32, device=dev)
        self.d_status = torch.empty(max_pkts, dtype=torch.uint8, device=dev)
        self.done = torch.cuda.Event()

    def close(self):
        for b in (self.host, self.h_off, self.h_len, self.h_first, self.h_status):
            b.free()


class TxChainPipeline:
    """Batched transmit of NetBuffer chains: the caller writes each
    datagram's head fragment — IP header then L4 header, checksum fields unset, as
    alloc_header leaves them (buf.rs:262-291) — back to back into ``heads()`` and its payload
    at a 16-byte-aligned offset of its choice into ``payloads()``, then ``send`` (or
    ``submit`` / ``complete``) with the head lengths and the payload offsets and lengths.
    One H2D copy of the used header bytes and one of the used payload bytes ->
    rns_tx_fill_chain_dev (pseudo-headers, L4 and IPv4 header checksums stored into the
    heads) -> D2H of the header region only -> rns_io_send_batch_chain (each datagram
    gathered from [head, payload], as send_packet's to_iovec + writev send a NetBuffer,
    netif.rs:51-98)."""

    HEAD_MAX = 128  # bytes per head fragment, at most (IPv4 with options + TCP with options)
    DEPTH = 2

    def __init__(self, device: int = 0, max_pkts: int = 65536, payload_bytes: int | None = None):
        self.max_pkts = max_pkts
        self.dev = torch.device(f"cuda:{device}")
        self.head_region = (self.HEAD_MAX * max_pkts + 4095) & ~4095
        self.payload_bytes = payload_bytes if payload_bytes is not None else MRU * max_pkts
        self._sets = [_ChainSet(self.dev, max_pkts, self.head_region, self.payload_bytes) for _ in range(self.DEPTH)]
        self._next = 0
        self._inflight: deque = deque()
        self._stream = None

    def heads(self) -> np.ndarray:
        """The free set's header region: head fragments back to back in datagram order."""
        if len(self._inflight) == self.DEPTH:
            raise RuntimeError("every buffer set is in flight: complete() one first")
        return self._sets[self._next].host.array[: self.head_region]

    def payloads(self) -> np.ndarray:
        """The free set's payload region (offsets passed to send / submit are relative to it)."""
        if len(self._inflight) == self.DEPTH:
            raise RuntimeError("every buffer set is in flight: complete() one first")
        return self._sets[self._next].host.array[self.head_region: self.head_region + self.payload_bytes]

    def pending(self) -> int:
        return len(self._inflight)

    def _describe(self, s: _ChainSet, head_len, pay_off, pay_len):
        """Chain descriptors [head, payload (if any)] per datagram into the set's pinned arrays;
        returns (n, fragments, header bytes used, payload bytes used)."""
        hl = np.ascontiguousarray(head_len, dtype=np.int64)
        po = np.ascontiguousarray(pay_off, dtype=np.int64)
        pl = np.ascontiguousarray(pay_len, dtype=np.int64)
        n = hl.shape[0]
        if po.shape[0] != n or pl.shape[0] != n:
            raise ValueError("head_len, pay_off and pay_len need one entry per datagram")
        if n > self.max_pkts:
            raise ValueError("more datagrams than the pipeline holds")
        if n and (hl.min() < 1 or hl.max() > self.HEAD_MAX or pl.min() < 0 or po.min() < 0 or
                  int((po + pl).max()) > self.payload_bytes):
            raise ValueError(f"head lengths must be 1..{self.HEAD_MAX} and payloads inside payloads()")
        hoff = np.zeros(n, dtype=np.int64)
        if n > 1:
            np.cumsum(hl[:-1], out=hoff[1:])
        nfr = 1 + (pl > 0)
        first = s.h_first.array.view(np.uint32)[: n + 1]
        first[0] = 0
        first[1:] = np.cumsum(nfr)
        nf = int(first[n])
        off = s.h_off.array.view(np.uint64)[:nf]
        ln = s.h_len.array.view(np.uint32)[:nf]
        f0 = first[:n].astype(np.int64)
        off[f0] = hoff.astype(np.uint64)
        ln[f0] = hl.astype(np.uint32)
        has = pl > 0
        off[f0[has] + 1] = (po[has] + self.head_region).astype(np.uint64)
        ln[f0[has] + 1] = pl[has].astype(np.uint32)
        hused = int(hoff[-1] + hl[-1]) if n else 0
        pused = int((po + pl).max()) if n else 0
        return n, nf, hused, pused

    def _queue(self, s: _ChainSet, n: int, nf: int, hused: int, pused: int) -> None:
        hr = self.head_region
        s.d_arena[:hused].copy_(torch.from_numpy(s.host.array[:hused]), non_blocking=True)
        if pused:
            s.d_arena[hr:hr + pused].copy_(torch.from_numpy(s.host.array[hr:hr + pused]), non_blocking=True)
        s.d_off[:nf].copy_(torch.from_numpy(s.h_off.array.view(np.int64)[:nf]), non_blocking=True)
        s.d_len[:nf].copy_(torch.from_numpy(s.h_len.array.view(np.int32)[:nf]), non_blocking=True)
        s.d_first[:n + 1].copy_(torch.from_numpy(s.h_first.array.view(np.int32)[:n + 1]), non_blocking=True)
        tx_fill_chain(s.d_arena, s.d_off[:nf], s.d_len[:nf], s.d_first[:n + 1], status=s.d_status[:n])
        torch.from_numpy(s.host.array[:hused]).copy_(s.d_arena[:hused], non_blocking=True)
        torch.from_numpy(s.h_status.array[:n]).copy_(s.d_status[:n], non_blocking=True)
        s.done.record()

    def _finish(self, fd: int, s: _ChainSet, n: int, nf: int) -> np.ndarray:
        s.done.synchronize()
        sent = send_batch_chain(fd, s.host.array, s.h_off.array.view(np.uint64)[:nf],
                                s.h_len.array.view(np.uint32)[:nf], s.h_first.array.view(np.uint32)[:n + 1])
        if sent != n:
            raise OSError(f"sent {sent} of {n} datagrams")
        return s.h_status.array[:n].copy()

    def send(self, fd: int, head_len, pay_off, pay_len) -> np.ndarray:
        """Finalize and send datagrams [0, n) of ``heads()`` / ``payloads()``; returns their
        RNS_TX_* status."""
        if self._inflight:
            raise RuntimeError("submitted batches pending: complete() them first")
        s = self._sets[self._next]
        n, nf, hused, pused = self._describe(s, head_len, pay_off, pay_len)
        if n == 0:
            return np.empty(0, dtype=np.uint8)
        with torch.cuda.device(self.dev):
            self._queue(s, n, nf, hused, pused)
        return self._finish(fd, s, n, nf)

    def submit(self, head_len, pay_off, pay_len) -> None:
        """Queue the GPU work for the free set's datagrams and hand out the other set."""
        if len(self._inflight) == self.DEPTH:
            raise RuntimeError("every buffer set is in flight: complete() one first")
        s = self._sets[self._next]
        n, nf, hused, pused = self._describe(s, head_len, pay_off, pay_len)
        with torch.cuda.device(self.dev):
            if self._stream is None:
                self._stream = torch.cuda.Stream(self.dev)
            with torch.cuda.stream(self._stream):
                if n:
                    self._queue(s, n, nf, hused, pused)
                else:
                    s.done.record()
        self._inflight.append((s, n, nf))
        self._next = (self._next + 1) % self.DEPTH

    def complete(self, fd: int) -> np.ndarray:
        """Wait for the oldest submitted batch, send it; returns its RNS_TX_* status."""
        if not self._inflight:
            raise RuntimeError("nothing submitted")
        s, n, nf = self._inflight.popleft()
        if n == 0:
            return np.empty(0, dtype=np.uint8)
        return self._finish(fd, s, n, nf)

    def close(self):
        for s in self._sets:
            s.close()
