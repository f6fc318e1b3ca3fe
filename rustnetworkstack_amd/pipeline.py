"""End-to-end batched receive and transmit.

Receive (RxPipeline): datagram fd -> pinned host arena -> HBM -> fused receive verify
-> per-packet verdicts.  Transmit (TxPipeline): pinned slots -> HBM -> transmit
finalize -> the changed header bytes back -> datagram fd.

The reference handles one packet per loop iteration on its receive thread
(packet_receive_thread lib.rs:26-31 -> recv_packet netif.rs:65-83 -> ip_input
ip.rs:38 -> checks ip.rs:76, tcp.rs:544).  Here one call moves every queued datagram
(rns_io_recv_batch into 2048-byte MRU slots, netif.rs:66), copies the used slots to
the GPU in one transfer and verifies them with one kernel (rns_rx_verify_dev).
"""
from __future__ import annotations

import numpy as np
import torch

from .batch import PinnedBuffer, recv_batch, rx_verify, send_batch, tx_fill

MRU = 2048  # netif.rs:66


class RxPipeline:
    def __init__(self, local_ipv4: bytes, local_ipv6: bytes, device: int = 0, max_pkts: int = 65536,
                 slot_bytes: int = MRU):
        self.local_ipv4, self.local_ipv6 = bytes(local_ipv4), bytes(local_ipv6)
        self.slot = slot_bytes
        self.max_pkts = max_pkts
        self.dev = torch.device(f"cuda:{device}")
        self.host = PinnedBuffer(slot_bytes * max_pkts)
        self.h_len = PinnedBuffer(4 * max_pkts)
        self.d_arena = torch.empty(slot_bytes * max_pkts, dtype=torch.uint8, device=self.dev)
        self.d_off = (torch.arange(max_pkts, dtype=torch.int64, device=self.dev) * slot_bytes).contiguous()
        self.d_len = torch.empty(max_pkts, dtype=torch.int32, device=self.dev)
        self.d_status = torch.empty(max_pkts, dtype=torch.uint8, device=self.dev)

    def receive(self, fd: int, timeout_ms: int = 0) -> tuple[np.ndarray, np.ndarray]:
        """One batch: returns (status uint8 [n], lengths uint32 [n]); packet i is in
        slot i of ``self.host.array``."""
        off, ln = recv_batch(fd, self.host.array, self.slot, self.max_pkts, timeout_ms)
        n = off.shape[0]
        if n == 0:
            return np.empty(0, dtype=np.uint8), ln
        hl = self.h_len.array.view(np.uint32)[:n]
        hl[:] = ln
        with torch.cuda.device(self.dev):
            # pinned host memory (rns_host_alloc): both copies are DMA transfers
            self.d_arena[: n * self.slot].copy_(torch.from_numpy(self.host.array[: n * self.slot]), non_blocking=True)
            self.d_len[:n].copy_(torch.from_numpy(hl.view(np.int32)), non_blocking=True)
            rx_verify(self.d_arena, self.d_off[:n], self.d_len[:n], self.local_ipv4, self.local_ipv6,
                      status=self.d_status[:n])
            status = self.d_status[:n].cpu().numpy()
        return status, ln

    def close(self):
        self.host.free()
        self.h_len.free()


class TxPipeline:
    """End-to-end batched transmit (transmit side): the caller builds
    datagrams in pinned MRU slots with their checksum fields unset (what tcp_output /
    udp_output / icmp_output_* and ip_output_v4 hand over before their checksum step)
    -> one H2D copy -> rns_tx_fill_dev (IPv4 header + L4 checksums, pseudo-headers on the
    device) -> D2H of each slot's first HEAD bytes (every byte the fill can change)
    -> rns_io_send_batch (one writev per datagram, like tun_send via send_packet,
    netif.rs:85-98)."""

    HEAD = 128  # the fill writes only below byte 96 of a slot-aligned datagram

    def __init__(self, device: int = 0, max_pkts: int = 65536, slot_bytes: int = MRU):
        self.slot = slot_bytes
        self.max_pkts = max_pkts
        self.dev = torch.device(f"cuda:{device}")
        self.host = PinnedBuffer(slot_bytes * max_pkts)
        self.h_len = PinnedBuffer(4 * max_pkts)
        self.h_head = PinnedBuffer(self.HEAD * max_pkts)
        self.d_arena = torch.empty(slot_bytes * max_pkts, dtype=torch.uint8, device=self.dev)
        self.d_off = (torch.arange(max_pkts, dtype=torch.int64, device=self.dev) * slot_bytes).contiguous()
        self.off = np.arange(max_pkts, dtype=np.uint64) * np.uint64(slot_bytes)
        self.d_len = torch.empty(max_pkts, dtype=torch.int32, device=self.dev)
        self.d_status = torch.empty(max_pkts, dtype=torch.uint8, device=self.dev)

    def slots(self) -> np.ndarray:
        """The pinned slots, shape (max_pkts, slot_bytes): datagram i goes in row i."""
        return self.host.array[: self.slot * self.max_pkts].reshape(self.max_pkts, self.slot)

    def send(self, fd: int, lengths: np.ndarray) -> np.ndarray:
        """Fill and send the datagrams in slots [0, n); returns their RNS_TX_* status."""
        n = int(lengths.shape[0])
        if n == 0:
            return np.empty(0, dtype=np.uint8)
        if n > self.max_pkts:
            raise ValueError("more datagrams than slots")
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        if int(ln.max()) > self.slot:
            raise ValueError("datagram longer than its slot")
        hl = self.h_len.array.view(np.uint32)[:n]
        hl[:] = ln
        head = self.h_head.array[: self.HEAD * n].reshape(n, self.HEAD)
        with torch.cuda.device(self.dev):
            self.d_arena[: n * self.slot].copy_(torch.from_numpy(self.host.array[: n * self.slot]), non_blocking=True)
            self.d_len[:n].copy_(torch.from_numpy(hl.view(np.int32)), non_blocking=True)
            tx_fill(self.d_arena, self.d_off[:n], self.d_len[:n], status=self.d_status[:n])
            heads = self.d_arena[: n * self.slot].view(n, self.slot)[:, : self.HEAD].contiguous()
            torch.from_numpy(head).copy_(heads, non_blocking=True)
            status = self.d_status[:n].cpu().numpy()   # synchronises: the heads have landed too
        self.slots()[:n, : self.HEAD] = head
        sent = send_batch(fd, self.host.array, self.off[:n], ln)
        if sent != n:
            raise OSError(f"sent {sent} of {n} datagrams")
        return status

    def close(self):
        self.host.free()
        self.h_len.free()
        self.h_head.free()
