/*
 * rns_checksum.h — C ABI of the MI355X-native Internet checksum path.
 *
 * Drop-in boundary for jbush001/RustNetworkStack's checksum core
 * (src/stack/util.rs:86-119, 180-207).  The reference binds native code with
 * `#[repr(C)]` structs and `extern "C"` functions returning int
 * (src/stack/netif.rs:24-37, built by build.rs:19-21); this header follows the
 * same convention: plain pointers and sizes, no HIP or torch types, status
 * codes instead of exceptions.  INTEGRATION.md shows the Rust `extern "C"`
 * block and build.rs lines a maintainer would add.
 *
 * Two groups of entry points:
 *
 *  1. Per-packet host calls with the reference's exact signatures and results.
 *     They run on the calling CPU thread (a GPU launch costs microseconds; one
 *     packet costs ~100 ns), are re-entrant, and are what util.rs's four
 *     functions forward to.  Where the reference panics they return a negative
 *     status; the Rust shim turns that back into the same panic.
 *
 *  2. Batch calls that run the hand-written gfx950 kernels over many packets at
 *     once: device-resident (descriptors + arena already in HBM) and
 *     host-resident (pinned staging, overlapped copies).  They never fall back
 *     to the CPU: without a usable GPU they return RNS_E_NODEVICE.
 *
 * Result semantics (both groups, bit-exact with util.rs:88-106): the value is
 * the reference's u32 accumulator — seed + sum of big-endian 16-bit words, an
 * odd final byte counted as (byte << 8), wrapping mod 2^32 like a release
 * build — folded end-around to 16 bits.  RNS_FLAG_COMPLEMENT XORs it with
 * 0xffff, which is what every call site stores or tests (ip.rs:76,158;
 * tcp.rs:848,970; udp.rs:168; icmp.rs:46,71,91,110).
 */
#ifndef RNS_CHECKSUM_H
#define RNS_CHECKSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RNS_ABI_VERSION 1

/* ---- status codes (0 = ok, < 0 = error; never abort) ------------------- */
#define RNS_OK            0
#define RNS_E_INVALID    (-1)  /* bad argument (NULL pointer, bad address length, ...)  */
#define RNS_E_EMPTY      (-2)  /* empty slice: the reference panics (util.rs:92)           */
#define RNS_E_BOUNDS     (-3)  /* a packet descriptor lies outside its arena               */
#define RNS_E_NODEVICE   (-4)  /* no usable gfx950 device / HIP runtime                     */
#define RNS_E_ORDER      (-5)  /* host batch: offsets not ascending                         */
#define RNS_E_TOOLARGE   (-6)  /* host batch: one packet larger than the staging chunk      */
#define RNS_E_IO         (-7)  /* batched I/O: read/write/poll failed (see errno)            */
#define RNS_E_HIP_BASE   (-1000) /* RNS_E_HIP_BASE - hipError_t: HIP runtime error          */

/* ---- flags for batch calls ---------------------------------------------- */
#define RNS_FLAG_COMPLEMENT 0x1u   /* store 0xffff ^ sum (the transmitted / verified value) */
#define RNS_FLAG_CHAIN_RUNS 0x2u   /* rns_csum_chain_dev: fragments are often views of one buffer (see there) */
#define RNS_FLAG_CHAIN_TX_PACKED 0x4u  /* chains: transmit-shaped, payloads packed (rns_csum_chain_fill_dev) */

/* Fragment of a packet, same layout as the reference's `#[repr(C)] struct IOVec
 * { base: *const u8, len: usize }` (netif.rs:24-29). */
typedef struct rns_iovec {
    const uint8_t *base;
    size_t len;
} rns_iovec;

/* IP address, the C form of `enum IPAddr { V4([u8;4]), V6([u8;16]) }`
 * (util.rs:22-26): version is 4 or 6; V4 uses bytes[0..4]. */
typedef struct rns_ipaddr {
    uint32_t version;
    uint8_t bytes[16];
} rns_ipaddr;

/* ========================================================================
 * 1. Per-packet host calls (util.rs)
 * ====================================================================== */

/* util.rs:88 `pub fn compute_ones_comp(in_checksum: u16, slice: &[u8]) -> u16`.
 * Returns the 16-bit sum (>= 0), or RNS_E_EMPTY for len == 0 / RNS_E_INVALID. */
int32_t rns_compute_ones_comp(uint16_t in_checksum, const uint8_t *slice, size_t len);

/* util.rs:108 `pub fn compute_checksum(slice: &[u8]) -> u16` = 0xffff ^ ones_comp(0, slice). */
int32_t rns_compute_checksum(const uint8_t *slice, size_t len);

/* util.rs:112 `pub fn compute_buffer_ones_comp(initial_sum: u16, buffer: &NetBuffer) -> u16`.
 * `frags` are the slices NetBuffer::iter yields (buf.rs:466-487), folded one at
 * a time, so an odd-length non-final fragment is zero-padded like the reference.
 * An empty fragment returns RNS_E_EMPTY (the reference would panic on it). */
int32_t rns_compute_buffer_ones_comp(uint16_t initial_sum, const rns_iovec *frags, size_t nfrags);

/* util.rs:180 `pub fn compute_pseudo_header_checksum(source_ip, dest_ip, length: usize,
 * protocol: u8) -> u16`.  Layout follows dest_ip's version (util.rs:186); a
 * source of the other version is RNS_E_INVALID (the reference panics in copy_to). */
int32_t rns_compute_pseudo_header_checksum(const rns_ipaddr *source_ip, const rns_ipaddr *dest_ip,
                                           uint64_t length, uint8_t protocol);

/* ========================================================================
 * 2. Batch calls (HIP kernels for gfx950)
 * ====================================================================== */

/* Device-resident batch.  All pointers are device pointers on the current HIP
 * device; `stream` is a hipStream_t (NULL = the null stream).  Packet i is the
 * bytes d_arena[d_off[i] .. d_off[i] + d_len[i]) at any byte alignment; its seed
 * is d_seed[i] (d_seed == NULL => 0).  d_out[i] receives the result.
 * A descriptor outside [0, arena_bytes) gets d_out[i] = 0 and is counted in
 * *d_bad (device u32, optional, not reset by the call).  len == 0 gives the seed
 * (the reference panics).  `len_hint` is the typical packet
 * length in bytes (0 = unknown): it only picks the lanes-per-packet shape.
 * Asynchronous: returns after the launch; errors of the launch itself are
 * returned, never raised. */
int rns_csum_batch_dev(const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_off,
                       const uint32_t *d_len, const uint16_t *d_seed, uint16_t *d_out, uint32_t n,
                       uint32_t flags, uint32_t len_hint, uint32_t *d_bad, void *stream);

/* Compact descriptors: as rns_csum_batch_dev (util.rs:88-110 per packet) with
 * 32-bit packet offsets (arenas below 4 GiB), 10 B of descriptors per packet
 * instead of 14.  Same results. */
int rns_csum_batch_dev_off32(const uint8_t *d_arena, uint64_t arena_bytes, const uint32_t *d_off32,
                             const uint32_t *d_len, const uint16_t *d_seed, uint16_t *d_out, uint32_t n,
                             uint32_t flags, uint32_t len_hint, uint32_t *d_bad, void *stream);

/* Packed descriptors: packets lie back to back in index order, packet i+1
 * starting at the first multiple of 2^align_log2 at or after the end of packet i
 * (align_log2 <= 12), as a batched receive packs datagrams into one arena.  Only
 * the lengths travel (d_len16: u16 per packet — an IP datagram's length field is
 * 16 bits) plus d_blk_off[b] = the offset of packet 64*b, one u64 per 64 packets
 * (rns_packed_layout computes them): 2.1 B of descriptors per packet instead of
 * 10 (off32) or 14.  Per packet exactly util.rs:88-110, as rns_csum_batch_dev;
 * a packet outside the arena gets 0 and is counted in *d_bad.  With align_log2 >= 4
 * every batch but one of tiny packets (len_hint <= 112) is streamed as whole 1 KiB
 * rows of its 64-packet blocks, whatever the packet sizes (the rows kernel). */
int rns_csum_batch_packed_dev(const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_blk_off,
                              const uint16_t *d_len16, uint32_t align_log2, const uint16_t *d_seed, uint16_t *d_out,
                              uint32_t n, uint32_t flags, uint32_t len_hint, uint32_t *d_bad, void *stream);

/* Host helper for the packed form: given the n lengths, the alignment and the
 * first packet's offset, writes the (n + 63) / 64 block offsets to blk_off and
 * the offset just past the last packet's padded end to *end (the arena size the
 * packing needs).  Optionally (off != NULL) every packet's offset.  CPU only. */
int rns_packed_layout(const uint16_t *len16, uint64_t n, uint32_t align_log2, uint64_t first_off, uint64_t *blk_off,
                      uint64_t *off, uint64_t *end);

/* Same, for packets at a fixed stride (no offset/length arrays to read):
 * packet i = d_arena[first_off + i*stride .. + len).  Offsets that would wrap 64 bits are
 * RNS_E_INVALID (also for rns_rx_verify_strided_dev). */
int rns_csum_batch_strided_dev(const uint8_t *d_arena, uint64_t arena_bytes, uint64_t first_off,
                               uint64_t stride, uint32_t len, const uint16_t *d_seed, uint16_t *d_out,
                               uint32_t n, uint32_t flags, uint32_t *d_bad, void *stream);

/* Fragment chains: util.rs:112 `compute_buffer_ones_comp` for a batch of
 * NetBuffer-style fragment lists (buf.rs:466-487).  Packet i is fragments
 * [d_first[i], d_first[i+1]) of (d_frag_off, d_frag_len) — d_first has n_pkts+1
 * entries; each fragment is folded on its own and the running sum is folded after
 * every fragment, exactly as the reference's loop: an odd-length non-final
 * fragment is zero-padded like the per-fragment call, and the result is exact for
 * ANY fragment count and fragment size (a fragment past 128 KiB wraps the u32
 * accumulator from the running sum, as util.rs:89-99 does in a release build).
 * One pass, one kernel; d_frag_sums is unused (the round-1 two-pass scratch; may
 * be NULL).  A packet whose range is malformed (end < start, end > n_frags) or
 * that has a fragment outside the arena gets 0 and is counted in *d_bad.  An empty
 * fragment contributes nothing (the reference panics on it).
 * RNS_FLAG_CHAIN_RUNS (a hint; results are identical without it): a packet whose
 * <= 4 fragments lie back to back in memory, every one but the last of even length,
 * <= 128 KiB in all, has the same result as that contiguous range (the fragments'
 * words pair identically), so the kernel checks each wave's packets for this and
 * sums a wave whose packets all qualify as contiguous packets.  Set it when the
 * fragments are views of whole receive buffers (c3 as [492, 512, 496]: 287 -> 263 us);
 * without such runs the check costs a descriptor round (shuffled 512-byte buffers:
 * 268 -> 283 us), so it is off by default. */
/* Packets per chain call, at most (both chain entries; the kernel indexes a wave's 64 x 8
 * packets in 32 bits): a larger n_pkts is RNS_E_INVALID. */
#define RNS_CHAIN_MAX_PACKETS (0xFFFFFFFFu - 512u)
int rns_csum_chain_dev(const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_frag_off,
                       const uint32_t *d_frag_len, uint32_t n_frags, const uint32_t *d_first,
                       const uint16_t *d_seed, uint16_t *d_out, uint32_t n_pkts, uint32_t flags,
                       uint32_t frag_len_hint, uint16_t *d_frag_sums, uint32_t *d_bad, void *stream);

/* Transmit fill over fragment chains, the shape the reference actually transmits:
 * tcp_output / udp_output / icmp_output_* (tcp.rs:957-973, udp.rs:158-171,
 * icmp.rs:87-112) checksum a NetBuffer whose FIRST fragment is the head fragment
 * alloc_header prepended (buf.rs:262-291, zero-filled, so the field counts as zero:
 * buf.rs:286-288), then set_be16 the result into header_mut() = that fragment.  Packet i
 * = the CSR chain of rns_csum_chain_dev; its field is at byte d_field[i] (NULL =>
 * field_off for every packet: TCP 16, UDP 6, ICMP 2) of fragment d_first[i].  The chain
 * is folded exactly as compute_buffer_ones_comp(d_seed[i], chain) with the field's two
 * bytes counted as zero, and the result (0xffff ^ sum with RNS_FLAG_COMPLEMENT, as every
 * call site stores it; UDP's 0 is stored as is) is stored big-endian into the field.
 * d_out (optional) receives the results.  A packet with no fragments, a malformed range,
 * a fragment outside the arena, or a head fragment too short for its field is left
 * untouched, gets d_out 0 and is counted in *d_bad.  Fragments of different packets
 * must not overlap a field.  RNS_FLAG_CHAIN_RUNS: the hint of rns_csum_chain_dev (the
 * head fragment then starts each run).  Lay the head fragments of consecutive packets
 * back to back in a header region (a batching transmit path's header arena): a wave's
 * 64 field stores then land in a few cache lines instead of 64 scattered ones.
 * RNS_FLAG_CHAIN_TX_PACKED (a hint for this entry and rns_csum_chain_dev; results are
 * identical without it): packets are [a head fragment with (start & 15) + length <= 64,
 * then payload fragments (at most 4) that form a run: back to back, even non-final
 * lengths, <= 65535 bytes], and the payloads of consecutive packets ascend at 16-byte-
 * aligned starts (a packed payload region).  Each 64-packet block's payloads then stream
 * as one region (the rows kernel) while every owner sums its own head; a block that does
 * not have this shape takes an exact per-packet loop (slow; use the hint only for such
 * batches: a batch whose mean fragment count per packet exceeds 5 ignores the hint and
 * runs the chain kernel). */
int rns_csum_chain_fill_dev(uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_frag_off,
                            const uint32_t *d_frag_len, uint32_t n_frags, const uint32_t *d_first,
                            const uint16_t *d_seed, const uint16_t *d_field, uint32_t field_off, uint16_t *d_out,
                            uint32_t n_pkts, uint32_t flags, uint32_t frag_len_hint, uint32_t *d_bad, void *stream);

/* Transmit in-place fill (tcp.rs:957-973, udp.rs:158-171, icmp.rs:87-112,
 * ip.rs:158-159): for packet i, sum d_arena[d_off[i] .. + d_len[i]) seeded with
 * d_seed[i], counting the 2-byte checksum field at packet offset d_field[i]
 * (d_field == NULL => field_off for every packet: TCP 16, UDP 6, ICMP 2, IPv4
 * header 10) as zero — the reference zero-fills it (buf.rs:286-288) — and store
 * the result (0xffff ^ sum with RNS_FLAG_COMPLEMENT, as every call site does)
 * big-endian into the field (set_be16).  UDP keeps the reference's behaviour of
 * storing 0 as-is (no RFC 768 0 -> 0xffff).  d_out (optional) also receives the
 * results.  Packets must not overlap.  A packet outside the arena or too short
 * for its field is left untouched, gets d_out 0, and is counted in *d_bad. */
int rns_csum_fill_dev(uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_off, const uint32_t *d_len,
                      const uint16_t *d_seed, const uint16_t *d_field, uint32_t field_off, uint16_t *d_out,
                      uint32_t n, uint32_t flags, uint32_t *d_bad, void *stream);

/* Transmit in-place fill of a PACKED transmit arena (the descriptor form of
 * rns_csum_batch_packed_dev: u16 lengths, d_blk_off[b] = offset of packet 64*b,
 * packets back to back at 2^align_log2 boundaries, align_log2 >= 4): per packet exactly
 * what rns_csum_fill_dev does (tcp.rs:957-973, udp.rs:158-171, icmp.rs:87-112,
 * ip.rs:158-159) — the field at d_field[i] (NULL => field_off) counted as zero, the
 * result stored big-endian into it, d_out (optional) and *d_bad as there.  One wave
 * streams each 64-packet block's bytes as whole 1 KiB rows (the rows kernel); the owner
 * of a packet rewrites the 32-byte sector around its field when it lies inside the
 * packet.  len_hint = the typical packet length (kernel depth).  align_log2 < 4 is
 * RNS_E_INVALID. */
int rns_csum_fill_packed_dev(uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_blk_off, const uint16_t *d_len16,
                             uint32_t align_log2, const uint16_t *d_seed, const uint16_t *d_field, uint32_t field_off,
                             uint16_t *d_out, uint32_t n, uint32_t flags, uint32_t len_hint, uint32_t *d_bad,
                             void *stream);

/* Receive verify (§8f row 1): for each received IP datagram
 * d_arena[d_off[i] .. + d_len[i]), the checks the stack applies before handing it
 * to the transport layer — ip_input_v4 header checksum (ip.rs:76-80), fragment
 * drop (ip.rs:84-87), protocol dispatch (ip.rs:123-131), TCP validate_checksum
 * with the pseudo-header built from the source address and the LOCAL address
 * (tcp.rs:838-850), ICMPv4 (icmp.rs:46-50), ICMPv6 (icmp.rs:62-75); UDP is not
 * verified by the stack (udp.rs:126-148).  As in the reference, the L4 length is
 * the buffer length minus the IP header (the total-length field is not used).
 * One fused pass over the datagram bytes.  d_status[i] gets RNS_RX_* bits;
 * d_l4_sum (optional) the complemented L4 sum. */
#define RNS_RX_IP_OK          0x01u  /* IPv4 header checksum verifies (always set for IPv6) */
#define RNS_RX_L4_OK          0x02u  /* TCP / ICMPv4 / ICMPv6 checksum verifies */
#define RNS_RX_L4_UNCHECKED   0x04u  /* UDP: the stack does not verify it */
#define RNS_RX_FRAGMENT       0x08u  /* IPv4 fragment: the stack drops it */
#define RNS_RX_UNKNOWN_PROTO  0x10u  /* protocol the stack drops */
#define RNS_RX_ACCEPT         0x40u  /* the stack would deliver it to its transport handler */
#define RNS_RX_MALFORMED      0x80u  /* bad version / too short: the reference drops or panics */
int rns_rx_verify_dev(const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_off, const uint32_t *d_len,
                      uint32_t n, const uint8_t *local_ipv4, const uint8_t *local_ipv6, uint8_t *d_status,
                      uint16_t *d_l4_sum, void *stream);

/* Receive verify of a PACKED receive arena (the descriptor form of
 * rns_csum_batch_packed_dev: u16 lengths, d_blk_off[b] = offset of datagram 64*b),
 * with datagrams starting on 16-byte boundaries (align_log2 >= 4; 2048-byte receive
 * slots qualify): per datagram exactly the checks and status bits of rns_rx_verify_dev
 * (ip.rs:65-131, tcp.rs:838-850, icmp.rs:44-75).  One wave streams each 64-datagram
 * block's bytes as whole 1 KiB rows whatever the datagram sizes (the stream kernel);
 * a block of ACK-sized datagrams (all <= 64 B) is read by its owners directly, which
 * keeps them at the plain checksum's rate.  align_log2 < 4 is RNS_E_INVALID. */
int rns_rx_verify_packed_dev(const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_blk_off,
                             const uint16_t *d_len16, uint32_t align_log2, uint32_t n, const uint8_t *local_ipv4,
                             const uint8_t *local_ipv6, uint8_t *d_status, uint16_t *d_l4_sum, void *stream);

/* Receive verify of datagrams at a FIXED STRIDE (a receive ring of fixed-size slots:
 * the reference's 2048-byte MRU buffers, netif.rs:66, or 64-byte ACK slots): datagram i
 * = d_arena[first_off + i * stride .. + d_len16[i]); per datagram exactly the checks and
 * status bits of rns_rx_verify_dev (ip.rs:65-131, tcp.rs:838-850, icmp.rs:44-75).  No
 * offsets travel and there is no per-block scan: with 16-byte-aligned slots every lane
 * loads its datagram's first 64 bytes beside its length, so an ACK-sized datagram costs
 * one memory round; longer datagrams are summed by a whole wave each.  Any stride and
 * alignment is accepted (datagrams may even overlap: nothing is written to the arena). */
int rns_rx_verify_strided_dev(const uint8_t *d_arena, uint64_t arena_bytes, uint64_t first_off, uint64_t stride,
                              const uint16_t *d_len16, uint32_t n, const uint8_t *local_ipv4, const uint8_t *local_ipv6,
                              uint8_t *d_status, uint16_t *d_l4_sum, void *stream);

/* Transmit finalize (SURVEY a6, §8f row 2 for whole datagrams): for each finished
 * outgoing IP datagram d_arena[d_off[i] .. + d_len[i]), the checksums the stack's
 * transmit path stores — tcp_output (tcp.rs:957-973: pseudo-header from the header's
 * source and destination, length as u16, field [16..18] of the segment), udp_output
 * (udp.rs:151-171, [6..8], 0 stored as is), icmp_output_v4 (icmp.rs:87-95, [2..4], no
 * pseudo-header), icmp_output_v6 (icmp.rs:97-112, [2..4], full length, protocol 58) and
 * ip_output_v4 (ip.rs:140-160, header[10..12] over IHL*4 bytes) — computed as if the
 * fields were zero (alloc_header zero-fills them, buf.rs:286-288) and stored big-endian
 * in place, with every pseudo-header formed on the device.  One pass over each
 * datagram's bytes.  Datagrams must not overlap.  d_status (optional) gets RNS_TX_*. */
#define RNS_TX_IP_FILLED      0x01u  /* IPv4 header checksum stored */
#define RNS_TX_L4_FILLED      0x02u  /* TCP / UDP / ICMP checksum stored */
#define RNS_TX_MALFORMED      0x80u  /* bad version / IHL / too short, or outside the arena: untouched */
int rns_tx_fill_dev(uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_off, const uint32_t *d_len,
                    uint32_t n, uint8_t *d_status, void *stream);

/* Transmit finalize of a PACKED transmit arena (the descriptor form of
 * rns_csum_batch_packed_dev: u16 lengths, d_blk_off[b] = offset of datagram 64*b, datagrams
 * back to back at 2^align_log2 boundaries, align_log2 >= 4): per datagram exactly what
 * rns_tx_fill_dev stores and reports (tcp.rs:957-973, udp.rs:151-171, icmp.rs:87-112,
 * ip.rs:140-160; both fields computed as zero, pseudo-headers from the header's own
 * addresses).  One wave streams each 64-datagram block as whole 1 KiB rows (the rows kernel)
 * while each owner holds its datagram's header chunks and stores its two fields with one
 * 2-byte store each.  len_hint = the typical datagram length (row depth; 0 = unknown).
 * d_status optional.  align_log2 < 4 is RNS_E_INVALID. */
int rns_tx_fill_packed_dev(uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_blk_off, const uint16_t *d_len16,
                           uint32_t align_log2, uint32_t n, uint8_t *d_status, uint32_t len_hint, void *stream);

/* Transmit finalize of datagrams held as NetBuffer chains — the reference's own transmit layout
 * (buf.rs:262-291, 385-420): datagram i = the CSR chain of rns_csum_chain_dev (fragments
 * [d_first[i], d_first[i+1]) of (d_frag_off, d_frag_len)), whose FIRST fragment is the head
 * fragment alloc_header built — the IP header and, behind it, the L4 header (both prepended
 * into one fragment) — followed by the payload fragments.  Per datagram what tcp_output /
 * udp_output / icmp_output_* and ip_output_v4 store (tcp.rs:957-973, udp.rs:151-171,
 * icmp.rs:87-112, ip.rs:140-160): the L4 checksum = compute_buffer_ones_comp(pseudo-header,
 * [head[hdr..], payload...]) folded per fragment as the reference folds it (an odd-length
 * fragment pads its last byte), pseudo-header from the head's addresses and the chain's total
 * length; the IPv4 header checksum over head[..IHL*4]; both fields computed as zero and stored
 * big-endian into the head fragment.  Only head bytes are written.  d_status (optional) gets
 * RNS_TX_*: MALFORMED (untouched) for a malformed range, no fragments, a fragment outside the
 * arena, or a head that does not hold the IP header; no L4 fill for a protocol the stack does
 * not checksum, a segment too short for its field, or a field past the head fragment.  Heads
 * of consecutive datagrams back to back in a header region and payloads back to back at
 * 16-byte-aligned starts (the shape of RNS_FLAG_CHAIN_TX_PACKED; heads of at most 80 bytes from
 * their 16-byte boundary, at most 4 payload fragments forming a run) stream as rows; any other
 * 64-datagram block takes an exact per-datagram loop (same results, slower).  n_pkts >
 * RNS_CHAIN_MAX_PACKETS is RNS_E_INVALID. */
int rns_tx_fill_chain_dev(uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_frag_off, const uint32_t *d_frag_len,
                          uint32_t n_frags, const uint32_t *d_first, uint32_t n_pkts, uint8_t *d_status, void *stream);

/* Tuning entry (bench / tests): explicit kernel shape.  variant bit 0: 0 = group
 * kernel (one lane stores each result), 1 = rounds kernel (a wave owns 64
 * consecutive packets, one coalesced result store); bit 1: nontemporal packet
 * loads; bit 2: mixed kernel (rounds kernel that sorts each wave's 64 packets
 * into size classes, each with its own shape; G and U are ignored); bit 3 (with
 * bit 0 only): rounds kernel with every round of a batch in flight (G <= 8, U <= 2);
 * bit 4 (with bit 0 only, not with bit 3): rounds kernel that loads the next wave
 * batch's descriptors before the current batch's data (G <= 8, U <= 2);
 * bits 8-11: at most that many 4-wave workgroups per CU (an occupancy cap, by LDS
 * reservation; 0 = none).
 * lanes_per_packet in {4,8,16,32,64} (2 too for the rounds kernel); unroll (16-byte
 * chunks in flight per lane per pass) in {1,2,4,8}; max_blocks = grid cap (0 = no
 * grid-stride loop). */
int rns_csum_batch_dev_cfg(const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_off,
                           const uint32_t *d_len, const uint16_t *d_seed, uint16_t *d_out, uint32_t n,
                           uint32_t flags, uint32_t variant, uint32_t lanes_per_packet, uint32_t unroll,
                           uint32_t max_blocks, uint32_t *d_bad, void *stream);

/* Host-resident batch through a staging context: chunked H2D copies, kernels and
 * D2H copies of the 2-byte results overlapped on several streams of `device`.
 * Offsets must be ascending.  Synchronous (returns when h_out is filled).
 * The whole batch is validated before anything is queued: a packet with
 * (offset mod 256) + length > chunk_bytes returns RNS_E_TOOLARGE (and out-of-arena /
 * descending descriptors RNS_E_BOUNDS / RNS_E_ORDER) with h_out untouched.
 * For full PCIe rate allocate h_arena with rns_host_alloc (pinned).  A context
 * serialises its own calls (internal mutex); use one per thread for concurrency. */
typedef struct rns_host_ctx rns_host_ctx;
int rns_host_ctx_create(int device, uint64_t chunk_bytes, uint32_t nstreams, rns_host_ctx **out);
int rns_host_ctx_destroy(rns_host_ctx *ctx);
int rns_csum_batch_host(rns_host_ctx *ctx, const uint8_t *h_arena, uint64_t arena_bytes,
                        const uint64_t *h_off, const uint32_t *h_len, const uint16_t *h_seed,
                        uint16_t *h_out, uint32_t n, uint32_t flags);

/* Multi-GPU batches.  Packets are independent, so the
 * batch is cut into contiguous packet ranges of about equal bytes, one per GPU,
 * with no collective: each GPU's results go straight to their slice of the output.
 * rns_csum_batch_multi_host: a host-resident batch over one staging context per
 * device (devices[] may repeat a device), ranges run concurrently, synchronous.
 * rns_csum_batch_multi_dev: each GPU's shard is already in its own HBM; launches
 * every shard on its device and stream and returns (asynchronous, like
 * rns_csum_batch_dev); the calling thread's current device is restored. */
typedef struct rns_multi_ctx rns_multi_ctx;
int rns_multi_ctx_create(const int *devices, uint32_t ndev, uint64_t chunk_bytes, uint32_t nstreams,
                         rns_multi_ctx **out);
int rns_multi_ctx_destroy(rns_multi_ctx *ctx);
int rns_csum_batch_multi_host(rns_multi_ctx *ctx, const uint8_t *h_arena, uint64_t arena_bytes,
                              const uint64_t *h_off, const uint32_t *h_len, const uint16_t *h_seed,
                              uint16_t *h_out, uint32_t n, uint32_t flags);
typedef struct rns_dev_batch {
    int device;                 /* HIP device of this shard */
    const uint8_t *d_arena;     /* this shard's arena, on `device` */
    uint64_t arena_bytes;
    const uint64_t *d_off;
    const uint32_t *d_len;
    const uint16_t *d_seed;     /* NULL: seed 0 */
    uint16_t *d_out;
    uint32_t n;
    uint32_t len_hint;          /* as rns_csum_batch_dev */
    uint32_t *d_bad;            /* optional */
    void *stream;               /* a stream of `device` (NULL: its default stream) */
} rns_dev_batch;
int rns_csum_batch_multi_dev(const rns_dev_batch *batches, uint32_t nbatches, uint32_t flags);

/* Batched datagram I/O.  The reference reads / writes one
 * packet per call on the TUN fd (recv_packet netif.rs:65-83 -> tun_recv tun.c:84-86;
 * send_packet netif.rs:85-98 -> tun_send tun.c:88-90).  rns_io_recv_batch waits up
 * to timeout_ms for the first datagram, then reads every datagram already queued
 * (up to max_pkts) into consecutive slot_bytes slots of h_arena (2048 = the
 * reference's MRU, netif.rs:66); h_off/h_len describe them.  A datagram longer
 * than its slot is dropped (on socket fds recv(MSG_TRUNC) reports its full length),
 * never handed on truncated; max_pkts is capped at INT_MAX.  Returns the number of
 * datagrams (0 on timeout) or RNS_E_IO.  Works on a TUN fd or any datagram fd; on a
 * socket fd up to 64 datagrams per recvmmsg call.
 * rns_io_send_batch writes n datagrams (sendmmsg on a socket fd, one writev per datagram
 * on a TUN fd); returns how many were written. */
int rns_io_recv_batch(int fd, uint8_t *h_arena, uint64_t slot_bytes, uint32_t max_pkts, uint64_t *h_off,
                      uint32_t *h_len, int timeout_ms);
int rns_io_send_batch(int fd, const uint8_t *h_arena, const uint64_t *h_off, const uint32_t *h_len, uint32_t n);
/* Batched send_packet of NetBuffer chains (netif.rs:85-98: to_iovec over the fragments, then
 * tun_send's writev, tun.c:88-90): datagram i = fragments [h_first[i], h_first[i+1]) of
 * (h_frag_off, h_frag_len), at least one and at most RNS_IO_MAX_FRAGS of them (the reference's
 * MAX_VECS, netif.rs:22), sent as ONE datagram gathered from its fragments — sendmmsg with one message per
 * datagram on a socket fd, one writev per datagram on a TUN fd.  The chains of
 * rns_tx_fill_chain_dev go out as they are (heads in a header region, payloads elsewhere).
 * Returns the datagrams sent; a malformed range or too many fragments is RNS_E_INVALID before
 * anything is sent. */
#define RNS_IO_MAX_FRAGS 8u
int rns_io_send_batch_chain(int fd, const uint8_t *h_arena, const uint64_t *h_frag_off, const uint32_t *h_frag_len,
                            const uint32_t *h_first, uint32_t n_pkts);

/* Batched receive straight into a PACKED arena (the descriptor form of
 * rns_rx_verify_packed_dev): every queued datagram (after waiting up to timeout_ms for the
 * first) goes to the next 16-byte boundary of h_arena, as long as a datagram of mru bytes
 * (<= 65535; the reference's MRU is 2048, netif.rs:66) still fits behind it and fewer than
 * max_pkts were read.  h_len16[i] = datagram i's length, h_blk_off[b] = the offset of
 * datagram 64*b, *h_end = the arena bytes used (the last datagram's end rounded up to 16:
 * what a copy to the GPU needs).  A datagram longer than mru is dropped.  On a socket fd
 * batches of up to 64 datagrams take one recvmmsg each; a TUN fd takes one read per
 * datagram.  Returns the number of datagrams (0 on timeout) or RNS_E_IO. */
int rns_io_recv_batch_packed(int fd, uint8_t *h_arena, uint64_t arena_bytes, uint32_t mru, uint32_t max_pkts,
                             uint16_t *h_len16, uint64_t *h_blk_off, uint64_t *h_end, int timeout_ms);

/* Pinned host memory for arenas handed to rns_csum_batch_host. */
int rns_host_alloc(uint64_t bytes, void **out);
int rns_host_free(void *p);

/* Deterministic synthetic packet bytes on the device: splitmix64 stream,
 * little-endian words, word i = mix(seed + (i+1)*0x9E3779B97F4A7C15) — the
 * generator oracle/oracle.py splitmix64_bytes restates on the CPU. */
int rns_fill_splitmix64_dev(uint8_t *d_buf, uint64_t nbytes, uint64_t seed, void *stream);

/* ---- introspection ------------------------------------------------------- */
int rns_abi_version(void);
const char *rns_strerror(int status);
const char *rns_build_info(void);
/* Kernel and shape rns_csum_batch_dev picks for a typical packet length. */
const char *rns_csum_shape_name(uint32_t len_hint);
int rns_device_count(void);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* RNS_CHECKSUM_H */
