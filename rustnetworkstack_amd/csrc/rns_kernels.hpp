// Batched Internet (RFC 1071) checksum for MI355X (gfx950, CDNA4).
//
// The reference computes compute_ones_comp (src/stack/util.rs:88-106) once per
// packet on whichever CPU thread handles it.  Here a batch of
// packets already resident in HBM is checksummed by one launch:
//
//   * a packet is owned by a GROUP of G lanes (G = 4..64, a power of two, so a
//     64-lane wavefront serves 64/G packets at once); the group streams the
//     packet as 16-byte aligned chunks, lane l taking chunks l, l+G, ...,
//     U chunks in flight per lane (global_load_dwordx4, fully coalesced);
//   * bytes outside [start, start+len) in the first / last chunk are masked
//     to zero, so packets may start at any byte offset and the odd final
//     byte is the zero-padded word the reference adds as byte << 8;
//   * each dword is split by two v_dot4_u32_u8 into the sum of the bytes that
//     are the HIGH half of a big-endian word and the sum of the LOW halves
//     (which is which depends on the packet start's parity).  The reference's
//     u32 accumulator is exactly  seed + 256*high + low  (mod 2^32), so the
//     per-lane u32 partials are summed with wrap-around across the group
//     (shuffle butterfly) and folded end-around exactly like util.rs:101-103:
//     bit-exact for every length, including the reference's wrap past 128 KiB;
//   * one lane per group stores the u16 result (optionally ^ 0xffff).
//
// This is a bandwidth-bound integer reduction (~1 byte of HBM per 0.5 VALU
// op): no MFMA, no LDS staging needed for the data itself.  Roofline: HBM read
// bandwidth; algorithmic bytes per packet = len + 2.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <type_traits>
#include <vector>

#include "rns_checksum.h"

namespace rns {

#ifndef RNS_BLOCK
#define RNS_BLOCK 256
#endif
constexpr int kBlock = RNS_BLOCK;  // threads per workgroup (A/B knob: 64..1024)

struct CsumArgs {
    const uint8_t *arena;      // 16-byte aligned base
    uint64_t arena_bytes;      // valid bytes from `arena` (after base_adjust)
    uint64_t base_adjust;      // added to every packet offset (caller base was not 16-aligned)
    const uint64_t *off;       // per-packet byte offsets (null in strided mode)
    const uint32_t *off32;     // compact form: 32-bit offsets for arenas < 4 GiB (used when non-null)
    const uint32_t *len;       // per-packet lengths (null in strided mode)
    const uint16_t *seed;      // per-packet seeds, null => 0
    uint16_t *out;
    uint32_t *bad;             // optional counter of rejected descriptors
    uint64_t first_off;        // strided mode
    uint64_t stride;
    uint32_t fixed_len;
    uint32_t n;
    uint32_t flags;
    const uint16_t *field;     // transmit fill: per-packet checksum field offset (null => field_off)
    uint32_t field_off;
    uint8_t *status;           // receive verify: RNS_RX_* per datagram
    uint16_t *l4_out;          // receive verify: complemented L4 sum (optional)
    uint32_t local4_sum;       // receive verify: BE word sums of the local addresses
    uint32_t local6_sum;
    const uint16_t *len16;     // packed form: u16 lengths, offsets implied (used when non-null)
    const uint64_t *blk_off;   // packed form: offset of packet 64*b, per block b of 64 packets
    uint32_t align_mask;       // packed form: packet starts are multiples of align_mask + 1
    const uint32_t *first;     // fragment chains: packet i = fragments [first[i], first[i+1]) (off/len = fragments)
    uint32_t n_frags;
    uint32_t chain_k;          // fragment chains: packets per lane (a wave owns 64*chain_k consecutive packets)
    uint32_t len_hint;         // packed form: the caller's typical packet length (kernel choice)
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Descriptor offset of packet p: the compact 32-bit form when the caller passed one
// (10 B of descriptors per packet instead of 14), else the 64-bit form.  The branch
// is on a kernel argument, so it is uniform.
__device__ __forceinline__ uint64_t desc_off(const CsumArgs &a, uint64_t p)
{
    return a.off32 ? static_cast<uint64_t>(a.off32[p]) : a.off[p];
}

// Packed form (rns_csum_batch_packed_dev): packets lie back to back in index order,
// each starting at the next multiple of (align_mask + 1) after the previous one's
// end, so a packet's offset is its 64-packet block's base plus the padded lengths
// of the packets before it in the block — an exclusive scan across the wave that
// owns the block (every lane calls this with p = base + lane, base a multiple of
// 64).  Descriptors: 2 B of length per packet + 8 B per 64 packets.
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF>
__device__ __forceinline__ uint32_t dpp_or_zero(uint32_t v)
{
    // lanes the masks disable, and lanes whose source lies outside the row, read 0
    return static_cast<uint32_t>(
        __builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, ROW_MASK, BANK_MASK, true));
}

// Exclusive prefix sum over the 64 lanes (the total must fit 32 bits): the classic
// gfx9 DPP scan (row_shr 1,2,3 / 4 / 8 within each row of 16, then row_bcast:15 and
// row_bcast:31 across rows) — VALU only, no LDS round trip.  packed_scan applies it
// to the lanes' padded lengths.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v)
{
    uint32_t x = v;
    x += dpp_or_zero<0x111>(v);              // row_shr:1
    x += dpp_or_zero<0x112>(v);              // row_shr:2
    x += dpp_or_zero<0x113>(v);              // row_shr:3
    x += dpp_or_zero<0x114, 0xF, 0xE>(x);    // row_shr:4, banks 1-3
    x += dpp_or_zero<0x118, 0xF, 0xC>(x);    // row_shr:8, banks 2-3
    x += dpp_or_zero<0x142, 0xA, 0xF>(x);    // row_bcast:15 into rows 1 and 3
    x += dpp_or_zero<0x143, 0xC, 0xF>(x);    // row_bcast:31 into rows 2 and 3
    return x - v;
}

__device__ __forceinline__ uint32_t packed_scan(const CsumArgs &a, uint32_t lane, uint32_t len)
{
    (void)lane;
    const uint32_t pad = (len + a.align_mask) & ~a.align_mask;  // < 2^17: the block's sum fits 32 bits
    return wave_excl_scan(pad);
}

__device__ __forceinline__ uint64_t packed_off(const CsumArgs &a, uint64_t base, uint32_t lane, uint32_t len)
{
    return a.blk_off[base >> 6] + packed_scan(a, lane, len);
}

// Cache-policy bits of the "nontemporal" buffer loads (gfx950 CPol: 1 = sc0, 2 = nt,
// 16 = sc1).  A/B knob: -DRNS_NT_AUX=...
#ifndef RNS_NT_AUX
#define RNS_NT_AUX 2
#endif
constexpr int kNtAux = RNS_NT_AUX;

// One 16-byte chunk.  NT = nontemporal (streamed once: do not keep it in the
// caches; the HBM read probe in tools/ measured +5..10 % for streaming reads).
template <bool NT>
__device__ __forceinline__ uint4 load_chunk(const uint8_t *p)
{
    if constexpr (NT) {
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return *reinterpret_cast<const uint4 *>(p);
    }
}

// Keep bytes [lo, hi) of the 4-byte dword at byte j4 = 4*j of a 16-byte chunk.
__device__ __forceinline__ uint32_t keep_bytes(uint32_t d, int lo, int hi, int j4)
{
    const int a = min(max(lo - j4, 0), 4);
    const int b = min(max(hi - j4, 0), 4);
    const uint32_t hm = static_cast<uint32_t>((1ull << (8 * b)) - 1);
    const uint32_t lm = static_cast<uint32_t>((1ull << (8 * a)) - 1);
    return d & hm & ~lm;  // b <= a gives 0
}

// Lanes of one wave exchanging data through LDS: the hardware executes a wave's LDS
// operations in order, but without a fence the compiler may treat another lane's
// store as a data race and forward this lane's own earlier store into a later load
// (it did: flag[lane] = 0 ... flag[t] = 1 ... flag[lane] was folded to 0).  A
// wavefront-scope fence costs no instruction and keeps the load.
__device__ __forceinline__ void wave_lds_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t v)
{
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1)
        v += static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), m, 64));
    return v;
}

template <int G, int U, bool STRIDED, bool NT>
__global__ __launch_bounds__(kBlock) void csum_batch_kernel(const CsumArgs a)
{
    static_assert(G >= 4 && G <= 64 && (G & (G - 1)) == 0, "G must be a power of two in [4,64]");
    constexpr uint32_t kGroups = kBlock / G;
    const uint32_t lane = threadIdx.x & (G - 1);
    const uint32_t grp_stride = gridDim.x * kGroups;

    for (uint32_t p = blockIdx.x * kGroups + threadIdx.x / G; p < a.n; p += grp_stride) {
        uint64_t start;
        uint32_t L;
        if constexpr (STRIDED) {
            start = a.first_off + static_cast<uint64_t>(p) * a.stride;
            L = a.fixed_len;
        } else {
            start = desc_off(a, p);
            L = a.len[p];
        }
        start += a.base_adjust;
        const bool ok = start <= a.arena_bytes && L <= a.arena_bytes - start;

        uint32_t hi_sum = 0, lo_sum = 0;
        if (ok && L != 0) {
            const uint32_t s = static_cast<uint32_t>(start & 15);
            const uint8_t *base = a.arena + (start - s);
            const uint64_t span = s + static_cast<uint64_t>(L);
            const uint32_t nch = static_cast<uint32_t>((span + 15) >> 4);
            const uint32_t last = nch - 1;
            const int e = static_cast<int>(span - (static_cast<uint64_t>(last) << 4));  // 1..16
            // Bytes at even offsets from the packet start are BE high halves.
            const uint32_t w_hi = (start & 1) ? 0x01000100u : 0x00010001u;
            const uint32_t w_lo = w_hi ^ 0x01010101u;

            for (uint32_t c0 = lane; c0 < nch; c0 += G * U) {
                uint4 v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t c = c0 + u * G;
                    if (c < nch)
                        v[u] = load_chunk<NT>(base + (static_cast<uint64_t>(c) << 4));
                    else
                        v[u] = make_uint4(0, 0, 0, 0);
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t c = c0 + u * G;
                    if ((c == 0 && s != 0) || (c == last && e != 16)) {
                        const int lo = (c == 0) ? static_cast<int>(s) : 0;
                        const int hi = (c == last) ? e : 16;
                        v[u].x = keep_bytes(v[u].x, lo, hi, 0);
                        v[u].y = keep_bytes(v[u].y, lo, hi, 4);
                        v[u].z = keep_bytes(v[u].z, lo, hi, 8);
                        v[u].w = keep_bytes(v[u].w, lo, hi, 12);
                    }
                    hi_sum = __builtin_amdgcn_udot4(v[u].x, w_hi, hi_sum, false);
                    lo_sum = __builtin_amdgcn_udot4(v[u].x, w_lo, lo_sum, false);
                    hi_sum = __builtin_amdgcn_udot4(v[u].y, w_hi, hi_sum, false);
                    lo_sum = __builtin_amdgcn_udot4(v[u].y, w_lo, lo_sum, false);
                    hi_sum = __builtin_amdgcn_udot4(v[u].z, w_hi, hi_sum, false);
                    lo_sum = __builtin_amdgcn_udot4(v[u].z, w_lo, lo_sum, false);
                    hi_sum = __builtin_amdgcn_udot4(v[u].w, w_hi, hi_sum, false);
                    lo_sum = __builtin_amdgcn_udot4(v[u].w, w_lo, lo_sum, false);
                }
            }
        }
        // sum of BE words of this lane's bytes, mod 2^32 (the reference's u32 wraps the same way)
        const uint32_t words = group_sum<G>((hi_sum << 8) + lo_sum);

        if (lane == 0) {
            const uint32_t sd = a.seed ? a.seed[p] : 0u;
            uint32_t acc = sd + words;  // util.rs:89-99 (mod 2^32)
            while (acc > 0xffff)        // util.rs:101-103
                acc = (acc & 0xffff) + (acc >> 16);
            if (a.flags & RNS_FLAG_COMPLEMENT)
                acc ^= 0xffff;
            if (!ok) {
                acc = 0;
                if (a.bad)
                    atomicAdd(a.bad, 1u);
            }
            a.out[p] = static_cast<uint16_t>(acc);
        }
    }
}


// ---------------------------------------------------------------------------
// v2: "rounds" kernel — a wavefront owns 64 CONSECUTIVE packets (a batch).
//
//   * one coalesced load of the batch's 64 descriptors (lane l: packet base+l);
//   * the batch is processed in G rounds; in round r, group g (G lanes) takes
//     packet base + r*P + g (P = 64/G packets at once), its descriptor
//     broadcast from lane r*P + g (readlane for G = 64, ds_bpermute otherwise);
//   * the first pass (G*U chunks) of round r+1 is loaded BEFORE round r is
//     consumed, so every wave keeps a pass of loads in flight while it masks,
//     dot4-sums and reduces;
//   * group sums use DPP (quad_perm, row_half_mirror, row_mirror) + ds_swizzle;
//     lane l collects the sum of ITS packet, adds the seed, folds, and the 64
//     results leave in ONE 128-byte store.  (v1's one-lane 2-byte stores from
//     many CUs made small-packet batches write-bound: ~4 packets/ns.)
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v)
{
    return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), CTRL, 0xF, 0xF, true));
}

// Sum over aligned groups of G lanes; every lane of a group receives its group's sum.
template <int G>
__device__ __forceinline__ uint32_t group_allreduce(uint32_t v)
{
    if constexpr (G >= 2) v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]: lane ^ 1
    if constexpr (G >= 4) v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]: lane ^ 2
    if constexpr (G >= 8) v += dpp_mov<0x141>(v);   // row_half_mirror: the other quad of 8
    if constexpr (G >= 16) v += dpp_mov<0x140>(v);  // row_mirror: the other half of 16
    if constexpr (G >= 32)                          // ds_swizzle bitmode xor 0x10: lane ^ 16
        v += static_cast<uint32_t>(__builtin_amdgcn_ds_swizzle(static_cast<int>(v), 0x401F));
    if constexpr (G >= 64)
        v = __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 32);
    return v;
}

template <int G>
__device__ __forceinline__ uint32_t bcast_from(uint32_t v, uint32_t src)
{
    if constexpr (G == 64)
        return __builtin_amdgcn_readlane(v, src);  // src is wave-uniform
    else
        return static_cast<uint32_t>(__shfl(static_cast<int>(v), static_cast<int>(src), 64));
}

// Packets up to this length cannot wrap the reference's u32 accumulator
// (seed + 65537 words * 0xffff <= 2^32 - 1): they take the one-op-per-dword
// v_sad_u16 path.  Longer packets take the exact dot4 path (wrap emulated).
constexpr uint32_t kNoWrapBytes = 131072;

// Byte offset that is out of range for every buffer descriptor we build, even
// after the compiler folds an immediate offset (<= 4095) into it.
constexpr uint32_t kOobOffset = 0xFFFFF000u;

// Buffer range checks are per dword: a dword that straddles num_records reads as
// zero.  The descriptor therefore covers the arena rounded up to whole 16-byte
// chunks (the bytes past arena_bytes share a chunk, hence a page, with valid
// bytes, and are masked away like every byte outside a packet).
__host__ __device__ __forceinline__ uint64_t buf_records(const CsumArgs &a) { return (a.arena_bytes + 15) & ~15ull; }

// Chunk stash (receive verify and transmit fill).  The word sum is linear in the
// bytes, so verify and fill run the PLAIN data pass over the whole packet; the few
// chunks their finish needs (a datagram's header, a packet's checksum field) are
// copied to LDS by the lanes that load them anyway, and the owner lane finishes
// from there: no extra memory round, no per-chunk header/field masking.
enum StashMode : int { kStashNone = 0, kStashHead = 1, kStashField = 2, kStashTx = 3 };
// Chunks stashed per packet: a datagram's first 5 chunks hold its first
// 16*5 - 15 = 65 >= 60 bytes (the longest IPv4 header) at any start offset; a
// field's chunks are the 32-byte sector that holds its first byte plus the next
// chunk (a field at the sector's last byte spills into it).
#ifndef RNS_FILL_BLOCK
#define RNS_FILL_BLOCK 32
#endif
// Transmit fill rewrites the largest aligned block (kFieldBlock, /2, ... 32 bytes)
// around the field that lies inside the packet; the stash holds that block's chunks
// plus the next one.
constexpr int kFieldBlock = RNS_FILL_BLOCK;
constexpr int kFieldChunks = kFieldBlock / 16;
static_assert(kFieldBlock >= 32 && kFieldBlock <= 128 && (kFieldBlock & (kFieldBlock - 1)) == 0, "fill block");
template <int MODE>
constexpr int kStashChunks = MODE == kStashHead ? 5 : MODE == kStashField ? kFieldChunks + 1 : MODE == kStashTx ? 6 : 0;

// First stashed chunk (relative to the packet's chunk 0) for a field whose first
// byte is in chunk cf: the chunk that starts the field's aligned kFieldBlock-byte
// block in MEMORY (chunk0 = the packet's chunk 0 index from the 16-byte aligned
// arena base; apar = that base's chunk index mod kFieldChunks).  May be negative.
__host__ __device__ __forceinline__ int field_block_lo(uint32_t cf, uint32_t chunk0, uint32_t apar)
{
    return static_cast<int>(cf) - static_cast<int>((apar + chunk0 + cf) & (kFieldChunks - 1));
}

struct Pkt {
    uint64_t start;       // packet byte offset from the 16-byte aligned arena base
    uint32_t nch;         // 16-byte chunks covering the packet (0 if empty)
    int s;                // first valid byte in chunk 0
    int e;                // bytes valid in the last chunk (1..16)
    bool big;             // > kNoWrapBytes: exact big-endian path
    int stash_lo;         // stash: first chunk to copy to LDS
    int stash_at;         // stash: LDS chunk index of that chunk's slot
};

__device__ __forceinline__ Pkt make_pkt(uint64_t start, uint32_t L)
{
    Pkt k;
    k.start = start;
    k.s = static_cast<int>(k.start & 15);
    const uint64_t span = static_cast<uint64_t>(k.s) + L;
    k.nch = L ? static_cast<uint32_t>((span + 15) >> 4) : 0u;
    k.e = static_cast<int>(span - (static_cast<uint64_t>(k.nch ? k.nch - 1 : 0) << 4));
    k.big = L > kNoWrapBytes;
    k.stash_lo = 0;
    k.stash_at = 0;
    return k;
}

// Stash slots of the packet at sorted position `slot`.  kStashField: `field` = its
// checksum field offset; the stash starts at the chunk that begins the field's
// 32-byte MEMORY sector (apar = parity of the arena base's 16-byte chunk index), so
// slots 0-1 are that sector whenever it lies inside the packet.
template <int MODE>
__device__ __forceinline__ void set_stash(Pkt &k, uint32_t slot, uint32_t field, uint32_t apar)
{
    if constexpr (MODE != kStashNone) {
        k.stash_at = static_cast<int>(slot) * kStashChunks<MODE>;
        if constexpr (MODE == kStashField) {
            const uint32_t cf = (static_cast<uint32_t>(k.s) + min(field, 1u << 30)) >> 4;
            k.stash_lo = field_block_lo(cf, static_cast<uint32_t>(k.start >> 4), apar);
        }
    }
}

template <int G, int MODE = kStashNone>
__device__ __forceinline__ Pkt fetch_pkt(uint64_t d_start, uint32_t d_len, uint32_t src, uint32_t d_aux = 0xFFFFFFFFu,
                                         uint32_t apar = 0)
{
    const uint32_t lo = bcast_from<G>(static_cast<uint32_t>(d_start), src);
    const uint32_t hi = bcast_from<G>(static_cast<uint32_t>(d_start >> 32), src);
    const uint32_t L = bcast_from<G>(d_len, src);
    const uint32_t x = MODE == kStashField ? bcast_from<G>(d_aux, src) : 0xFFFFFFFFu;
    Pkt k = make_pkt((static_cast<uint64_t>(hi) << 32) | lo, L);
    set_stash<MODE>(k, src, x, apar);
    return k;
}

__device__ __forceinline__ uint32_t arena_parity(const CsumArgs &a)
{
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>(a.arena) >> 4) & (kFieldChunks - 1);
}

// Loads of one pass: chunk c = c0 + u*G of the packet, for u < U.  Branch-free:
// a chunk past the packet's end reads zeros (buffer path: out-of-range offset;
// global path: re-reads the packet's first chunk, then selects zero), so the
// compiler can count outstanding loads exactly and keep the next round's
// pass in flight while this one is consumed.
template <int G, int U, bool NT, bool BUF, int N = U>
__device__ __forceinline__ void issue_pass(const CsumArgs &a, __amdgpu_buffer_rsrc_t rsrc, const Pkt &k, uint32_t c0,
                                           uint4 (&v)[N])
{
    const uint64_t first = k.start - static_cast<uint64_t>(k.s);  // 16-aligned offset of chunk 0
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t c = c0 + u * G;
        const bool in = c < k.nch;
        if constexpr (BUF) {
            const uint32_t off = in ? static_cast<uint32_t>(first + (static_cast<uint64_t>(c) << 4)) : kOobOffset;
            const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, NT ? kNtAux : 0);
            v[u] = make_uint4(x.x, x.y, x.z, x.w);
        } else {
            const uint8_t *ptr = a.arena + first + (in ? (static_cast<uint64_t>(c) << 4) : 0);
            const uint4 x = load_chunk<NT>(ptr);  // nch == 0 never reaches here (see caller)
            v[u] = in ? x : make_uint4(0, 0, 0, 0);
        }
    }
}

template <int G, int U, int N = U>
__device__ __forceinline__ void mask_edges(const Pkt &k, uint32_t c0, uint4 (&v)[N])
{
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t c = c0 + u * G;
        // (a chunk-aligned start or end needs no mask: with 16-byte-aligned packet
        // starts the head chunk is skipped by the whole wave)
        if ((c == 0 && k.s != 0) || (c + 1 == k.nch && k.e != 16)) {
            const int lo = (c == 0) ? k.s : 0;
            const int hi = (c + 1 == k.nch) ? k.e : 16;
            v[u].x = keep_bytes(v[u].x, lo, hi, 0);
            v[u].y = keep_bytes(v[u].y, lo, hi, 4);
            v[u].z = keep_bytes(v[u].z, lo, hi, 8);
            v[u].w = keep_bytes(v[u].w, lo, hi, 12);
        }
    }
}

// Copy the chunks of this pass that the finish needs to their LDS slots (after
// edge masking: only bytes outside the packet were zeroed, and the finish reads
// none of those).  Chunks past the packet's end are never written: their slot may
// belong to a valid packet of another group.
template <int MODE, int G, int U, int N = U>
__device__ __forceinline__ void stash_chunks(const Pkt &k, uint32_t c0, const uint4 (&v)[N], uint4 *st)
{
    if constexpr (MODE != kStashNone) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = c0 + u * G;
            const uint32_t i = c - static_cast<uint32_t>(k.stash_lo);
            if (i < static_cast<uint32_t>(kStashChunks<MODE>) && c < k.nch)
                st[k.stash_at + static_cast<int>(i)] = v[u];
        }
    }
}

// Little-endian 16-bit word sum (v_sad_u16: lo16 + hi16 + acc, one op per dword).
template <int U, int N = U>
__device__ __forceinline__ uint32_t sum_le(const uint4 (&v)[N], uint32_t acc)
{
#pragma unroll
    for (int u = 0; u < U; ++u) {
        acc = __builtin_amdgcn_sad_u16(v[u].x, 0, acc);
        acc = __builtin_amdgcn_sad_u16(v[u].y, 0, acc);
        acc = __builtin_amdgcn_sad_u16(v[u].z, 0, acc);
        acc = __builtin_amdgcn_sad_u16(v[u].w, 0, acc);
    }
    return acc;
}

// Exact big-endian word sum mod 2^32: 256 * (high-half bytes) + (low-half bytes).
template <int U, int N = U>
__device__ __forceinline__ void sum_be(const uint4 (&v)[N], uint32_t w_hi, uint32_t &hs, uint32_t &ls)
{
    const uint32_t w_lo = w_hi ^ 0x01010101u;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        hs = __builtin_amdgcn_udot4(v[u].x, w_hi, hs, false);
        ls = __builtin_amdgcn_udot4(v[u].x, w_lo, ls, false);
        hs = __builtin_amdgcn_udot4(v[u].y, w_hi, hs, false);
        ls = __builtin_amdgcn_udot4(v[u].y, w_lo, ls, false);
        hs = __builtin_amdgcn_udot4(v[u].z, w_hi, hs, false);
        ls = __builtin_amdgcn_udot4(v[u].z, w_lo, ls, false);
        hs = __builtin_amdgcn_udot4(v[u].w, w_hi, hs, false);
        ls = __builtin_amdgcn_udot4(v[u].w, w_lo, ls, false);
    }
}

// One packet's contribution from this lane.  `v` holds the (prefetched) first pass.
// MODE != kStashNone: the chunks the finish needs are also copied to LDS (`st`).
template <int G, int U, bool NT, bool BUF, int N = U, int MODE = kStashNone>
__device__ __forceinline__ uint32_t packet_partial(const CsumArgs &a, __amdgpu_buffer_rsrc_t rsrc, const Pkt &k,
                                                   uint32_t sub, uint4 (&v)[N], uint4 *st = nullptr)
{
    constexpr uint32_t kPass = G * U;
    mask_edges<G, U, N>(k, sub, v);
    stash_chunks<MODE, G, U, N>(k, sub, v, st);
    if (!k.big) {
        uint32_t acc = sum_le<U, N>(v, 0u);
        for (uint32_t c0 = kPass + sub; c0 < k.nch; c0 += kPass) {  // packets longer than one pass (reuse v)
            issue_pass<G, U, NT, BUF, N>(a, rsrc, k, c0, v);
            mask_edges<G, U, N>(k, c0, v);
            stash_chunks<MODE, G, U, N>(k, c0, v, st);
            acc = sum_le<U, N>(v, acc);
        }
        return acc;  // LE-word sum, exact (< 2^32 for a packet of <= 128 KiB)
    }
    const uint32_t w_hi = (k.start & 1) ? 0x01000100u : 0x00010001u;
    uint32_t hs = 0, ls = 0;
    sum_be<U, N>(v, w_hi, hs, ls);
    for (uint32_t c0 = kPass + sub; c0 < k.nch; c0 += kPass) {
        issue_pass<G, U, NT, BUF, N>(a, rsrc, k, c0, v);
        mask_edges<G, U, N>(k, c0, v);
        stash_chunks<MODE, G, U, N>(k, c0, v, st);
        sum_be<U, N>(v, w_hi, hs, ls);
    }
    return (hs << 8) + ls;  // BE-word sum mod 2^32, exactly the reference's accumulator
}

// Owner-lane finish: seed + this packet's word sum -> the reference's folded u16.
// odd: the packet starts at an odd offset; big: longer than kNoWrapBytes (BE sum).
__device__ __forceinline__ uint16_t finalize_bits(uint32_t mine, bool odd, bool big, uint32_t d_seed, bool d_ok,
                                                  uint32_t flags)
{
    uint32_t acc;
    if (!big) {
        // seed + BE words, no wrap possible: equals seed + G where G is the LE
        // sum folded and byte-swapped (a packet at an odd offset is already in
        // BE order relative to the aligned words) — RFC 1071 §2(B).
        uint32_t x = mine;
        while (x > 0xffff)
            x = (x & 0xffff) + (x >> 16);
        const uint32_t g = odd ? x : (((x & 0xff) << 8) | (x >> 8));
        acc = d_seed + g;
        acc = (acc & 0xffff) + (acc >> 16);  // <= 0x1fffe: one end-around step folds it
    } else {
        acc = d_seed + mine;  // util.rs:89-99 (mod 2^32)
        while (acc > 0xffff)  // util.rs:101-103
            acc = (acc & 0xffff) + (acc >> 16);
    }
    if (flags & RNS_FLAG_COMPLEMENT)
        acc ^= 0xffff;
    return d_ok ? static_cast<uint16_t>(acc) : static_cast<uint16_t>(0);
}

__device__ __forceinline__ uint16_t finalize(uint32_t mine, uint64_t d_start, uint32_t d_len, uint32_t d_seed,
                                             bool d_ok, uint32_t flags)
{
    return finalize_bits(mine, d_start & 1, d_len > kNoWrapBytes, d_seed, d_ok, flags);
}

// D = rounds in flight: 1 = the next round's first pass is issued before the current
// round is consumed; D = G (small G only) = all rounds of the batch are issued up
// front, so a batch of tiny packets costs one memory latency instead of G.
// PF: the next wave batch's descriptors are loaded (branch-free) before the current
// batch's data, so a wave's descriptor latency overlaps its previous batch instead of
// preceding each batch's first data load (tiny packets: a batch is only G rounds).
template <int G, int U, bool STRIDED, bool NT, bool BUF, int D = 1, bool PACKED = false, bool PF = false>
__global__ __launch_bounds__(kBlock) void csum_rounds_kernel(const CsumArgs a)
{
    static_assert(G >= 2 && G <= 64 && (G & (G - 1)) == 0, "G must be a power of two in [2,64]");
    static_assert(D == 1 || (D == G && G <= 8), "deep prefetch: every round of a small-G batch");
    constexpr uint32_t P = 64 / G;  // packets per round
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t sub = lane & (G - 1);
    const uint32_t grp = lane / G;
    const uint32_t wave = (blockIdx.x * kBlock + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * kBlock) >> 6;
    // Whole-arena buffer descriptor (used only when BUF: the arena fits a 32-bit offset).
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.arena), static_cast<short>(0), static_cast<int>(BUF ? buf_records(a) : 0), 0x00020000);

    const uint64_t wstride = static_cast<uint64_t>(nwaves) * 64;
    // PF: raw descriptors of the batch at `base` (packed: the length and the block base)
    uint64_t r_off = 0;
    uint32_t r_len = 0, r_seed = 0;
    auto fetch_raw = [&](uint64_t b) {
        const uint64_t q = b + lane < a.n ? b + lane : a.n - 1;  // branch-free: past the end re-reads the last
        if constexpr (PACKED) {
            r_len = a.len16[q];
            r_off = a.blk_off[(b < a.n ? b : a.n - 1) >> 6];
        } else if constexpr (!STRIDED) {
            r_off = desc_off(a, q);
            r_len = a.len[q];
        }
        r_seed = a.seed ? a.seed[q] : 0u;
    };
    if constexpr (PF)
        fetch_raw(static_cast<uint64_t>(wave) * 64);

    for (uint64_t base = static_cast<uint64_t>(wave) * 64; base < a.n; base += wstride) {
        const uint64_t p = base + lane;
        const bool live = p < a.n;
        uint64_t d_start = 0;
        uint32_t d_len = 0, d_seed = 0;
        if constexpr (PF) {
            const uint64_t c_off = r_off;
            const uint32_t c_len = r_len, c_seed = r_seed;
            fetch_raw(base + wstride);  // the next batch's descriptors, in flight during this one
            d_seed = live ? c_seed : 0u;
            if constexpr (STRIDED) {
                d_start = a.first_off + p * a.stride;
                d_len = live ? a.fixed_len : 0u;
            } else if constexpr (PACKED) {
                d_len = live ? c_len : 0u;
                d_start = c_off + packed_scan(a, lane, d_len);
            } else {
                d_start = live ? c_off : 0;
                d_len = live ? c_len : 0u;
            }
        } else {
            if (live) {
                if constexpr (STRIDED) {
                    d_start = a.first_off + p * a.stride;
                    d_len = a.fixed_len;
                } else if constexpr (!PACKED) {
                    d_start = desc_off(a, p);
                    d_len = a.len[p];
                }
                d_seed = a.seed ? a.seed[p] : 0u;
            }
            if constexpr (PACKED) {  // lengths only, offsets from the wave's scan
                d_len = live ? a.len16[p] : 0u;
                d_start = packed_off(a, base, lane, d_len);
            }
        }
        d_start += a.base_adjust;
        const bool d_ok = d_start <= a.arena_bytes && d_len <= a.arena_bytes - d_start;
        if (!d_ok || d_len == 0) {  // nothing to read; chunk 0 of offset 0 is a safe address
            d_len = 0;
            d_start = 0;
        }

        uint32_t mine = 0;  // this lane's packet: LE sum (<= 128 KiB) or BE sum (longer)
        if constexpr (D > 1) {
            Pkt k[D];
            uint4 v[D][U];
#pragma unroll
            for (int r = 0; r < D; ++r) {
                k[r] = fetch_pkt<G>(d_start, d_len, r * P + grp);
                issue_pass<G, U, NT, BUF>(a, rsrc, k[r], sub, v[r]);
            }
#pragma unroll
            for (int r = 0; r < D; ++r) {  // consumed oldest first: each wait leaves the later rounds in flight
                const uint32_t words = group_allreduce<G>(packet_partial<G, U, NT, BUF>(a, rsrc, k[r], sub, v[r]));
                const uint32_t t = bcast_from<G>(words, (lane % P) * G);
                mine = (lane / P == static_cast<uint32_t>(r)) ? t : mine;
            }
        }
        Pkt cur = fetch_pkt<G>(d_start, d_len, grp);
        uint4 v[U];
        if constexpr (D == 1)
            issue_pass<G, U, NT, BUF>(a, rsrc, cur, sub, v);
        for (uint32_t r = 0; r < (D == 1 ? G : 0); ++r) {
            // Prefetch the next round's first pass.  Unconditional on purpose: on the
            // last round it loads an empty packet (no memory traffic on the buffer
            // path), so every path through the loop has the same loads outstanding
            // and the compiler waits only for the pass it consumes (vmcnt(U)).
            const bool has_next = r + 1 < G;
            Pkt nxt = fetch_pkt<G>(d_start, d_len, (has_next ? r + 1 : r) * P + grp);
            nxt.nch = has_next ? nxt.nch : 0u;
            uint4 w[U];
            issue_pass<G, U, NT, BUF>(a, rsrc, nxt, sub, w);
            const uint32_t words = group_allreduce<G>(packet_partial<G, U, NT, BUF>(a, rsrc, cur, sub, v));
            if constexpr (G == 64) {
                mine = (lane == r) ? words : mine;
            } else {
                const uint32_t t = bcast_from<G>(words, (lane % P) * G);  // group (lane % P)'s sum
                mine = (lane / P == r) ? t : mine;
            }
            cur = nxt;
#pragma unroll
            for (int u = 0; u < U; ++u)
                v[u] = w[u];
        }
        const uint16_t acc = finalize(mine, d_start, d_len, d_seed, d_ok, a.flags);
        // 64 consecutive u16: one 128-byte store (nontemporal stores measured 12.88 -> 13.21 us on
        // c2, r03; the ordinary policy stays)
        if (live)
            a.out[p] = static_cast<uint16_t>(acc);
        if (a.bad) {
            const uint64_t rejected = __ballot(live && !d_ok);
            if (rejected && lane == 0)
                atomicAdd(a.bad, static_cast<uint32_t>(__popcll(rejected)));
        }
    }
}

// ---------------------------------------------------------------------------
// v3: "mixed" kernel — the rounds kernel for batches whose packet sizes vary
// (IMIX).  A wavefront still owns 64 consecutive packets, but first SORTS them
// by size class inside the wave (ballot + mbcnt ranks, one ds_permute per
// descriptor word), then runs each class with its own lanes-per-packet shape,
// so a 40 B packet never holds 16 lanes idle while a 1500 B packet finishes.
// Results return to the owner lane (its class, round and group are known from
// its rank) and leave in one 128-byte store, as in v2.
// ---------------------------------------------------------------------------
struct ClassRun {
    uint32_t off;   // first sorted position of the class (wave-uniform)
    uint32_t cnt;   // packets in the class (wave-uniform)
};

// Size classes (16-byte chunks a packet spans) and the shape each class runs with.
// (A/B builds override these: -DRNS_CLASS_MAX=4,16,32,64,128 -DRNS_CLASS_LOG2G=2,2,3,4,5,6
//  -DRNS_CLASS_U=1,4,4,4,4,4 — the class count follows RNS_CLASS_MAX, at most 6)
#ifndef RNS_CLASS_MAX
#define RNS_CLASS_MAX 4, 16, 64, 128
#endif
#ifndef RNS_CLASS_LOG2G
#define RNS_CLASS_LOG2G 2, 2, 4, 5, 6
#endif
#ifndef RNS_CLASS_U
#define RNS_CLASS_U 1, 4, 4, 4, 4
#endif
constexpr uint32_t kClassMaxList[] = {RNS_CLASS_MAX};                 // above the last: jumbo
constexpr uint32_t kNumClasses = sizeof(kClassMaxList) / sizeof(kClassMaxList[0]) + 1;
static_assert(kNumClasses <= 6, "at most 6 size classes");
inline constexpr const uint32_t (&kClassMax)[kNumClasses - 1] = kClassMaxList;
constexpr uint32_t kClassLog2G[kNumClasses] = {RNS_CLASS_LOG2G};   // lanes per packet 4, 4, 16, 32, 64
constexpr uint32_t kClassU[kNumClasses] = {RNS_CLASS_U};           // chunks in flight per lane
constexpr int umax_of(int i = 0, int m = 1)
{
    return i == static_cast<int>(kNumClasses) ? m : umax_of(i + 1, m > static_cast<int>(kClassU[i]) ? m : static_cast<int>(kClassU[i]));
}
constexpr int kUMax = umax_of();  // chunk slots of the widest class

// Round 0 of class n (wave-uniform; kNumClasses = none), issued with the class's
// runtime shape into the shared buffer: the last round of the previous class
// calls this, so a class starts with its first pass already in flight.
template <bool NT, bool BUF, int MODE>
__device__ __forceinline__ Pkt prefetch_class(const CsumArgs &a, __amdgpu_buffer_rsrc_t rsrc, uint32_t n,
                                              const ClassRun (&cr)[kNumClasses], uint64_t s_start, uint32_t s_len,
                                              uint32_t s_aux, uint32_t lane, uint4 (&w)[kUMax])
{
    uint32_t lg = 6, U = 0, off = 0, cnt = 0;
#pragma unroll
    for (uint32_t c = 0; c < kNumClasses; ++c)
        if (n == c) {
            lg = kClassLog2G[c];
            U = kClassU[c];
            off = cr[c].off;
            cnt = cr[c].cnt;
        }
    const uint32_t G = 1u << lg;
    const uint32_t sub = lane & (G - 1);
    const uint32_t grp = lane >> lg;
    const bool valid = grp < cnt;
    const int src = static_cast<int>(off + (valid ? grp : 0u));
    const uint32_t lo = static_cast<uint32_t>(__shfl(static_cast<int>(static_cast<uint32_t>(s_start)), src, 64));
    const uint32_t hi = static_cast<uint32_t>(__shfl(static_cast<int>(static_cast<uint32_t>(s_start >> 32)), src, 64));
    const uint32_t L = static_cast<uint32_t>(__shfl(static_cast<int>(s_len), src, 64));
    const uint32_t x = MODE == kStashField ? static_cast<uint32_t>(__shfl(static_cast<int>(s_aux), src, 64)) : 0xFFFFFFFFu;
    Pkt k = make_pkt((static_cast<uint64_t>(hi) << 32) | lo, L);
    set_stash<MODE>(k, static_cast<uint32_t>(src), x, arena_parity(a));
    k.nch = valid ? k.nch : 0u;
    const uint64_t first = k.start - static_cast<uint64_t>(k.s);
#pragma unroll
    for (int u = 0; u < kUMax; ++u) {
        const uint32_t c = sub + u * G;
        const bool in = static_cast<uint32_t>(u) < U && c < k.nch;
        if constexpr (BUF) {
            const uint32_t o = in ? static_cast<uint32_t>(first + (static_cast<uint64_t>(c) << 4)) : kOobOffset;
            const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o, 0, NT ? kNtAux : 0);
            w[u] = make_uint4(x.x, x.y, x.z, x.w);
        } else {
            const uint4 x = load_chunk<NT>(a.arena + first + (in ? (static_cast<uint64_t>(c) << 4) : 0));
            w[u] = in ? x : make_uint4(0, 0, 0, 0);
        }
    }
    return k;
}

// Transmit fill (kStashField): where the field's bytes sit in the stashed block, their
// word contribution (they count as zero, buf.rs:286-288), and the largest aligned
// block around the field that lies inside the packet (rewritten whole: no partial-
// sector write).  sb = the packet's stash; the block starts at stash chunk 0.
struct FillSite {
    uint64_t blk;      // offset (from a.arena) of the stashed block around the field
    uint32_t f_rel;    // the field's first byte in that block (0 .. kFieldBlock-1)
    uint32_t w_size;   // bytes of the largest aligned block inside the packet (0: none)
    uint32_t contrib;  // the field's two bytes as the packet's word sum holds them
};

__device__ __forceinline__ FillSite fill_site(const CsumArgs &a, uint64_t d_start, uint32_t d_len, uint32_t d_field,
                                              bool big, const uint8_t *sb, bool ok)
{
    FillSite f;
    const uint32_t s = static_cast<uint32_t>(d_start & 15);
    const uint32_t fpos = s + d_field;  // from chunk 0's first byte
    const int lo = field_block_lo(fpos >> 4, static_cast<uint32_t>(d_start >> 4), arena_parity(a));
    f.f_rel = fpos - 16u * static_cast<uint32_t>(lo);
    f.blk = d_start - s + static_cast<uint64_t>(16 * static_cast<int64_t>(lo));
    const uint32_t b0 = ok ? sb[f.f_rel] : 0u, b1 = ok ? sb[f.f_rel + 1] : 0u;
    // LE words pair aligned bytes; the exact BE path pairs from the packet start
    const bool hi_first = big ? !(d_field & 1) : (fpos & 1);
    f.contrib = hi_first ? (b0 << 8) + b1 : b0 + (b1 << 8);
    f.w_size = 0;
#pragma unroll
    for (uint32_t bs = 32; bs <= static_cast<uint32_t>(kFieldBlock); bs *= 2) {
        const uint64_t b = f.blk + (f.f_rel & ~(bs - 1));  // the bs-byte block holding the field
        const bool in = lo >= 0 && b >= d_start && b + bs <= d_start + d_len && (f.f_rel & (bs - 1)) != bs - 1;
        f.w_size = in ? bs : f.w_size;
    }
    return f;
}

// A transmit block store: the ordinary cache policy (nontemporal stores were 11-25 % slower:
// the scattered writes gain from being combined in the caches, profiles/archive/r02/r02_fill_ntstore_ab.json).
__device__ __forceinline__ void store_block(uint4 *p, uint4 v) { *p = v; }

// set_be16(&mut header[f..f+2], checksum): rewrite the block from the stash (stp =
// the packet's stash chunks) with the field patched in, or store the two bytes.
__device__ __forceinline__ void fill_store(const CsumArgs &a, const FillSite &f, uint64_t d_start, uint32_t d_field,
                                           uint16_t res, const uint4 *stp)
{
    uint8_t *arena_w = const_cast<uint8_t *>(a.arena);
    const uint32_t be = (res >> 8) | ((res & 0xffu) << 8);
    if (f.w_size) {
        // The whole block belongs to this packet (packets never overlap) and its
        // bytes are in the stash: rewrite it entirely, since a full-sector write
        // needs no read-modify-write at the memory side.
        const uint32_t c_lo = (f.f_rel & ~(f.w_size - 1)) >> 4, c_hi = c_lo + (f.w_size >> 4);
#pragma unroll
        for (uint32_t i = 0; i < static_cast<uint32_t>(kFieldChunks); ++i) {
            if (i >= c_lo && i < c_hi) {
                const uint4 c = stp[i];
                uint32_t w[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
                for (uint32_t k = 0; k < 2; ++k) {  // bytes f_rel and f_rel+1
                    const uint32_t bpos = f.f_rel + k - 16 * i, sh = (bpos & 3) * 8;
                    const uint32_t byte = (be >> (8 * k)) & 0xffu;
#pragma unroll
                    for (uint32_t d = 0; d < 4; ++d)
                        if (bpos < 16 && d == (bpos >> 2))
                            w[d] = (w[d] & ~(0xffu << sh)) | (byte << sh);
                }
                store_block(reinterpret_cast<uint4 *>(arena_w + f.blk + 16 * i), make_uint4(w[0], w[1], w[2], w[3]));
            }
        }
    } else {
        uint8_t *q = arena_w + d_start + d_field;
        q[0] = static_cast<uint8_t>(res >> 8);
        q[1] = static_cast<uint8_t>(res);
    }
}

// All rounds of class C.  On entry (cur, v) hold round 0's prefetched first pass;
// on exit they hold the first pass of class `next` (the next non-empty class).
template <uint32_t C, bool NT, bool BUF, int MODE>
__device__ __forceinline__ void run_class(const CsumArgs &a, __amdgpu_buffer_rsrc_t rsrc,
                                          const ClassRun (&cr)[kNumClasses], uint32_t next, uint64_t s_start,
                                          uint32_t s_len, uint32_t s_aux, bool in_class, uint32_t rank,
                                          uint32_t lane, Pkt &cur, uint4 (&v)[kUMax], uint32_t &mine, uint4 *st)
{
    constexpr int G = 1 << kClassLog2G[C];
    constexpr int U = static_cast<int>(kClassU[C]);
    constexpr uint32_t P = 64 / G;
    const uint32_t sub = lane & (G - 1);
    const uint32_t grp = lane / G;
    const uint32_t rounds = (cr[C].cnt + P - 1) / P;
    if (rounds == 0)
        return;  // (cur, v) already hold the next class's prefetch
    auto fetch = [&](uint32_t r) {  // group `grp` of round r: sorted position off + r*P + grp
        const uint32_t i = r * P + grp;
        Pkt k = fetch_pkt<G, MODE>(s_start, s_len, cr[C].off + (i < cr[C].cnt ? i : 0), s_aux, arena_parity(a));
        k.nch = (i < cr[C].cnt) ? k.nch : 0u;
        return k;
    };
    auto finish = [&](uint32_t r) {  // consume round r from (cur, v), route each sum to its owner lane
        const uint32_t words = group_allreduce<G>(packet_partial<G, U, NT, BUF, kUMax, MODE>(a, rsrc, cur, sub, v, st));
        if constexpr (G == 64) {
            mine = (in_class && rank == r) ? words : mine;  // wave-uniform sum
        } else {
            const int src = static_cast<int>((rank % P) * G);
            const uint32_t t = static_cast<uint32_t>(__shfl(static_cast<int>(words), src, 64));
            mine = (in_class && rank / P == r) ? t : mine;
        }
    };
    for (uint32_t r = 0; r + 1 < rounds; ++r) {
        const Pkt nxt = fetch(r + 1);
        uint4 w[kUMax];
        issue_pass<G, U, NT, BUF, kUMax>(a, rsrc, nxt, sub, w);  // in-class prefetch (vmcnt stays exact)
        finish(r);
        cur = nxt;
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = w[u];
    }
    uint4 w[kUMax];
    const Pkt nxt = prefetch_class<NT, BUF, MODE>(a, rsrc, next, cr, s_start, s_len, s_aux, lane, w);
    finish(rounds - 1);
    cur = nxt;
#pragma unroll
    for (int u = 0; u < kUMax; ++u)
        v[u] = w[u];
}

// The tiny class (<= 4 chunks: IMIX's 40-byte packets, TCP ACKs) in rounds of 64
// packets instead of 16: a group of 4 lanes takes FOUR packets per round, one per
// chunk slot (slot q of group g = the class's packet r*64 + q*16 + g; lane `sub`
// loads chunk `sub` of each), so the class's whole share of a wave batch is one
// memory round (IMIX: ~37 of 64 packets; G4/U1 took 3).  Each slot is reduced in
// its group; lane 4g + q keeps slot q's sum, and each owner lane pulls its packet's
// with one shuffle.  Issues its own round 0 (it is always the first class) and, like
// run_class, leaves the next class's first pass in flight in (cur, v).
constexpr uint32_t kTinyQ = 4;
static_assert(kClassLog2G[0] == 2 && kClassMax[0] <= 4, "tiny class shape");

template <bool NT, bool BUF, int MODE>
__device__ __forceinline__ void run_tiny(const CsumArgs &a, __amdgpu_buffer_rsrc_t rsrc,
                                         const ClassRun (&cr)[kNumClasses], uint32_t next, uint64_t s_start,
                                         uint32_t s_len, uint32_t s_aux, bool in_class, uint32_t rank, uint32_t lane,
                                         Pkt &cur, uint4 (&v)[kUMax], uint32_t &mine, uint4 *st)
{
    // A class pass covers 64 descriptors, so the class is ONE round (cnt <= 64).
    constexpr int G = 4, Q = 4;
    const uint32_t sub = lane & (G - 1);
    const uint32_t grp = lane / G;
    const uint32_t cnt = cr[0].cnt;
    // per slot q: the bytes [lo, hi) of this lane's chunk that lie inside the packet,
    // byte q of bnd = lo | (hi - 1) << 4 (one VGPR for all four); the stash modes also
    // keep the packet (its stash slots)
    uint32_t bnd = 0;
    Pkt k[MODE != kStashNone ? Q : 1];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const uint32_t i = q * 16 + grp;
        Pkt kq = fetch_pkt<G, MODE>(s_start, s_len, cr[0].off + (i < cnt ? i : 0), s_aux, arena_parity(a));
        kq.nch = (i < cnt) ? kq.nch : 0u;
        uint4 one[1];
        issue_pass<G, 1, NT, BUF, 1>(a, rsrc, kq, sub, one);
        v[q] = one[0];
        const uint32_t lo = sub == 0 ? static_cast<uint32_t>(kq.s) : 0u;
        const uint32_t hi = sub + 1 == kq.nch ? static_cast<uint32_t>(kq.e) : 16u;
        const uint32_t b = sub < kq.nch ? (lo | ((hi - 1) << 4)) : 0xF0u;  // absent chunks already read as zeros
        bnd |= b << (8 * q);
        if constexpr (MODE != kStashNone)
            k[q] = kq;
    }
    uint4 w[kUMax];
    cur = prefetch_class<NT, BUF, MODE>(a, rsrc, next, cr, s_start, s_len, s_aux, lane, w);  // next class in flight
    uint32_t sel = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        uint4 x = v[q];
        const int lo = static_cast<int>((bnd >> (8 * q)) & 15u), hi = static_cast<int>((bnd >> (8 * q + 4)) & 15u) + 1;
        if (lo != 0 || hi != 16) {
            x.x = keep_bytes(x.x, lo, hi, 0);
            x.y = keep_bytes(x.y, lo, hi, 4);
            x.z = keep_bytes(x.z, lo, hi, 8);
            x.w = keep_bytes(x.w, lo, hi, 12);
        }
        if constexpr (MODE != kStashNone) {
            const uint4 one[1] = {x};
            stash_chunks<MODE, G, 1, 1>(k[q], sub, one, st);
        }
        uint32_t s = __builtin_amdgcn_sad_u16(x.x, 0, 0u);  // <= 64 bytes: never the BE path
        s = __builtin_amdgcn_sad_u16(x.y, 0, s);
        s = __builtin_amdgcn_sad_u16(x.z, 0, s);
        s = __builtin_amdgcn_sad_u16(x.w, 0, s);
        const uint32_t words = group_allreduce<G>(s);
        sel = (sub == static_cast<uint32_t>(q)) ? words : sel;
    }
    const int src = static_cast<int>(((rank & 15u) << 2) | ((rank >> 4) & 3u));  // lane 4g + q of the owner's slot
    const uint32_t t = static_cast<uint32_t>(__shfl(static_cast<int>(sel), src, 64));
    mine = in_class ? t : mine;
#pragma unroll
    for (int u = 0; u < kUMax; ++u)
        v[u] = w[u];
}

// The size-class data pass over one wave batch: lane l holds one descriptor
// (d_start, d_len; d_aux = the field offset for kStashField; d_len 0 = nothing to
// read) and receives that packet's word sum — the LE sum for packets <= 128 KiB,
// the exact BE sum mod 2^32 above.  The wave sorts its 64 descriptors by size class
// (ballot + mbcnt ranks, ds_permute), runs every class's rounds with its own shape,
// and routes each sum back to its owner lane.  pos = the lane's sorted position
// (its stash slot).
template <bool NT, bool BUF, int MODE, bool TINY = (kTinyQ > 1)>
__device__ __forceinline__ uint32_t wave_class_pass(const CsumArgs &a, __amdgpu_buffer_rsrc_t rsrc, uint64_t d_start,
                                                    uint32_t d_len, uint32_t d_aux, uint32_t lane, uint4 *st,
                                                    uint32_t &pos)
{
    // size class of this lane's packet (kNumClasses: empty, no rounds at all — e.g. the
    // fragments the chain kernel merged into their run's first); ranks within the
    // class; sorted position (empty packets last)
    const uint32_t nch = d_len ? static_cast<uint32_t>(((d_start & 15) + d_len + 15) >> 4) : 0u;
    uint32_t cls = kNumClasses - 1;
#pragma unroll
    for (int c = kNumClasses - 2; c >= 0; --c)
        cls = (nch <= kClassMax[c]) ? static_cast<uint32_t>(c) : cls;
    cls = nch ? cls : kNumClasses;
    uint32_t rank = 0, off = 0;
    pos = 0;
    ClassRun cr[kNumClasses];
#pragma unroll
    for (uint32_t c = 0; c < kNumClasses; ++c) {
        const uint64_t m = __ballot(cls == c);
        const uint32_t below = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
        if (cls == c) {
            rank = below;
            pos = off + below;
        }
        cr[c] = ClassRun{off, static_cast<uint32_t>(__popcll(m))};
        off += cr[c].cnt;
    }
    {
        const uint64_t m = __ballot(cls == kNumClasses);
        if (cls == kNumClasses)
            pos = off + __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                  __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
    }
    // next non-empty class after each class (wave-uniform); kNumClasses = none
    uint32_t next[kNumClasses + 1];
    next[kNumClasses] = kNumClasses;
#pragma unroll
    for (int c = kNumClasses - 1; c >= 0; --c)
        next[c] = cr[c].cnt ? static_cast<uint32_t>(c) : next[c + 1];
    // sort the descriptors by class: lane `pos` receives this lane's packet
    const int addr = static_cast<int>(pos * 4);
    const uint32_t s_lo = static_cast<uint32_t>(
        __builtin_amdgcn_ds_permute(addr, static_cast<int>(static_cast<uint32_t>(d_start))));
    const uint32_t s_hi = static_cast<uint32_t>(
        __builtin_amdgcn_ds_permute(addr, static_cast<int>(static_cast<uint32_t>(d_start >> 32))));
    const uint32_t s_len = static_cast<uint32_t>(__builtin_amdgcn_ds_permute(addr, static_cast<int>(d_len)));
    const uint64_t s_start = (static_cast<uint64_t>(s_hi) << 32) | s_lo;
    const uint32_t s_aux = MODE == kStashField
        ? static_cast<uint32_t>(__builtin_amdgcn_ds_permute(addr, static_cast<int>(d_aux))) : 0u;

    uint32_t mine = 0;
    uint4 v[kUMax];
    Pkt cur;
#define RNS_RUN_CLASS(C)                                                                                  \
    run_class<C, NT, BUF, MODE>(a, rsrc, cr, next[C + 1], s_start, s_len, s_aux, cls == C, rank, lane, \
                                cur, v, mine, st)
    if (TINY && cr[0].cnt) {  // the tiny class issues its own first round
        run_tiny<NT, BUF, MODE>(a, rsrc, cr, next[1], s_start, s_len, s_aux, cls == 0, rank, lane, cur, v, mine, st);
    } else {
        cur = prefetch_class<NT, BUF, MODE>(a, rsrc, next[0], cr, s_start, s_len, s_aux, lane, v);
        if (!TINY)
            RNS_RUN_CLASS(0);
    }
    RNS_RUN_CLASS(1);
    RNS_RUN_CLASS(2);
    RNS_RUN_CLASS(3);
    RNS_RUN_CLASS(4);
    if constexpr (kNumClasses > 5)
        RNS_RUN_CLASS(5 % kNumClasses);
#undef RNS_RUN_CLASS
    return mine;
}

// ---------------------------------------------------------------------------
// Receive verify (§8f row 1), fused into the mixed kernel (kStashHead): the checks
// ip_input_v4 (ip.rs:65-92), ip_input_v6 (ip.rs:114-121), ip_input_common
// (ip.rs:123-131), tcp::validate_checksum (tcp.rs:838-850), icmp_input_v4
// (icmp.rs:44-50) and icmp_input_v6 (icmp.rs:62-75) apply to a received datagram.
// A wave takes 64 datagrams, one per owner lane.  The data pass is the plain one
// over the WHOLE datagram (its LE word sum T); the lanes that load a datagram's
// first 5 chunks also copy them to LDS.  The owner lane then parses the header from
// LDS and sums the header bytes H itself (<= 60 bytes), so the L4 segment's sum is
// T - H: the word sum is linear in the bytes, and the header length (IHL*4 or 40) is
// even, so the L4 bytes pair exactly as the reference's separate call over the
// trimmed packet pairs them.  The L4 seed is the pseudo-header sum with dest = the
// LOCAL address, as the reference passes netif::get_ipaddr().
// ---------------------------------------------------------------------------
// Receive verify's owner-lane finish takes a short path for 16-byte-aligned datagrams
// (header dwords as stashed; a 20-byte IPv4 header summed without byte masks).

enum : uint32_t {
    kMetaV4 = 1, kMetaV6 = 2, kMetaFrag = 4, kMetaMalformed = 8,
    kMetaL4Checked = 16, kMetaUnchecked = 32, kMetaUnknown = 64,
};

__device__ __forceinline__ uint32_t fold16(uint32_t x)
{
    while (x > 0xffff)
        x = (x & 0xffff) + (x >> 16);
    return x;
}

struct RxParse {
    uint32_t meta;  // kMeta* bits
    uint32_t hdr;   // IP header bytes (IHL*4 or 40)
    uint32_t ph;    // L4 seed: pseudo-header sum (TCP, ICMPv6) or 0 (ICMPv4)
};

// The first 24 bytes of a datagram (every field rx_parse reads) as six dwords in
// datagram byte order, from the stashed chunks 0..2 (s = start & 15).
__device__ __forceinline__ void head_from_stash(const uint4 (&ch)[3], uint32_t s, uint32_t (&h)[6])
{
    const uint32_t w[12] = {ch[0].x, ch[0].y, ch[0].z, ch[0].w, ch[1].x, ch[1].y,
                            ch[1].z, ch[1].w, ch[2].x, ch[2].y, ch[2].z, ch[2].w};
    const uint32_t q = s >> 2, sh = s & 3;
    uint32_t d[7];
#pragma unroll
    for (int k = 0; k < 7; ++k)
        d[k] = q == 0 ? w[k] : q == 1 ? w[k + 1] : q == 2 ? w[k + 2] : w[k + 3];
#pragma unroll
    for (int k = 0; k < 6; ++k)
        h[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
}

// Word sums of bytes [lo, hi) of the stashed chunks (byte index from chunk 0's
// first byte; hi <= 80): LE words at aligned positions (v_sad_u16), or the exact
// big-endian words relative to a packet start of parity `odd` (256*hi + lo bytes).
template <int NCH>
__device__ __forceinline__ uint32_t stash_sum_le(const uint4 (&ch)[NCH], int lo, int hi)
{
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        acc = __builtin_amdgcn_sad_u16(keep_bytes(ch[c].x, lo - 16 * c, hi - 16 * c, 0), 0, acc);
        acc = __builtin_amdgcn_sad_u16(keep_bytes(ch[c].y, lo - 16 * c, hi - 16 * c, 4), 0, acc);
        acc = __builtin_amdgcn_sad_u16(keep_bytes(ch[c].z, lo - 16 * c, hi - 16 * c, 8), 0, acc);
        acc = __builtin_amdgcn_sad_u16(keep_bytes(ch[c].w, lo - 16 * c, hi - 16 * c, 12), 0, acc);
    }
    return acc;
}

template <int NCH>
__device__ __forceinline__ uint32_t stash_sum_be(const uint4 (&ch)[NCH], int lo, int hi, bool odd)
{
    uint4 m[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c)
        m[c] = make_uint4(keep_bytes(ch[c].x, lo - 16 * c, hi - 16 * c, 0),
                          keep_bytes(ch[c].y, lo - 16 * c, hi - 16 * c, 4),
                          keep_bytes(ch[c].z, lo - 16 * c, hi - 16 * c, 8),
                          keep_bytes(ch[c].w, lo - 16 * c, hi - 16 * c, 12));
    uint32_t hs = 0, ls = 0;
    sum_be<NCH, NCH>(m, odd ? 0x01000100u : 0x00010001u, hs, ls);
    return (hs << 8) + ls;
}

// h = the datagram's first 24 bytes (head_from_stash), L = its length (the buffer length,
// as the stack sees it).
__device__ __forceinline__ RxParse rx_parse(const uint32_t (&h)[6], uint32_t L, uint32_t local4_sum,
                                            uint32_t local6_sum)
{
    RxParse r{kMetaMalformed, 0u, 0u};
    if (L == 0)
        return r;
    auto p = [&](int i) -> uint32_t { return (h[i >> 2] >> (8 * (i & 3))) & 0xffu; };
    const uint32_t version = p(0) >> 4;                      // ip.rs:40
    uint32_t proto = 0, src_sum = 0;
    bool v4src = false;
    if (version == 4) {
        r.hdr = (p(0) & 0xf) * 4u;                           // ip.rs:71
        if (r.hdr == 0 || L < 16 || r.hdr > L)               // empty slice / header index / trim_head panic
            return r;
        r.meta = kMetaV4;
        if (((p(6) << 8 | p(7)) & 0x3fff) != 0)  // ip.rs:84-87
            r.meta |= kMetaFrag;
        proto = p(9);                                        // ip.rs:89
        src_sum = (p(12) << 8 | p(13)) + (p(14) << 8 | p(15));
        v4src = true;
    } else if (version == 6) {
        r.hdr = 40;
        if (L < 40)                                          // trim_head(IPV6_HEADER_LEN) would panic
            return r;
        r.meta = kMetaV6;
        proto = p(6);                                        // ip.rs:116
        for (int k = 8; k < 24; k += 2)                      // source address, ip.rs:117
            src_sum += p(k) << 8 | p(k + 1);
    } else {
        return r;                                            // "IP: Invalid version field"
    }
    const uint32_t l4len = L - r.hdr;                        // packet.len() after trim_head
    if (proto == 6) {                                        // tcp.rs:838-850: dest = local address of src's family
        r.ph = v4src ? fold16(src_sum + local4_sum + 6 + (l4len & 0xffff))
                     : fold16(src_sum + local6_sum + (l4len >> 16) + (l4len & 0xffff) + 6);
        r.meta |= kMetaL4Checked;
    } else if (proto == 1) {                                 // icmp.rs:46: no pseudo header
        r.meta |= kMetaL4Checked;
    } else if (proto == 58) {                                // icmp.rs:63-68: dest = local IPv6
        if (v4src) {
            r.meta = kMetaMalformed;                         // V4 source in a V6 pseudo-header: copy_to panics
            return r;
        }
        r.ph = fold16(src_sum + local6_sum + (l4len >> 16) + (l4len & 0xffff) + 58);
        r.meta |= kMetaL4Checked;
    } else if (proto == 17) {
        r.meta |= kMetaUnchecked;                            // udp.rs:126-148 never verifies
    } else {
        r.meta |= kMetaUnknown;                              // ip.rs:129 "Unknown protocol"
    }
    return r;
}

// hdr_res / l4_res: complemented sums (0 = verifies).
__device__ __forceinline__ uint8_t rx_verdict(uint32_t m, uint32_t hdr_res, uint32_t l4_res)
{
    if (m & kMetaMalformed)
        return RNS_RX_MALFORMED;
    uint32_t st = 0;
    if ((m & kMetaV6) || hdr_res == 0)                       // compute_checksum(header) == 0 (ip.rs:76-80)
        st |= RNS_RX_IP_OK;
    if (m & kMetaFrag)
        st |= RNS_RX_FRAGMENT;
    if ((m & kMetaL4Checked) && l4_res == 0)                 // buffer sum ^ 0xffff == 0
        st |= RNS_RX_L4_OK;
    if (m & kMetaUnchecked)
        st |= RNS_RX_L4_UNCHECKED;
    if (m & kMetaUnknown)
        st |= RNS_RX_UNKNOWN_PROTO;
    if ((st & RNS_RX_IP_OK) && !(st & RNS_RX_FRAGMENT) && (st & (RNS_RX_L4_OK | RNS_RX_L4_UNCHECKED)))
        st |= RNS_RX_ACCEPT;
    return static_cast<uint8_t>(st);
}

// Receive verify, owner-lane finish for one datagram: mine = the whole datagram's word
// sum T (LE for <= 128 KiB, exact BE mod 2^32 above), own = its stashed chunks 0..NS-1
// from the 16-byte-aligned chunk holding its first byte (bytes outside the datagram read
// as zero; a chunk past NS reads as zero), s = start & 15.  Header H from the stash (seed
// 0, <= 60 bytes); L4 = T - H, seeded with the pseudo-header sum.  Both parts start at
// the datagram's parity (the header length is even).  Returns the RNS_RX_* status;
// l4_res = the complemented L4 sum.
template <int NS>
__device__ __forceinline__ uint8_t rx_finish(const CsumArgs &a, const uint4 *own, uint32_t mine, uint32_t s,
                                             uint32_t d_len, bool odd, bool big, bool present, uint32_t &l4_res)
{
    uint4 ch[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        ch[i] = own[i];
    uint32_t head[6];
    if (s == 0) {  // 16-byte-aligned datagram: the dwords as they are
        const uint32_t w6[6] = {ch[0].x, ch[0].y, ch[0].z, ch[0].w, ch[1].x, ch[1].y};
#pragma unroll
        for (int k = 0; k < 6; ++k)
            head[k] = w6[k];
    } else {
        head_from_stash(ch, s, head);
    }
    const RxParse rp = present ? rx_parse(head, d_len, a.local4_sum, a.local6_sum) : RxParse{kMetaMalformed, 0u, 0u};
    uint32_t hdr_res = 0;
    l4_res = 0;
    if (!(rp.meta & kMetaMalformed)) {
        const int hlo = static_cast<int>(s), hhi = hlo + static_cast<int>(rp.hdr);  // <= 15 + 60
        uint32_t H;
        if (hlo == 0 && hhi == 20) {  // aligned IPv4 header, no options: 5 dwords
            H = __builtin_amdgcn_sad_u16(ch[0].x, 0, 0u);
            H = __builtin_amdgcn_sad_u16(ch[0].y, 0, H);
            H = __builtin_amdgcn_sad_u16(ch[0].z, 0, H);
            H = __builtin_amdgcn_sad_u16(ch[0].w, 0, H);
            H = __builtin_amdgcn_sad_u16(ch[1].x, 0, H);
        } else {
            H = stash_sum_le(ch, hlo, hhi);
        }
        uint4 tail[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
        if (hhi > 48) {  // IPv6 past offset 8, IPv4 with options: header bytes in chunks 3-4
            tail[0] = own[3];
            if constexpr (NS > 4)
                tail[1] = own[4];
            H += stash_sum_le(tail, hlo - 48, hhi - 48);
        }
        hdr_res = finalize_bits(H, odd, false, 0u, true, RNS_FLAG_COMPLEMENT);
        if (rp.meta & kMetaL4Checked) {
            uint32_t l4 = mine - H;
            if (big) {  // > 128 KiB (rare): the exact big-endian sums, mod 2^32
                const uint4 all[5] = {ch[0], ch[1], ch[2], tail[0], tail[1]};
                l4 = mine - stash_sum_be(all, hlo, hhi, odd);
            }
            l4_res = finalize_bits(l4, odd, big, rp.ph, true, RNS_FLAG_COMPLEMENT);
        }
    }
    return rx_verdict(rp.meta, hdr_res, l4_res);
}

// One packet's descriptor.  Loads are branch-free (an index past the batch re-reads
// its last packet and the result is discarded), so no wait is forced at a branch merge.
// With a buffer descriptor (arena < 4 GiB) the offset is held in 32 bits: one past
// 4 GiB becomes 0xFFFFFFFF, still outside the arena, so it is still rejected.
template <bool BUF>
struct Desc {
    typename std::conditional<BUF, uint32_t, uint64_t>::type off;
    uint32_t len, field;
};

template <bool STRIDED, bool FILL, bool BUF, bool PACKED = false>
__device__ __forceinline__ Desc<BUF> load_desc(const CsumArgs &a, uint64_t p)
{
    const bool live = p < a.n;
    const uint64_t q = live ? p : a.n - 1;
    uint64_t off;
    Desc<BUF> d;
    if constexpr (STRIDED) {
        off = a.first_off + q * a.stride;
        d.len = a.fixed_len;
    } else if constexpr (PACKED) {  // lengths only, offsets from the wave's scan
        d.len = live ? a.len16[q] : 0u;
        off = packed_off(a, p & ~63ull, static_cast<uint32_t>(p & 63), d.len);
    } else {
        off = desc_off(a, q);
        d.len = a.len[q];
    }
    if constexpr (BUF)
        d.off = off > 0xFFFFFFFFull ? 0xFFFFFFFFu : static_cast<uint32_t>(off);
    else
        d.off = off;
    d.field = FILL ? (a.field ? static_cast<uint32_t>(a.field[q]) : a.field_off) : 0xFFFFFFFFu;
    d.off = live ? d.off : 0;
    d.len = live ? d.len : 0u;
    return d;
}

// Workgroup size of the mixed kernel: one wave.  Receive verify and transmit fill hold
// an LDS stash per wave, and LDS is freed per WORKGROUP, so one-wave workgroups let a
// CU refill as soon as any wave finishes (IMIX verify 590 -> 559 us).  The plain batch
// has no LDS, but a new workgroup still waits for a slot for ALL its waves: one-wave
// workgroups took IMIX from 440-456 to 424-430 us per pipelined step (c3 equal;
// profiles/r02_block_ab.json).  A/B knob: -DRNS_MIXED_PLAIN_BLOCK=256.
#ifndef RNS_MIXED_PLAIN_BLOCK
#define RNS_MIXED_PLAIN_BLOCK 64
#endif
template <bool STASH>
constexpr int kMixedBlock = STASH ? 64 : RNS_MIXED_PLAIN_BLOCK;

// FILL (transmit in-place fill, tcp.rs:957-973 / udp.rs:158-171 / icmp.rs:87-112 /
// ip.rs:158-159): the checksum is that of the packet with its 2-byte field zeroed
// (alloc_header zero-fills it, buf.rs:286-288).  The data pass sums the whole packet;
// the owner lane subtracts the field's word contribution (its bytes from the stash),
// folds, and stores the (complemented) result into the field big-endian (set_be16,
// util.rs:132-135) after the whole wave has read its 64 packets.
// RX: receive verify (see above).
template <bool STRIDED, bool NT, bool BUF, bool FILL, bool RX = false, bool TX = false, bool PACKED = false>
#ifndef RNS_MIXED_OCC
#define RNS_MIXED_OCC 4
#endif
#ifndef RNS_STASH_OCC  // waves/SIMD bound of the stash modes (receive verify, transmit fill/finalize)
#define RNS_STASH_OCC 4
#endif
#ifndef RNS_FILL_OCC  // waves/SIMD bound of transmit fill / finalize: 3 (4 spilled 8-84 B/lane; equal
#define RNS_FILL_OCC 3      // time: c3 fill 346 / 348 us, IMIX 788 / 785, session r04b)
#endif
__global__ __launch_bounds__(kMixedBlock<FILL || RX || TX>, (BUF && !FILL && !RX && !TX) ? RNS_MIXED_OCC
                                                             : (FILL || TX)                 ? RNS_FILL_OCC
                                                                                            : RNS_STASH_OCC) void
csum_mixed_kernel(const CsumArgs a)
{
    static_assert(int(FILL) + int(RX) + int(TX) <= 1 && !(STRIDED && (RX || TX)), "one mode at a time");
    constexpr int kMode = RX ? kStashHead : FILL ? kStashField : TX ? kStashTx : kStashNone;
    constexpr int kNS = kStashChunks<kMode>;
    constexpr uint32_t kPer = 64;  // packets per wave batch
    // per wave: kNS chunks for each of its 64 packets, indexed by sorted position
    constexpr int BLK = kMixedBlock<FILL || RX || TX>;
    __shared__ uint4 stash_lds[kNS ? (BLK / 64) * kPer * kNS : 1];
    uint4 *const st = stash_lds + (threadIdx.x >> 6) * (kPer * kNS);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * BLK + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * BLK) >> 6;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.arena), static_cast<short>(0), static_cast<int>(BUF ? buf_records(a) : 0), 0x00020000);

    // (Loading the descriptors one wave batch ahead was measured slower: the extra
    // live registers spill at 4 waves/SIMD and the spill forces a wait on the loads.)
    const uint64_t wstep = static_cast<uint64_t>(nwaves) * kPer;

    // Packed form: the next wave batch's lengths (and block base) are loaded together
    // with this batch's seeds after the class pass — one memory latency between two
    // batches instead of two, and nothing extra is live during the class pass.
    constexpr bool kPf = PACKED;  // packed: the next wave batch's lengths loaded beside this batch's seeds
    uint32_t nx_len = 0;
    uint64_t nx_blk = 0;
    auto load_next = [&](uint64_t b) {  // branch-free: past the end re-reads the last packet
        const uint64_t q = b + lane < a.n ? b + lane : a.n - 1;
        nx_len = a.len16[q];
        nx_blk = a.blk_off[(b < a.n ? b : a.n - 1) >> 6];
    };
    if constexpr (kPf)
        load_next(static_cast<uint64_t>(wave) * kPer);

    for (uint64_t base = static_cast<uint64_t>(wave) * kPer; base < a.n; base += wstep) {
        const uint64_t p = base + lane;
        const bool live = p < a.n;
        Desc<BUF> cd;
        if constexpr (kPf) {
            cd.len = live ? nx_len : 0u;
            const uint64_t off = nx_blk + packed_scan(a, lane, cd.len);
            cd.off = BUF ? (off > 0xFFFFFFFFull ? 0xFFFFFFFFu : static_cast<uint32_t>(off)) : off;
            cd.off = live ? cd.off : 0;
            cd.field = 0xFFFFFFFFu;
        } else {
            cd = load_desc<STRIDED, FILL, BUF, PACKED>(a, p);
        }
        uint64_t d_start = cd.off + a.base_adjust;
        // the seed is first needed after the data pass: loaded here, its latency is hidden
        uint32_t d_len = cd.len;
        // (packed form: loaded after the class pass — held across it, the seed spilled to scratch)
        uint32_t d_seed = (!PACKED && a.seed && live) ? a.seed[p] : 0u;
        const uint32_t d_field = cd.field;  // FILL: the field offset
        bool d_ok = d_start <= a.arena_bytes && d_len <= a.arena_bytes - d_start;
        if constexpr (FILL) {
            d_ok = d_ok && d_len >= 2 && d_field <= d_len - 2;  // header[f..f+2] must exist
            // (stores happen after the wave read all 64 packets: a store between a
            // prefetch and its consumer would serialise the in-order vmcnt waits)
        }
        if (!d_ok || d_len == 0) {
            d_len = 0;
            d_start = 0;
        }
        const bool odd = d_start & 1, big = d_len > kNoWrapBytes;  // all finalize needs of (start, len)
        uint32_t pos;
        uint32_t mine = wave_class_pass<NT, BUF, kMode>(a, rsrc, d_start, d_len, d_field, lane, st, pos);

        if constexpr (TX) {
            // Transmit finalize: mine = the whole datagram's word sum.  From the stash
            // (chunks 0-5: >= 81 bytes past any start offset): parse the header, sum the
            // IPv4 header H and take the L4 segment as mine - H; both fields count as zero.
            const uint4 *own = st + pos * kNS;
            wave_lds_fence();  // the stash was written by other lanes of this wave
            const uint32_t s = static_cast<uint32_t>(d_start & 15);
            uint8_t status = RNS_TX_MALFORMED;
            uint32_t ipf = 0xFFFFFFFFu, l4f = 0xFFFFFFFFu;  // field offsets in the datagram (none)
            uint32_t ipc = 0, l4c = 0;
            if (live && d_len != 0) {
                const uint8_t *b = reinterpret_cast<const uint8_t *>(own) + s;  // datagram byte i = b[i], i < 96 - s
                const uint32_t version = b[0] >> 4;
                uint32_t hdr = 0, proto = 0, field = 0xFFFFFFFFu, seed = 0;
                bool ok = false;
                const uint32_t L = d_len;
                auto be16 = [&](uint32_t i) { return (static_cast<uint32_t>(b[i]) << 8) | b[i + 1]; };
                if (version == 4) {
                    hdr = (b[0] & 0xFu) * 4u;
                    ok = hdr >= 20 && hdr <= L;
                    proto = b[9];
                } else if (version == 6) {
                    hdr = 40;
                    ok = L >= 40;
                    proto = b[6];
                }
                if (ok) {
                    const uint32_t seg = L - hdr;
                    uint32_t addr = 0;  // BE word sum of source + destination (tcp.rs:958-966: local = header source)
                    if (version == 4) {
                        for (uint32_t i = 12; i < 20; i += 2)
                            addr += be16(i);
                    } else {
                        for (uint32_t i = 8; i < 40; i += 2)
                            addr += be16(i);
                    }
                    const uint32_t l16 = seg & 0xFFFFu;  // packet.len() as u16 (tcp.rs:942, udp.rs:152)
                    if (proto == 6 || proto == 17) {
                        field = proto == 6 ? 16u : 6u;
                        seed = fold16(addr + proto + l16);  // v4: len16; v6: len32 whose high half is 0
                    } else if (proto == 1 && version == 4) {
                        field = 2;  // icmp_output_v4: no pseudo-header
                    } else if (proto == 58 && version == 6) {
                        field = 2;  // icmp_output_v6: full length, protocol 58
                        seed = fold16(addr + 58 + (seg >> 16) + (seg & 0xFFFFu));
                    }
                    status = 0;
                    // header sum (<= 60 bytes, chunks 0-4) and the fields' own words
                    uint4 ch[5];
#pragma unroll
                    for (int i = 0; i < 5; ++i)
                        ch[i] = own[i];
                    const int hlo = static_cast<int>(s), hhi = hlo + static_cast<int>(hdr);
                    const uint32_t H = stash_sum_le(ch, hlo, hhi);
                    // a field's two bytes, as the LE words (aligned pairing) or BE words (packet pairing) hold them
                    auto le_contrib = [&](uint32_t f) {
                        const uint32_t b0 = b[f], b1 = b[f + 1];
                        return ((s + f) & 1) ? (b0 << 8) + b1 : b0 + (b1 << 8);
                    };
                    if (version == 4) {  // ip_output_v4 (ip.rs:158-159): over the header, [10..12] as zero
                        ipf = 10;
                        ipc = finalize_bits(H - le_contrib(10), odd, false, 0u, true, RNS_FLAG_COMPLEMENT);
                        status |= RNS_TX_IP_FILLED;
                    }
                    if (field != 0xFFFFFFFFu && seg >= field + 2) {
                        l4f = hdr + field;
                        uint32_t l4 = mine - H - le_contrib(l4f);
                        if (big) {  // > 128 KiB: the exact big-endian sums mod 2^32
                            const uint32_t b0 = b[l4f], b1 = b[l4f + 1];
                            l4 = mine - stash_sum_be(ch, hlo, hhi, odd) - ((b0 << 8) + b1);  // l4f even: a BE word
                        }
                        l4c = finalize_bits(l4, odd, big, seed, true, RNS_FLAG_COMPLEMENT);
                        status |= RNS_TX_L4_FILLED;
                    }
                }
            }
            if (live && a.status)
                a.status[p] = status;
            // store the fields: patch the stash, then rewrite each field's 32-byte memory
            // sector from it when the sector lies inside the datagram and the stash, else
            // store the two bytes (set_be16, util.rs:132-135)
            uint8_t *own_b = reinterpret_cast<uint8_t *>(st + pos * kNS);
            uint8_t *arena_w = const_cast<uint8_t *>(a.arena);
            const uint32_t fld[2] = {ipf, l4f}, val[2] = {ipc, l4c};
#pragma unroll
            for (int k = 0; k < 2; ++k)
                if (fld[k] != 0xFFFFFFFFu) {
                    own_b[s + fld[k]] = static_cast<uint8_t>(val[k] >> 8);
                    own_b[s + fld[k] + 1] = static_cast<uint8_t>(val[k]);
                }
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (fld[k] == 0xFFFFFFFFu)
                    continue;
                const uint32_t fpos = s + fld[k];  // from chunk 0's first byte
                const int lo = static_cast<int>(fpos >> 4) -
                               static_cast<int>((arena_parity(a) + static_cast<uint32_t>(d_start >> 4) + (fpos >> 4)) & 1u);
                const uint64_t sec = d_start - s + static_cast<uint64_t>(16 * static_cast<int64_t>(lo));
                const bool whole = lo >= 0 && lo + 2 <= kNS && sec >= d_start && sec + 32 <= d_start + d_len &&
                                   (fpos - 16u * static_cast<uint32_t>(lo)) != 31u;
                if (whole) {
                    uint4 *sp = reinterpret_cast<uint4 *>(arena_w + sec);
                    store_block(sp, own[lo]);
                    store_block(sp + 1, own[lo + 1]);
                } else {
                    arena_w[d_start + fld[k]] = static_cast<uint8_t>(val[k] >> 8);
                    arena_w[d_start + fld[k] + 1] = static_cast<uint8_t>(val[k]);
                }
            }
            continue;
        }
        if constexpr (RX) {
            // mine = the whole datagram's word sum T (see rx_finish)
            wave_lds_fence();  // the stash was written by other lanes of this wave
            uint32_t l4_res = 0;
            const uint8_t stv = rx_finish<kNS>(a, st + pos * kNS, mine, static_cast<uint32_t>(d_start & 15), d_len, odd,
                                               big, live && d_len != 0, l4_res);
            if (live) {
                a.status[p] = stv;
                if (a.l4_out)
                    a.l4_out[p] = static_cast<uint16_t>(l4_res);
            }
            continue;
        }
        FillSite fs{};
        if constexpr (FILL) {  // take the field's bytes out of the sum: it counts as zero
            wave_lds_fence();  // the stash was written by other lanes of this wave
            fs = fill_site(a, d_start, d_len, d_field, big, reinterpret_cast<const uint8_t *>(st + pos * kNS), d_ok);
            mine -= fs.contrib;
        }
        if constexpr (PACKED) {
            d_seed = (a.seed && live) ? a.seed[p] : 0u;
            if constexpr (kPf)
                load_next(base + wstep);  // in flight while this batch finishes and stores
        }
        const uint16_t res = finalize_bits(mine, odd, big, d_seed, d_ok, a.flags);
        if (live && a.out) {
            // nontemporal result stores in the plain class kernel (c3 232.4 -> 229.5 us per step, r03l)
            if constexpr (!FILL && !RX && !TX)
                __builtin_nontemporal_store(res, a.out + p);
            else
                a.out[p] = res;  // 64 consecutive u16: one 128-byte store
        }
        if constexpr (FILL) {
            if (live && d_ok)  // set_be16(&mut header[f..f+2], checksum), after the wave read its 64 packets
                fill_store(a, fs, d_start, d_field, res, st + pos * kNS);
        }
        if (a.bad) {
            const uint64_t rejected = __ballot(live && !d_ok);
            if (rejected && lane == 0)
                atomicAdd(a.bad, static_cast<uint32_t>(__popcll(rejected)));
        }
    }
}

// ---------------------------------------------------------------------------
// Fragment chains (util.rs:112-119 compute_buffer_ones_comp over NetBuffer
// fragments, buf.rs:466-487), in ONE pass.  A wave owns 64 consecutive packets;
// their fragments [F0, F1) (CSR `first`) stream through the size-class pass 64 at
// a time, each fragment paired from its own start exactly as the per-fragment call
// pairs it.  Each owner lane then applies the reference's step to its own
// fragments, in order, fetching their sums from the lanes that computed them:
//   fragment <= 128 KiB: sum = fold(sum + fold(W)).  No u32 wrap is possible, so
//     this is util.rs:89-103 with in_checksum = sum (same residue mod 0xffff, zero
//     iff both are zero);
//   longer: sum = fold((sum + W) mod 2^32), W = the exact BE word sum mod 2^32 —
//     the reference's wrapping u32 accumulator itself.
// Exact for any fragment count and size; no second kernel.  At 4 waves/SIMD every
// instantiation spills 8-44 B/lane (8 on the default path); 3 waves/SIMD spills nothing
// and is 4-7 % slower on c3 chains (session r04b), so 4 stays (tools/scratch_report.sh).
// ---------------------------------------------------------------------------
// Inclusive max over the 64 lanes (Hillis-Steele over DPP row shifts, then the row broadcasts).
// DPP, not __shfl_xor: the shuffles' lane-address registers are loop invariants the compiler
// hoisted and then spilled in the chain kernel (round 5).
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v)
{
    uint32_t x = v;
    x = max(x, dpp_or_zero<0x111>(x));           // row_shr:1
    x = max(x, dpp_or_zero<0x112>(x));           // row_shr:2
    x = max(x, dpp_or_zero<0x114>(x));           // row_shr:4
    x = max(x, dpp_or_zero<0x118>(x));           // row_shr:8
    x = max(x, dpp_or_zero<0x142, 0xA, 0xF>(x));  // row_bcast:15 into rows 1 and 3
    x = max(x, dpp_or_zero<0x143, 0xC, 0xF>(x));  // row_bcast:31 into rows 2 and 3
    return x;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
    return __builtin_amdgcn_readlane(wave_incl_max(v), 63);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) { return ~wave_max_u32(~v); }

constexpr uint32_t kChainMaxK = 8;  // packets per lane, at most

// The one-round tiny class (run_tiny) in the chain kernel's class pass: only for
// short fragments (the temporal instantiation, mean fragment < 384 B: IMIX chains
// 870 -> 800 us in 512-byte buffers).  With NetBuffer-sized fragments there are no
// tiny ones, and its registers made the kernel spill (c3 chains 292 -> 321 us).
#ifndef RNS_CHAIN_TINY
#define RNS_CHAIN_TINY 1
#endif
constexpr bool kChainTiny = RNS_CHAIN_TINY && kTinyQ > 1;

// Packets whose fragments form one run (RNS_FLAG_CHAIN_RUNS; A/B knob: -DRNS_CHAIN_RUNS=0).
//
// util.rs:112-119 folds after every fragment, each fragment's BE words paired from
// its own start.  When fragment f starts where f-1 ends and f-1 has EVEN length, f's
// words pair exactly as they do counted from f-1's start, so for fragments of at
// most 128 KiB (no u32 wrap) fold(fold(s + W[f-1]) + W[f]) == fold(s + fold(W[f-1] +
// W[f])): the same residue mod 0xffff, zero iff everything is zero.  A packet whose
// fragments (at most kRunFrags) are such a run — the pieces of one receive buffer, as
// the IP-trimmed views of a packet are — is therefore ONE contiguous unit of at most
// 128 KiB.  When every packet of a wave batch is, the wave runs the class pass over
// its 64 packets (as the plain batch kernel does) instead of over their fragments.
// Opt-in: the check is a round of descriptor loads before the class pass, which a
// layout without runs pays for nothing (profiles/r02_chain_runs_ab.json).
#ifndef RNS_CHAIN_RUNS
#define RNS_CHAIN_RUNS 1
#endif
constexpr bool kChainRuns = RNS_CHAIN_RUNS != 0;
constexpr uint32_t kRunFrags = 4;
constexpr uint32_t kNoRun = 0xFFFFFFFFu;

// The bytes of packet [f0, f1)'s run, or kNoRun.  Its (<= kRunFrags) descriptors are
// loaded up front: one memory latency, not one per fragment.
__device__ __forceinline__ uint32_t fragment_run(const CsumArgs &a, uint32_t f0, uint32_t f1, uint64_t &start)
{
    const uint32_t nfr = f1 - f0;
    if (nfr > kRunFrags)
        return kNoRun;
    uint64_t o[kRunFrags];
    uint32_t l[kRunFrags];
#pragma unroll
    for (uint32_t j = 0; j < kRunFrags; ++j) {
        o[j] = 0;
        l[j] = 0;
        if (j < nfr) {
            o[j] = a.off[f0 + j] + a.base_adjust;
            l[j] = a.len[f0 + j];
        }
    }
    uint32_t tot = 0;
    bool run = true;
#pragma unroll
    for (uint32_t j = 0; j < kRunFrags; ++j) {
        if (j < nfr) {
            const bool in = o[j] <= a.arena_bytes && l[j] <= a.arena_bytes - o[j];
            const bool joins = j == 0 || (o[j] == o[j - 1] + l[j - 1] && !(l[j - 1] & 1));
            run = run && in && joins && l[j] <= kNoWrapBytes;
            tot += run ? l[j] : 0u;
        }
    }
    start = o[0];
    return run && tot <= kNoWrapBytes ? tot : kNoRun;
}

// Waves/SIMD of the chain kernel (every instantiation free of scratch: tools/scratch_report.sh,
// profiles/r05_resources.txt): 4 (128 VGPRs) for the nontemporal buffer forms — NetBuffer-sized
// fragments, c3 chains 4-7 % faster than at 3 (session r04b) — and 3 (168 VGPRs) for the rest:
// at 4 the temporal runs / fill forms and the 64-bit addresses of arenas of 4 GiB and more
// spill 8-20 B/lane.  The temporal plain checksum (IMIX-like fragments) fits 4 without scratch
// too and has both: the launcher picks by the chain shape (OCC below).  -DRNS_CHAIN_OCC=n
// forces n for every instantiation (A/B builds).
template <bool NT, bool BUF, uint32_t KMAX, bool RUNS, bool FILL, int OCC>
constexpr int chain_occ()
{
#ifdef RNS_CHAIN_OCC
    return RNS_CHAIN_OCC;
#else
    return OCC ? OCC : (NT && BUF) ? 4 : 3;
#endif
}
// Workgroup size of the chain kernel: one wave.  Its per-packet state is LDS, which is
// freed per workgroup, as for the mixed kernel's stash modes: IMIX chains 640 -> 608 us
// packed, 839 -> 771 us in 512-byte buffers, c3 equal (profiles/r02_block_ab.json).
constexpr int kChainBlock = 64;
#ifndef RNS_CHAIN_WINDOW  // arenas of 4 GiB or more: buffer loads through a per-pass window
#define RNS_CHAIN_WINDOW 1
#endif
// RUNS: the RNS_FLAG_CHAIN_RUNS instantiation (buffer path only).  A separate kernel:
// compiled into the plain one, the run check cost it ~5 % (registers) even unused.
template <bool NT, bool BUF, uint32_t KMAX, bool RUNS = false, bool FILL = false, int OCC = 0>
__global__ __launch_bounds__(kChainBlock, (chain_occ<NT, BUF, KMAX, RUNS, FILL, OCC>())) void csum_chain_kernel(const CsumArgs a)
{
    static_assert(!RUNS || BUF, "runs: buffer path only");
    // A wave owns K*64 consecutive packets (K = a.chain_k, chosen by the host from the
    // mean fragment count so the wave's fragments fill whole 64-fragment batches).
    // Per-packet state is parked in LDS across the class pass (which needs every VGPR
    // of a 4-waves/SIMD budget): the fragment range and the running sum (bit 31 = a
    // bad descriptor seen).
    // RUNS: [3] the packet's run bytes (fragment_run), [4] its start
    // FILL: [kPk - 1] the field's contribution to the head fragment's raw sum
    constexpr int kPk = (RUNS ? 5 : 3) + (FILL ? 1 : 0);
    constexpr int kPf = kPk - 1;
    __shared__ uint32_t pk_lds[kChainBlock / 64][kPk][KMAX * 64];
    const uint32_t lane = threadIdx.x & 63;
    uint32_t (&pk)[kPk][KMAX * 64] = pk_lds[threadIdx.x >> 6];
    // A wave stops looking for runs after a batch without them (the check costs a round
    // of descriptor loads): the fragment path is exact for every batch anyway.
    bool try_runs = RUNS;
    const uint32_t wave = (blockIdx.x * kChainBlock + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * kChainBlock) >> 6;
    const uint32_t K = KMAX == 1 ? 1u : a.chain_k;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.arena), static_cast<short>(0), static_cast<int>(BUF ? buf_records(a) : 0), 0x00020000);
    constexpr uint32_t kBad = 0x80000000u;
    const uint64_t per_wave = 64ull * K;

    // (the packet index in 32 bits — a.n < 2^32 — with the step taken in 64 bits, so the loop
    // cannot wrap: one VGPR less across the class pass)
    const uint64_t first_pkt = static_cast<uint64_t>(wave) * per_wave, step = static_cast<uint64_t>(nwaves) * per_wave;
    if (first_pkt >= a.n)
        return;
    for (uint32_t base = static_cast<uint32_t>(first_pkt);;) {
        uint32_t lo_all = 0xFFFFFFFFu, hi_all = 0u;
        bool runs_all = true;
        for (uint32_t q = 0; q < K; ++q) {
            const uint64_t p = base + q * 64 + lane;  // (32-bit add: the host caps a.n at 2^32 - 64 * kChainMaxK)
            const bool live = p < a.n;
            uint32_t f0 = live ? a.first[p] : 0u, f1 = live ? a.first[p + 1] : 0u;
            const bool ok = f0 <= f1 && f1 <= a.n_frags;
            if (!ok)
                f0 = f1 = 0;
            const uint32_t acc = (a.seed && live) ? a.seed[p] : 0u;  // util.rs:113 (sum = initial_sum)
            lo_all = f0 < f1 ? min(lo_all, f0) : lo_all;
            hi_all = f0 < f1 ? max(hi_all, f1) : hi_all;
            pk[0][q * 64 + lane] = f0;
            pk[1][q * 64 + lane] = f1;
            bool fok = true;
            if constexpr (FILL) {
                // the field in the head fragment f0: its bytes' share of that fragment's raw sum
                // (LE words paired by absolute parity; the exact BE words past 128 KiB)
                uint32_t fc = 0;
                fok = false;
                if (ok && f0 < f1) {
                    const uint64_t ho = a.off[f0] + a.base_adjust;
                    const uint32_t hl = a.len[f0];
                    const uint32_t fo = a.field ? static_cast<uint32_t>(a.field[p]) : a.field_off;
                    fok = ho <= a.arena_bytes && hl <= a.arena_bytes - ho && fo <= hl && hl - fo >= 2u;
                    if (fok) {
                        const uint64_t fp = ho + fo;
                        const uint32_t b0 = a.arena[fp], b1 = a.arena[fp + 1];
                        fc = hl > kNoWrapBytes ? ((fo & 1u) ? b0 | (b1 << 8) : (b0 << 8) | b1)
                                               : (b0 << ((fp & 1) * 8)) + (b1 << (((fp + 1) & 1) * 8));
                    }
                }
                pk[kPf][q * 64 + lane] = fc;
            }
            pk[2][q * 64 + lane] = acc | (ok && fok ? 0u : kBad);
            if constexpr (RUNS) {
                uint64_t rs = 0;
                const uint32_t run = (ok && try_runs) ? fragment_run(a, f0, f1, rs) : kNoRun;
                pk[RUNS ? 3 : 0][q * 64 + lane] = run;
                pk[RUNS ? 4 : 0][q * 64 + lane] = static_cast<uint32_t>(rs);  // < 4 GiB on the buffer path
                runs_all = runs_all && run != kNoRun;
            }
        }
        // the wave's fragments: the union of its packets' ranges (contiguous for a CSR list)
        const uint32_t F0 = wave_min_u32(lo_all), F1 = wave_max_u32(hi_all);
        // every packet one run: K class passes over packets; else passes over fragments
        const bool by_packet = RUNS && try_runs && !__ballot(!runs_all);
        try_runs = by_packet;
        const uint32_t passes = by_packet ? K : (F1 - F0 + 63) / 64;  // (F1 >= F0, equal if no fragments)
        for (uint32_t it = 0; it < passes; ++it) {
            const uint32_t fb = F0 + 64u * it;  // < F1 <= n_frags: 32 bits
            uint64_t d_start = 0;
            uint32_t d_len = 0;
            if (by_packet) {
                const uint32_t i = it * 64 + lane;
                d_len = pk[RUNS ? 3 : 0][i];
                d_start = pk[RUNS ? 4 : 0][i] - a.base_adjust;  // (base_adjust added back below)
            } else if (static_cast<uint64_t>(fb) + lane < F1) {
                d_start = a.off[static_cast<uint64_t>(fb) + lane];
                d_len = a.len[static_cast<uint64_t>(fb) + lane];
            }
            d_start += a.base_adjust;
            const bool d_ok = d_start <= a.arena_bytes && d_len <= a.arena_bytes - d_start;
            if (!d_ok || d_len == 0) {  // an empty fragment adds nothing (the reference panics on it)
                d_len = 0;
                d_start = 0;
            }
            const bool big = d_len > kNoWrapBytes, odd = d_start & 1;
            uint32_t pos;
            uint32_t w;
            if constexpr (!BUF && RNS_CHAIN_WINDOW) {
                // arenas of 4 GiB or more: a pass whose 64 fragments lie within one window below
                // the buffer range (NetBuffers in order: 64 consecutive 512-byte buffers) loads
                // through a buffer descriptor based at the window's 16-byte-aligned start (IMIX
                // in 512-byte NetBuffers, a 6.4 GB arena: 751-753 -> 700-701 us; shuffled buffers,
                // every pass 64-bit: 780-782 -> 793-795, the two paths' code; sessions r05p, r05q)
                const uint32_t lo_hi = d_len ? static_cast<uint32_t>(d_start >> 32) : 0xFFFFFFFFu;
                const uint32_t wlh = wave_min_u32(lo_hi);
                const uint32_t wll = wave_min_u32(d_len && lo_hi == wlh ? static_cast<uint32_t>(d_start) & ~15u : 0xFFFFFFFFu);
                const uint64_t end = d_len ? d_start + d_len : 0;
                const uint32_t ehi = wave_max_u32(static_cast<uint32_t>(end >> 32));
                const uint32_t elo = wave_max_u32(static_cast<uint32_t>(end >> 32) == ehi ? static_cast<uint32_t>(end) : 0u);
                const uint64_t wlo = (static_cast<uint64_t>(wlh) << 32) | wll, whi = (static_cast<uint64_t>(ehi) << 32) | elo;
                if (whi <= wlo || whi - wlo <= kOobOffset - 4096u) {  // (no fragment: whi = 0)
                    const uint64_t wb = whi > wlo ? wlo : 0;
                    const uint64_t recs_w = buf_records(a) - wb;
                    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
                        const_cast<uint8_t *>(a.arena) + wb, static_cast<short>(0),
                        static_cast<int>(recs_w < kOobOffset ? recs_w : kOobOffset), 0x00020000);
                    w = wave_class_pass<NT, true, kStashNone, kChainTiny && !NT>(a, rw, d_len ? d_start - wb : 0, d_len, 0u,
                                                                                  lane, nullptr, pos);
                } else {
                    w = wave_class_pass<NT, false, kStashNone, kChainTiny && !NT>(a, rsrc, d_start, d_len, 0u, lane, nullptr,
                                                                                   pos);
                }
            } else {
                w = wave_class_pass<NT, BUF, kStashNone, kChainTiny && !NT>(a, rsrc, d_start, d_len, 0u, lane, nullptr, pos);
            }
            uint32_t g = w;  // big: BE sum mod 2^32; else the folded BE sum (RFC 1071 §2(B), as finalize_bits)
            if (!big) {
                const uint32_t x = fold16(w);
                g = odd ? x : (((x & 0xff) << 8) | (x >> 8));
            }
            const uint32_t gflag = (big ? 1u : 0u) | (d_ok ? 0u : 2u) | (FILL && odd ? 4u : 0u);
            wave_lds_fence();
            if (by_packet) {  // the lane's packet is its run: one fold (never big, never bad)
                const uint32_t i = it * 64 + lane;
                uint32_t gr = g;
                if constexpr (FILL) {  // the run starts with the head fragment: the field out of it
                    const uint32_t x = fold16(w - pk[kPf][i]);
                    gr = odd ? x : (((x & 0xff) << 8) | (x >> 8));
                }
                const uint32_t s = (pk[2][i] & 0xffffu) + gr;
                pk[2][i] = ((s & 0xffff) + (s >> 16)) | (FILL ? pk[2][i] & kBad : 0u);
                continue;
            }
            // owner lanes: each packet's fragments inside [fb, fb + 64), in order
            for (uint32_t q = 0; q < K; ++q) {
                const uint32_t i = q * 64 + lane;
                uint32_t t = max(pk[0][i], fb);
                const uint32_t hi = static_cast<uint32_t>(min(static_cast<uint64_t>(pk[1][i]), static_cast<uint64_t>(fb) + 64));
                if (!__ballot(t < hi))
                    continue;
                uint32_t acc = pk[2][i];
                const uint32_t head = FILL ? pk[0][i] : 0u, fc = FILL ? pk[kPf][i] : 0u;
                do {
                    const bool act = t < hi;
                    const int src = act ? static_cast<int>(t - fb) : 0;
                    uint32_t gv = static_cast<uint32_t>(__shfl(static_cast<int>(g), src, 64));
                    const uint32_t fv = static_cast<uint32_t>(__shfl(static_cast<int>(gflag), src, 64));
                    if constexpr (FILL) {  // the head fragment: its raw sum without the field, folded here
                        const uint32_t wv = static_cast<uint32_t>(__shfl(static_cast<int>(w), src, 64)) - fc;
                        const uint32_t x = fold16(wv);
                        gv = t != head ? gv : (fv & 1u) ? wv : (fv & 4u) ? x : (((x & 0xff) << 8) | (x >> 8));
                    }
                    if (act) {
                        const uint32_t bad = (acc & kBad) | ((fv & 2u) ? kBad : 0u);
                        uint32_t s = (acc & 0xffffu) + gv;  // big: util.rs:89-99 mod 2^32; else <= 0x1fffe
                        if (fv & 1u) {
                            while (s > 0xffff)  // util.rs:101-103
                                s = (s & 0xffff) + (s >> 16);
                        } else {
                            s = (s & 0xffff) + (s >> 16);  // one end-around step folds it
                        }
                        acc = s | bad;
                        ++t;
                    }
                } while (__ballot(t < hi));
                pk[2][i] = acc;
            }
        }
        wave_lds_fence();
        for (uint32_t q = 0; q < K; ++q) {
            const uint64_t p = base + q * 64 + lane;
            const uint32_t acc = pk[2][q * 64 + lane];
            uint32_t r = acc & 0xffffu;
            if (a.flags & RNS_FLAG_COMPLEMENT)
                r ^= 0xffff;
            const bool ok = !(acc & kBad);
            if constexpr (FILL) {
                if (p < a.n && ok) {  // set_be16(&mut header[fo..fo + 2], result), header = fragment f0
                    const uint32_t fo = a.field ? static_cast<uint32_t>(a.field[p]) : a.field_off;
                    const uint64_t fp = a.off[pk[0][q * 64 + lane]] + a.base_adjust + fo;
                    uint8_t *w8 = const_cast<uint8_t *>(a.arena);
                    if (fp & 1) {
                        w8[fp] = static_cast<uint8_t>(r >> 8);
                        w8[fp + 1] = static_cast<uint8_t>(r);
                    } else {
                        *reinterpret_cast<uint16_t *>(w8 + fp) = static_cast<uint16_t>(((r & 0xff) << 8) | (r >> 8));
                    }
                }
            }
            if (p < a.n && (!FILL || a.out))
                a.out[p] = static_cast<uint16_t>(ok ? r : 0u);  // 64 consecutive u16: one 128-byte store
            if (a.bad) {
                const uint64_t rejected = __ballot(p < a.n && !ok);
                if (rejected && lane == 0)
                    atomicAdd(a.bad, static_cast<uint32_t>(__popcll(rejected)));
            }
        }
        wave_lds_fence();  // the next batch rewrites pk
        const uint64_t next = static_cast<uint64_t>(base) + step;
        if (next >= a.n)
            break;
        base = static_cast<uint32_t>(next);
    }
}

// ---------------------------------------------------------------------------
// v4: "stream" kernel — the packed form with 16-byte-aligned packets (align_log2 >= 4).
//
// A wave owns a 64-packet block.  Its packets lie back to back from blk_off[b], each
// starting on a 16-byte boundary, so the block is one contiguous REGION of the arena
// in which every 16-byte chunk belongs to exactly one packet (its tail chunk also
// holds the padding up to the next boundary).  The wave streams the region as rows
// of 64 chunks — lane l loads chunk 64k + l of row k, one fully coalesced 1 KiB load
// per row, D rows in flight — whatever the packet sizes: no size classes, no sort, no
// partially used loads.  Per row every lane sums its chunk's LE 16-bit words
// (v_sad_u16), a DPP scan turns the row into prefix sums P, and the region prefix at
// each packet's LAST chunk is kept.  A packet's word sum is the difference of the
// prefixes at its own last chunk and at the previous non-empty packet's.  Packets
// are at most 65535 bytes (u16 lengths), so every packet's LE sum is exact in u32 and
// the u32 prefixes may wrap: the difference is exact.
//
// Per row: the owners whose packet ends in the row publish (row tag, packet, valid
// bytes) to an LDS slot indexed by the lane that loads that chunk; every lane reads its
// slot, zeroes the padding bytes of an end chunk, and an end lane stores its prefix to
// pend[packet].  ~25 VALU + 3 LDS operations per KiB, one VMEM load per KiB.
//
// A block whose region does not start 16-byte aligned (a first packet at an unaligned
// offset, or an unaligned arena base) takes a simple per-packet wave loop instead.
// ---------------------------------------------------------------------------
// Inclusive prefix sum over the 64 lanes (wave_excl_scan's DPP sequence).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
    uint32_t x = v;
    x += dpp_or_zero<0x111>(v);              // row_shr:1
    x += dpp_or_zero<0x112>(v);              // row_shr:2
    x += dpp_or_zero<0x113>(v);              // row_shr:3
    x += dpp_or_zero<0x114, 0xF, 0xE>(x);    // row_shr:4, banks 1-3
    x += dpp_or_zero<0x118, 0xF, 0xC>(x);    // row_shr:8, banks 2-3
    x += dpp_or_zero<0x142, 0xA, 0xF>(x);    // row_bcast:15 into rows 1 and 3
    x += dpp_or_zero<0x143, 0xC, 0xF>(x);    // row_bcast:31 into rows 2 and 3
    return x;
}

// Keep the first c (1..16) bytes of a chunk: the 128-bit mask (1 << 8c) - 1 as two
// 64-bit halves (shift counts stay in 0..63).
__device__ __forceinline__ uint4 keep_first(uint4 v, uint32_t c)
{
    const uint32_t bits = c * 8u;                                    // 8..128
    const uint64_t lo = ~0ull >> (64u - min(bits, 64u));
    const uint64_t hi = bits > 64u ? ~0ull >> ((128u - bits) & 63u) : 0ull;
    v.x &= static_cast<uint32_t>(lo);
    v.y &= static_cast<uint32_t>(lo >> 32);
    v.z &= static_cast<uint32_t>(hi);
    v.w &= static_cast<uint32_t>(hi >> 32);
    return v;
}

#ifndef RNS_STREAM_NT  // nontemporal loads in the stream kernel
#define RNS_STREAM_NT 1
#endif
#ifndef RNS_STREAM_OUT_AUX  // cache-policy bits of the result buffer stores (17 = sc0 | sc1)
#define RNS_STREAM_OUT_AUX 17
#endif
// Result stores: buffer stores with the policy bits above (arrays below 2^30 entries; larger
// ones: nontemporal stores).  IMIX, isolated dispatch: plain stores 472 us, nontemporal
// 454-461, sc0|sc1 455.9 (r03i, r03o; sc0 alone 474, sc1 457, sc1|nt 461-466, sc0|nt 459-460).
// The stream kernel's rows in flight: 8 since its rows start line-aligned (IMIX verify 472.3-472.8
// -> 468.0-470.3 us, c3 235.9 -> 234.5; 6: 476.9; r04af), and its waves/SIMD bound (its finish
// needs registers).
constexpr int kStreamD = 8;
constexpr int kStreamRxOcc = 6;

// Chunk i of the datagram of len bytes whose 16-byte-aligned chunk 0 is at byte offset off
// (zero, with no load, for a chunk wholly past the end; the last chunk is not masked).
template <bool BUF>
__device__ __forceinline__ uint4 own_chunk(const CsumArgs &a, __amdgpu_buffer_rsrc_t rsrc, uint64_t recs, uint64_t off,
                                           uint32_t len, uint32_t i)
{
    const uint64_t o = off + 16u * i;
    const bool in = 16u * i < len && o + 16 <= recs;
    uint4 x;
    if constexpr (BUF) {
        const u32x4 y = __builtin_amdgcn_raw_buffer_load_b128(rsrc, in ? static_cast<uint32_t>(o) : kOobOffset, 0, 0);
        x = make_uint4(y.x, y.y, y.z, y.w);
    } else {
        const uint4 y = load_chunk<false>(a.arena + (in ? o : 0));
        x = in ? y : make_uint4(0, 0, 0, 0);
    }
    return x;
}

// Receive verify (rns_rx_verify_packed_dev).  The lanes that load a datagram's first 4
// chunks (64 bytes: every IPv4 header incl. options, the IPv6 header) also copy them to an
// LDS stash, and the owner finishes exactly as the class kernel's receive verify does
// (rx_finish).  A unit whose datagrams all fit 4 chunks (ACK-sized: 64 B TCP/IPv4 with
// options) skips the rows: each owner loads its datagram whole and finishes from registers
// (64 B datagrams: 13.3 -> 12.1 us per step, session r04b).  (Round 3's plain mode of this
// kernel gave way to csum_rows_kernel in round 4; forms that gave a wave several units were
// measured slower in round 3 and removed.)  One wave per 64-datagram unit.
template <bool NT, bool BUF>
__global__ __launch_bounds__(64, kStreamRxOcc) void csum_stream_kernel(const CsumArgs a)
{
    constexpr int kNS = 4;  // stash chunks per datagram (16-byte-aligned: its first 64 bytes)
    // entry bits: [31:17] row tag, [16] head chunk, [15:14] head index, [13] end chunk,
    // [12] first chunk, [11:4] packet (of the wave's 64), [3:0] valid bytes - 1 (end chunk)
    constexpr uint32_t kTagShift = 17, kHead = 1u << 16, kEnd = 1u << 13, kStart = 1u << 12;
    __shared__ uint32_t tab[64];     // per row: the entry of the chunk lane l loads
    __shared__ uint32_t pend[64];    // per packet: the region prefix through its last chunk
    __shared__ uint32_t pstart[64];  // per packet: the region prefix before its first chunk
    __shared__ uint4 stash[64 * kNS];
    const uint32_t lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.arena), static_cast<short>(0), static_cast<int>(BUF ? buf_records(a) : 0), 0x00020000);
    const uint64_t recs = buf_records(a);
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * 64;
    const uint64_t p = base + lane;
    const bool live = p < a.n;
    const uint64_t q = live ? p : a.n - 1;  // branch-free descriptor loads
    // (the block offset is loaded per lane at an index the compiler cannot prove uniform: a
    // uniform load is moved to SGPRs right away, with a vmcnt(0) wait for every row in flight)
    const uint32_t zero_v = __builtin_amdgcn_mbcnt_lo(0u, 0u);
    const uint64_t r0v = a.blk_off[(base >> 6) + zero_v];
    const uint32_t len = live ? static_cast<uint32_t>(a.len16[q]) : 0u;
    // (the lane intrinsics return int: widen through uint32_t, or an offset past 2 GiB sign-extends)
    const uint64_t r0 =
        ((static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(r0v >> 32))))
          << 32) |
         static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(r0v)))) +
        a.base_adjust;  // the wave's first packet
    const uint32_t pad = (len + a.align_mask) & ~a.align_mask;
    const uint32_t incl = wave_incl_scan(pad);
    const uint32_t excl = incl - pad;
    const uint32_t total = __builtin_amdgcn_readlane(incl, 63);  // the region's bytes
    uint32_t mine = 0;
    bool odd = false;

    if ((r0 & 15) == 0 && !__ballot(len > 64)) {
        // ---- ACK-sized unit: every owner takes its datagram whole ----
        const uint64_t start = r0 + excl;
        const bool ok = start <= a.arena_bytes && len <= a.arena_bytes - start;
        uint4 own[kNS + 1];
#pragma unroll
        for (int i = 0; i < 4; ++i)  // all four loads in flight before the first is used
            own[i] = own_chunk<BUF>(a, rsrc, recs, start, len, i);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint4 x = own[i];
            if (16u * i + 16u > len)  // rx_finish sees zeros past the end, as from the stash
                x = 16u * i < len ? keep_first(x, len - 16u * i) : make_uint4(0, 0, 0, 0);
            own[i] = x;
            mine = __builtin_amdgcn_sad_u16(x.x, 0, mine);
            mine = __builtin_amdgcn_sad_u16(x.y, 0, mine);
            mine = __builtin_amdgcn_sad_u16(x.z, 0, mine);
            mine = __builtin_amdgcn_sad_u16(x.w, 0, mine);
        }
        own[4] = make_uint4(0, 0, 0, 0);
        uint32_t l4_res = 0;
        const uint8_t stv = rx_finish<kNS + 1>(a, own, mine, 0u, len, false, false, live && ok && len != 0, l4_res);
        if (live) {
            a.status[p] = stv;
            if (a.l4_out)
                a.l4_out[p] = static_cast<uint16_t>(l4_res);
        }
        return;
    }
    if ((r0 & 15) == 0) {
        // ---- stream path ----
        // (rows from the 128-byte line below the region, as csum_rows_kernel)
        const uint32_t la = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(a.arena) + r0) & 127u;
        const uint32_t lead = la <= r0 ? la : 0u;  // (IMIX verify 473.6-473.7 -> 469.5-471.5 us: r04y)
        const uint64_t rb = r0 - lead;
        const uint32_t nrows = (total + lead + 1023) >> 10;
        tab[lane] = 0xFFFFFFFFu;  // tag 0x7FFF: never a row
        wave_lds_fence();
        uint32_t carry = 0;
        uint4 v[kStreamD];
        auto issue = [&](uint32_t k, uint4 &dst) {  // row k: chunk 64k + lane of the region
            const uint64_t off = rb + (static_cast<uint64_t>(k) << 10) + (lane << 4);
            const bool in = k < nrows && off + 16 <= recs;
            if constexpr (BUF) {
                const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(
                    rsrc, in ? static_cast<uint32_t>(off) : kOobOffset, 0, NT ? kNtAux : 0);
                dst = make_uint4(x.x, x.y, x.z, x.w);
            } else {
                const uint4 x = load_chunk<NT>(a.arena + (in ? off : 0));
                dst = in ? x : make_uint4(0, 0, 0, 0);
            }
        };
        // (issue order pinned: the loop consumes v[0] first, so its load must be the oldest
        // on entry as on the back edge, or the compiler waits for all of them)
#pragma unroll
        for (int j = 0; j < kStreamD; ++j) {
            issue(j, v[j]);
            __builtin_amdgcn_sched_barrier(0);
        }
        const uint32_t c0 = (excl + lead) >> 4;
        const uint32_t e = (excl + lead + len - 1) >> 4;
        const uint32_t ent = (lane << 4) | ((len - 1) & 15u);
        const bool ne = len != 0;
        for (uint32_t k0 = 0; k0 < nrows; k0 += kStreamD) {
#pragma unroll
            for (int j = 0; j < kStreamD; ++j) {
                const uint32_t k = k0 + j;
                const uint32_t tag = k << kTagShift;
                // owners publish at the lanes that load their chunks in row k: the first chunk
                // (padding chunks between packets, align_log2 > 4, belong to no packet, so a
                // packet's sum is its end prefix minus its own start prefix), the last chunk
                // (its valid bytes) and, receive verify, the first 4 chunks (the stash)
#pragma unroll
                for (uint32_t h = 0; h < 4; ++h) {
                    const uint32_t c = c0 + h;
                    if (ne && c <= e && (c >> 6) == k)
                        tab[c & 63] = tag | kHead | (h << 14) | (h == 0 ? kStart : 0u) | (c == e ? kEnd : 0u) | ent;
                }
                if (ne && e >= c0 + 4 && (e >> 6) == k)
                    tab[e & 63] = tag | kEnd | ent;
                wave_lds_fence();
                const uint32_t t = tab[lane];
                const bool mark = (t >> kTagShift) == k;
                const bool is_end = mark && (t & kEnd);
                const uint32_t pk = (t >> 4) & 0xFFu;
                uint4 x = v[j];
                if (__ballot(is_end && (t & 15u) != 15u))  // a partial end chunk in this row
                    x = keep_first(x, is_end ? (t & 15u) + 1u : 16u);
                if (mark && (t & kHead))
                    stash[pk * kNS + ((t >> 14) & 3u)] = x;
                uint32_t s = __builtin_amdgcn_sad_u16(x.x, 0, 0u);
                s = __builtin_amdgcn_sad_u16(x.y, 0, s);
                s = __builtin_amdgcn_sad_u16(x.z, 0, s);
                s = __builtin_amdgcn_sad_u16(x.w, 0, s);
                // the row D ahead into the registers this row just freed (past the region: no
                // memory traffic).  Issued only after the row is consumed, so the loop-carried
                // registers need no copy — a copy at the back edge waits for every load in flight.
                __builtin_amdgcn_sched_barrier(0);
                issue(k + kStreamD, v[j]);
                __builtin_amdgcn_sched_barrier(0);
                const uint32_t inc = wave_incl_scan(s);
                if (mark && (t & kStart))
                    pstart[pk] = carry + inc - s;
                if (is_end)
                    pend[pk] = carry + inc;
                carry += __builtin_amdgcn_readlane(inc, 63);
                wave_lds_fence();
            }
        }
        // a packet's sum: the region prefix through its last chunk minus the prefix before its
        // first (u32 differences: exact, a packet's LE sum is < 2^32)
        mine = len ? pend[lane] - pstart[lane] : 0u;
    } else {
        // ---- unaligned region (rare): the whole wave sums one packet at a time ----
        const uint64_t start = r0 + excl;
        const bool ok = start <= a.arena_bytes && len <= a.arena_bytes - start;
        uint64_t todo = __ballot(len != 0 && ok);
        while (todo) {
            const uint32_t o = static_cast<uint32_t>(__builtin_ctzll(todo));
            todo &= todo - 1;
            const uint64_t st =
                (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(start >> 32), o)))
                 << 32) |
                static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(start), o));
            const uint32_t L = __builtin_amdgcn_readlane(len, o);
            const Pkt k = make_pkt(st, L);
            uint32_t acc = 0;
            for (uint32_t cc = 0; cc < k.nch; cc += 64) {
                uint4 w[1];
                issue_pass<64, 1, NT, BUF, 1>(a, rsrc, k, cc + lane, w);
                mask_edges<64, 1, 1>(k, cc + lane, w);
                acc = sum_le<1, 1>(w, acc);
            }
            const uint32_t sum = group_allreduce<64>(acc);
            mine = lane == o ? sum : mine;
        }
        odd = r0 & 1;  // every packet of the range shares the region start's misalignment
        // each owner takes its header from the 16-byte boundary below its start: 5 chunks hold
        // its first 65-80 bytes, masked to the datagram
        const uint64_t b0 = start & ~15ull;
        const uint32_t s0 = static_cast<uint32_t>(start & 15);
        uint4 own[5];
#pragma unroll
        for (int i = 0; i < 5; ++i)
            own[i] = own_chunk<BUF>(a, rsrc, recs, b0, (len && ok) ? s0 + len : 0u, i);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int lo = static_cast<int>(s0) - 16 * i, hi = static_cast<int>(s0 + len) - 16 * i;
            own[i] = make_uint4(keep_bytes(own[i].x, lo, hi, 0), keep_bytes(own[i].y, lo, hi, 4),
                                keep_bytes(own[i].z, lo, hi, 8), keep_bytes(own[i].w, lo, hi, 12));
        }
        uint32_t l4_res = 0;
        const uint8_t stv = rx_finish<5>(a, own, mine, s0, len, odd, false, live && ok && len != 0, l4_res);
        if (live) {
            a.status[p] = stv;
            if (a.l4_out)
                a.l4_out[p] = static_cast<uint16_t>(l4_res);
        }
        return;
    }
    wave_lds_fence();
    const uint64_t start = r0 + excl;
    const bool ok = start <= a.arena_bytes && len <= a.arena_bytes - start;
    uint32_t l4_res = 0;
    const uint8_t stv = rx_finish<kNS>(a, stash + lane * kNS, mine, static_cast<uint32_t>(start & 15), len, odd, false,
                                       live && ok && len != 0, l4_res);
    if (live) {
        a.status[p] = stv;
        if (a.l4_out)
            a.l4_out[p] = static_cast<uint16_t>(l4_res);
    }
}

// Three measured choices shape the row stream (round 4; the losing forms are gone):
//  * the owner's end-chunk load is issued a group of rows ahead of its row, not up front
//    (c3 isolated 228.2-229.4 -> 224.8 us, traffic 1.030 -> 1.006x; session r04q);
//  * rows start at the 128-byte line below the region (IMIX 445.8-446.0 -> 436.6-437.5 us,
//    0.809 -> 0.825, traffic 1.042 -> 1.034x; session r04w);
//  * lanes past the region's end in its last row load nothing (IMIX isolated 451.7-453.3 ->
//    447.9-448.4 us, traffic 1.062 -> 1.042x; session r04r).
// The rows decomposition over one region that starts 16-byte aligned at r0 (an offset from
// a.arena) and holds total bytes (a multiple of 16; ceil(total / 1 KiB) rows): the lane's packet covers chunks c0..e of the region (its
// start 16-byte aligned, len bytes, len 0: none).  Returns the packet's LE word sum (pairs by
// absolute parity).  csum_rows_kernel's aligned path and the chain kernel's runs (below).
#ifndef RNS_ROWS_WINDOW  // arenas of 4 GiB or more: the rows through a buffer window (1) or 64-bit loads (0)
#define RNS_ROWS_WINDOW 1
#endif
struct NoHook {
    __device__ __forceinline__ void operator()() const {}
};
// `after_first` runs once the first D rows are issued (a caller's own earlier loads are then
// the oldest in flight: consuming them waits for exactly those, not for the rows).
// NH > 0 (receive verify): the owner also loads its packet's first NH chunks into hv[] (those
// inside the packet; the others read as zero), like its end chunk: a group of rows ahead of
// the row that streams them, so each line is fetched once.
template <bool NT, bool BUF, int D, int NH = 0, typename Hook = NoHook>
__device__ __forceinline__ uint32_t rows_region_sum(const CsumArgs &a, const __amdgpu_buffer_rsrc_t rsrc, uint64_t recs,
                                                   uint64_t r0, uint32_t total, uint32_t c0, uint32_t e, uint32_t len,
                                                   uint4 *hv = nullptr, Hook after_first = Hook{})
{
    {
        // start the row stream at the 128-byte line below the region (the few bytes before it
        // belong to no packet of this unit; prefix differences cancel them), so every 1 KiB row
        // covers 8 whole lines, not 9 — IMIX regions end anywhere on a 16-byte boundary
        const uint32_t la = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(a.arena) + r0) & 127u;  // absolute
        const uint32_t lead = la <= r0 ? la : 0u;
        r0 -= lead;
        total += lead;
        c0 += lead >> 4;
        e += lead >> 4;
    }
    const uint32_t nrows = (total + 1023) >> 10;
    const uint32_t lane = threadIdx.x & 63u;
    // the owner's end chunk (pulling it from its row instead, four ds_bpermute per row, measured
    // 2x slower: session r04g)
    uint4 endv = make_uint4(0, 0, 0, 0);
    constexpr bool kLate = BUF;
    const uint32_t row_e = len ? e >> 6 : 0xFFFFFFFFu;
    // the owners load their end chunks a group of D rows ahead of the rows
    // that hold them (one exec-masked load per group: its line is then still in L2 when the row
    // streams it), not all before the first row
    const uint32_t row_h = len ? c0 >> 6 : 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < NH; ++i)
        hv[i] = make_uint4(0, 0, 0, 0);
    auto load_end_late = [&](uint32_t k) {  // end chunks in rows [k, k + D)
        if constexpr (kLate) {
            if (row_e - k < static_cast<uint32_t>(D)) {
                const uint32_t off = static_cast<uint32_t>(r0) + (e << 4);
                const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off + 16u <= recs ? off : kOobOffset, 0, 0);
                endv = make_uint4(x.x, x.y, x.z, x.w);
            }
            if constexpr (NH > 0) {  // the packet's first chunks, a group ahead of their row
                if (row_h - k < static_cast<uint32_t>(D)) {
#pragma unroll
                    for (int i = 0; i < NH; ++i) {
                        const uint32_t off = static_cast<uint32_t>(r0) + ((c0 + i) << 4);
                        const bool in = 16u * i < len && off + 16u <= recs;
                        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, in ? off : kOobOffset, 0, 0);
                        hv[i] = make_uint4(x.x, x.y, x.z, x.w);
                    }
                }
            }
        }
    };
    if constexpr (!kLate) {
#pragma unroll
        for (int i = 0; i < NH; ++i)
            hv[i] = own_chunk<BUF>(a, rsrc, recs, r0 + (static_cast<uint64_t>(c0) << 4), len, i);
        const uint64_t off = r0 + (static_cast<uint64_t>(e) << 4);
        const bool in = len != 0 && off + 16 <= recs;
        if constexpr (BUF) {
            const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, in ? static_cast<uint32_t>(off) : kOobOffset,
                                                                  0, 0);
            endv = make_uint4(x.x, x.y, x.z, x.w);
        } else {
            const uint4 x = load_chunk<false>(a.arena + (in ? off : 0));
            endv = in ? x : make_uint4(0, 0, 0, 0);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t vlane = lane << 4;
    uint4 v[D];
    auto issue = [&](uint32_t k, uint4 &dst) {  // row k: chunk 64k + lane of the region
        if constexpr (BUF) {
            // lanes past the region's end load nothing (a row past it: no traffic at all); the next
            // unit's wave streams those bytes, often on another XCD's L2
            const uint32_t rel = (k << 10) + vlane;
            const uint32_t o = rel < total ? static_cast<uint32_t>(r0) + rel : kOobOffset;
            const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o, 0, NT ? kNtAux : 0);
            dst = make_uint4(x.x, x.y, x.z, x.w);
        } else {
            const uint64_t off = r0 + (static_cast<uint64_t>(k) << 10) + vlane;
            const bool in = k < nrows && off + 16 <= recs;
            const uint4 x = load_chunk<NT>(a.arena + (in ? off : 0));
            dst = in ? x : make_uint4(0, 0, 0, 0);
        }
    };
    load_end_late(0);
#pragma unroll
    for (int j = 0; j < D; ++j) {
        issue(j, v[j]);
        __builtin_amdgcn_sched_barrier(0);
    }
    after_first();
    __builtin_amdgcn_sched_barrier(0);
    // the owner's partial end chunk (its padding bytes never count)
    auto end_part = [&]() -> uint32_t {
        uint32_t part = 0;
        if (len) {
            const uint4 x = keep_first(endv, ((len - 1) & 15u) + 1u);
            part = __builtin_amdgcn_sad_u16(x.x, 0, 0u);
            part = __builtin_amdgcn_sad_u16(x.y, 0, part);
            part = __builtin_amdgcn_sad_u16(x.z, 0, part);
            part = __builtin_amdgcn_sad_u16(x.w, 0, part);
        }
        return part;
    };
    uint32_t part = kLate ? 0u : end_part();
    // capture points: P(c0 - 1) and P(e - 1) (row, source lane); e == c0 takes the
    // start's point twice (the difference is 0), c0 == 0 never captures (P(-1) = 0)
    const uint32_t ca = c0 - 1u;
    const uint32_t cb = e > c0 ? e - 1u : ca;
    const uint32_t row_a = c0 ? ca >> 6 : 0xFFFFFFFFu, row_b = (e > c0 || c0) ? cb >> 6 : 0xFFFFFFFFu;
    const int src_a = static_cast<int>((ca & 63u) << 2), src_b = static_cast<int>((cb & 63u) << 2);
    uint32_t pa = 0, pb = 0, carry = 0;
    for (uint32_t k0 = 0; k0 < nrows; k0 += D) {
        load_end_late(k0 + D);  // (the rows this group issues)
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const uint32_t k = k0 + j;
            const uint4 x = v[j];
            uint32_t s = __builtin_amdgcn_sad_u16(x.x, 0, 0u);
            s = __builtin_amdgcn_sad_u16(x.y, 0, s);
            s = __builtin_amdgcn_sad_u16(x.z, 0, s);
            s = __builtin_amdgcn_sad_u16(x.w, 0, s);
            // the row D ahead into the registers this row just freed (issued after the row
            // is consumed: no loop-carried copy, exact vmcnt(D-1) waits)
            __builtin_amdgcn_sched_barrier(0);
            issue(k + D, v[j]);
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t inc = wave_incl_scan(s);
            const uint32_t ta = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src_a, static_cast<int>(inc)));
            const uint32_t tb = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src_b, static_cast<int>(inc)));
            pa = row_a == k ? carry + ta : pa;
            pb = row_b == k ? carry + tb : pb;
            carry += __builtin_amdgcn_readlane(inc, 63);
        }
    }
    if constexpr (kLate)
        part = end_part();
    return len ? pb - pa + part : 0u;
}

// The region sum on any arena: past 4 GiB (BUF = false) through a buffer descriptor based at the
// region's 128-byte line (a region is at most 64 packets of 64 KiB: far below the buffer range),
// so the rows keep buffer loads with their range checks and cache-policy bits instead of 64-bit
// addresses (per isolated dispatch, session r05s: 3M x 1500 B 815 -> 684 us, 16M IMIX 945 -> 864,
// the transmit-packed chain checksum of 16M IMIX 1263 -> 945).
template <bool NT, bool BUF, int D, int NH = 0, typename Hook = NoHook>
__device__ __forceinline__ uint32_t rows_region_sum_any(const CsumArgs &a, const __amdgpu_buffer_rsrc_t rsrc, uint64_t recs,
                                                       uint64_t r0, uint32_t total, uint32_t c0, uint32_t e, uint32_t len,
                                                       uint4 *hv = nullptr, Hook after_first = Hook{})
{
    if constexpr (BUF || !RNS_ROWS_WINDOW) {
        return rows_region_sum<NT, BUF, D, NH>(a, rsrc, recs, r0, total, c0, e, len, hv, after_first);
    } else {
        const uint32_t la = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(a.arena) + r0) & 127u;
        const uint64_t wb = la <= r0 ? r0 - la : 0;  // the line the rows start at (absolute alignment kept)
        CsumArgs aw = a;
        aw.arena = a.arena + wb;
        aw.arena_bytes = a.arena_bytes - wb;
        const uint64_t rw_recs = recs - wb;
        const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(aw.arena), static_cast<short>(0),
            static_cast<int>(rw_recs < kOobOffset ? rw_recs : static_cast<uint64_t>(kOobOffset)), 0x00020000);
        return rows_region_sum<NT, true, D, NH>(aw, rw, rw_recs, r0 - wb, total, c0, e, len, hv, after_first);
    }
}

// ---------------------------------------------------------------------------
// Row stream with owner captures (round 4; the packed form's plain checksum for
// 16-byte-aligned packets above the tiny class: c3, c4, IMIX).
//
// A wave owns 64 consecutive packets and streams their bytes as ONE region, row k =
// the region's k-th KiB (64 lanes x 16 B), D rows in flight — as csum_stream_kernel,
// without its per-row LDS table.  The loading lanes know nothing about packets: each
// sums its whole chunk (4 v_sad_u16), and one DPP scan per row gives the region's
// inclusive prefix P at every chunk.  Packet p (chunks c0..e, 16-aligned start) needs
// only two of those prefixes and its own end chunk:
//     sum_p = P(e - 1) - P(c0 - 1) + (the first ((len - 1) & 15) + 1 bytes of chunk e)
// (P(-1) = 0; e == c0: the end chunk alone).  The owner lane pulls P(c0 - 1) and
// P(e - 1) from the lanes that hold them with ds_bpermute in the rows they fall in, and
// loads its end chunk itself one group of D rows before the row that streams it (the line
// is fetched once), so the end chunk's padding bytes never need a per-row mask.  Rows start
// at the 128-byte line below the region and lanes past its end load nothing.  Per KiB: 4 sad + the scan + two captures, no LDS memory, no fences
// (csum_stream_kernel: a table publish, two wave fences, the masks; 57 VALU/KB).
// u32 differences are exact: a packet's LE word sum is < 2^32.
// ---------------------------------------------------------------------------
// Rows in flight D: 8 at 8 waves/SIMD, or 16 at 4 waves/SIMD for MTU-sized and longer packets
// (c3 isolated 230.2-231.0 -> 227.8-227.9 us; IMIX 445.6-447.6 -> 454-456, so IMIX keeps 8;
// D = 12 at 5 waves/SIMD in between; two or four 64-packet sets per wave slower on IMIX:
// session r04g).
//
// FILL (transmit in-place fill of a packed arena, rns_csum_fill_packed_dev): the field
// (2 bytes at packet offset field[p] / field_off) counts as zero (buf.rs:286-288) and
// receives the result big-endian (tcp.rs:970-973).  The owner loads the 32-byte sector
// around its field with its end chunk, takes the field's bytes out of the row sum, and
// rewrites the whole sector when it lies inside the packet (a full-sector write: no
// read-modify-write at the memory side), else stores the two bytes.
#ifndef RNS_ROWS_FILL_OCC  // waves/SIMD bound of the fill form at D = 8 (8 spills its sector registers)
#define RNS_ROWS_FILL_OCC 6
#endif
#ifndef RNS_ROWS_FILL_BLOCK  // bytes of the aligned block around the field the fill loads and rewrites
#define RNS_ROWS_FILL_BLOCK 32
#endif
// (Two-byte stores, nontemporal and sc0|sc1 block stores were measured and cost the same or more:
// profiles/r04_fill_store_ab.json.)
template <bool NT, bool BUF, int D, bool FILL = false>
__global__ __launch_bounds__(64, D >= 16 ? 4 : FILL ? RNS_ROWS_FILL_OCC : 8) void csum_rows_kernel(const CsumArgs a)
{
    const uint32_t lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.arena), static_cast<short>(0), static_cast<int>(BUF ? buf_records(a) : 0), 0x00020000);
    const uint64_t recs = buf_records(a);
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * 64;
    const uint64_t p = base + lane;
    const bool live = p < a.n;
    const uint64_t q = live ? p : a.n - 1;  // branch-free descriptor loads
    // (the block offset is loaded per lane at an index the compiler cannot prove uniform:
    // a uniform load goes to SGPRs with a vmcnt(0) wait right away)
    const uint32_t zero_v = __builtin_amdgcn_mbcnt_lo(0u, 0u);
    const uint64_t r0v = a.blk_off[(base >> 6) + zero_v];
    const uint32_t len = live ? static_cast<uint32_t>(a.len16[q]) : 0u;
    const uint32_t seed = (a.seed && live) ? static_cast<uint32_t>(a.seed[q]) : 0u;
    const uint64_t r0 =
        ((static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(r0v >> 32))))
          << 32) |
         static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(r0v)))) +
        a.base_adjust;  // the wave's first packet
    const uint32_t pad = (len + a.align_mask) & ~a.align_mask;
    const uint32_t incl = wave_incl_scan(pad);
    const uint32_t excl = incl - pad;
    const uint32_t total = __builtin_amdgcn_readlane(incl, 63);  // the region's bytes
    const uint64_t start = r0 + excl;
    const bool ok = start <= a.arena_bytes && len <= a.arena_bytes - start;
    // transmit fill: the field, the aligned block of FB bytes around it (a.arena is 16-aligned;
    // the block's alignment is absolute) and whether it lies inside the packet
    constexpr uint32_t FB = FILL ? RNS_ROWS_FILL_BLOCK : 16u, FC = FB / 16u;
    uint32_t fo = 0;
    if constexpr (FILL)
        fo = a.field ? static_cast<uint32_t>(a.field[q]) : a.field_off;
    const bool fok = FILL && live && ok && fo <= len && len - fo >= 2u;  // (no u32 wrap for any field_off)
    const uint64_t fpos = start + fo, fch = fpos & ~15ull;
    const uint32_t back = ((static_cast<uint32_t>(reinterpret_cast<uintptr_t>(a.arena) >> 4) +
                            static_cast<uint32_t>(fch >> 4)) & (FC - 1u)) * 16u;
    const uint64_t sec = fch - back;
    const bool sec_ok = fok && fch >= back && sec + FB <= recs;
    const uint32_t rel = static_cast<uint32_t>(fpos - sec);  // the field's first byte in the block
    uint4 sv[FC];
    uint32_t fb0 = 0, fb1 = 0;  // the field's bytes when the block does not hold both
    if constexpr (FILL) {
#pragma unroll
        for (uint32_t i = 0; i < FC; ++i) {
            if constexpr (BUF) {
                const uint32_t o = sec_ok ? static_cast<uint32_t>(sec) + 16u * i : kOobOffset;
                const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o, 0, 0);
                sv[i] = make_uint4(x.x, x.y, x.z, x.w);
            } else {
                sv[i] = sec_ok ? load_chunk<false>(a.arena + sec + 16u * i) : make_uint4(0, 0, 0, 0);
            }
        }
        if (fok && (!sec_ok || rel == FB - 1u)) {  // rare: odd field at a block end, or the arena's first chunk
            fb0 = a.arena[fpos];
            fb1 = a.arena[fpos + 1];
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    uint32_t mine = 0;
    bool odd = false;
    if ((r0 & 15) == 0) {
        const uint32_t c0 = excl >> 4;
        const uint32_t e = len ? (excl + len - 1) >> 4 : c0;
        mine = rows_region_sum_any<NT, BUF, D>(a, rsrc, recs, r0, total, c0, e, len);
    } else {
        // ---- unaligned region (rare): the whole wave sums one packet at a time ----
        const uint64_t start = r0 + excl;
        const bool ok = start <= a.arena_bytes && len <= a.arena_bytes - start;
        uint64_t todo = __ballot(len != 0 && ok);
        while (todo) {
            const uint32_t o = static_cast<uint32_t>(__builtin_ctzll(todo));
            todo &= todo - 1;
            const uint64_t st =
                (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(start >> 32), o)))
                 << 32) |
                static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(start), o));
            const uint32_t L = __builtin_amdgcn_readlane(len, o);
            const Pkt k = make_pkt(st, L);
            uint32_t acc = 0;
            for (uint32_t cc = 0; cc < k.nch; cc += 64) {
                uint4 w[1];
                issue_pass<64, 1, NT, BUF, 1>(a, rsrc, k, cc + lane, w);
                mask_edges<64, 1, 1>(k, cc + lane, w);
                acc = sum_le<1, 1>(w, acc);
            }
            const uint32_t sum = group_allreduce<64>(acc);
            mine = lane == o ? sum : mine;
        }
        odd = r0 & 1;  // every packet of the range shares the region start's misalignment
    }
    if constexpr (FILL) {
        // the field's bytes out of the sum (LE words pair bytes by absolute parity)
        uint32_t w[4 * FC];
#pragma unroll
        for (uint32_t i = 0; i < FC; ++i) {
            w[4 * i] = sv[i].x;
            w[4 * i + 1] = sv[i].y;
            w[4 * i + 2] = sv[i].z;
            w[4 * i + 3] = sv[i].w;
        }
        uint32_t b0 = fb0, b1 = fb1;
        if (sec_ok && rel != FB - 1u) {
            uint32_t d0 = 0, d1 = 0;
#pragma unroll
            for (uint32_t d = 0; d < 4 * FC; ++d) {
                d0 = (rel >> 2) == d ? w[d] : d0;
                d1 = ((rel + 1u) >> 2) == d ? w[d] : d1;
            }
            b0 = (d0 >> ((rel & 3u) * 8u)) & 0xffu;
            b1 = (d1 >> (((rel + 1u) & 3u) * 8u)) & 0xffu;
        }
        mine -= fok ? (b0 << ((fpos & 1) * 8)) + (b1 << (((fpos + 1) & 1) * 8)) : 0u;
        const uint16_t r = finalize_bits(mine, odd, false, seed, ok && fok, a.flags);
        // set_be16(&mut packet[fo..fo + 2], result): rewrite the largest aligned block (FB, ..., 32
        // bytes) around the field that lies inside the packet, else store the two bytes
        const uint32_t hi = static_cast<uint32_t>(r) >> 8, lo = static_cast<uint32_t>(r) & 0xffu;
        uint8_t *arena_w = const_cast<uint8_t *>(a.arena);
        uint32_t wsz = 0;  // bytes of the block rewritten
#pragma unroll
        for (uint32_t bs = 32; bs <= FB; bs *= 2) {
            const uint64_t bb = sec + (rel & ~(bs - 1u));
            wsz = sec_ok && (rel & (bs - 1u)) != bs - 1u && bb >= start && bb + bs <= start + len ? bs : wsz;
        }
        if (wsz) {
#pragma unroll
            for (uint32_t d = 0; d < 4 * FC; ++d) {
                const uint32_t s0 = (rel & 3u) * 8u, s1 = ((rel + 1u) & 3u) * 8u;
                w[d] = (rel >> 2) == d ? (w[d] & ~(0xffu << s0)) | (hi << s0) : w[d];
                w[d] = ((rel + 1u) >> 2) == d ? (w[d] & ~(0xffu << s1)) | (lo << s1) : w[d];
            }
            const uint32_t c_lo = (rel & ~(wsz - 1u)) >> 4, c_hi = c_lo + (wsz >> 4);
#pragma unroll
            for (uint32_t i = 0; i < FC; ++i)
                if (i >= c_lo && i < c_hi)
                    store_block(reinterpret_cast<uint4 *>(arena_w + sec + 16u * i),
                                make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]));
        } else if (fok) {
            arena_w[fpos] = static_cast<uint8_t>(hi);
            arena_w[fpos + 1] = static_cast<uint8_t>(lo);
        }
    }
    const uint16_t res = finalize_bits(mine, odd, false, seed, ok && (!FILL || fok), a.flags);
    if (live && (!FILL || a.out)) {
        if (a.n < (1u << 30)) {  // buffer store, sc0|sc1 (the stream kernel's measured best, r03o)
            const __amdgpu_buffer_rsrc_t out_rsrc = __builtin_amdgcn_make_buffer_rsrc(
                static_cast<void *>(a.out), static_cast<short>(0), static_cast<int>(2u * a.n), 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b16(res, out_rsrc, static_cast<uint32_t>(2 * p), 0, RNS_STREAM_OUT_AUX);
        } else {
            __builtin_nontemporal_store(res, a.out + p);
        }
    }
    if (a.bad) {
        const uint64_t rejected = __ballot(live && !(ok && (!FILL || fok)));
        if (rejected && lane == 0)
            atomicAdd(a.bad, static_cast<uint32_t>(__popcll(rejected)));
    }
}

// ---------------------------------------------------------------------------
// Tiny fixed-size packets at a fixed stride (rns_csum_batch_strided_dev, c2: 2^20 x 64 B):
// packet i = arena[first_off + i * stride, + len) with len <= 64 and 16-byte-aligned starts,
// so a packet is at most 4 chunks and a wave's 64 packets are 4 rows of 16 packets x 4 chunks
// whose addresses the lanes compute themselves — no descriptors but the seeds, no per-round
// broadcast (the rounds kernel's fetch_pkt), every row of every batch in flight at once.  A
// quad of lanes sums its packet (two DPP steps); the owner lane pulls its packet's sum with one
// ds_bpermute per row and finishes (util.rs:88-106: the LE sum folded and byte-swapped — the
// starts are even — plus the seed, folded).
// ---------------------------------------------------------------------------
template <bool BUF, int B>
__global__ __launch_bounds__(64) void csum_strided_tiny_kernel(const CsumArgs a)
{
    const uint32_t lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.arena), static_cast<short>(0), static_cast<int>(BUF ? buf_records(a) : 0), 0x00020000);
    const uint64_t recs = buf_records(a);
    const uint32_t L = a.fixed_len;  // 1..64
    const uint32_t j = lane & 3u;
    const uint32_t jb = 16u * j;
    const uint64_t start0 = a.first_off + a.base_adjust;
    // the seeds first, with the rows (issued where they are used they cost the wave a second
    // memory latency after its rows: 12.24-12.29 -> 12.06-12.08 us per isolated dispatch, r05m)
    uint32_t sd[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const uint64_t p = (static_cast<uint64_t>(blockIdx.x) * B + b) * 64 + lane;
        sd[b] = 0;
        if (a.seed)
            sd[b] = a.seed[p < a.n ? p : a.n - 1];
    }
    uint4 v[B][4];
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const uint64_t base = (static_cast<uint64_t>(blockIdx.x) * B + b) * 64;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint64_t q = base + 16u * r + (lane >> 2);
            const uint64_t o = start0 + q * a.stride + jb;
            const bool in = q < a.n && jb < L && o + 16 <= recs;
            if constexpr (BUF) {
                const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, in ? static_cast<uint32_t>(o) : kOobOffset, 0,
                                                                      kNtAux);
                v[b][r] = make_uint4(x.x, x.y, x.z, x.w);
            } else {
                const uint4 x = load_chunk<true>(a.arena + (in ? o : 0));
                v[b][r] = in ? x : make_uint4(0, 0, 0, 0);
            }
        }
    }
    const int src = static_cast<int>((lane & 15u) << 4);  // lane 4 * (p & 15) of the owner's row
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const uint64_t base = (static_cast<uint64_t>(blockIdx.x) * B + b) * 64;
        const uint64_t p = base + lane;
        uint32_t mine = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            uint4 x = v[b][r];
            if (jb + 16u > L)  // the packet's last chunk: its bytes past len never count
                x = jb < L ? keep_first(x, L - jb) : make_uint4(0, 0, 0, 0);
            uint32_t t = __builtin_amdgcn_sad_u16(x.x, 0, 0u);
            t = __builtin_amdgcn_sad_u16(x.y, 0, t);
            t = __builtin_amdgcn_sad_u16(x.z, 0, t);
            t = __builtin_amdgcn_sad_u16(x.w, 0, t);
            t = group_allreduce<4>(t);
            const uint32_t got = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(t)));
            mine = (lane >> 4) == static_cast<uint32_t>(r) ? got : mine;
        }
        if (p < a.n) {
            const uint64_t st = start0 + p * a.stride;
            const bool ok = st <= a.arena_bytes && L <= a.arena_bytes - st;
            a.out[p] = finalize_bits(mine, false, false, sd[b], ok, a.flags);  // 64 consecutive u16: one 128-byte store
        }
        if (a.bad) {
            const uint64_t st = start0 + p * a.stride;
            const uint64_t rejected = __ballot(p < a.n && !(st <= a.arena_bytes && L <= a.arena_bytes - st));
            if (rejected && lane == 0)
                atomicAdd(a.bad, static_cast<uint32_t>(__popcll(rejected)));
        }
    }
}

// ---------------------------------------------------------------------------
// Receive verify through the rows decomposition (rns_rx_verify_packed_dev, round 5):
// ip_input_v4 (ip.rs:65-92), ip_input_v6 (ip.rs:114-121), tcp::validate_checksum
// (tcp.rs:838-850), icmp_input_v4/v6 (icmp.rs:44-75) over a packed arena of datagrams.  The
// whole datagram's word sum T comes from csum_rows_kernel's rows (P(e-1) - P(c0-1) + the
// owner's end chunk: no LDS table, no fences); each owner also loads its datagram's first 4
// chunks (64 bytes: every IPv4 header incl. options, the IPv6 header) a group of rows ahead
// of the row that streams them, as it loads its end chunk, and finishes exactly as the class
// kernel's receive verify does (rx_finish: header sum H, pseudo-header from the header's own
// addresses, L4 = T - H).  A unit of ACK-sized datagrams (all <= 64 B) skips the rows: each
// owner loads its datagram whole; a unit that does not start 16-byte aligned takes the
// per-datagram wave loop.
// ---------------------------------------------------------------------------
#ifndef RNS_ROWS_RX_OCC  // waves/SIMD bound of the receive form (its header chunks need registers)
#define RNS_ROWS_RX_OCC 6  // (78 VGPRs, no scratch; 5 with all 4 header chunks loaded with the rows)
#endif
// (Arenas of ACK-sized datagrams — at most 128 arena bytes per datagram — go to csum_stream_kernel,
// whose identical ACK path measured faster there: 64-byte datagrams 14.54-14.64 us per isolated
// dispatch against 15.03-15.25 for this kernel, at 6 or 8 waves/SIMD, with or without an LDS
// reservation like the stream kernel's; sessions r05g, r05h.)
template <bool NT, bool BUF, int D>
__global__ __launch_bounds__(64, RNS_ROWS_RX_OCC) void csum_rows_rx_kernel(const CsumArgs a)
{
    constexpr int kNS = 4;  // header chunks per datagram (16-byte-aligned: its first 64 bytes)
    const uint32_t lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.arena), static_cast<short>(0), static_cast<int>(BUF ? buf_records(a) : 0), 0x00020000);
    const uint64_t recs = buf_records(a);
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * 64;
    const uint64_t p = base + lane;
    const bool live = p < a.n;
    const uint64_t q = live ? p : a.n - 1;  // branch-free descriptor loads
    const uint32_t zero_v = __builtin_amdgcn_mbcnt_lo(0u, 0u);
    const uint64_t r0v = a.blk_off[(base >> 6) + zero_v];
    const uint32_t len = live ? static_cast<uint32_t>(a.len16[q]) : 0u;
    const uint64_t r0 =
        ((static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(r0v >> 32))))
          << 32) |
         static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(r0v)))) +
        a.base_adjust;  // the wave's first datagram
    const uint32_t pad = (len + a.align_mask) & ~a.align_mask;
    const uint32_t incl = wave_incl_scan(pad);
    const uint32_t excl = incl - pad;
    const uint32_t total = __builtin_amdgcn_readlane(incl, 63);  // the region's bytes
    const uint64_t start = r0 + excl;
    const bool ok = start <= a.arena_bytes && len <= a.arena_bytes - start;
    uint32_t mine = 0;
    uint4 own[kNS + 1];
    own[kNS] = make_uint4(0, 0, 0, 0);
    // the owner's finish (rx_finish), called in each path with that path's start offset and
    // parity: constants on the aligned paths, so their finish keeps only the aligned code
    auto finish = [&](uint32_t s0, bool odd) {
        uint32_t l4_res = 0;
        const uint8_t stv = rx_finish<kNS + 1>(a, own, mine, s0, len, odd, false, live && ok && len != 0, l4_res);
        if (live) {
            a.status[p] = stv;
            if (a.l4_out)
                a.l4_out[p] = static_cast<uint16_t>(l4_res);
        }
    };
    if ((r0 & 15) == 0 && !__ballot(len > 64)) {
        // ---- ACK-sized unit: every owner takes its datagram whole ----
#pragma unroll
        for (int i = 0; i < kNS; ++i)  // all four loads in flight before the first is used
            own[i] = own_chunk<BUF>(a, rsrc, recs, start, len, i);
#pragma unroll
        for (int i = 0; i < kNS; ++i) {
            uint4 x = own[i];
            if (16u * i + 16u > len)  // rx_finish sees zeros past the end
                x = 16u * i < len ? keep_first(x, len - 16u * i) : make_uint4(0, 0, 0, 0);
            own[i] = x;
            mine = __builtin_amdgcn_sad_u16(x.x, 0, mine);
            mine = __builtin_amdgcn_sad_u16(x.y, 0, mine);
            mine = __builtin_amdgcn_sad_u16(x.z, 0, mine);
            mine = __builtin_amdgcn_sad_u16(x.w, 0, mine);
        }
        finish(0u, false);
    } else if ((r0 & 15) == 0) {
        // ---- the rows: T, and the owner's first chunks loaded a group ahead ----
        const uint32_t c0 = excl >> 4;
        const uint32_t e = len ? (excl + len - 1) >> 4 : c0;
        // (3 header chunks with the rows, the 4th only where needed: 78 VGPRs, 6 waves/SIMD — IMIX
        // 448.0-448.4 -> 444.8-445.0 us, c3 isolated 234.1-234.3 -> 232.6-232.7 against all 4 at 5
        // waves/SIMD, session r05j)
        mine = rows_region_sum_any<NT, BUF, D, 3>(a, rsrc, recs, r0, total, c0, e, len, own);
        {
            // bytes 48..63 belong to the header only of an IPv4 datagram with more than 28 bytes of
            // options (IHL > 12); the IPv6 header is 40 bytes: those few owners load chunk 3 now
            const uint32_t b0 = own[0].x & 0xffu;
            const bool need = live && len > 48 && (b0 >> 4) == 4 && (b0 & 15u) > 12;
            if (__ballot(need))
                own[3] = need ? own_chunk<BUF>(a, rsrc, recs, start, len, 3) : make_uint4(0, 0, 0, 0);
            else
                own[3] = make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < kNS; ++i)  // zeros past the datagram's end (the region's next bytes)
            if (16u * i + 16u > len)
                own[i] = 16u * i < len ? keep_first(own[i], len - 16u * i) : make_uint4(0, 0, 0, 0);
        finish(0u, false);
    } else {
        // ---- unaligned region (rare): the whole wave sums one datagram at a time ----
        uint64_t todo = __ballot(len != 0 && ok);
        while (todo) {
            const uint32_t o = static_cast<uint32_t>(__builtin_ctzll(todo));
            todo &= todo - 1;
            const uint64_t st =
                (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(start >> 32), o)))
                 << 32) |
                static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(start), o));
            const uint32_t L = __builtin_amdgcn_readlane(len, o);
            const Pkt k = make_pkt(st, L);
            uint32_t acc = 0;
            for (uint32_t cc = 0; cc < k.nch; cc += 64) {
                uint4 w[1];
                issue_pass<64, 1, NT, BUF, 1>(a, rsrc, k, cc + lane, w);
                mask_edges<64, 1, 1>(k, cc + lane, w);
                acc = sum_le<1, 1>(w, acc);
            }
            const uint32_t sum = group_allreduce<64>(acc);
            mine = lane == o ? sum : mine;
        }
        // each owner takes its header from the 16-byte boundary below its start: 5 chunks hold
        // its first 65-80 bytes, masked to the datagram
        const uint64_t b0 = start & ~15ull;
        const uint32_t s0 = static_cast<uint32_t>(start & 15);
#pragma unroll
        for (int i = 0; i < kNS + 1; ++i)
            own[i] = own_chunk<BUF>(a, rsrc, recs, b0, (len && ok) ? s0 + len : 0u, i);
#pragma unroll
        for (int i = 0; i < kNS + 1; ++i) {
            const int lo = static_cast<int>(s0) - 16 * i, hi = static_cast<int>(s0 + len) - 16 * i;
            own[i] = make_uint4(keep_bytes(own[i].x, lo, hi, 0), keep_bytes(own[i].y, lo, hi, 4),
                                keep_bytes(own[i].z, lo, hi, 8), keep_bytes(own[i].w, lo, hi, 12));
        }
        finish(s0, r0 & 1);  // every datagram of the range shares the region start's misalignment
    }
}

// ---------------------------------------------------------------------------
// Transmit-shaped chains (RNS_FLAG_CHAIN_TX_PACKED; rns_csum_chain_dev and
// rns_csum_chain_fill_dev).  What tcp_output checksums (tcp.rs:938-973) is a head fragment
// (the TCP header alloc_header prepended, buf.rs:262-291) followed by the payload.  A batching
// transmit path keeps the heads of consecutive packets back to back in a header region and the
// payloads back to back, 16-byte aligned, in a payload region.  Then a wave's 64 payloads are
// ONE region and stream as csum_rows_kernel's rows (P(e-1) - P(c0-1) + the owner's end chunk),
// while each owner loads its own head (at most 4 chunks; the 64 heads of a wave are one
// contiguous run, so those loads coalesce) and, for the fill, stores its field into it:
// 64 two-byte stores into one short run of lines instead of 64 scattered writes.
//
// The chain is folded as compute_buffer_ones_comp does (util.rs:112-119): acc = fold(seed +
// G(head)), then fold(acc + G(payload)) — the payload's fragments form a run (back to back,
// even non-final lengths: their words pair as one slice's), so the payload is
// one contiguous sum; G(x) is the folded sum in big-endian order (zero iff all bytes zero).
// With the fill the field's two bytes are taken out of the head's exact sum before the fold.
//
// Every lane classifies its packet from its first 1 + kRunFrags descriptors (one round of
// loads after first[]).  A wave whose packets all have that shape (or a defined rejection:
// malformed range, no fragments, a fragment outside the arena, a head too short for its
// field) and whose payloads ascend at 16-byte starts with bounded gaps takes the rows; any
// other wave takes an exact per-packet loop (the whole wave sums one fragment at a time,
// big-endian words mod 2^32: util.rs:88-106 literally), so the hint never changes a result.
// ---------------------------------------------------------------------------
#ifndef RNS_TXROWS_OCC  // waves/SIMD bound of the transmit-rows kernel
#define RNS_TXROWS_OCC 5  // (zero scratch at 86-89 VGPRs; 6 spills 32-116 B/lane)
#endif
constexpr uint32_t kTxHeadMax = 64;  // (head start & 15) + head length: at most 4 chunks

__device__ __forceinline__ uint32_t bswap16_u32(uint32_t x) { return ((x & 0xff) << 8) | (x >> 8); }

template <bool NT, bool BUF, int D, bool FILL>
__global__ __launch_bounds__(64, RNS_TXROWS_OCC) void csum_txrows_kernel(const CsumArgs a)
{
    const uint32_t lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.arena), static_cast<short>(0), static_cast<int>(BUF ? buf_records(a) : 0), 0x00020000);
    const uint64_t recs = buf_records(a);
    const uint64_t p = static_cast<uint64_t>(blockIdx.x) * 64 + lane;
    const bool live = p < a.n;
    const uint32_t f0 = live ? a.first[p] : 0u, f1 = live ? a.first[p + 1] : 0u;
    const bool rng_ok = f0 <= f1 && f1 <= a.n_frags;
    const uint32_t nfr = live && rng_ok ? f1 - f0 : 0u;
    const uint32_t seed = (a.seed && live) ? static_cast<uint32_t>(a.seed[p]) : 0u;
    uint32_t fo = 0;
    if constexpr (FILL)
        fo = live ? (a.field ? static_cast<uint32_t>(a.field[p]) : a.field_off) : 0u;
    // the head and up to kRunFrags payload fragments: one round of descriptor loads
    constexpr uint32_t kF = 1 + kRunFrags;
    uint64_t o[kF];
    uint32_t l[kF];
#pragma unroll
    for (uint32_t j = 0; j < kF; ++j) {
        o[j] = 0;
        l[j] = 0;
        if (j < nfr) {
            o[j] = a.off[f0 + j] + a.base_adjust;
            l[j] = a.len[f0 + j];
        }
    }
    bool all_in = true, run = nfr <= kF;
    uint32_t plen = 0;
#pragma unroll
    for (uint32_t j = 0; j < kF; ++j) {
        if (j < nfr) {
            const bool in = o[j] <= a.arena_bytes && l[j] <= a.arena_bytes - o[j];
            all_in = all_in && in;
            if (j >= 1) {
                run = run && (j == 1 || (o[j] == o[j - 1] + l[j - 1] && !(l[j - 1] & 1u)));
                plen += l[j];
            }
        }
    }
    const uint32_t hl = l[0];
    // defined rejections (every path): bad range, a fragment outside the arena and, for the fill,
    // no fragments or a head too short for the field — the packet gets 0, is counted and is left
    // untouched.  (The checksum of a packet without fragments is its seed, as the reference's
    // loop over no fragments returns initial_sum.)
    bool bad = live && (!rng_ok || (nfr <= kF && !all_in));
    if constexpr (FILL)
        bad = bad || (live && (nfr == 0 || !(fo <= hl && hl - fo >= 2u)));
    const bool has_pay = live && !bad && plen != 0;
    const uint64_t po = o[1];
    const bool shape = !live || bad ||
                       (run && plen <= 0xFFFFu && (o[0] & 15u) + hl <= kTxHeadMax && (!has_pay || (po & 15u) == 0));
    // the wave's payload region: ascending, 16-byte starts, gaps bounded (else the exact loop)
    const uint64_t pm = __ballot(has_pay);
    uint64_t r0 = 0;
    uint32_t rel = 0, c0 = 0, e = 0, total = 0;
    bool region = true;
    if (pm) {
        const uint32_t fl = static_cast<uint32_t>(__builtin_ctzll(pm));
        r0 = (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(po >> 32), fl)))
              << 32) |
             static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(po), fl));
        const uint64_t rel64 = has_pay ? po - r0 : 0;
        const uint32_t pad = has_pay ? (plen + 15u) & ~15u : 0u;
        const bool near = rel64 < (1ull << 30);
        rel = static_cast<uint32_t>(rel64);
        const uint32_t end = has_pay && near ? rel + pad : 0u;
        const uint32_t incl = wave_incl_max(end);
        const uint32_t before = static_cast<uint32_t>(__shfl(static_cast<int>(incl), static_cast<int>(lane) - 1, 64));
        const bool asc = !has_pay || (near && (lane == 0 || rel >= before));
        total = __builtin_amdgcn_readlane(incl, 63);
        const uint32_t sum_pad = __builtin_amdgcn_readlane(wave_incl_scan(pad), 63);
        region = !__ballot(!asc) && total <= 2u * sum_pad + 4096u;
        c0 = has_pay ? rel >> 4 : 0u;
        e = has_pay ? (rel + plen - 1u) >> 4 : 0u;
    }
    const bool fast = !__ballot(!shape) && region;
    uint32_t res = 0;  // the folded sum (before the complement)
    if (fast) {
        // the owner's head: its chunks issued before the rows, consumed after the first group
        const uint64_t hb = o[0] & ~15ull;
        const uint32_t hs = static_cast<uint32_t>(o[0] & 15u), span = live && !bad ? hs + hl : 0u;
        uint4 h[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i)
            h[i] = own_chunk<BUF>(a, rsrc, recs, hb, span, i);
        uint32_t acc1 = 0;
        auto head = [&]() {
            uint32_t hsum = 0;
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i) {
                const int lo = static_cast<int>(hs) - 16 * static_cast<int>(i), hi = static_cast<int>(span) - 16 * static_cast<int>(i);
                hsum = __builtin_amdgcn_sad_u16(keep_bytes(h[i].x, lo, hi, 0), 0, hsum);
                hsum = __builtin_amdgcn_sad_u16(keep_bytes(h[i].y, lo, hi, 4), 0, hsum);
                hsum = __builtin_amdgcn_sad_u16(keep_bytes(h[i].z, lo, hi, 8), 0, hsum);
                hsum = __builtin_amdgcn_sad_u16(keep_bytes(h[i].w, lo, hi, 12), 0, hsum);
            }
            if constexpr (FILL) {  // the field counts as zero (buf.rs:286-288)
                const uint32_t w[16] = {h[0].x, h[0].y, h[0].z, h[0].w, h[1].x, h[1].y, h[1].z, h[1].w,
                                        h[2].x, h[2].y, h[2].z, h[2].w, h[3].x, h[3].y, h[3].z, h[3].w};
                const uint32_t q0 = hs + fo, q1 = q0 + 1u;  // < 64 for a packet that is not rejected
                uint32_t d0 = 0, d1 = 0;
#pragma unroll
                for (uint32_t d = 0; d < 16; ++d) {
                    d0 = (q0 >> 2) == d ? w[d] : d0;
                    d1 = (q1 >> 2) == d ? w[d] : d1;
                }
                const uint32_t b0 = (d0 >> ((q0 & 3u) * 8u)) & 0xffu, b1 = (d1 >> ((q1 & 3u) * 8u)) & 0xffu;
                hsum -= (live && !bad) ? (b0 << ((q0 & 1u) * 8u)) + (b1 << ((q1 & 1u) * 8u)) : 0u;
            }
            const uint32_t x = fold16(hsum);
            const uint32_t g = (o[0] & 1u) ? x : bswap16_u32(x);
            const uint32_t t = seed + g;  // util.rs:89-103 with in_checksum = seed (no wrap: <= 0x1fffe)
            acc1 = (t & 0xffff) + (t >> 16);
        };
        uint32_t mine = 0;
        if (pm) {
            mine = rows_region_sum_any<NT, BUF, D>(a, rsrc, recs, r0, total, c0, e, has_pay ? plen : 0u, nullptr, head);
        } else {
            head();
        }
        const uint32_t x = fold16(mine);
        const uint32_t t = acc1 + bswap16_u32(x);  // the payload starts 16-byte aligned: even
        res = has_pay ? (t & 0xffff) + (t >> 16) : acc1;
    } else {
        // ---- the exact per-packet loop: the whole wave sums one fragment at a time ----
        uint64_t todo = __ballot(live && rng_ok && nfr != 0 && !bad);
        bool lbad = bad;
        res = seed;  // (a packet without fragments)
        while (todo) {
            const uint32_t ow = static_cast<uint32_t>(__builtin_ctzll(todo));
            todo &= todo - 1;
            const uint32_t F0 = __builtin_amdgcn_readlane(f0, ow), F1 = __builtin_amdgcn_readlane(f1, ow);
            const uint32_t FO = __builtin_amdgcn_readlane(fo, ow);
            uint32_t acc = __builtin_amdgcn_readlane(seed, ow);
            bool pbad = false;
            for (uint32_t f = F0; f < F1; ++f) {
                const uint64_t st = a.off[f] + a.base_adjust;
                const uint32_t L = a.len[f];
                if (!(st <= a.arena_bytes && L <= a.arena_bytes - st)) {
                    pbad = true;
                    break;
                }
                if (L == 0)  // an empty fragment adds nothing (the reference panics on it)
                    continue;
                const Pkt k = make_pkt(st, L);
                const uint32_t w_hi = (st & 1) ? 0x01000100u : 0x00010001u;
                const uint64_t fpos = st + FO;  // FILL: the field in the head fragment (f == F0)
                uint32_t hsb = 0, lsb = 0;
                for (uint32_t cc = 0; cc < k.nch; cc += 64) {
                    uint4 w[1];
                    issue_pass<64, 1, NT, BUF, 1>(a, rsrc, k, cc + lane, w);
                    mask_edges<64, 1, 1>(k, cc + lane, w);
                    if (FILL && f == F0) {
                        const uint64_t cs = (st & ~15ull) + (static_cast<uint64_t>(cc + lane) << 4);
                        const int lo = static_cast<int>(static_cast<int64_t>(fpos) - static_cast<int64_t>(cs));
                        if (lo > -2 && lo < 16) {  // zero the field's bytes in this chunk
                            // (keep_bytes keeps [lo, hi) of a dword: here everything but [lo, lo + 2))
                            w[0].x &= ~keep_bytes(0xffffffffu, lo, lo + 2, 0);
                            w[0].y &= ~keep_bytes(0xffffffffu, lo, lo + 2, 4);
                            w[0].z &= ~keep_bytes(0xffffffffu, lo, lo + 2, 8);
                            w[0].w &= ~keep_bytes(0xffffffffu, lo, lo + 2, 12);
                        }
                    }
                    sum_be<1, 1>(w, w_hi, hsb, lsb);
                }
                const uint32_t words = group_allreduce<64>((hsb << 8) + lsb);  // BE words mod 2^32
                acc += words;                                                   // util.rs:89-99
                while (acc > 0xffff)                                            // util.rs:101-103
                    acc = (acc & 0xffff) + (acc >> 16);
            }
            if (lane == ow) {
                res = acc;
                lbad = pbad;
            }
        }
        bad = lbad;
    }
    const bool okp = live && !bad;
    const uint32_t r = (a.flags & RNS_FLAG_COMPLEMENT) ? res ^ 0xffffu : res;
    // (field stores as buffer stores with the result stores' sc0|sc1 bits: IMIX 604.4 -> 598.4 us,
    // c3 251.0 -> 245.7 against ordinary stores; nontemporal 595.8 / 246.4: session r05e)
    if constexpr (FILL) {
        if (okp) {  // set_be16(&mut header[fo..fo + 2], result): the head fragment's bytes
            uint8_t *w8 = const_cast<uint8_t *>(a.arena);
            const uint64_t fp = o[0] + fo;
            if (fp & 1) {
                w8[fp] = static_cast<uint8_t>(r >> 8);
                w8[fp + 1] = static_cast<uint8_t>(r);
            } else if (BUF) {
                __builtin_amdgcn_raw_buffer_store_b16(static_cast<uint16_t>(bswap16_u32(r & 0xffffu)), rsrc,
                                                      static_cast<uint32_t>(fp), 0, RNS_STREAM_OUT_AUX);
            } else {
                *reinterpret_cast<uint16_t *>(w8 + fp) = static_cast<uint16_t>(bswap16_u32(r & 0xffffu));
            }
        }
    }
    if (live && a.out) {
        const uint16_t v = okp ? static_cast<uint16_t>(r) : static_cast<uint16_t>(0);
        if (a.n < (1u << 30)) {
            const __amdgpu_buffer_rsrc_t out_rsrc = __builtin_amdgcn_make_buffer_rsrc(
                static_cast<void *>(a.out), static_cast<short>(0), static_cast<int>(2u * a.n), 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b16(v, out_rsrc, static_cast<uint32_t>(2 * p), 0, RNS_STREAM_OUT_AUX);
        } else {
            __builtin_nontemporal_store(v, a.out + p);
        }
    }
    if (a.bad) {
        const uint64_t rejected = __ballot(live && !okp);
        if (rejected && lane == 0)
            atomicAdd(a.bad, static_cast<uint32_t>(__popcll(rejected)));
    }
}

}  // namespace rns
