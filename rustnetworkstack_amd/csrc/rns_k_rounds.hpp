// The rounds kernel (v2): a wave owns 64 consecutive packets, one size class per launch.
// (One part of rns_kernels.hpp: the parts are included in order, each after the one it builds on.)
#pragma once

#include "rns_k_common.hpp"

namespace rns {

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

}  // namespace rns
