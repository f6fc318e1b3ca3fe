// Common device code of the checksum kernels (one part of rns_kernels.hpp, whose header
// comment describes the approach): kernel arguments, load / mask / sum primitives, the wave
// reductions and the one-lane-group-per-packet batch kernel (v1).
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

}  // namespace rns
