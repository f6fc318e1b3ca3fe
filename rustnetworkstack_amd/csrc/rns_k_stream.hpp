// The packed form's row machinery: the stream kernel (v4, receive verify of ACK-sized units) and
// the rows decomposition (rows_region_sum) the round-4/5 kernels share.
// (One part of rns_kernels.hpp: the parts are included in order, each after the one it builds on.)
#pragma once

#include "rns_k_chain.hpp"

namespace rns {

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
// absolute parity).  Used by csum_rows_kernel, csum_rows_rx_kernel and csum_txrows_kernel (rns_k_rows.hpp).
struct NoHook {
    __device__ __forceinline__ void operator()() const {}
};
// `after_first` runs once the first D rows are issued (a caller's own earlier loads are then
// the oldest in flight: consuming them waits for exactly those, not for the rows).
// NH > 0 (receive verify): the owner also loads its packet's first NH chunks into hv[] (those
// inside the packet; the others read as zero), like its end chunk: a group of rows ahead of
// the row that streams them, so each line is fetched once.
// Buffer loads only: rsrc covers the region (rows_region_sum below gives arenas of 4 GiB or
// more a descriptor based at the region).
template <bool NT, int D, int NH, typename Hook>
__device__ __forceinline__ uint32_t rows_stream(const CsumArgs &a, const __amdgpu_buffer_rsrc_t rsrc, uint64_t recs,
                                               uint64_t r0, uint32_t total, uint32_t c0, uint32_t e, uint32_t len,
                                               uint4 *hv, Hook after_first)
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
    const uint32_t row_e = len ? e >> 6 : 0xFFFFFFFFu;
    // the owners load their end chunks a group of D rows ahead of the rows
    // that hold them (one exec-masked load per group: its line is then still in L2 when the row
    // streams it), not all before the first row
    const uint32_t row_h = len ? c0 >> 6 : 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < NH; ++i)
        hv[i] = make_uint4(0, 0, 0, 0);
    auto load_end_late = [&](uint32_t k) {  // end chunks in rows [k, k + D)
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
    };
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t vlane = lane << 4;
    uint4 v[D];
    auto issue = [&](uint32_t k, uint4 &dst) {  // row k: chunk 64k + lane of the region
        // lanes past the region's end load nothing (a row past it: no traffic at all); the next
        // unit's wave streams those bytes, often on another XCD's L2
        const uint32_t rel = (k << 10) + vlane;
        const uint32_t o = rel < total ? static_cast<uint32_t>(r0) + rel : kOobOffset;
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o, 0, NT ? kNtAux : 0);
        dst = make_uint4(x.x, x.y, x.z, x.w);
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
    uint32_t part = 0;
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
    part = end_part();
    return len ? pb - pa + part : 0u;
}

// The region sum: on an arena below 4 GiB (BUF) through the arena's buffer descriptor; past 4 GiB
// through a buffer descriptor based at the
// region's 128-byte line (a region is at most 64 packets of 64 KiB: far below the buffer range),
// so the rows keep buffer loads with their range checks and cache-policy bits instead of 64-bit
// addresses (per isolated dispatch, session r05s: 3M x 1500 B 815 -> 684 us, 16M IMIX 945 -> 864,
// the transmit-packed chain checksum of 16M IMIX 1263 -> 945).
template <bool NT, bool BUF, int D, int NH = 0, typename Hook = NoHook>
__device__ __forceinline__ uint32_t rows_region_sum(const CsumArgs &a, const __amdgpu_buffer_rsrc_t rsrc, uint64_t recs,
                                                   uint64_t r0, uint32_t total, uint32_t c0, uint32_t e, uint32_t len,
                                                   uint4 *hv = nullptr, Hook after_first = Hook{})
{
    if constexpr (BUF) {
        return rows_stream<NT, D, NH>(a, rsrc, recs, r0, total, c0, e, len, hv, after_first);
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
        return rows_stream<NT, D, NH>(aw, rw, rw_recs, r0 - wb, total, c0, e, len, hv, after_first);
    }
}

}  // namespace rns
