// The rows kernels: packed checksum and fill, the strided tiny kernel, receive verify through
// the rows, the transmit-shaped chains.
// (One part of rns_kernels.hpp: the parts are included in order, each after the one it builds on.)
#pragma once

#include "rns_k_stream.hpp"

namespace rns {

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
        mine = rows_region_sum<NT, BUF, D>(a, rsrc, recs, r0, total, c0, e, len);
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
        mine = rows_region_sum<NT, BUF, D, 3>(a, rsrc, recs, r0, total, c0, e, len, own);
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
// Receive verify of datagrams at a fixed stride (rns_rx_verify_strided_dev, round 6):
// datagram i = arena[first_off + i * stride, + len16[i]) — a receive ring of fixed-size slots
// (64-byte ACK slots, or the reference's 2048-byte MRU buffers, netif.rs:66).  No block offsets
// and no scan: the lanes compute every address themselves.  With 16-byte-aligned slots a
// 64-datagram batch is read as csum_strided_tiny_kernel reads c2 — 4 rows, lane 4k + j loading
// chunk j of datagram 16r + k in row r (one coalesced KiB per row for 64-byte slots) — and
// lane 4k + j OWNS datagram 16j + k, so everything a datagram's finish needs stays in its quad:
// per row the quad sums its datagram's first 64 bytes (T) and its header bytes (H, IHL from
// byte 0 broadcast in the quad), and the owner (quad lane r) takes T, H and the first 24 bytes
// with quad DPP moves — no LDS, no ds_bpermute.  (Lane-per-datagram loads, as the packed
// form's ACK path does, measured 15.1-15.6 us per isolated dispatch on 1M x 64 B: r06b.)  A
// datagram longer than 64 bytes has its whole sum taken by the wave, one datagram at a time
// (as the packed kernels' unaligned path); its header is in the quad's 64 bytes.  Unaligned
// slots take that loop for every datagram and load their header chunks from the 16-byte
// boundary below the start.  B 64-datagram batches per wave.
// ---------------------------------------------------------------------------
constexpr int kStridedRxB = 1;    // 64-datagram batches per wave (k_packed.hip: launch_strided_rx)
constexpr int kStridedRxOcc = 8;  // waves/SIMD bound (48 VGPRs: 10 fit)
template <bool BUF, int B>
__global__ __launch_bounds__(64, kStridedRxOcc) void csum_strided_rx_kernel(const CsumArgs a)
{
    const uint32_t lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a.arena), static_cast<short>(0), static_cast<int>(BUF ? buf_records(a) : 0), 0x00020000);
    const uint64_t recs = buf_records(a);
    const uint64_t start0 = a.first_off + a.base_adjust;
    const bool aligned = ((start0 | a.stride) & 15) == 0;  // uniform: kernel arguments
    const uint32_t k = lane >> 2, j = lane & 3;
    const uint32_t dl = 16u * j + k;  // the datagram this lane owns, in its batch
    uint32_t len[B];
    uint4 x[B][4];  // row r: chunk j of datagram 16r + k
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const uint64_t base = (static_cast<uint64_t>(blockIdx.x) * B + b) * 64;
        const uint64_t p = base + dl;
        len[b] = p < a.n ? static_cast<uint32_t>(a.len16[p]) : 0u;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint64_t q = base + 16u * r + k;
            const uint64_t o = start0 + q * a.stride + 16u * j;
            const bool in = aligned && q < a.n && o + 16 <= recs;
            if constexpr (BUF) {
                const u32x4 y = __builtin_amdgcn_raw_buffer_load_b128(rsrc, in ? static_cast<uint32_t>(o) : kOobOffset,
                                                                      0, kNtAux);
                x[b][r] = make_uint4(y.x, y.y, y.z, y.w);
            } else {
                const uint4 y = load_chunk<true>(a.arena + (in ? o : 0));
                x[b][r] = in ? y : make_uint4(0, 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const uint64_t p = (static_cast<uint64_t>(blockIdx.x) * B + b) * 64 + dl;
        const bool live = p < a.n;
        const uint32_t L = len[b];
        const uint64_t start = start0 + p * a.stride;
        const bool ok = start <= a.arena_bytes && L <= a.arena_bytes - start;
        const bool present = live && ok && L != 0;
        uint32_t mine = 0;
        uint8_t stv;
        uint32_t l4_res = 0;
        if (aligned) {
            uint32_t H = 0, head[6] = {0, 0, 0, 0, 0, 0};
            auto row = [&](auto rc) {
                constexpr int r = decltype(rc)::value;
                const uint32_t Lr = dpp_mov<r * 0x55>(L);  // the row's datagram 16r + k: owned by quad lane r
                uint4 xm = x[b][r];
                if (16u * j + 16u > Lr)  // bytes past the datagram never count
                    xm = 16u * j < Lr ? keep_first(xm, Lr - 16u * j) : make_uint4(0, 0, 0, 0);
                uint32_t t = __builtin_amdgcn_sad_u16(xm.x, 0, 0u);
                t = __builtin_amdgcn_sad_u16(xm.y, 0, t);
                t = __builtin_amdgcn_sad_u16(xm.z, 0, t);
                t = __builtin_amdgcn_sad_u16(xm.w, 0, t);
                t = group_allreduce<4>(t);
                const uint32_t c0x = dpp_mov<0x00>(xm.x), c0y = dpp_mov<0x00>(xm.y);  // chunk 0 (quad lane 0)
                const uint32_t c0z = dpp_mov<0x00>(xm.z), c0w = dpp_mov<0x00>(xm.w);
                const uint32_t c1x = dpp_mov<0x55>(xm.x), c1y = dpp_mov<0x55>(xm.y);  // chunk 1 (quad lane 1)
                if (j == static_cast<uint32_t>(r)) {
                    mine = t;
                    head[0] = c0x;
                    head[1] = c0y;
                    head[2] = c0z;
                    head[3] = c0w;
                    head[4] = c1x;
                    head[5] = c1y;
                }
            };
            row(std::integral_constant<int, 0>{});
            row(std::integral_constant<int, 1>{});
            row(std::integral_constant<int, 2>{});
            row(std::integral_constant<int, 3>{});
            // H, the header's word sum (IHL*4 bytes, or 40 for IPv6): from the owner's first 20
            // bytes when no datagram of the wave has a longer header (IPv4 without options, the
            // ACK case), else per row from the quad's chunks like T
            const uint32_t hb0 = head[0] & 0xffu, hv = hb0 >> 4;
            const uint32_t hdr = hv == 4 ? (hb0 & 15u) * 4u : hv == 6 ? 40u : 0u;  // <= 60
            if (!__ballot(present && hdr > 20u)) {
#pragma unroll
                for (uint32_t d = 0; d < 5; ++d)
                    H = __builtin_amdgcn_sad_u16(4u * d < hdr ? head[d] : 0u, 0, H);
            } else {
                auto hrow = [&](auto rc) {
                    constexpr int r = decltype(rc)::value;
                    const uint32_t hr = dpp_mov<r * 0x55>(hdr);  // the row's datagram's header length
                    const uint4 xv = x[b][r];
                    uint4 hm = make_uint4(0, 0, 0, 0);
                    if (16u * j < hr)
                        hm = 16u * j + 16u <= hr ? xv : keep_first(xv, hr - 16u * j);
                    uint32_t h = __builtin_amdgcn_sad_u16(hm.x, 0, 0u);
                    h = __builtin_amdgcn_sad_u16(hm.y, 0, h);
                    h = __builtin_amdgcn_sad_u16(hm.z, 0, h);
                    h = __builtin_amdgcn_sad_u16(hm.w, 0, h);
                    h = group_allreduce<4>(h);
                    H = j == static_cast<uint32_t>(r) ? h : H;
                };
                hrow(std::integral_constant<int, 0>{});
                hrow(std::integral_constant<int, 1>{});
                hrow(std::integral_constant<int, 2>{});
                hrow(std::integral_constant<int, 3>{});
            }
            uint64_t todo = __ballot(present && L > 64);
            while (todo) {  // longer datagrams: the whole wave sums one at a time
                const uint32_t o = static_cast<uint32_t>(__builtin_ctzll(todo));
                todo &= todo - 1;
                const uint64_t sto =
                    (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(start >> 32), o)))
                     << 32) |
                    static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(start), o));
                const Pkt pk = make_pkt(sto, __builtin_amdgcn_readlane(L, o));
                uint32_t acc = 0;
                for (uint32_t cc = 0; cc < pk.nch; cc += 64) {
                    uint4 w[1];
                    issue_pass<64, 1, true, BUF, 1>(a, rsrc, pk, cc + lane, w);
                    mask_edges<64, 1, 1>(pk, cc + lane, w);
                    acc = sum_le<1, 1>(w, acc);
                }
                const uint32_t sum = group_allreduce<64>(acc);
                mine = lane == o ? sum : mine;
            }
            // rx_finish with H and the header dwords from the quad (16-byte-aligned: even starts)
            const RxParse rp = present ? rx_parse(head, L, a.local4_sum, a.local6_sum) : RxParse{kMetaMalformed, 0u, 0u};
            uint32_t hdr_res = 0;
            if (!(rp.meta & kMetaMalformed)) {
                hdr_res = finalize_bits(H, false, false, 0u, true, RNS_FLAG_COMPLEMENT);
                if (rp.meta & kMetaL4Checked)
                    l4_res = finalize_bits(mine - H, false, false, rp.ph, true, RNS_FLAG_COMPLEMENT);
            }
            stv = rx_verdict(rp.meta, hdr_res, l4_res);
        } else {
            // ---- unaligned slots (rare): the whole wave sums one datagram at a time ----
            uint64_t todo = __ballot(present);
            while (todo) {
                const uint32_t o = static_cast<uint32_t>(__builtin_ctzll(todo));
                todo &= todo - 1;
                const uint64_t sto =
                    (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(start >> 32), o)))
                     << 32) |
                    static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(start), o));
                const Pkt pk = make_pkt(sto, __builtin_amdgcn_readlane(L, o));
                uint32_t acc = 0;
                for (uint32_t cc = 0; cc < pk.nch; cc += 64) {
                    uint4 w[1];
                    issue_pass<64, 1, true, BUF, 1>(a, rsrc, pk, cc + lane, w);
                    mask_edges<64, 1, 1>(pk, cc + lane, w);
                    acc = sum_le<1, 1>(w, acc);
                }
                const uint32_t sum = group_allreduce<64>(acc);
                mine = lane == o ? sum : mine;
            }
            // the header from the 16-byte boundary below the start: 5 chunks hold its first
            // 65-80 bytes, masked to the datagram
            const uint64_t b0 = start & ~15ull;
            const uint32_t s0 = static_cast<uint32_t>(start & 15);
            uint4 hd[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                hd[i] = own_chunk<BUF>(a, rsrc, recs, b0, present ? s0 + L : 0u, i);
                const int lo = static_cast<int>(s0) - 16 * i, hi = static_cast<int>(s0 + L) - 16 * i;
                hd[i] = make_uint4(keep_bytes(hd[i].x, lo, hi, 0), keep_bytes(hd[i].y, lo, hi, 4),
                                   keep_bytes(hd[i].z, lo, hi, 8), keep_bytes(hd[i].w, lo, hi, 12));
            }
            stv = rx_finish<5>(a, hd, mine, s0, L, start & 1, false, present, l4_res);
        }
        if (live) {  // lane 4k + j: datagram 16j + k (a permutation of 64 consecutive entries)
            a.status[p] = stv;
            if (a.l4_out)
                a.l4_out[p] = static_cast<uint16_t>(l4_res);
        }
    }
}

// ---------------------------------------------------------------------------
// Transmit finalize through the rows decomposition (rns_tx_fill_packed_dev, round 6):
// tcp_output (tcp.rs:957-973), udp_output (udp.rs:151-171), icmp_output_v4/v6
// (icmp.rs:87-112) and ip_output_v4 (ip.rs:140-160) over a packed arena of finished
// datagrams.  The datagram's word sum T comes from the rows as in csum_rows_rx_kernel, and
// its owner holds the first 3 chunks (loaded a group of rows ahead of the row that streams
// them) — the IPv4 header without options, both fields of an IPv4 datagram, both addresses
// of either family; chunks 3-4 are loaded only by the owners that need them (IPv4 options,
// TCP over IPv6).  The owner parses the header, takes the header sum H and the two fields'
// bytes out of T (both fields count as zero: buf.rs:286-288), forms the pseudo-header from
// the header's own addresses and stores each result with one 2-byte store (two-byte stores
// measured no dearer than sector rewrites: profiles/r04_fill_store_ab.json).  The stash
// kernel this replaces needed a class pass, an LDS stash and two 32-byte sector rewrites.
// ---------------------------------------------------------------------------
#ifndef RNS_ROWS_TX_OCC  // waves/SIMD bound of the transmit form
#define RNS_ROWS_TX_OCC 6
#endif
#ifndef RNS_ROWS_TX_FIELD_AUX  // cache-policy bits of the packed finalize's field stores: plain (c3 305.2 /
#define RNS_ROWS_TX_FIELD_AUX 0  // IMIX 809.8 us; nontemporal 322.1 / 836.1, sc0|sc1 310.5 / 820.8: r06w)
#endif
constexpr uint32_t kNoField = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t bswap16_u32(uint32_t x) { return ((x & 0xff) << 8) | (x >> 8); }

// Two big-endian 16-bit words of a dword held little-endian (bytes b0 b1 b2 b3): b0b1 + b2b3.
__device__ __forceinline__ uint32_t be2(uint32_t d)
{
    const uint32_t x = ((d & 0x00ff00ffu) << 8) | ((d >> 8) & 0x00ff00ffu);
    return (x & 0xffffu) + (x >> 16);
}

// The first 40 bytes of a datagram (version, IHL, protocol and both addresses of either
// family) as ten dwords in datagram byte order, from its chunks (s = start & 15; chunk 0 is
// the 16-byte boundary at or below the start; s > 0 needs NS >= 4).
template <int NS>
__device__ __forceinline__ void head40(const uint4 (&ch)[NS], uint32_t s, uint32_t (&h)[10])
{
    uint32_t w[4 * NS];
#pragma unroll
    for (int c = 0; c < NS; ++c) {
        w[4 * c] = ch[c].x;
        w[4 * c + 1] = ch[c].y;
        w[4 * c + 2] = ch[c].z;
        w[4 * c + 3] = ch[c].w;
    }
    if (s == 0) {
#pragma unroll
        for (int k = 0; k < 10; ++k)
            h[k] = w[k];
        return;
    }
    if constexpr (NS >= 4) {
        const uint32_t q = s >> 2, sh = s & 3;
        uint32_t d[11];
#pragma unroll
        for (int k = 0; k < 11; ++k)
            d[k] = q == 0 ? w[k] : q == 1 ? w[k + 1] : q == 2 ? w[k + 2] : w[k + 3];
#pragma unroll
        for (int k = 0; k < 10; ++k)
            h[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
    }
}

// The transmit path's reading of a datagram of L bytes whose first 40 bytes are h (head40)
// and whose IP header must lie within its first hl bytes: the IP header length, the L4 field
// (offset after the IP header: TCP 16, UDP 6, ICMPv4 / ICMPv6 2; kNoField for a protocol the
// stack does not checksum) and the pseudo-header sum the L4 output routine seeds with
// (tcp.rs:957-966, udp.rs:158-165, icmp.rs:97-104; none for ICMPv4, icmp.rs:87-95).  False:
// a datagram the stack cannot produce (bad version, IHL < 5, header past hl).
__device__ __forceinline__ bool tx_parse(const uint32_t (&h)[10], uint32_t L, uint32_t hl, uint32_t &hdr,
                                         uint32_t &field, uint32_t &seed, bool &v4)
{
    const uint32_t b0 = h[0] & 0xffu, version = b0 >> 4;
    uint32_t proto, addr;  // addr: BE word sum of source + destination (tcp.rs:958-966)
    if (version == 4) {
        hdr = (b0 & 15u) * 4u;
        if (hdr < 20 || hdr > hl)
            return false;
        proto = (h[2] >> 8) & 0xffu;            // header[9]
        addr = be2(h[3]) + be2(h[4]);            // header[12..20]
    } else if (version == 6) {
        hdr = 40;
        if (hl < 40)
            return false;
        proto = (h[1] >> 16) & 0xffu;           // header[6]
        addr = 0;
#pragma unroll
        for (int k = 2; k < 10; ++k)             // header[8..40]
            addr += be2(h[k]);
    } else {
        return false;
    }
    v4 = version == 4;
    const uint32_t seg = L - hdr, l16 = seg & 0xffffu;  // packet.len() as u16 (tcp.rs:942, udp.rs:152)
    field = kNoField;
    seed = 0;
    if (proto == 6 || proto == 17) {
        field = proto == 6 ? 16u : 6u;
        seed = fold16(addr + proto + l16);
    } else if (proto == 1 && v4) {
        field = 2;  // icmp_output_v4: no pseudo-header
    } else if (proto == 58 && !v4) {
        field = 2;  // icmp_output_v6: full length, protocol 58
        seed = fold16(addr + 58 + (seg >> 16) + (seg & 0xffffu));
    }
    return true;
}

// Owner-lane finish of transmit finalize for one datagram of L bytes: ch = its chunks from
// the 16-byte boundary at or below its start (raw memory bytes; s = start & 15; NS chunks
// hold bytes up to s + 78: the TCP field behind a 60-byte IPv4 header), mine = the
// datagram's word sum T (LE words at absolute pairing; L <= 65535, so no u32 wrap), odd =
// start & 1.  Exactly the stash kernel's transmit finish (csum_mixed_kernel, TX mode) and
// oracle.tx_fill_ref: fld[0] = 10 for IPv4 (ip_output_v4 over IHL*4 bytes), fld[1] = the
// L4 field (TCP 16, UDP 6, ICMPv4 / ICMPv6 2, after the IP header) when the segment holds
// it; val[] = the values to store big-endian (complemented; UDP's 0 stored as is).
template <int NS>
__device__ __forceinline__ uint8_t tx_finish(const uint4 (&ch)[NS], uint32_t mine, uint32_t s, uint32_t L, bool odd,
                                             bool present, uint32_t (&fld)[2], uint32_t (&val)[2])
{
    fld[0] = fld[1] = kNoField;
    val[0] = val[1] = 0;
    if (!present)
        return RNS_TX_MALFORMED;
    uint32_t h[10];
    head40(ch, s, h);
    uint32_t hdr, field, seed;
    bool v4;
    if (!tx_parse(h, L, L, hdr, field, seed, v4))
        return RNS_TX_MALFORMED;
    const uint32_t seg = L - hdr;
    const int lo = static_cast<int>(s);
    const uint32_t H = stash_sum_le(ch, lo, lo + static_cast<int>(hdr));
    uint8_t st = 0;
    if (v4) {  // compute_checksum(header) with header[10..12] as zero
        fld[0] = 10;
        val[0] = finalize_bits(H - stash_sum_le(ch, lo + 10, lo + 12), odd, false, 0u, true, RNS_FLAG_COMPLEMENT);
        st |= RNS_TX_IP_FILLED;
    }
    if (field != kNoField && seg >= field + 2) {
        const uint32_t f = hdr + field;
        fld[1] = f;
        const uint32_t l4 = mine - H - stash_sum_le(ch, lo + static_cast<int>(f), lo + static_cast<int>(f) + 2);
        val[1] = finalize_bits(l4, odd, false, seed, true, RNS_FLAG_COMPLEMENT);
        st |= RNS_TX_L4_FILLED;
    }
    return st;
}

// The head fragment's part of a chain's transmit finalize (csum_txrows_kernel FIN mode): ch =
// the head's chunks from the 16-byte boundary at or below its start (s = start & 15), hl = its
// length (the IP header and, behind it, the L4 header: alloc_header prepends both into one
// fragment, buf.rs:262-291), L = the datagram's length over every fragment.  ipv = the IPv4
// header checksum to store at head + 10 (ip.rs:140-160); l4f = the L4 field's offset in the
// head (kNoField: no L4 fill — a protocol the stack does not checksum, a segment too short
// for its field, or a field past the head fragment); hsum = the LE word sum of the head's L4
// part with the field as zero (valid when s + hl <= 16 * NS); seed = the pseudo-header sum.
// The L4 part starts at an even distance from the head's start (IHL*4 or 40), so hsum pairs
// exactly as that part would alone.
template <int NS>
__device__ __forceinline__ uint8_t chain_tx_head(const uint4 (&ch)[NS], uint32_t s, uint32_t hl, uint32_t L, bool odd,
                                                 bool present, uint32_t &ipv, uint32_t &l4f, uint32_t &hsum,
                                                 uint32_t &seed, uint32_t &hdr)
{
    ipv = 0;
    l4f = kNoField;
    hsum = 0;
    seed = 0;
    hdr = 0;
    if (!present)
        return RNS_TX_MALFORMED;
    uint32_t h[10];
    head40(ch, s, h);
    uint32_t field;
    bool v4;
    if (!tx_parse(h, L, hl, hdr, field, seed, v4))
        return RNS_TX_MALFORMED;
    const int lo = static_cast<int>(s);
    uint8_t st = 0;
    if (v4) {
        const uint32_t H = stash_sum_le(ch, lo, lo + static_cast<int>(hdr)) - stash_sum_le(ch, lo + 10, lo + 12);
        ipv = finalize_bits(H, odd, false, 0u, true, RNS_FLAG_COMPLEMENT);
        st |= RNS_TX_IP_FILLED;
    }
    if (field != kNoField && L - hdr >= field + 2 && hdr + field + 2 <= hl) {
        l4f = hdr + field;
        const int f = lo + static_cast<int>(l4f);
        hsum = stash_sum_le(ch, lo + static_cast<int>(hdr), lo + static_cast<int>(hl)) - stash_sum_le(ch, f, f + 2);
        st |= RNS_TX_L4_FILLED;
    }
    return st;
}

// set_be16 of a finished field at absolute arena offset fp (util.rs:132-135); AUX = the buffer
// store's cache-policy bits
template <bool BUF, int AUX = 0>
__device__ __forceinline__ void store_field(const CsumArgs &a, __amdgpu_buffer_rsrc_t rsrc, uint64_t fp, uint32_t v)
{
    uint8_t *w8 = const_cast<uint8_t *>(a.arena);
    if (fp & 1) {
        w8[fp] = static_cast<uint8_t>(v >> 8);
        w8[fp + 1] = static_cast<uint8_t>(v);
    } else if constexpr (BUF) {
        __builtin_amdgcn_raw_buffer_store_b16(static_cast<uint16_t>(bswap16_u32(v & 0xffffu)), rsrc,
                                              static_cast<uint32_t>(fp), 0, AUX);
    } else {
        *reinterpret_cast<uint16_t *>(w8 + fp) = static_cast<uint16_t>(bswap16_u32(v & 0xffffu));
    }
}

// (Rewriting each field's whole 64-byte memory segment from the owner's chunks where the segment
// lies inside the datagram — full-segment writes instead of partial ones, which the store probe
// measured cheaper on cold lines — was slower: c3 322.6-323.0 / IMIX 823.4-826.7 us against
// 305.8-306.6 / 810.7-812.8, parity green; it reloads chunks 3-5 after the rows: session r06e.)
template <bool NT, bool BUF, int D>
__global__ __launch_bounds__(64, D >= 16 ? 4 : RNS_ROWS_TX_OCC) void csum_rows_tx_kernel(const CsumArgs a)
{
    constexpr int kNS = 5;  // chunks 0-4: bytes 0..79 of a 16-byte-aligned datagram
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
    const bool present = live && ok && len != 0;
    uint32_t mine = 0;
    uint8_t st = RNS_TX_MALFORMED;
    uint32_t fld[2], val[2];
    // the bytes a datagram's finish reads past chunk 2 (from its first chunk): IPv4 options
    // past byte 48, or an L4 field ending past it (TCP over IPv6, TCP / UDP behind options)
    auto need_bytes = [&](const uint4 c0) -> uint32_t {
        const uint32_t b0 = c0.x & 0xffu, v = b0 >> 4;
        const uint32_t proto = v == 4 ? (c0.z >> 8) & 0xffu : (c0.y >> 16) & 0xffu;
        const uint32_t hdr = v == 4 ? (b0 & 15u) * 4u : 40u;
        const uint32_t fend = hdr + (proto == 6 ? 18u : proto == 17 ? 8u : 4u);
        return v == 4 || v == 6 ? max(hdr, fend) : 0u;
    };
    if ((r0 & 15) == 0) {
        uint4 own[kNS];
#pragma unroll
        for (int i = 3; i < kNS; ++i)
            own[i] = make_uint4(0, 0, 0, 0);
        if (!__ballot(len > 64)) {
            // ---- ACK-sized unit: every owner takes its datagram whole ----
#pragma unroll
            for (int i = 0; i < 4; ++i)
                own[i] = own_chunk<BUF>(a, rsrc, recs, start, len, i);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint4 x = own[i];
                if (16u * i + 16u > len)  // the sum sees none of the bytes past the end
                    x = 16u * i < len ? keep_first(x, len - 16u * i) : make_uint4(0, 0, 0, 0);
                mine = __builtin_amdgcn_sad_u16(x.x, 0, mine);
                mine = __builtin_amdgcn_sad_u16(x.y, 0, mine);
                mine = __builtin_amdgcn_sad_u16(x.z, 0, mine);
                mine = __builtin_amdgcn_sad_u16(x.w, 0, mine);
            }
        } else {
            // ---- the rows: T, and the owner's first 3 chunks loaded a group ahead ----
            const uint32_t c0 = excl >> 4;
            const uint32_t e = len ? (excl + len - 1) >> 4 : c0;
            mine = rows_region_sum<NT, BUF, D, 3>(a, rsrc, recs, r0, total, c0, e, len, own);
            const uint32_t nb = present ? need_bytes(own[0]) : 0u;
            if (__ballot(nb > 48)) {
                own[3] = nb > 48 ? own_chunk<BUF>(a, rsrc, recs, start, len, 3) : make_uint4(0, 0, 0, 0);
                own[4] = nb > 64 ? own_chunk<BUF>(a, rsrc, recs, start, len, 4) : make_uint4(0, 0, 0, 0);
            }
        }
        st = tx_finish<kNS>(own, mine, 0u, len, false, present, fld, val);
    } else {
        // ---- unaligned region (rare): the whole wave sums one datagram at a time ----
        uint64_t todo = __ballot(present);
        while (todo) {
            const uint32_t o = static_cast<uint32_t>(__builtin_ctzll(todo));
            todo &= todo - 1;
            const uint64_t sto =
                (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(start >> 32), o)))
                 << 32) |
                static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(start), o));
            const uint32_t L = __builtin_amdgcn_readlane(len, o);
            const Pkt k = make_pkt(sto, L);
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
        // each owner takes chunks 0-5 from the 16-byte boundary below its start (its first
        // 81-96 bytes)
        const uint64_t b0 = start & ~15ull;
        const uint32_t s0 = static_cast<uint32_t>(start & 15);
        uint4 own[6];
#pragma unroll
        for (int i = 0; i < 6; ++i)
            own[i] = own_chunk<BUF>(a, rsrc, recs, b0, present ? s0 + len : 0u, i);
        st = tx_finish<6>(own, mine, s0, len, start & 1, present, fld, val);
    }
    // (after the wave's loads: a store between a load and its use would join the in-order
    // vmcnt queue)
#pragma unroll
    for (int k = 0; k < 2; ++k)
        if (fld[k] != kNoField)
            store_field<BUF, RNS_ROWS_TX_FIELD_AUX>(a, rsrc, start + fld[k], val[k]);
    if (live && a.status)
        a.status[p] = st;
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
//
// FIN (rns_tx_fill_chain_dev): the whole transmit finalize of such chains — the head fragment
// holds the IP header and the L4 header behind it (alloc_header prepends both into one fragment,
// buf.rs:262-291), so the owner parses its head (chain_tx_head), forms the pseudo-header from the
// head's addresses and the chain's length, sums the head's L4 part, and stores the L4 field and
// the IPv4 header checksum into the head: tcp.rs:957-973, udp.rs:151-171, icmp.rs:87-112,
// ip.rs:140-160 over [head[hdr..], payload...] exactly as compute_buffer_ones_comp folds it.
// Heads of up to 80 bytes from their 16-byte boundary (an IPv6 + TCP head at any start) take
// the rows; the status byte goes to a.status.
// ---------------------------------------------------------------------------
#ifndef RNS_TXROWS_OCC  // waves/SIMD bound of the transmit-rows kernel
#define RNS_TXROWS_OCC 5  // (zero scratch at 86-89 VGPRs; 6 spills 32-116 B/lane)
#endif
constexpr uint32_t kTxHeadMax = 64;  // (head start & 15) + head length: at most 4 chunks (5 for FIN)
#ifndef RNS_TXFIN_RUN_AUX  // cache-policy bits of the run write-back's chunk stores: nontemporal (c3 277.3 ->
#define RNS_TXFIN_RUN_AUX kNtAux  // 270.1 us cold, IMIX 626.4 -> 624.7; plain stores 282.2 / 634.6: r06t)
#endif
#ifndef RNS_TXFIN_RUNWRITE  // FIN: write a wave's back-to-back heads back as whole chunks
#define RNS_TXFIN_RUNWRITE 1  // (IMIX 652.1-652.2 -> 632.5 us, c3 257.3 -> 256.0 against two 2-byte
#endif                        //  stores per head: session r06h, txops / txops_rw)

template <bool NT, bool BUF, int D, bool FILL, bool FIN = false>
__global__ __launch_bounds__(64, RNS_TXROWS_OCC) void csum_txrows_kernel(const CsumArgs a)
{
    static_assert(!(FILL && FIN), "FIN finds its fields itself");
    constexpr uint32_t kNH = FIN ? 5u : 4u;  // head chunks the fast path holds
    constexpr uint32_t kHeadMax = 16u * kNH;
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
    if constexpr (FIN)
        bad = bad || (live && nfr == 0);
    const bool has_pay = live && !bad && plen != 0;
    const uint64_t po = o[1];
    const bool shape = !live || bad ||
                       (run && plen <= 0xFFFFu && (o[0] & 15u) + hl <= kHeadMax && (!has_pay || (po & 15u) == 0));
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
    uint32_t fst = RNS_TX_MALFORMED, ipv = 0, l4f = kNoField;  // FIN: status, IPv4 checksum, L4 field
    // FIN run write-back (RNS_TXFIN_RUNWRITE): a fast wave whose heads lie back to back (one run)
    // stages its raw head chunks in LDS, patches its fields there and writes the run's whole
    // 16-byte chunks back (full 64-byte segments, about half the write requests of two field
    // stores per head); fields in the run's partial edge chunks take the 2-byte stores.
    // (the same write-back for the one-field fill measured no gain: c3 246.8 / IMIX 598.0 us against
    // 246.1 / 597.8, session r06n — its 20-byte heads already leave one request per 64-byte segment)
    constexpr bool kRunWrite = FIN && RNS_TXFIN_RUNWRITE != 0;
    bool runw = false;
    uint64_t b0 = 0, r1 = 0;  // the run's first chunk boundary, its end
    if constexpr (kRunWrite) {
        const uint64_t hend = o[0] + hl;
        const uint64_t pe = (static_cast<uint64_t>(static_cast<uint32_t>(
                                 __shfl(static_cast<int>(hend >> 32), static_cast<int>(lane) - 1, 64)))
                             << 32) |
                            static_cast<uint32_t>(__shfl(static_cast<int>(hend), static_cast<int>(lane) - 1, 64));
        const bool contig = !live || (!bad && (lane == 0 || o[0] == pe));
        runw = fast && !__ballot(!contig);
        const uint32_t last = 63u - static_cast<uint32_t>(__builtin_clzll(__ballot(live)));
        b0 = ((static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(o[0] >> 32))))
               << 32) |
              static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(o[0])))) &
             ~15ull;
        r1 = (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(hend >> 32), last)))
              << 32) |
             static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(hend), last));
    }
    __shared__ uint4 run_lds[kRunWrite ? 64u * kNH + 1u : 1u];
    if (fast) {
        // the owner's head: its chunks issued before the rows, consumed after the first group
        const uint64_t hb = o[0] & ~15ull;
        const uint32_t hs = static_cast<uint32_t>(o[0] & 15u), span = live && !bad ? hs + hl : 0u;
        uint4 h[kNH];
#pragma unroll
        for (uint32_t i = 0; i < kNH; ++i)
            h[i] = own_chunk<BUF>(a, rsrc, recs, hb, span, i);
        uint32_t acc1 = 0;
        auto head = [&]() {
            uint32_t hsum = 0, sd = seed;
            if constexpr (kRunWrite) {
                if (runw) {  // the raw chunks the head touches (neighbours' bytes in them are raw too)
                    const uint32_t q = static_cast<uint32_t>((hb - b0) >> 4);
#pragma unroll
                    for (uint32_t i = 0; i < kNH; ++i)
                        if (16u * i < span)
                            run_lds[q + i] = h[i];
                }
            }
            if constexpr (FIN) {
                uint32_t hd;
                fst = chain_tx_head<kNH>(h, hs, hl, hl + plen, (o[0] & 1u) != 0, live && !bad, ipv, l4f, hsum, sd, hd);
            } else {
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i) {
                const int lo = static_cast<int>(hs) - 16 * static_cast<int>(i), hi = static_cast<int>(span) - 16 * static_cast<int>(i);
                hsum = __builtin_amdgcn_sad_u16(keep_bytes(h[i].x, lo, hi, 0), 0, hsum);
                hsum = __builtin_amdgcn_sad_u16(keep_bytes(h[i].y, lo, hi, 4), 0, hsum);
                hsum = __builtin_amdgcn_sad_u16(keep_bytes(h[i].z, lo, hi, 8), 0, hsum);
                hsum = __builtin_amdgcn_sad_u16(keep_bytes(h[i].w, lo, hi, 12), 0, hsum);
            }
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
            const uint32_t t = sd + g;  // util.rs:89-103 with in_checksum = seed (no wrap: <= 0x1fffe)
            acc1 = (t & 0xffff) + (t >> 16);
        };
        uint32_t mine = 0;
        if (pm) {
            mine = rows_region_sum<NT, BUF, D>(a, rsrc, recs, r0, total, c0, e, has_pay ? plen : 0u, nullptr, head);
        } else {
            head();
        }
        const uint32_t x = fold16(mine);
        const uint32_t t = acc1 + bswap16_u32(x);  // the payload starts 16-byte aligned: even
        res = has_pay ? (t & 0xffff) + (t >> 16) : acc1;
    } else {
        // ---- the exact per-packet loop: the whole wave sums one fragment at a time ----
        uint32_t sd = seed, hd = 0;
        if constexpr (FIN) {
            // the chain's length, and every fragment (not just the first kF) inside the arena
            uint32_t lt = 0;
            bool in = true;
            if (live && rng_ok) {
                for (uint32_t f = f0; f < f1; ++f) {
                    const uint64_t so = a.off[f] + a.base_adjust;
                    const uint32_t lf = a.len[f];
                    in = in && so <= a.arena_bytes && lf <= a.arena_bytes - so;
                    lt += lf;
                }
            }
            bad = bad || (live && !in);
            // the head's first 81-96 bytes from its 16-byte boundary: the IP header and the L4 field
            const uint64_t hb = o[0] & ~15ull;
            const uint32_t s0 = static_cast<uint32_t>(o[0] & 15u);
            uint4 own[6];
#pragma unroll
            for (int i = 0; i < 6; ++i)
                own[i] = own_chunk<BUF>(a, rsrc, recs, hb, live && !bad ? s0 + hl : 0u, i);
            uint32_t hsum;
            fst = chain_tx_head<6>(own, s0, hl, lt, (o[0] & 1u) != 0, live && !bad, ipv, l4f, hsum, sd, hd);
        }
        uint64_t todo = FIN ? __ballot(live && !bad && l4f != kNoField) : __ballot(live && rng_ok && nfr != 0 && !bad);
        bool lbad = bad;
        res = sd;  // (a packet without fragments)
        while (todo) {
            const uint32_t ow = static_cast<uint32_t>(__builtin_ctzll(todo));
            todo &= todo - 1;
            const uint32_t F0 = __builtin_amdgcn_readlane(f0, ow), F1 = __builtin_amdgcn_readlane(f1, ow);
            // FIN: the L4 part of the head starts HD bytes in, its field FO bytes after that
            const uint32_t HD = FIN ? __builtin_amdgcn_readlane(hd, ow) : 0u;
            const uint32_t FO = FIN ? __builtin_amdgcn_readlane(l4f, ow) - HD : __builtin_amdgcn_readlane(fo, ow);
            uint32_t acc = __builtin_amdgcn_readlane(sd, ow);
            bool pbad = false;
            for (uint32_t f = F0; f < F1; ++f) {
                uint64_t st = a.off[f] + a.base_adjust;
                uint32_t L = a.len[f];
                if (!(st <= a.arena_bytes && L <= a.arena_bytes - st)) {
                    pbad = true;
                    break;
                }
                if (FIN && f == F0) {  // the IP header was prepended after the L4 checksum
                    st += HD;
                    L -= HD;
                }
                if (L == 0)  // an empty fragment adds nothing (the reference panics on it)
                    continue;
                const Pkt k = make_pkt(st, L);
                const uint32_t w_hi = (st & 1) ? 0x01000100u : 0x00010001u;
                const uint64_t fpos = st + FO;  // FILL / FIN: the field in the head fragment (f == F0)
                uint32_t hsb = 0, lsb = 0;
                for (uint32_t cc = 0; cc < k.nch; cc += 64) {
                    uint4 w[1];
                    issue_pass<64, 1, NT, BUF, 1>(a, rsrc, k, cc + lane, w);
                    mask_edges<64, 1, 1>(k, cc + lane, w);
                    if ((FILL || FIN) && f == F0) {
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
    const uint32_t r = (FIN || (a.flags & RNS_FLAG_COMPLEMENT)) ? res ^ 0xffffu : res;
    // the fields to store (set_be16 into header_mut()): FIN the L4 field, then ip.rs:158-159's
    // IPv4 header checksum; FILL the caller's field
    constexpr uint64_t kNoPos = ~0ull;
    uint64_t fpos[2] = {kNoPos, kNoPos};
    uint32_t fval[2] = {0u, 0u};
    if constexpr (FIN) {
        if (okp && (fst & RNS_TX_L4_FILLED)) {
            fpos[0] = o[0] + l4f;
            fval[0] = r;
        }
        if (okp && (fst & RNS_TX_IP_FILLED)) {
            fpos[1] = o[0] + 10;
            fval[1] = ipv;
        }
    }
    if constexpr (FILL) {
        if (okp) {
            fpos[0] = o[0] + fo;
            fval[0] = r;
        }
    }
    uint64_t c0w = 0, c1w = 0;  // the run's whole chunks [c0w, c1w) (run write-back)
    if constexpr (kRunWrite) {
        if (runw) {
            uint8_t *l8 = reinterpret_cast<uint8_t *>(run_lds);
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (fpos[k] != kNoPos) {
                    l8[fpos[k] - b0] = static_cast<uint8_t>(fval[k] >> 8);
                    l8[fpos[k] - b0 + 1] = static_cast<uint8_t>(fval[k]);
                }
            }
            __syncthreads();
            c0w = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(o[0] & 15u)) == 0 ? b0 : b0 + 16;
            c1w = r1 & ~15ull;
            uint8_t *w8 = const_cast<uint8_t *>(a.arena);
            for (uint64_t c = c0w + 16u * lane; c < c1w; c += 1024u) {
                const uint4 v = run_lds[(c - b0) >> 4];
                if constexpr (BUF) {
                    const u32x4 y = {v.x, v.y, v.z, v.w};
                    __builtin_amdgcn_raw_buffer_store_b128(y, rsrc, static_cast<uint32_t>(c), 0, RNS_TXFIN_RUN_AUX);
                } else {
                    *reinterpret_cast<uint4 *>(w8 + c) = v;
                }
            }
        }
    }
    // (field stores as buffer stores with the result stores' sc0|sc1 bits: IMIX 604.4 -> 598.4 us,
    // c3 251.0 -> 245.7 against ordinary stores; nontemporal 595.8 / 246.4: session r05e; with the
    // run write-back only the fields not wholly inside its chunks)
#pragma unroll
    for (int k = 0; k < 2; ++k)
        if (fpos[k] != kNoPos && (!runw || fpos[k] < c0w || fpos[k] + 2 > c1w))
            store_field<BUF, RNS_STREAM_OUT_AUX>(a, rsrc, fpos[k], fval[k]);
    if constexpr (FIN) {
        if (live && a.status)
            a.status[p] = okp ? static_cast<uint8_t>(fst) : static_cast<uint8_t>(RNS_TX_MALFORMED);
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
