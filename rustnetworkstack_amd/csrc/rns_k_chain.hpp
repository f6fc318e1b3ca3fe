// Fragment chains (util.rs:112-119 over NetBuffer chains): the chain kernel.
// (One part of rns_kernels.hpp: the parts are included in order, each after the one it builds on.)
#pragma once

#include "rns_k_mixed.hpp"

namespace rns {

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
            if constexpr (!BUF) {
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

}  // namespace rns
