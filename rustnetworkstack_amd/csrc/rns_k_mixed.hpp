// The mixed / class kernel (v3): per-wave size classes, the chunk stash, receive verify and the
// transmit fills over explicit descriptors.
// (One part of rns_kernels.hpp: the parts are included in order, each after the one it builds on.)
#pragma once

#include "rns_k_rounds.hpp"

namespace rns {

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

}  // namespace rns
