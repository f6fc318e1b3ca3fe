// The C ABI (include/rns_checksum.h): argument checks, the batch descriptors -> CsumArgs,
// the host-resident pipeline and multi-device contexts.  The kernels are in rns_kernels.hpp
// and are launched from the k_*.hip translation units (rns_launch.hpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "rns_launch.hpp"

using namespace rns;

namespace {

__global__ __launch_bounds__(kBlock) void splitmix64_fill_kernel(uint8_t *buf, uint64_t nbytes, uint64_t seed)
{
    const uint64_t nwords = (nbytes + 7) / 8;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < nwords; i += stride) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z = z ^ (z >> 31);
        if ((i + 1) * 8 <= nbytes) {
            reinterpret_cast<uint64_t *>(buf)[i] = z;
        } else {
            for (uint64_t b = i * 8; b < nbytes; ++b)
                buf[b] = static_cast<uint8_t>(z >> (8 * (b - i * 8)));
        }
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// host-resident pipeline context
// ---------------------------------------------------------------------------
struct rns_host_ctx {
    struct Slot {
        hipStream_t stream = nullptr;
        hipEvent_t done = nullptr;
        uint8_t *d_arena = nullptr;
        uint64_t *d_off = nullptr;
        uint32_t *d_len = nullptr;
        uint16_t *d_seed = nullptr;
        uint16_t *d_out = nullptr;
        uint64_t *h_off = nullptr;  // pinned descriptor staging
        uint32_t *h_len = nullptr;
        uint16_t *h_seed = nullptr;
        uint16_t *h_out = nullptr;
        bool busy = false;
        uint32_t i0 = 0, cnt = 0;
    };
    int device = 0;
    uint64_t chunk_bytes = 0;
    uint32_t chunk_packets = 0;
    std::vector<Slot> slots;
    std::mutex mu;
};

namespace {

void free_ctx(rns_host_ctx *c)
{
    if (!c)
        return;
    (void)hipSetDevice(c->device);
    for (auto &s : c->slots) {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        if (s.done) (void)hipEventDestroy(s.done);
        if (s.stream) (void)hipStreamDestroy(s.stream);
        (void)hipFree(s.d_arena); (void)hipFree(s.d_off); (void)hipFree(s.d_len);
        (void)hipFree(s.d_seed); (void)hipFree(s.d_out);
        (void)hipHostFree(s.h_off); (void)hipHostFree(s.h_len);
        (void)hipHostFree(s.h_seed); (void)hipHostFree(s.h_out);
    }
    delete c;
}

int drain_slot(rns_host_ctx::Slot &s, uint16_t *h_out)
{
    if (!s.busy)
        return RNS_OK;
    s.busy = false;
    int st = hip_status(hipEventSynchronize(s.done));
    if (st == RNS_OK)
        std::memcpy(h_out + s.i0, s.h_out, static_cast<size_t>(s.cnt) * sizeof(uint16_t));
    return st;
}

}  // namespace

// A strided call's offsets first_off + i * stride (+ the base adjustment) must not wrap 64 bits:
// a wrapped offset would name bytes inside the arena that are not packet i's.
static bool strided_fits(uint64_t first_off, uint64_t stride, uint32_t n)
{
    const uint64_t room = ~0ull - 16u - first_off;
    return first_off <= ~0ull - 16u && (n <= 1 || stride <= room / (n - 1));
}

extern "C" {

int rns_csum_batch_dev_cfg(const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_off,
                           const uint32_t *d_len, const uint16_t *d_seed, uint16_t *d_out, uint32_t n,
                           uint32_t flags, uint32_t variant, uint32_t lanes_per_packet, uint32_t unroll,
                           uint32_t max_blocks, uint32_t *d_bad, void *stream)
{
    if (n == 0)
        return RNS_OK;
    if (!d_arena || !d_off || !d_len || !d_out)
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    CsumArgs a{};
    set_arena(a, d_arena, arena_bytes);
    a.off = d_off;
    a.len = d_len;
    a.seed = d_seed;
    a.out = d_out;
    a.bad = d_bad;
    a.n = n;
    a.flags = flags;
    return dispatch<false>(a, variant, lanes_per_packet, unroll, max_blocks, static_cast<hipStream_t>(stream));
}

int rns_csum_batch_dev(const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_off,
                       const uint32_t *d_len, const uint16_t *d_seed, uint16_t *d_out, uint32_t n,
                       uint32_t flags, uint32_t len_hint, uint32_t *d_bad, void *stream)
{
    const Shape sh = pick_shape(len_hint);
    return rns_csum_batch_dev_cfg(d_arena, arena_bytes, d_off, d_len, d_seed, d_out, n, flags, sh.variant, sh.G,
                                  sh.U, sh.max_blocks, d_bad, stream);
}

int rns_csum_batch_dev_off32(const uint8_t *d_arena, uint64_t arena_bytes, const uint32_t *d_off32,
                             const uint32_t *d_len, const uint16_t *d_seed, uint16_t *d_out, uint32_t n,
                             uint32_t flags, uint32_t len_hint, uint32_t *d_bad, void *stream)
{
    if (n == 0)
        return RNS_OK;
    if (!d_arena || !d_off32 || !d_len || !d_out)
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    const Shape sh = pick_shape(len_hint);
    CsumArgs a{};
    set_arena(a, d_arena, arena_bytes);
    a.off32 = d_off32;
    a.len = d_len;
    a.seed = d_seed;
    a.out = d_out;
    a.bad = d_bad;
    a.n = n;
    a.flags = flags;
    return dispatch<false>(a, sh.variant, sh.G, sh.U, sh.max_blocks, static_cast<hipStream_t>(stream));
}

int rns_csum_batch_packed_dev(const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_blk_off,
                              const uint16_t *d_len16, uint32_t align_log2, const uint16_t *d_seed, uint16_t *d_out,
                              uint32_t n, uint32_t flags, uint32_t len_hint, uint32_t *d_bad, void *stream)
{
    if (n == 0)
        return RNS_OK;
    if (!d_arena || !d_blk_off || !d_len16 || !d_out || align_log2 > 12)
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    Shape sh = pick_shape(len_hint);
    if ((sh.variant & 5u) == 0)  // the group kernel has no 64-packet wave batches: mixed kernel, nontemporal
        sh = Shape{6u, 0u, 0u, 0u};

    CsumArgs a{};
    set_arena(a, d_arena, arena_bytes);
    a.len16 = d_len16;
    a.blk_off = d_blk_off;
    a.align_mask = (1u << align_log2) - 1u;
    a.seed = d_seed;
    a.out = d_out;
    a.bad = d_bad;
    a.n = n;
    a.flags = flags;
    a.len_hint = len_hint;
    return dispatch_packed(a, sh, static_cast<hipStream_t>(stream));
}

int rns_csum_batch_strided_dev(const uint8_t *d_arena, uint64_t arena_bytes, uint64_t first_off,
                               uint64_t stride, uint32_t len, const uint16_t *d_seed, uint16_t *d_out,
                               uint32_t n, uint32_t flags, uint32_t *d_bad, void *stream)
{
    if (n == 0)
        return RNS_OK;
    if (!d_arena || !d_out || !strided_fits(first_off, stride, n))
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    CsumArgs a{};
    set_arena(a, d_arena, arena_bytes);
    a.seed = d_seed;
    a.out = d_out;
    a.bad = d_bad;
    a.first_off = first_off;
    a.stride = stride;
    a.fixed_len = len;
    a.n = n;
    a.flags = flags;
    // packets of at most 64 bytes at 16-byte-aligned starts: the strided tiny kernel (c2 isolated
    // 12.83-12.94 -> 12.24-12.29 us against the rounds kernel: sessions r05g, r05h)
    if (len != 0 && len <= 64 && ((first_off + a.base_adjust) & 15) == 0 && (stride & 15) == 0)
        return launch_strided_tiny(a, static_cast<hipStream_t>(stream));
    const Shape sh = pick_shape(len);
    return dispatch<true>(a, sh.variant, sh.G, sh.U, sh.max_blocks, static_cast<hipStream_t>(stream));
}

}  // extern "C"

// Fragment chains: the chain kernel's arguments and launch (checksum or head-fragment fill).
template <bool FILL>
static int chain_launch(CsumArgs &a, const uint64_t *d_frag_off, const uint32_t *d_frag_len, uint32_t n_frags,
                        const uint32_t *d_first, uint32_t n_pkts, uint32_t flags, uint32_t frag_len_hint,
                        hipStream_t stream)
{
    // the chain kernel adds packet indices in 32 bits (a VGPR less across its class pass): its
    // last wave's base + 64 * K + lane must not wrap
    static_assert(RNS_CHAIN_MAX_PACKETS == 0xFFFFFFFFu - 64u * kChainMaxK, "rns_checksum.h's chain cap");
    if (n_pkts > RNS_CHAIN_MAX_PACKETS)
        return RNS_E_INVALID;
    a.off = d_frag_off;
    a.len = d_frag_len;
    a.n = n_pkts;
    a.flags = flags;
    a.first = d_first;
    a.n_frags = n_frags;
    // Packets per lane K: the wave's K*64 packets should bring whole 64-fragment
    // batches (a partial batch runs the class rounds for few bytes), so pick the K
    // in 1..8 whose expected fragment count K*mean fills its batches best.
    const double mean = static_cast<double>(n_frags) / static_cast<double>(n_pkts);
    uint32_t K = 1;
    double best = -1.0;
    for (uint32_t k = 1; k <= kChainMaxK; ++k) {
        const double fr = k * mean, fill = fr > 0 ? fr / std::ceil(fr) : 1.0;
        if (fill > best + 0.02) {
            best = fill;
            K = k;
        }
    }
    a.chain_k = K;
    // transmit-shaped chains: heads + a packed payload region.  A batch whose mean fragment
    // count already exceeds the shape (a head + kRunFrags payload fragments) has most of its
    // waves in the transmit-rows kernel's exact per-packet loop — far slower than the chain
    // kernel on the same chains — so the hint is ignored there (same results either way).
    if ((flags & RNS_FLAG_CHAIN_TX_PACKED) && mean <= 1.0 + kRunFrags)
        return launch_txrows<FILL>(a, stream);
    // Nontemporal loads for NetBuffer-sized fragments (c3 as 3 fragments: 298 -> 289 us
    // packed back to back, 281 -> 261 us in 512-byte buffers), not for IMIX's mix of
    // 40-byte packets and 512-byte fragments (646 -> 670 us): profiles/archive/r02/r02_chain_ab.json.
#ifndef RNS_CHAIN_NT_FROM  // fragment-length hints from this take the nontemporal instantiation
#define RNS_CHAIN_NT_FROM 384u
#endif
    const bool nt = (frag_len_hint ? frag_len_hint : 512u) >= RNS_CHAIN_NT_FROM;
    // RNS_FLAG_CHAIN_RUNS: the run-checking kernel (buffer path; a hint, ignored otherwise)
    const bool runs = kChainRuns && (flags & RNS_FLAG_CHAIN_RUNS) && buf_records(a) < kOobOffset;
    return launch_chain<FILL>(a, K, nt, runs, stream);
}

extern "C" {

int rns_csum_chain_dev(const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_frag_off,
                       const uint32_t *d_frag_len, uint32_t n_frags, const uint32_t *d_first,
                       const uint16_t *d_seed, uint16_t *d_out, uint32_t n_pkts, uint32_t flags,
                       uint32_t frag_len_hint, uint16_t *d_frag_sums, uint32_t *d_bad, void *stream)
{
    (void)d_frag_sums;  // scratch of the two-pass form (round 1); the one-pass kernel needs none
    if (n_pkts == 0)
        return RNS_OK;
    if (!d_arena || !d_first || !d_out || (n_frags && (!d_frag_off || !d_frag_len)))
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    CsumArgs a{};
    set_arena(a, d_arena, arena_bytes);
    a.seed = d_seed;
    a.out = d_out;
    a.bad = d_bad;
    return chain_launch<false>(a, d_frag_off, d_frag_len, n_frags, d_first, n_pkts, flags, frag_len_hint,
                               static_cast<hipStream_t>(stream));
}

int rns_csum_chain_fill_dev(uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_frag_off,
                            const uint32_t *d_frag_len, uint32_t n_frags, const uint32_t *d_first,
                            const uint16_t *d_seed, const uint16_t *d_field, uint32_t field_off, uint16_t *d_out,
                            uint32_t n_pkts, uint32_t flags, uint32_t frag_len_hint, uint32_t *d_bad, void *stream)
{
    if (n_pkts == 0)
        return RNS_OK;
    if (!d_arena || !d_first || (n_frags && (!d_frag_off || !d_frag_len)))
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    CsumArgs a{};
    set_arena(a, d_arena, arena_bytes);
    a.seed = d_seed;
    a.out = d_out;
    a.bad = d_bad;
    a.field = d_field;
    a.field_off = field_off;
    return chain_launch<true>(a, d_frag_off, d_frag_len, n_frags, d_first, n_pkts, flags, frag_len_hint,
                              static_cast<hipStream_t>(stream));
}

// Grid of the stash-mode kernels (one 64-datagram batch per one-wave workgroup).  Batches
// of tiny datagrams (arena bytes per datagram <= 128: ACK-sized) run on a capped grid, each
// wave looping over several batches: one-batch waves are mostly launch ramp there (64 B
// verify 18.9 -> 17.2-17.8 us per step); larger datagrams keep one wave per batch (a cap
// measured 3-6 % slower on IMIX; profiles/r02_rx_cap_ab.json).
constexpr uint64_t kRxGridCap = 4096;  // the cap for tiny datagrams
// Receive verify and transmit finalize take the cap (64 B finalize 35.2-36.3 -> 33.3 us);
// the single-field fill does not (64 B fill 28.9-29.2 us without, 29.8-30.0 with it:
// profiles/r02_tx_cap_ab.json).
static uint64_t stash_blocks(uint64_t n, uint64_t arena_bytes, bool tiny_cap)
{
    constexpr int BLK = kMixedBlock<true>;
    uint64_t blocks = ((n + 63) / 64 + BLK / 64 - 1) / (BLK / 64);
    const bool cap = tiny_cap && arena_bytes / n <= 128;
    if (cap && blocks > kRxGridCap)
        blocks = kRxGridCap;
    return blocks;
}

int rns_csum_fill_dev(uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_off, const uint32_t *d_len,
                      const uint16_t *d_seed, const uint16_t *d_field, uint32_t field_off, uint16_t *d_out,
                      uint32_t n, uint32_t flags, uint32_t *d_bad, void *stream)
{
    if (n == 0)
        return RNS_OK;
    if (!d_arena || !d_off || !d_len)
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    CsumArgs a{};
    set_arena(a, d_arena, arena_bytes);
    a.off = d_off;
    a.len = d_len;
    a.seed = d_seed;
    a.out = d_out;
    a.bad = d_bad;
    a.n = n;
    a.flags = flags;
    a.field = d_field;
    a.field_off = field_off;
    return launch_fill(a, dim3(static_cast<uint32_t>(stash_blocks(n, arena_bytes, false))),
                       static_cast<hipStream_t>(stream));
}

int rns_csum_fill_packed_dev(uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_blk_off, const uint16_t *d_len16,
                             uint32_t align_log2, const uint16_t *d_seed, const uint16_t *d_field, uint32_t field_off,
                             uint16_t *d_out, uint32_t n, uint32_t flags, uint32_t len_hint, uint32_t *d_bad,
                             void *stream)
{
    if (n == 0)
        return RNS_OK;
    if (!d_arena || !d_blk_off || !d_len16 || align_log2 < 4 || align_log2 > 12)
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    CsumArgs a{};
    set_arena(a, d_arena, arena_bytes);
    a.len16 = d_len16;
    a.blk_off = d_blk_off;
    a.align_mask = (1u << align_log2) - 1u;
    a.seed = d_seed;
    a.out = d_out;
    a.bad = d_bad;
    a.n = n;
    a.flags = flags;
    a.field = d_field;
    a.field_off = field_off;
    a.len_hint = len_hint;
    return launch_fill_packed(a, static_cast<hipStream_t>(stream));
}

static uint32_t be_sum(const uint8_t *p, int nbytes)
{
    uint32_t s = 0;
    for (int k = 0; k < nbytes; k += 2)
        s += static_cast<uint32_t>(p[k]) << 8 | p[k + 1];
    return s;
}

int rns_rx_verify_dev(const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_off, const uint32_t *d_len,
                      uint32_t n, const uint8_t *local_ipv4, const uint8_t *local_ipv6, uint8_t *d_status,
                      uint16_t *d_l4_sum, void *stream)
{
    if (n == 0)
        return RNS_OK;
    if (!d_arena || !d_off || !d_len || !d_status || !local_ipv4 || !local_ipv6)
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    CsumArgs a{};
    set_arena(a, d_arena, arena_bytes);
    a.off = d_off;
    a.len = d_len;
    a.n = n;
    a.flags = RNS_FLAG_COMPLEMENT;
    a.status = d_status;
    a.l4_out = d_l4_sum;
    a.local4_sum = be_sum(local_ipv4, 4);
    a.local6_sum = be_sum(local_ipv6, 16);
    return launch_rx(a, dim3(static_cast<uint32_t>(stash_blocks(n, arena_bytes, true))),
                     static_cast<hipStream_t>(stream));
}

int rns_rx_verify_packed_dev(const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_blk_off,
                             const uint16_t *d_len16, uint32_t align_log2, uint32_t n, const uint8_t *local_ipv4,
                             const uint8_t *local_ipv6, uint8_t *d_status, uint16_t *d_l4_sum, void *stream)
{
    if (n == 0)
        return RNS_OK;
    if (!d_arena || !d_blk_off || !d_len16 || !d_status || !local_ipv4 || !local_ipv6 || align_log2 < 4 ||
        align_log2 > 12)
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    CsumArgs a{};
    set_arena(a, d_arena, arena_bytes);
    a.len16 = d_len16;
    a.blk_off = d_blk_off;
    a.align_mask = (1u << align_log2) - 1u;
    a.n = n;
    a.flags = RNS_FLAG_COMPLEMENT;
    a.status = d_status;
    a.l4_out = d_l4_sum;
    a.local4_sum = be_sum(local_ipv4, 4);
    a.local6_sum = be_sum(local_ipv6, 16);
    return launch_stream_rx(a, static_cast<hipStream_t>(stream));
}

int rns_rx_verify_strided_dev(const uint8_t *d_arena, uint64_t arena_bytes, uint64_t first_off, uint64_t stride,
                              const uint16_t *d_len16, uint32_t n, const uint8_t *local_ipv4, const uint8_t *local_ipv6,
                              uint8_t *d_status, uint16_t *d_l4_sum, void *stream)
{
    if (n == 0)
        return RNS_OK;
    if (!d_arena || !d_len16 || !d_status || !local_ipv4 || !local_ipv6 || !strided_fits(first_off, stride, n))
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    CsumArgs a{};
    set_arena(a, d_arena, arena_bytes);
    a.len16 = d_len16;
    a.first_off = first_off;
    a.stride = stride;
    a.n = n;
    a.flags = RNS_FLAG_COMPLEMENT;
    a.status = d_status;
    a.l4_out = d_l4_sum;
    a.local4_sum = be_sum(local_ipv4, 4);
    a.local6_sum = be_sum(local_ipv6, 16);
    return launch_strided_rx(a, static_cast<hipStream_t>(stream));
}

int rns_tx_fill_packed_dev(uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_blk_off, const uint16_t *d_len16,
                           uint32_t align_log2, uint32_t n, uint8_t *d_status, uint32_t len_hint, void *stream)
{
    if (n == 0)
        return RNS_OK;
    if (!d_arena || !d_blk_off || !d_len16 || align_log2 < 4 || align_log2 > 12)
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    CsumArgs a{};
    set_arena(a, d_arena, arena_bytes);
    a.len16 = d_len16;
    a.blk_off = d_blk_off;
    a.align_mask = (1u << align_log2) - 1u;
    a.n = n;
    a.flags = RNS_FLAG_COMPLEMENT;
    a.status = d_status;
    a.len_hint = len_hint;
    return launch_tx_packed(a, static_cast<hipStream_t>(stream));
}

int rns_tx_fill_chain_dev(uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_frag_off, const uint32_t *d_frag_len,
                          uint32_t n_frags, const uint32_t *d_first, uint32_t n_pkts, uint8_t *d_status, void *stream)
{
    if (n_pkts == 0)
        return RNS_OK;
    if (!d_arena || !d_first || (n_frags && (!d_frag_off || !d_frag_len)) || n_pkts > RNS_CHAIN_MAX_PACKETS)
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    CsumArgs a{};
    set_arena(a, d_arena, arena_bytes);
    a.off = d_frag_off;
    a.len = d_frag_len;
    a.first = d_first;
    a.n_frags = n_frags;
    a.n = n_pkts;
    a.flags = RNS_FLAG_COMPLEMENT;
    a.status = d_status;
    return launch_txfin(a, static_cast<hipStream_t>(stream));
}

int rns_tx_fill_dev(uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_off, const uint32_t *d_len,
                    uint32_t n, uint8_t *d_status, void *stream)
{
    if (n == 0)
        return RNS_OK;
    if (!d_arena || !d_off || !d_len)
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    CsumArgs a{};
    set_arena(a, d_arena, arena_bytes);
    a.off = d_off;
    a.len = d_len;
    a.n = n;
    a.flags = RNS_FLAG_COMPLEMENT;
    a.status = d_status;
    return launch_tx(a, dim3(static_cast<uint32_t>(stash_blocks(n, arena_bytes, true))),
                     static_cast<hipStream_t>(stream));
}

int rns_host_ctx_create(int device, uint64_t chunk_bytes, uint32_t nstreams, rns_host_ctx **out)
{
    if (!out || nstreams == 0 || nstreams > 16 || chunk_bytes < 4096)
        return RNS_E_INVALID;
    *out = nullptr;
    if (int st = check_device())
        return st;
    int st = hip_status(hipSetDevice(device));
    if (st)
        return st;
    rns_host_ctx *c = new (std::nothrow) rns_host_ctx;
    if (!c)
        return RNS_E_INVALID;
    c->device = device;
    c->chunk_bytes = (chunk_bytes + 255) & ~255ull;
    c->chunk_packets = static_cast<uint32_t>(std::min<uint64_t>(c->chunk_bytes / 16, 1u << 24));
    c->slots.resize(nstreams);
    const size_t np = c->chunk_packets;
    for (auto &s : c->slots) {
        hipError_t e = hipSuccess;
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&s.d_arena), c->chunk_bytes + 256);
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&s.d_off), np * sizeof(uint64_t));
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&s.d_len), np * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&s.d_seed), np * sizeof(uint16_t));
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&s.d_out), np * sizeof(uint16_t));
        if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&s.h_off), np * sizeof(uint64_t), 0);
        if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&s.h_len), np * sizeof(uint32_t), 0);
        if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&s.h_seed), np * sizeof(uint16_t), 0);
        if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&s.h_out), np * sizeof(uint16_t), 0);
        if (e != hipSuccess) {
            free_ctx(c);
            return hip_status(e);
        }
    }
    *out = c;
    return RNS_OK;
}

int rns_host_ctx_destroy(rns_host_ctx *ctx)
{
    free_ctx(ctx);
    return RNS_OK;
}

int rns_csum_batch_host(rns_host_ctx *ctx, const uint8_t *h_arena, uint64_t arena_bytes,
                        const uint64_t *h_off, const uint32_t *h_len, const uint16_t *h_seed,
                        uint16_t *h_out, uint32_t n, uint32_t flags)
{
    if (!ctx)
        return RNS_E_INVALID;
    if (n == 0)
        return RNS_OK;
    if (!h_arena || !h_off || !h_len || !h_out)
        return RNS_E_INVALID;
    // Validate the whole batch first so a bad descriptor never reaches the device and
    // nothing is queued for a batch that cannot finish.  A chunk starts at its first
    // packet's offset rounded down to 256 bytes, so a packet fits a staging chunk iff
    // (off mod 256) + len <= chunk_bytes.
    for (uint32_t i = 0; i < n; ++i) {
        if (h_off[i] > arena_bytes || h_len[i] > arena_bytes - h_off[i])
            return RNS_E_BOUNDS;
        if (i && h_off[i] < h_off[i - 1])
            return RNS_E_ORDER;
        if ((h_off[i] & 255u) + h_len[i] > ctx->chunk_bytes)
            return RNS_E_TOOLARGE;
    }
    std::lock_guard<std::mutex> lock(ctx->mu);
    int st = hip_status(hipSetDevice(ctx->device));
    if (st)
        return st;
    const size_t nslots = ctx->slots.size();
    size_t k = 0;
    uint32_t i0 = 0;
    while (i0 < n && st == RNS_OK) {
        // Chunk: packets [i0, i1) whose bytes fit one staging buffer.
        const uint64_t lo = h_off[i0] & ~255ull;  // keeps 16-byte alignment and byte parity
        uint64_t hi = lo;
        uint32_t i1 = i0;
        while (i1 < n && i1 - i0 < ctx->chunk_packets) {
            const uint64_t end = std::max(hi, h_off[i1] + h_len[i1]);
            if (end - lo > ctx->chunk_bytes)
                break;
            hi = end;
            ++i1;
        }
        if (i1 == i0) {  // (excluded by the validation pass; never leave queued slots undrained)
            st = RNS_E_TOOLARGE;
            break;
        }
        auto &s = ctx->slots[k++ % nslots];
        st = drain_slot(s, h_out);
        if (st)
            break;
        const uint32_t cnt = i1 - i0;
        std::memcpy(s.h_off, h_off + i0, cnt * sizeof(uint64_t));
        std::memcpy(s.h_len, h_len + i0, cnt * sizeof(uint32_t));
        if (h_seed)
            std::memcpy(s.h_seed, h_seed + i0, cnt * sizeof(uint16_t));
        hipError_t e = hipMemcpyAsync(s.d_arena, h_arena + lo, hi - lo, hipMemcpyHostToDevice, s.stream);
        if (e == hipSuccess) e = hipMemcpyAsync(s.d_off, s.h_off, cnt * sizeof(uint64_t), hipMemcpyHostToDevice, s.stream);
        if (e == hipSuccess) e = hipMemcpyAsync(s.d_len, s.h_len, cnt * sizeof(uint32_t), hipMemcpyHostToDevice, s.stream);
        if (e == hipSuccess && h_seed)
            e = hipMemcpyAsync(s.d_seed, s.h_seed, cnt * sizeof(uint16_t), hipMemcpyHostToDevice, s.stream);
        if (e != hipSuccess) {
            st = hip_status(e);
            break;
        }
        // Offsets stay absolute: the kernel sees arena = staging - lo (never dereferenced below staging).
        CsumArgs a{};
        a.arena = s.d_arena - lo;
        a.arena_bytes = hi;
        a.base_adjust = 0;
        a.off = s.d_off;
        a.len = s.d_len;
        a.seed = h_seed ? s.d_seed : nullptr;
        a.out = s.d_out;
        a.n = cnt;
        a.flags = flags;
        const Shape sh = pick_shape(static_cast<uint32_t>(std::min<uint64_t>((hi - lo) / cnt, 1u << 30)));
        st = dispatch<false>(a, sh.variant, sh.G, sh.U, sh.max_blocks, s.stream);
        if (st)
            break;
        e = hipMemcpyAsync(s.h_out, s.d_out, cnt * sizeof(uint16_t), hipMemcpyDeviceToHost, s.stream);
        if (e == hipSuccess) e = hipEventRecord(s.done, s.stream);
        if (e != hipSuccess) {
            st = hip_status(e);
            break;
        }
        s.busy = true;
        s.i0 = i0;
        s.cnt = cnt;
        i0 = i1;
    }
    for (auto &s : ctx->slots) {
        int d = drain_slot(s, h_out);
        if (st == RNS_OK)
            st = d;
    }
    return st;
}

// ---------------------------------------------------------------------------
// Multi-GPU batches: packets are independent, so a batch
// is cut into contiguous packet ranges of about equal BYTES, one per GPU; each GPU
// checksums its range from its own HBM (device-resident) or through its own
// staging context and PCIe link (host-resident).  No bytes cross xGMI and no
// collective is needed: each range's results land in their slice of h_out.
// ---------------------------------------------------------------------------
struct rns_multi_ctx {
    std::vector<rns_host_ctx *> ctx;
};

int rns_multi_ctx_create(const int *devices, uint32_t ndev, uint64_t chunk_bytes, uint32_t nstreams,
                         rns_multi_ctx **out)
{
    if (!out || !devices || ndev == 0 || ndev > 64)
        return RNS_E_INVALID;
    *out = nullptr;
    rns_multi_ctx *m = new (std::nothrow) rns_multi_ctx;
    if (!m)
        return RNS_E_INVALID;
    for (uint32_t i = 0; i < ndev; ++i) {
        rns_host_ctx *c = nullptr;
        const int st = rns_host_ctx_create(devices[i], chunk_bytes, nstreams, &c);
        if (st) {
            rns_multi_ctx_destroy(m);
            return st;
        }
        m->ctx.push_back(c);
    }
    *out = m;
    return RNS_OK;
}

int rns_multi_ctx_destroy(rns_multi_ctx *ctx)
{
    if (ctx) {
        for (rns_host_ctx *c : ctx->ctx)
            rns_host_ctx_destroy(c);
        delete ctx;
    }
    return RNS_OK;
}

extern "C++" {
namespace {
// Cut [0, n) into `parts` contiguous ranges of about equal byte totals: bounds[0..parts].
std::vector<uint32_t> split_by_bytes(const uint32_t *len, uint32_t n, uint32_t parts)
{
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i)
        total += len[i];
    std::vector<uint32_t> bounds(parts + 1, n);
    bounds[0] = 0;
    uint64_t acc = 0;
    uint32_t i = 0;
    for (uint32_t k = 1; k < parts; ++k) {
        const uint64_t target = total * k / parts;
        while (i < n && acc + len[i] <= target)
            acc += len[i++];
        bounds[k] = std::max(i, bounds[k - 1]);
    }
    return bounds;
}
}  // namespace
}  // extern "C++"

int rns_csum_batch_multi_host(rns_multi_ctx *ctx, const uint8_t *h_arena, uint64_t arena_bytes,
                              const uint64_t *h_off, const uint32_t *h_len, const uint16_t *h_seed,
                              uint16_t *h_out, uint32_t n, uint32_t flags)
{
    if (!ctx || ctx->ctx.empty())
        return RNS_E_INVALID;
    if (n == 0)
        return RNS_OK;
    if (!h_arena || !h_off || !h_len || !h_out)
        return RNS_E_INVALID;
    const uint32_t parts = static_cast<uint32_t>(ctx->ctx.size());
    const std::vector<uint32_t> b = split_by_bytes(h_len, n, parts);
    std::vector<int> st(parts, RNS_OK);
    auto run = [&](uint32_t k) {
        const uint32_t i0 = b[k], cnt = b[k + 1] - b[k];
        if (cnt)
            st[k] = rns_csum_batch_host(ctx->ctx[k], h_arena, arena_bytes, h_off + i0, h_len + i0,
                                        h_seed ? h_seed + i0 : nullptr, h_out + i0, cnt, flags);
    };
    std::vector<std::thread> workers;
    for (uint32_t k = 1; k < parts; ++k) {
        try {
            workers.emplace_back(run, k);
        } catch (...) {
            run(k);  // no thread available: run this range inline
        }
    }
    run(0);
    for (auto &w : workers)
        w.join();
    for (int x : st)
        if (x)
            return x;
    return RNS_OK;
}

int rns_csum_batch_multi_dev(const rns_dev_batch *batches, uint32_t nbatches, uint32_t flags)
{
    if (nbatches == 0)
        return RNS_OK;
    if (!batches)
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess)
        return RNS_E_NODEVICE;
    int st = RNS_OK;
    for (uint32_t k = 0; k < nbatches && st == RNS_OK; ++k) {  // launches are asynchronous: GPUs run together
        const rns_dev_batch &d = batches[k];
        st = hip_status(hipSetDevice(d.device));
        if (st == RNS_OK)
            st = rns_csum_batch_dev(d.d_arena, d.arena_bytes, d.d_off, d.d_len, d.d_seed, d.d_out, d.n, flags,
                                    d.len_hint, d.d_bad, d.stream);
    }
    (void)hipSetDevice(prev);
    return st;
}

int rns_host_alloc(uint64_t bytes, void **out)
{
    if (!out)
        return RNS_E_INVALID;
    *out = nullptr;
    if (int st = check_device())
        return st;
    return hip_status(hipHostMalloc(out, bytes, 0));
}

int rns_host_free(void *p) { return hip_status(hipHostFree(p)); }

int rns_fill_splitmix64_dev(uint8_t *d_buf, uint64_t nbytes, uint64_t seed, void *stream)
{
    if (nbytes == 0)
        return RNS_OK;
    if (!d_buf || (reinterpret_cast<uintptr_t>(d_buf) & 7))
        return RNS_E_INVALID;
    if (int st = check_device())
        return st;
    const uint64_t words = (nbytes + 7) / 8;
    const uint32_t blocks = static_cast<uint32_t>(std::min<uint64_t>((words + kBlock - 1) / kBlock, 8192));
    hipLaunchKernelGGL(splitmix64_fill_kernel, dim3(blocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                       d_buf, nbytes, seed);
    return hip_status(hipGetLastError());
}

const char *rns_csum_shape_name(uint32_t len_hint)
{
    static const char *const names[] = {"csum_batch_kernel",     "csum_rounds_kernel",     "csum_batch_kernel[nt]",
                                        "csum_rounds_kernel[nt]", "csum_mixed_kernel",      "csum_mixed_kernel",
                                        "csum_mixed_kernel[nt]",  "csum_mixed_kernel[nt]"};
    static thread_local char buf[96];
    const Shape sh = pick_shape(len_hint);
    if (sh.variant & 4)
        std::snprintf(buf, sizeof(buf), "%s (size classes G/U 4/1 x 4 packets, 4/4, 16/4, 32/4, 64/4)", names[sh.variant & 7]);
    else
        std::snprintf(buf, sizeof(buf), "%s<G=%u,U=%u>%s%s", names[sh.variant & 7], sh.G, sh.U,
                      (sh.variant & 8) ? " all rounds in flight" : (sh.variant & 16) ? " descriptors prefetched" : "",
                      sh.max_blocks ? " grid-capped" : "");
    return buf;
}

const char *rns_build_info(void)
{
    return "rns_checksum abi=1 offload-arch=gfx950 kernels=csum_rows_kernel (packed form: 1 KiB rows per 64-packet "
           "region, owners capture two region prefixes and sum their own end chunk; fill mode), csum_rows_rx_kernel "
           "(packed receive verify: the rows plus each owner's header chunks loaded a group ahead), csum_stream_kernel "
           "(receive verify of ACK-sized arenas: owners load their datagrams whole), csum_strided_rx_kernel (receive "
           "verify of fixed-size slots: quad-coalesced rows), csum_rows_tx_kernel (packed transmit finalize through the "
           "rows), csum_txrows_kernel (transmit-shaped chains: packed payload rows + owner-loaded head fragments; "
           "head-fragment fill; whole finalize of NetBuffer chains with the heads written back from LDS), "
           "csum_strided_tiny_kernel "
           "(fixed-size packets <= 64 B at a fixed stride), csum_mixed_kernel (per-wave size-class sort; verify / fill / "
           "transmit-finalize stash modes), csum_rounds_kernel, csum_batch_kernel, csum_chain_kernel (one pass, "
           "per-fragment fold; head-fragment fill) (v_sad_u16 LE sums, v_dot4 BE sums past 128 KiB, wave64, DPP "
           "reductions)";
}

int rns_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

}  // extern "C"
