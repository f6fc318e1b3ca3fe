// Fragment chains (rns_csum_chain_dev) and their head-fragment fill (rns_csum_chain_fill_dev):
// the one-pass class kernel, K packets per lane.
#include "rns_launch.hpp"

namespace rns {

template <bool FILL>
int launch_chain(const CsumArgs &a, uint32_t K, bool nt, bool runs, hipStream_t st)
{
    const uint64_t waves = (static_cast<uint64_t>(a.n) + 64 * K - 1) / (64 * K);
    const dim3 grid(static_cast<uint32_t>((waves + kChainBlock / 64 - 1) / (kChainBlock / 64))), block(kChainBlock);
    const bool buf = buf_records(a) < kOobOffset;
    // The temporal plain checksum (IMIX-like fragments) at 4 waves/SIMD for chains of 3+ packets
    // per lane or 2+ fragments per packet (IMIX [492, 512, rest] chains 640 -> 598 us, IMIX
    // transmit chains in 512-byte fragments 900 -> 790), else at 3 (IMIX in 512-byte NetBuffers
    // 811 -> 754, [head, payload] chains 658 -> 620; session r05f, both forms free of scratch).
    const double mean = static_cast<double>(a.n_frags) / static_cast<double>(a.n);
    const bool deep = !FILL && (K >= 3 || (K == 2 && mean >= 2.0));
#define RNS_CHAIN_LAUNCH(KM)                                                                      \
    if (runs && nt)                                                                               \
        hipLaunchKernelGGL((csum_chain_kernel<true, true, KM, true, FILL>), grid, block, 0, st, a);  \
    else if (runs)                                                                                \
        hipLaunchKernelGGL((csum_chain_kernel<false, true, KM, true, FILL>), grid, block, 0, st, a); \
    else if (nt && buf)                                                                           \
        hipLaunchKernelGGL((csum_chain_kernel<true, true, KM, false, FILL>), grid, block, 0, st, a); \
    else if (nt)                                                                                  \
        hipLaunchKernelGGL((csum_chain_kernel<true, false, KM, false, FILL>), grid, block, 0, st, a); \
    else if (buf && deep)                                                                         \
        hipLaunchKernelGGL((csum_chain_kernel<false, true, KM, false, FILL, FILL ? 0 : 4>), grid, block, 0, st, a); \
    else if (buf)                                                                                 \
        hipLaunchKernelGGL((csum_chain_kernel<false, true, KM, false, FILL>), grid, block, 0, st, a); \
    else                                                                                          \
        hipLaunchKernelGGL((csum_chain_kernel<false, false, KM, false, FILL>), grid, block, 0, st, a);
    if (K == 1) {
        RNS_CHAIN_LAUNCH(1)
    } else {
        RNS_CHAIN_LAUNCH(kChainMaxK)
    }
#undef RNS_CHAIN_LAUNCH
    return hip_status(hipGetLastError());
}

// RNS_FLAG_CHAIN_TX_PACKED: the transmit-rows kernel (one wave per 64 packets).
#ifndef RNS_TXROWS_D  // payload rows in flight per wave
#define RNS_TXROWS_D 8
#endif
template <bool FILL>
int launch_txrows(const CsumArgs &a, hipStream_t st)
{
    constexpr bool NT = RNS_STREAM_NT != 0;
    const dim3 grid(static_cast<uint32_t>((static_cast<uint64_t>(a.n) + 63) / 64)), block(64);
    if (buf_records(a) < kOobOffset)
        hipLaunchKernelGGL((csum_txrows_kernel<NT, true, RNS_TXROWS_D, FILL>), grid, block, 0, st, a);
    else
        hipLaunchKernelGGL((csum_txrows_kernel<NT, false, RNS_TXROWS_D, FILL>), grid, block, 0, st, a);
    return hip_status(hipGetLastError());
}

// Transmit finalize of chains (rns_tx_fill_chain_dev): the transmit-rows kernel in FIN mode, whatever the
// batch's shape (a wave without the transmit-packed shape takes its exact per-packet loop).
int launch_txfin(const CsumArgs &a, hipStream_t st)
{
    constexpr bool NT = RNS_STREAM_NT != 0;
    const dim3 grid(static_cast<uint32_t>((static_cast<uint64_t>(a.n) + 63) / 64)), block(64);
    if (buf_records(a) < kOobOffset)
        hipLaunchKernelGGL((csum_txrows_kernel<NT, true, RNS_TXROWS_D, false, true>), grid, block, 0, st, a);
    else
        hipLaunchKernelGGL((csum_txrows_kernel<NT, false, RNS_TXROWS_D, false, true>), grid, block, 0, st, a);
    return hip_status(hipGetLastError());
}

template int launch_chain<false>(const CsumArgs &, uint32_t, bool, bool, hipStream_t);
template int launch_chain<true>(const CsumArgs &, uint32_t, bool, bool, hipStream_t);
template int launch_txrows<false>(const CsumArgs &, hipStream_t);
template int launch_txrows<true>(const CsumArgs &, hipStream_t);

}  // namespace rns
