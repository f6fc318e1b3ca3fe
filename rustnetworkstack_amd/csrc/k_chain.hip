// Fragment chains (rns_csum_chain_dev): the one-pass class kernel, K packets per lane.
#include "rns_launch.hpp"

namespace rns {

int launch_chain(const CsumArgs &a, uint32_t K, bool nt, bool runs, hipStream_t st)
{
    const uint64_t waves = (static_cast<uint64_t>(a.n) + 64 * K - 1) / (64 * K);
    const dim3 grid(static_cast<uint32_t>((waves + kChainBlock / 64 - 1) / (kChainBlock / 64))), block(kChainBlock);
    const bool buf = buf_records(a) < kOobOffset;
#define RNS_CHAIN_LAUNCH(KM)                                                                      \
    if (runs && nt)                                                                               \
        hipLaunchKernelGGL((csum_chain_kernel<true, true, KM, true>), grid, block, 0, st, a);     \
    else if (runs)                                                                                \
        hipLaunchKernelGGL((csum_chain_kernel<false, true, KM, true>), grid, block, 0, st, a);    \
    else if (nt && buf)                                                                           \
        hipLaunchKernelGGL((csum_chain_kernel<true, true, KM>), grid, block, 0, st, a);           \
    else if (nt)                                                                                  \
        hipLaunchKernelGGL((csum_chain_kernel<true, false, KM>), grid, block, 0, st, a);          \
    else if (buf)                                                                                 \
        hipLaunchKernelGGL((csum_chain_kernel<false, true, KM>), grid, block, 0, st, a);          \
    else                                                                                          \
        hipLaunchKernelGGL((csum_chain_kernel<false, false, KM>), grid, block, 0, st, a);
    if (K == 1) {
        RNS_CHAIN_LAUNCH(1)
    } else {
        RNS_CHAIN_LAUNCH(kChainMaxK)
    }
#undef RNS_CHAIN_LAUNCH
    return hip_status(hipGetLastError());
}

}  // namespace rns
