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
#define RNS_CHAIN_LAUNCH(KM)                                                                      \
    if (runs && nt)                                                                               \
        hipLaunchKernelGGL((csum_chain_kernel<true, true, KM, true, FILL>), grid, block, 0, st, a);  \
    else if (runs)                                                                                \
        hipLaunchKernelGGL((csum_chain_kernel<false, true, KM, true, FILL>), grid, block, 0, st, a); \
    else if (nt && buf)                                                                           \
        hipLaunchKernelGGL((csum_chain_kernel<true, true, KM, false, FILL>), grid, block, 0, st, a); \
    else if (nt)                                                                                  \
        hipLaunchKernelGGL((csum_chain_kernel<true, false, KM, false, FILL>), grid, block, 0, st, a); \
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

template int launch_chain<false>(const CsumArgs &, uint32_t, bool, bool, hipStream_t);
template int launch_chain<true>(const CsumArgs &, uint32_t, bool, bool, hipStream_t);

}  // namespace rns
