// The class kernel's stash modes on one-wave workgroups: transmit fill (rns_csum_fill_dev),
// receive verify (rns_rx_verify_dev) and transmit finalize (rns_tx_fill_dev).
#include "rns_launch.hpp"

namespace rns {

int launch_fill(const CsumArgs &a, dim3 grid, hipStream_t st)
{
    const dim3 block(kMixedBlock<true>);
    if (buf_records(a) < kOobOffset)
        hipLaunchKernelGGL((csum_mixed_kernel<false, false, true, true>), grid, block, 0, st, a);
    else
        hipLaunchKernelGGL((csum_mixed_kernel<false, false, false, true>), grid, block, 0, st, a);
    return hip_status(hipGetLastError());
}

int launch_rx(const CsumArgs &a, dim3 grid, hipStream_t st)
{
    const dim3 block(kMixedBlock<true>);
    if (buf_records(a) < kOobOffset)  // nontemporal loads
        hipLaunchKernelGGL((csum_mixed_kernel<false, true, true, false, true>), grid, block, 0, st, a);
    else
        hipLaunchKernelGGL((csum_mixed_kernel<false, true, false, false, true>), grid, block, 0, st, a);
    return hip_status(hipGetLastError());
}

int launch_tx(const CsumArgs &a, dim3 grid, hipStream_t st)
{
    const dim3 block(kMixedBlock<true>);
    if (buf_records(a) < kOobOffset)
        hipLaunchKernelGGL((csum_mixed_kernel<false, false, true, false, false, true>), grid, block, 0, st, a);
    else
        hipLaunchKernelGGL((csum_mixed_kernel<false, false, false, false, false, true>), grid, block, 0, st, a);
    return hip_status(hipGetLastError());
}

}  // namespace rns
