// The explicit-descriptor kernels by shape (rns_csum_batch_dev / _off32 / _strided / _cfg).
#include "rns_launch.hpp"

namespace rns {

// Kernel variants: bit 0 = rounds kernel (1) / group kernel (0); bit 1 = nontemporal loads;
// bit 2 = mixed kernel; bit 3 = rounds kernel with every round in flight; bit 4 = rounds
// kernel with the next batch's descriptors prefetched.
template <int G, int U, bool S>
int launch_shape(const CsumArgs &a, uint32_t variant, uint32_t max_blocks, hipStream_t st)
{
    uint64_t blocks;
    if ((variant & 5) == 0) {
        constexpr uint32_t kGroups = kBlock / G;
        blocks = (static_cast<uint64_t>(a.n) + kGroups - 1) / kGroups;
    } else {
        const uint64_t batches = (static_cast<uint64_t>(a.n) + 63) / 64;  // one wave per 64 packets
        const uint64_t wpb = ((variant & 4) ? kMixedBlock<false> : kBlock) / 64;  // waves per workgroup
        blocks = (batches + wpb - 1) / wpb;
    }
    if (max_blocks != 0 && blocks > max_blocks)
        blocks = max_blocks;
    if (blocks == 0)
        return RNS_OK;
    const dim3 grid(static_cast<uint32_t>(blocks)), block((variant & 4) ? kMixedBlock<false> : kBlock);
    const bool nt = (variant & 2) != 0;
    const bool buf = buf_records(a) < kOobOffset;  // buffer loads need a 32-bit offset range
    // Variant bits 8-11 (tuning): at most that many workgroups per CU, i.e. waves per
    // SIMD for 4-wave workgroups, by reserving LDS (160 KB per CU on gfx950).
    const uint32_t cap = (variant >> 8) & 15u;
    const size_t lds = cap ? ((160u << 10) / cap) - (2u << 10) : 0u;
    variant &= 0xffu;
    if (variant & 4) {
        if (nt && buf)
            hipLaunchKernelGGL((csum_mixed_kernel<S, true, true, false>), grid, block, lds, st, a);
        else if (nt)
            hipLaunchKernelGGL((csum_mixed_kernel<S, true, false, false>), grid, block, lds, st, a);
        else if (buf)
            hipLaunchKernelGGL((csum_mixed_kernel<S, false, true, false>), grid, block, lds, st, a);
        else
            hipLaunchKernelGGL((csum_mixed_kernel<S, false, false, false>), grid, block, lds, st, a);
    } else if ((variant & 1) == 0) {
        if constexpr (G >= 4) {
            if (nt)
                hipLaunchKernelGGL((csum_batch_kernel<G, U, S, true>), grid, block, lds, st, a);
            else
                hipLaunchKernelGGL((csum_batch_kernel<G, U, S, false>), grid, block, lds, st, a);
        } else {
            return RNS_E_INVALID;
        }
    } else if (variant & 8) {  // rounds kernel, every round in flight (tiny packets)
        if constexpr (G <= 8 && U <= 2) {
            if (nt && buf)
                hipLaunchKernelGGL((csum_rounds_kernel<G, U, S, true, true, G>), grid, block, lds, st, a);
            else if (nt)
                hipLaunchKernelGGL((csum_rounds_kernel<G, U, S, true, false, G>), grid, block, lds, st, a);
            else if (buf)
                hipLaunchKernelGGL((csum_rounds_kernel<G, U, S, false, true, G>), grid, block, lds, st, a);
            else
                hipLaunchKernelGGL((csum_rounds_kernel<G, U, S, false, false, G>), grid, block, lds, st, a);
        } else {
            return RNS_E_INVALID;
        }
    } else if (variant & 16) {  // rounds kernel, next batch's descriptors prefetched (tiny packets)
        if constexpr (G <= 8 && U <= 2) {
            if (nt && buf)
                hipLaunchKernelGGL((csum_rounds_kernel<G, U, S, true, true, 1, false, true>), grid, block, lds, st, a);
            else if (nt)
                hipLaunchKernelGGL((csum_rounds_kernel<G, U, S, true, false, 1, false, true>), grid, block, lds, st, a);
            else if (buf)
                hipLaunchKernelGGL((csum_rounds_kernel<G, U, S, false, true, 1, false, true>), grid, block, lds, st, a);
            else
                hipLaunchKernelGGL((csum_rounds_kernel<G, U, S, false, false, 1, false, true>), grid, block, lds, st,
                                   a);
        } else {
            return RNS_E_INVALID;
        }
    } else {
        if (nt && buf)
            hipLaunchKernelGGL((csum_rounds_kernel<G, U, S, true, true>), grid, block, lds, st, a);
        else if (nt)
            hipLaunchKernelGGL((csum_rounds_kernel<G, U, S, true, false>), grid, block, lds, st, a);
        else if (buf)
            hipLaunchKernelGGL((csum_rounds_kernel<G, U, S, false, true>), grid, block, lds, st, a);
        else
            hipLaunchKernelGGL((csum_rounds_kernel<G, U, S, false, false>), grid, block, lds, st, a);
    }
    return hip_status(hipGetLastError());
}

template <bool S>
int dispatch(const CsumArgs &a, uint32_t variant, uint32_t G, uint32_t U, uint32_t max_blocks, hipStream_t st)
{
    const uint32_t v = variant & 0xffu;  // bits 8-11: occupancy cap (launch_shape)
    // bit 3 (deep prefetch) and bit 4 (descriptor prefetch): rounds kernel only, not both
    if (v > 31 || (variant >> 12) || ((v & 24) && (v & 5) != 1) || (v & 24) == 24)
        return RNS_E_INVALID;
    if (variant & 4)  // the mixed kernel picks its own per-class shapes
        return launch_shape<64, 4, S>(a, variant, max_blocks, st);
#define RNS_SHAPE(g, u) \
    if (G == g && U == u) return launch_shape<g, u, S>(a, variant, max_blocks, st);
    if (variant & 1) {  // lanes_per_packet 2: rounds kernel only
        RNS_SHAPE(2, 1) RNS_SHAPE(2, 2) RNS_SHAPE(2, 4)
    }
    RNS_SHAPE(4, 1) RNS_SHAPE(4, 2) RNS_SHAPE(4, 4) RNS_SHAPE(4, 8)
    RNS_SHAPE(8, 1) RNS_SHAPE(8, 2) RNS_SHAPE(8, 4) RNS_SHAPE(8, 8)
    RNS_SHAPE(16, 1) RNS_SHAPE(16, 2) RNS_SHAPE(16, 4) RNS_SHAPE(16, 8)
    RNS_SHAPE(32, 1) RNS_SHAPE(32, 2) RNS_SHAPE(32, 4) RNS_SHAPE(32, 8)
    RNS_SHAPE(64, 1) RNS_SHAPE(64, 2) RNS_SHAPE(64, 4) RNS_SHAPE(64, 8)
#undef RNS_SHAPE
    return RNS_E_INVALID;
}

template int dispatch<false>(const CsumArgs &, uint32_t, uint32_t, uint32_t, uint32_t, hipStream_t);
template int dispatch<true>(const CsumArgs &, uint32_t, uint32_t, uint32_t, uint32_t, hipStream_t);

// Tiny fixed-size packets at a fixed 16-byte-aligned stride: csum_strided_tiny_kernel.
int launch_strided_tiny(const CsumArgs &a, hipStream_t st)
{
    // two 64-packet batches per wave: c2 isolated 12.56-12.59 -> 12.24-12.29 us, per step equal
    // (10.76-11.5 / 10.97-11.14); four: 13.55-13.65 (session r05h)
    constexpr int B = 2;
    const dim3 grid(static_cast<uint32_t>((static_cast<uint64_t>(a.n) + 64 * B - 1) / (64 * B))), block(64);
    if (buf_records(a) < kOobOffset)
        hipLaunchKernelGGL((csum_strided_tiny_kernel<true, B>), grid, block, 0, st, a);
    else
        hipLaunchKernelGGL((csum_strided_tiny_kernel<false, B>), grid, block, 0, st, a);
    return hip_status(hipGetLastError());
}

}  // namespace rns
