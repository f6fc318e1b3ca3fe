// The packed form (rns_csum_batch_packed_dev) and packed receive verify.
#include "rns_launch.hpp"

#ifndef RNS_ROWS_DEEP_FROM  // typical lengths from this take D = 16 rows in flight at 4 waves/SIMD
#define RNS_ROWS_DEEP_FROM 1024u
#endif

namespace rns {

// The packed form's kernels (separate instantiations, so the explicit-descriptor
// kernels carry no packed-form code): the mixed kernel, or for tiny packets the
// rounds kernel with pick_shape's G=4, U=1 shape.
// Receive verify's stream launch: one wave per 64-datagram unit.
#ifndef RNS_RX_ROWS_D  // rows in flight of the receive form
#define RNS_RX_ROWS_D 8
#endif
// Packed receive verify: the rows receive kernel (round 5: IMIX 468.1 -> 449.2-450.3 us, c3
// 230.4 -> 225.0-226.2 per step against the stream kernel), except for arenas of ACK-sized
// datagrams (at most 128 arena bytes per datagram), where the stream kernel's ACK path measured
// faster (14.54-14.64 vs 15.03-15.25 us per isolated dispatch; sessions r05c-r05h; a kernel of
// its own, 1 or 2 units per wave at 6-8 waves/SIMD: 15.2-19.5 against 14.7-14.9, r05n).
int launch_stream_rx(const CsumArgs &a, hipStream_t st)
{
    const dim3 grid(static_cast<uint32_t>((static_cast<uint64_t>(a.n) + 63) / 64)), block(64);
    constexpr bool NT = RNS_STREAM_NT != 0;
    const bool ack = a.arena_bytes / a.n <= 128, buf = buf_records(a) < kOobOffset;
    if (ack && buf)
        hipLaunchKernelGGL((csum_stream_kernel<NT, true>), grid, block, 0, st, a);
    else if (ack)
        hipLaunchKernelGGL((csum_stream_kernel<NT, false>), grid, block, 0, st, a);
    else if (buf)
        hipLaunchKernelGGL((csum_rows_rx_kernel<NT, true, RNS_RX_ROWS_D>), grid, block, 0, st, a);
    else
        hipLaunchKernelGGL((csum_rows_rx_kernel<NT, false, RNS_RX_ROWS_D>), grid, block, 0, st, a);
    return hip_status(hipGetLastError());
}

int dispatch_packed(const CsumArgs &a, const Shape &sh, hipStream_t st)
{
    const bool nt = (sh.variant & 2u) != 0, buf = buf_records(a) < kOobOffset;
    // 16-byte-aligned packets (align_log2 >= 4) of any typical length above the tiny rounds
    // kernel's, or unknown: the rows kernel.  Measured against the kernels it replaced (session
    // r04d, isolated dispatch): c3 1500 B 231.5 vs 238.5-239.2 us (class kernel), c4 9000 B
    // 344.4-345.1 vs 346.4-347.1 (group kernel, u32 offsets), IMIX 451-453 vs 456 (round 3's
    // stream kernel).  Tiny packets keep the rounds kernel (c2: 13.2-13.7 vs 14.0-14.8 us with
    // round 3's stream kernel).
    // (tiny packets through the rows kernel: c2 19.6 vs 13.8 us per isolated dispatch, a 4 KiB unit
    // is all prologue: profiles/r04_unit_size_and_tiny.json)
    const bool tiny = (sh.variant & ~16u) == 3u && sh.G == 4u && sh.U == 1u;
    if (a.align_mask >= 15u && !tiny) {
        constexpr bool NT = RNS_STREAM_NT != 0;
        const dim3 grid(static_cast<uint32_t>((static_cast<uint64_t>(a.n) + 63) / 64)), block(64);
        if (a.len_hint >= RNS_ROWS_DEEP_FROM) {
            if (buf)
                hipLaunchKernelGGL((csum_rows_kernel<NT, true, 16>), grid, block, 0, st, a);
            else
                hipLaunchKernelGGL((csum_rows_kernel<NT, false, 16>), grid, block, 0, st, a);
        } else {
            if (buf)
                hipLaunchKernelGGL((csum_rows_kernel<NT, true, 8>), grid, block, 0, st, a);
            else
                hipLaunchKernelGGL((csum_rows_kernel<NT, false, 8>), grid, block, 0, st, a);
        }
        return hip_status(hipGetLastError());
    }
    const uint64_t batches = (static_cast<uint64_t>(a.n) + 63) / 64;  // one wave per 64 packets
    const uint64_t wpb = ((sh.variant & 4u) ? kMixedBlock<false> : kBlock) / 64;  // waves per workgroup
    uint64_t blocks = (batches + wpb - 1) / wpb;
    if (sh.max_blocks != 0 && blocks > sh.max_blocks)
        blocks = sh.max_blocks;
    const dim3 grid(static_cast<uint32_t>(blocks)), block((sh.variant & 4u) ? kMixedBlock<false> : kBlock);
    if (sh.variant & 4u) {
        if (nt && buf)
            hipLaunchKernelGGL((csum_mixed_kernel<false, true, true, false, false, false, true>), grid, block, 0, st, a);
        else if (nt)
            hipLaunchKernelGGL((csum_mixed_kernel<false, true, false, false, false, false, true>), grid, block, 0, st, a);
        else if (buf)
            hipLaunchKernelGGL((csum_mixed_kernel<false, false, true, false, false, false, true>), grid, block, 0, st, a);
        else
            hipLaunchKernelGGL((csum_mixed_kernel<false, false, false, false, false, false, true>), grid, block, 0, st,
                               a);
    } else if ((sh.variant & ~16u) == 3u && sh.G == 4u && sh.U == 1u) {  // c2: 13.46 -> 13.36 us with prefetch
        const bool pf = (sh.variant & 16u) != 0;
        if (buf && pf)
            hipLaunchKernelGGL((csum_rounds_kernel<4, 1, false, true, true, 1, true, true>), grid, block, 0,
                               st, a);
        else if (buf)
            hipLaunchKernelGGL((csum_rounds_kernel<4, 1, false, true, true, 1, true>), grid, block, 0, st, a);
        else if (pf)
            hipLaunchKernelGGL((csum_rounds_kernel<4, 1, false, true, false, 1, true, true>), grid, block, 0, st, a);
        else
            hipLaunchKernelGGL((csum_rounds_kernel<4, 1, false, true, false, 1, true>), grid, block, 0, st, a);
    } else {
        return RNS_E_INVALID;
    }
    return hip_status(hipGetLastError());
}

// Transmit fill of a packed arena (align_log2 >= 4): the rows kernel in fill mode, D by the
// typical length as for the plain checksum.
// (Temporal row loads, so that a field's line is still in L2 when its store comes, measured
// slower on c3 and equal on IMIX: fill 344.4 / 762.3 us, finalize 360.8 / 808.8 against
// 303.8 / 764.2 and 306.7 / 810.9 with nontemporal rows; session r06d.)
int launch_fill_packed(const CsumArgs &a, hipStream_t st)
{
    constexpr bool NT = RNS_STREAM_NT != 0;
    const bool buf = buf_records(a) < kOobOffset;
    const dim3 grid(static_cast<uint32_t>((static_cast<uint64_t>(a.n) + 63) / 64)), block(64);
    if (a.len_hint >= RNS_ROWS_DEEP_FROM) {
        if (buf)
            hipLaunchKernelGGL((csum_rows_kernel<NT, true, 16, true>), grid, block, 0, st, a);
        else
            hipLaunchKernelGGL((csum_rows_kernel<NT, false, 16, true>), grid, block, 0, st, a);
    } else {
        if (buf)
            hipLaunchKernelGGL((csum_rows_kernel<NT, true, 8, true>), grid, block, 0, st, a);
        else
            hipLaunchKernelGGL((csum_rows_kernel<NT, false, 8, true>), grid, block, 0, st, a);
    }
    return hip_status(hipGetLastError());
}

// Transmit finalize of a packed arena (align_log2 >= 4): the rows transmit kernel, D by the
// typical length as for the plain checksum.
#ifndef RNS_TX_ROWS_DEEP_FROM  // typical lengths from this take D = 16 rows at 4 waves/SIMD
#define RNS_TX_ROWS_DEEP_FROM 1024u
#endif
int launch_tx_packed(const CsumArgs &a, hipStream_t st)
{
    constexpr bool NT = RNS_STREAM_NT != 0;
    const bool buf = buf_records(a) < kOobOffset;
    const dim3 grid(static_cast<uint32_t>((static_cast<uint64_t>(a.n) + 63) / 64)), block(64);
    if (a.len_hint >= RNS_TX_ROWS_DEEP_FROM) {
        if (buf)
            hipLaunchKernelGGL((csum_rows_tx_kernel<NT, true, 16>), grid, block, 0, st, a);
        else
            hipLaunchKernelGGL((csum_rows_tx_kernel<NT, false, 16>), grid, block, 0, st, a);
    } else {
        if (buf)
            hipLaunchKernelGGL((csum_rows_tx_kernel<NT, true, 8>), grid, block, 0, st, a);
        else
            hipLaunchKernelGGL((csum_rows_tx_kernel<NT, false, 8>), grid, block, 0, st, a);
    }
    return hip_status(hipGetLastError());
}

// Receive verify of datagrams at a fixed stride: B batches of 64 per one-wave workgroup (one:
// 48 VGPRs, 10 waves/SIMD; two batches per wave need 81 VGPRs and a second generation of waves,
// 16.4 us per isolated 64-byte dispatch against 14.0: sessions r06c, r06d).
int launch_strided_rx(const CsumArgs &a, hipStream_t st)
{
    constexpr int B = kStridedRxB;
    const dim3 grid(static_cast<uint32_t>((static_cast<uint64_t>(a.n) + 64 * B - 1) / (64 * B))), block(64);
    if (buf_records(a) < kOobOffset)
        hipLaunchKernelGGL((csum_strided_rx_kernel<true, B>), grid, block, 0, st, a);
    else
        hipLaunchKernelGGL((csum_strided_rx_kernel<false, B>), grid, block, 0, st, a);
    return hip_status(hipGetLastError());
}

}  // namespace rns
