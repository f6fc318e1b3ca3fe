// Host-side launchers of the checksum kernels (rns_kernels.hpp), one translation unit per
// kernel family so the build compiles them in parallel: k_shapes.hip (the explicit-descriptor
// shapes and the tuning entry), k_packed.hip (the packed form), k_chain.hip (fragment chains),
// k_stash.hip (transmit fill / receive verify / transmit finalize).  rns_checksum.hip holds the
// C ABI.
#pragma once

#include "rns_kernels.hpp"

namespace rns {

inline int hip_status(hipError_t e) { return e == hipSuccess ? RNS_OK : RNS_E_HIP_BASE - static_cast<int>(e); }

// Kernel shape for a typical (mean) packet length, in 16-byte chunks, from the
// interleaved shape sweeps on MI355X (tools/sweep_shapes.py, profiles/r01_sweep*.json):
//   <= 8 chunks   (64 B)        rounds, nontemporal, G=4, U=1, grid 2048,     (c2)
//                               next batch's descriptors prefetched
//   <= 48 chunks  (IMIX mean)   mixed (per-wave size-class sort)              (c5)
//   <= 160 chunks (1500 B)      mixed, nontemporal (= rounds G=32,U=4 here)   (c3, headline)
//   longer        (9000 B)      group, nontemporal, G=64, U=4                 (c4)
// The mixed kernel is the robust choice for any size distribution; the other
// two win by a few percent on batches of uniformly tiny / jumbo packets.
struct Shape {
    uint32_t variant, G, U, max_blocks;
};

// (round 6: the grid caps and the tiny variant are constants, no longer build knobs — every
// shipped shape is one the GPU parity suite runs; the other settings were measured slower:
// a grid cap on the mixed kernel, variant 11 for tiny packets, profiles/archive/r01-r02)
constexpr uint32_t kTinyVariant = 19u;  // rounds, nontemporal, next batch's descriptors prefetched
constexpr uint32_t kTinyGrid = 2048u;   // workgroups (4 waves each) for tiny packets
inline Shape pick_shape(uint32_t len_hint)
{
    const uint32_t chunks = len_hint ? (len_hint + 15) / 16 + 1 : 96;
    if (chunks <= 8)  // rounds, nontemporal, next batch's descriptors prefetched (c2: 15.1 -> 14.4 us)
        return Shape{kTinyVariant, 4u, 1u, kTinyGrid};
    if (chunks <= 48)
        return Shape{4u, 0u, 0u, 0u};  // mixed kernel, one wave per 64-packet batch
    if (chunks <= 160)
        return Shape{6u, 0u, 0u, 0u};
    return Shape{2u, 64u, 4u, 0u};
}

inline int check_device()
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        return RNS_E_NODEVICE;
    }
    return RNS_OK;
}

// Fill CsumArgs for a caller arena base that may not be 16-byte aligned.
inline void set_arena(CsumArgs &a, const uint8_t *arena, uint64_t arena_bytes)
{
    const uintptr_t p = reinterpret_cast<uintptr_t>(arena);
    a.base_adjust = p & 15;
    a.arena = reinterpret_cast<const uint8_t *>(p - a.base_adjust);
    a.arena_bytes = arena_bytes + a.base_adjust;
}


// k_shapes.hip: the explicit-descriptor kernels by (variant, lanes per packet, chunks in flight)
template <bool S>
int dispatch(const CsumArgs &a, uint32_t variant, uint32_t G, uint32_t U, uint32_t max_blocks, hipStream_t st);
extern template int dispatch<false>(const CsumArgs &, uint32_t, uint32_t, uint32_t, uint32_t, hipStream_t);
extern template int dispatch<true>(const CsumArgs &, uint32_t, uint32_t, uint32_t, uint32_t, hipStream_t);
int launch_strided_tiny(const CsumArgs &a, hipStream_t st);
// k_packed.hip
int dispatch_packed(const CsumArgs &a, const Shape &sh, hipStream_t st);
int launch_fill_packed(const CsumArgs &a, hipStream_t st);
int launch_stream_rx(const CsumArgs &a, hipStream_t st);
int launch_tx_packed(const CsumArgs &a, hipStream_t st);
int launch_strided_rx(const CsumArgs &a, hipStream_t st);
// k_chain.hip: K packets per lane (1..kChainMaxK); FILL = the head-fragment fill
template <bool FILL>
int launch_chain(const CsumArgs &a, uint32_t K, bool nt, bool runs, hipStream_t st);
extern template int launch_chain<false>(const CsumArgs &, uint32_t, bool, bool, hipStream_t);
extern template int launch_chain<true>(const CsumArgs &, uint32_t, bool, bool, hipStream_t);
template <bool FILL>
int launch_txrows(const CsumArgs &a, hipStream_t st);
extern template int launch_txrows<false>(const CsumArgs &, hipStream_t);
extern template int launch_txrows<true>(const CsumArgs &, hipStream_t);
int launch_txfin(const CsumArgs &a, hipStream_t st);
// k_stash.hip: the class kernel's stash modes on one-wave workgroups
int launch_fill(const CsumArgs &a, dim3 grid, hipStream_t st);
int launch_rx(const CsumArgs &a, dim3 grid, hipStream_t st);
int launch_tx(const CsumArgs &a, dim3 grid, hipStream_t st);

}  // namespace rns
