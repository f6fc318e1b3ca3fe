// Scattered-store probe for MI355X: what does the transmit fill's one small store per
// packet cost, alone and fused behind a streaming read of the packets?
//
//   hipcc --offload-arch=gfx950 -O3 tools/store_probe.hip -o tools/store_probe
//   ./tools/store_probe [packets] [stride]
//
// Packets of `stride` bytes back to back (default 2^20 x 1504 B, the c3 arena); the
// "field" is at byte 16 of each packet.  Variants:
//   scatter{2,16,32,64}  one lane per packet stores N bytes at the field (aligned block)
//   read                 one wave per 64 packets streams their bytes (16 B/lane, 4 in flight)
//   read+store{2,32}     the same, then each lane stores into one packet's field
//   read+compact         the same, then one coalesced 128-B store of 64 u16 results
//   read+store{64,128}   the same, each lane rewriting the whole aligned 64-B / 128-B block around its
//                        packet's field (round 6: are full-block writes cheaper than partial ones?)
//   read_xcd             read, with blocks renumbered so each XCD streams a contiguous eighth
//   glds{4,8,16}         the slab through an LDS ring with global_load_lds (DEPTH-1 KB blocks in flight)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int B>
__global__ __launch_bounds__(256) void scatter(uint8_t *arena, uint32_t n, uint32_t stride, uint32_t v)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    const uint64_t f = static_cast<uint64_t>(i) * stride + 16;
    if constexpr (B == 2) {
        *reinterpret_cast<uint16_t *>(arena + f) = static_cast<uint16_t>(v);
    } else {
        uint4 *q = reinterpret_cast<uint4 *>(arena + (f & ~static_cast<uint64_t>(B - 1)));
#pragma unroll
        for (int k = 0; k < B / 16; ++k)
            q[k] = make_uint4(v, v + k, v, v);
    }
}

// XCD-contiguous block order: dispatch sends block b to XCD b % 8, so block b takes
// slab (b % 8) * (nblk / 8) + b / 8 and each XCD streams one contiguous eighth.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nblk)
{
    const uint32_t per = nblk / 8;
    return (b < per * 8) ? (b % 8) * per + b / 8 : b;
}

// MODE 0: read only; 1: + 2-byte field store; 2: + 32-byte sector store; 3: + compact u16 store
// (MODE 7: + 64-byte block store; MODE 8: + 128-byte line store)
// at the end of the wave's slab.  MODE 4: the lane that loaded a packet's field chunk
// rewrites that 16-B chunk right after consuming it; MODE 5: the same store issued one
// iteration later, after the next iteration's loads (so no load waits for it).
// CACHE: buffer-load cache policy bits (0 = default, 2 = nontemporal).
template <int MODE, int CACHE = 2, bool XCD = false>
__global__ __launch_bounds__(256) void read_store(uint8_t *arena, uint32_t n, uint32_t stride, uint16_t *out)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t blk = XCD ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t wave = (blk * 256 + threadIdx.x) >> 6;
    const uint64_t p0 = static_cast<uint64_t>(wave) * 64;
    if (p0 >= n)
        return;
    const uint32_t np = min(64u, n - static_cast<uint32_t>(p0));
    uint64_t b0 = p0 * stride;
    if constexpr (MODE == 6) {  // a dependent per-wave descriptor load before the slab (always 0 here)
        const uint64_t dep = reinterpret_cast<const uint64_t *>(out)[(p0 + lane) % n / 4];
        b0 += __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(dep & 0));
        b0 += static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(dep)) == 0x7fffffffu);
    }
    const uint64_t nch = (static_cast<uint64_t>(np) * stride) >> 4;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(arena + b0, 0, static_cast<int>(nch * 16), 0x00020000);
    const uint32_t fch = 16 / 16, sch = stride / 16;  // the field's chunk within a packet; chunks per packet
    uint32_t acc = 0;
    bool pend = false;
    uint64_t pc = 0;
    u32x4 pv = {0, 0, 0, 0};
    for (uint64_t c = lane; c < nch; c += 256) {
        u32x4 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            x[u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, static_cast<uint32_t>((c + 64 * u) * 16), 0, CACHE);
        if constexpr (MODE == 5) {
            if (pend)
                *reinterpret_cast<u32x4 *>(arena + b0 + pc * 16) = pv;
            pend = false;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            acc = __builtin_amdgcn_sad_u16(x[u].x, 0, acc);
            acc = __builtin_amdgcn_sad_u16(x[u].y, 0, acc);
            acc = __builtin_amdgcn_sad_u16(x[u].z, 0, acc);
            acc = __builtin_amdgcn_sad_u16(x[u].w, 0, acc);
            if constexpr (MODE == 4 || MODE == 5) {
                const uint64_t cc = c + 64 * u;
                if (cc < nch && cc % sch == fch) {
                    u32x4 y = x[u];
                    y.x = acc;
                    if constexpr (MODE == 4) {
                        *reinterpret_cast<u32x4 *>(arena + b0 + cc * 16) = y;
                    } else {
                        pend = true;
                        pc = cc;
                        pv = y;
                    }
                }
            }
        }
    }
    if constexpr (MODE == 5) {
        if (pend)
            *reinterpret_cast<u32x4 *>(arena + b0 + pc * 16) = pv;
    }
    if constexpr (MODE == 4 || MODE == 5)
        return;
    if (lane >= np)
        return;
    const uint64_t f = (p0 + lane) * stride + 16;
    if constexpr (MODE == 0 || MODE == 6) {
        if (acc == 0x12345678u)
            out[p0 + lane] = 1;
    } else if constexpr (MODE == 1) {
        *reinterpret_cast<uint16_t *>(arena + f) = static_cast<uint16_t>(acc);
    } else if constexpr (MODE == 2) {
        uint4 *q = reinterpret_cast<uint4 *>(arena + (f & ~31ull));
        q[0] = make_uint4(acc, acc, acc, acc);
        q[1] = make_uint4(acc, 0, acc, 0);
    } else if constexpr (MODE == 7 || MODE == 8) {
        constexpr uint32_t BS = MODE == 7 ? 64 : 128;
        uint4 *q = reinterpret_cast<uint4 *>(arena + (f & ~static_cast<uint64_t>(BS - 1)));
#pragma unroll
        for (uint32_t k = 0; k < BS / 16; ++k)
            q[k] = make_uint4(acc, k, acc, k);
    } else {
        out[p0 + lane] = static_cast<uint16_t>(acc);
    }
}

// LDS-DMA streaming: each wave streams its slab in 1 KB blocks with global_load_lds
// (16 B per lane, no VGPR destination) into a DEPTH-block LDS ring, DEPTH-1 blocks in
// flight, one counted vmcnt wait per block, then ds_read_b128 + v_sad_u16.
template <int DEPTH>
__global__ __launch_bounds__(256) void read_glds(const uint8_t *arena, uint32_t n, uint32_t stride, uint16_t *out)
{
    extern __shared__ uint4 ring[];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
    const uint64_t p0 = static_cast<uint64_t>(wave) * 64;
    if (p0 >= n)
        return;
    const uint32_t np = min(64u, n - static_cast<uint32_t>(p0));
    const uint8_t *base = arena + p0 * stride;
    const uint32_t nblk = static_cast<uint32_t>((static_cast<uint64_t>(np) * stride) >> 10);
    typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
    lds_u32x4 *myring = (lds_u32x4 *)(ring + wv * DEPTH * 64);  // addrspacecast: ds_read, not flat
    auto issue = [&](uint32_t blk) {  // past the end: re-read the last block (keeps the count constant)
        const uint32_t b = blk < nblk ? blk : nblk - 1;
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(base + static_cast<uint64_t>(b) * 1024 + lane * 16),
                                         (__attribute__((address_space(3))) void *)(myring + (blk % DEPTH) * 64),
                                         16, 0, 2);
    };
#pragma unroll
    for (int d = 0; d < DEPTH - 1; ++d)
        issue(d);
    uint32_t acc = 0;
    for (uint32_t b = 0; b < nblk; ++b) {
        issue(b + DEPTH - 1);
        // vmcnt(DEPTH-1): block b has landed (gfx9 encoding: vmcnt[3:0], expcnt 7, lgkmcnt 15)
        __builtin_amdgcn_s_waitcnt((DEPTH - 1) | 0xF70);
        __asm__ volatile("" ::: "memory");
        const u32x4 x = *(volatile lds_u32x4 *)(myring + (b % DEPTH) * 64 + lane);
        acc = __builtin_amdgcn_sad_u16(x.x, 0, acc);
        acc = __builtin_amdgcn_sad_u16(x.y, 0, acc);
        acc = __builtin_amdgcn_sad_u16(x.z, 0, acc);
        acc = __builtin_amdgcn_sad_u16(x.w, 0, acc);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the read is done before the slot is refilled
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // drain the DMA before the wave ends
    if (acc == 0x12345678u)
        out[p0 + lane] = 1;
}

template <class F>
static float time_ms(F launch, int iters)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i)
        launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / iters;
}

int main(int argc, char **argv)
{
    const uint32_t n = argc > 1 ? static_cast<uint32_t>(std::strtoul(argv[1], nullptr, 0)) : (1u << 20);
    const uint32_t stride = argc > 2 ? static_cast<uint32_t>(std::strtoul(argv[2], nullptr, 0)) : 1504u;
    if (stride % 32 != 0 && stride % 16 != 0) {
        std::fprintf(stderr, "stride must be a multiple of 16\n");
        return 1;
    }
    const uint64_t bytes = static_cast<uint64_t>(n) * stride;
    uint8_t *arena;
    uint16_t *out;
    CHECK(hipMalloc(&arena, bytes + 256));
    CHECK(hipMalloc(&out, static_cast<size_t>(n) * 2 + 64));
    CHECK(hipMemset(out, 0, static_cast<size_t>(n) * 2 + 64));
    CHECK(hipMemset(arena, 0x5a, bytes));
    const int iters = 20;
    const uint32_t sblocks = (n + 255) / 256, rblocks = (n + 255) / 256;  // read: 4 waves of 64 packets per block
    std::printf("{\"packets\": %u, \"stride\": %u, \"bytes\": %llu, \"results\": [\n", n, stride,
                static_cast<unsigned long long>(bytes));
    bool first = true;
    auto report = [&](const char *name, float ms) {
        std::printf("%s{\"variant\": \"%s\", \"us\": %.1f, \"read_GBps\": %.1f}\n", first ? "" : ",", name, ms * 1e3,
                    bytes / (ms * 1e-3) / 1e9);
        first = false;
    };
    for (int rep = 0; rep < 2; ++rep) {
        report("scatter2", time_ms([&] { scatter<2><<<sblocks, 256>>>(arena, n, stride, 7); }, iters));
        report("scatter16", time_ms([&] { scatter<16><<<sblocks, 256>>>(arena, n, stride, 7); }, iters));
        report("scatter32", time_ms([&] { scatter<32><<<sblocks, 256>>>(arena, n, stride, 7); }, iters));
        report("scatter64", time_ms([&] { scatter<64><<<sblocks, 256>>>(arena, n, stride, 7); }, iters));
        report("scatter128", time_ms([&] { scatter<128><<<sblocks, 256>>>(arena, n, stride, 7); }, iters));
        report("read", time_ms([&] { read_store<0><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        report("read+store2", time_ms([&] { read_store<1><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        report("read+store32", time_ms([&] { read_store<2><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        report("read+compact", time_ms([&] { read_store<3><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        report("read+store64", time_ms([&] { read_store<7><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        report("read+store128", time_ms([&] { read_store<8><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        report("read_plain+store2", time_ms([&] { read_store<1, 0><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        report("read_plain+store64", time_ms([&] { read_store<7, 0><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        report("read+dep_desc", time_ms([&] { read_store<6><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        // occupancy capped by dynamic LDS per 4-wave workgroup (160 KB per CU)
        report("read_occ4", time_ms([&] { read_store<0><<<rblocks, 256, 40 << 10>>>(arena, n, stride, out); }, iters));
        report("read_occ3", time_ms([&] { read_store<0><<<rblocks, 256, 52 << 10>>>(arena, n, stride, out); }, iters));
        report("read_occ2", time_ms([&] { read_store<0><<<rblocks, 256, 80 << 10>>>(arena, n, stride, out); }, iters));
        report("read+inline16", time_ms([&] { read_store<4><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        report("read+deferred16", time_ms([&] { read_store<5><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        report("read_plain", time_ms([&] { read_store<0, 0><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        report("read_plain+store32", time_ms([&] { read_store<2, 0><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        report("read_plain+inline16", time_ms([&] { read_store<4, 0><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        report("read_plain+deferred16", time_ms([&] { read_store<5, 0><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        report("read_xcd", time_ms([&] { read_store<0, 2, true><<<rblocks, 256>>>(arena, n, stride, out); }, iters));
        report("read_xcd_occ2", time_ms([&] { read_store<0, 2, true><<<rblocks, 256, 80 << 10>>>(arena, n, stride, out); }, iters));
        report("glds4", time_ms([&] { read_glds<4><<<rblocks, 256, 4 * 4 * 1024>>>(arena, n, stride, out); }, iters));
        report("glds8", time_ms([&] { read_glds<8><<<rblocks, 256, 4 * 8 * 1024>>>(arena, n, stride, out); }, iters));
        report("glds8_occ2", time_ms([&] { read_glds<8><<<rblocks, 256, 80 << 10>>>(arena, n, stride, out); }, iters));
        report("glds16", time_ms([&] { read_glds<16><<<rblocks, 256, 4 * 16 * 1024>>>(arena, n, stride, out); }, iters));
        report("read;scatter32", time_ms([&] {
                   read_store<3><<<rblocks, 256>>>(arena, n, stride, out);
                   scatter<32><<<sblocks, 256>>>(arena, n, stride, 7);
               }, iters));
    }
    std::printf("]}\n");
    CHECK(hipFree(arena));
    CHECK(hipFree(out));
    return 0;
}
