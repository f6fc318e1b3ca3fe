// Streaming-read ceiling probe for MI355X: how fast can ONE kernel read a large
// buffer from HBM with 16 B/lane coalesced loads?  This is the practical roof the
// checksum kernel is compared with (the spec peak is 8 TB/s; MI355X_MICROARCH.md
// measured 6.29 TB/s for a float4 copy).  Each variant sums the dwords it reads
// (v_dot4 like the checksum) so nothing is dead-code-eliminated.
//
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_read_probe.hip -o tools/hbm_read_probe
//   ./tools/hbm_read_probe [bytes]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 load_nt(const uint4 *q)
{
    u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(q));
    return make_uint4(v.x, v.y, v.z, v.w);
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void read_grid_stride(const uint4 *__restrict__ p, uint64_t n16, uint32_t *out)
{
    uint32_t acc = 0;
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
    uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = NT ? load_nt(p + i + u * stride) : p[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc = __builtin_amdgcn_udot4(v[u].x, 0x01010101u, acc, false);
            acc = __builtin_amdgcn_udot4(v[u].y, 0x01010101u, acc, false);
            acc = __builtin_amdgcn_udot4(v[u].z, 0x01010101u, acc, false);
            acc = __builtin_amdgcn_udot4(v[u].w, 0x01010101u, acc, false);
        }
    }
    for (; i < n16; i += stride) {
        uint4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 0x12345678u)
        out[0] = acc;  // practically never: keeps the loads live
}

// One block per contiguous slab (each block streams its own 1500*64-ish region).
template <int U>
__global__ __launch_bounds__(256) void read_slabs(const uint4 *__restrict__ p, uint64_t n16, uint64_t slab16,
                                                  uint32_t *out)
{
    uint32_t acc = 0;
    const uint64_t b0 = static_cast<uint64_t>(blockIdx.x) * slab16;
    const uint64_t b1 = b0 + slab16 < n16 ? b0 + slab16 : n16;
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += 256 * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = (i + u * 256 < b1) ? p[i + u * 256] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc = __builtin_amdgcn_udot4(v[u].x, 0x01010101u, acc, false);
            acc = __builtin_amdgcn_udot4(v[u].y, 0x01010101u, acc, false);
            acc = __builtin_amdgcn_udot4(v[u].z, 0x01010101u, acc, false);
            acc = __builtin_amdgcn_udot4(v[u].w, 0x01010101u, acc, false);
        }
    }
    if (acc == 0x12345678u)
        out[0] = acc;
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
    const uint64_t bytes = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : (1500ull << 20);
    const uint64_t n16 = bytes / 16;
    uint4 *p;
    uint32_t *out;
    CHECK(hipMalloc(&p, n16 * 16));
    CHECK(hipMalloc(&out, 4));
    CHECK(hipMemset(p, 0x5a, n16 * 16));
    const int iters = 20;
    std::printf("{\"bytes\": %llu, \"results\": [\n", (unsigned long long)(n16 * 16));
    bool first = true;
    auto report = [&](const char *name, int grid, float ms) {
        std::printf("%s{\"variant\": \"%s\", \"grid\": %d, \"us\": %.1f, \"GBps\": %.1f}\n", first ? "" : ",", name,
                    grid, ms * 1e3, (n16 * 16) / (ms * 1e-3) / 1e9);
        first = false;
    };
    for (int grid : {1024, 2048, 4096, 8192, 16384}) {
        report("grid_stride_U1", grid, time_ms([&] { read_grid_stride<1, false><<<grid, 256>>>(p, n16, out); }, iters));
        report("grid_stride_U2", grid, time_ms([&] { read_grid_stride<2, false><<<grid, 256>>>(p, n16, out); }, iters));
        report("grid_stride_U4", grid, time_ms([&] { read_grid_stride<4, false><<<grid, 256>>>(p, n16, out); }, iters));
        report("grid_stride_U4_nt", grid, time_ms([&] { read_grid_stride<4, true><<<grid, 256>>>(p, n16, out); }, iters));
        report("grid_stride_U8", grid, time_ms([&] { read_grid_stride<8, false><<<grid, 256>>>(p, n16, out); }, iters));
    }
    for (uint64_t slab : {4096ull, 16384ull, 65536ull}) {  // slab in 16-B units
        int grid = static_cast<int>((n16 + slab - 1) / slab);
        char name[64];
        std::snprintf(name, sizeof(name), "slabs_%lluKiB_U4", (unsigned long long)(slab * 16 / 1024));
        report(name, grid, time_ms([&] { read_slabs<4><<<grid, 256>>>(p, n16, slab, out); }, iters));
    }
    std::printf("]}\n");
    CHECK(hipFree(p));
    CHECK(hipFree(out));
    return 0;
}
