// Per-XCD timing probe: does one XCD finish a streaming read later than the others?
//
//   hipcc --offload-arch=gfx950 -O3 tools/xcd_probe.hip -o tools/xcd_probe
//   ./tools/xcd_probe [waves] [bytes_per_wave] [reps] [shift]
//
// Each wave (one 64-lane workgroup) streams its own contiguous slice with 16-byte loads, 16 KiB
// in flight (the rows kernel's D = 16), and records its XCD (HW_REG_XCC_ID), its first and last
// realtime-counter reads (100 MHz) into a per-wave record with vector stores.  Defaults: the
// c4 shape (4096 waves x 576 KiB, one generation of 4 waves/SIMD); 16384 x 96 KiB is c3's.
// Prints one JSON line per rep: per XCD the wave count, mean start, mean / max end (us after
// the earliest start), and the kernel span.
#include <hip/hip_runtime.h>

#include <algorithm>
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

__global__ __launch_bounds__(64, 4) void stream_probe(const uint8_t *arena, uint64_t per_wave, uint64_t *rec,
                                                      uint32_t *sink, uint32_t shift)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    // XCC_ID: hwreg 20, bits [3:0]
    const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
    // (shift: block b streams slice (b + shift) mod grid — does the slowness follow the XCD or the addresses?)
    const uint8_t *base = arena + static_cast<uint64_t>((blockIdx.x + shift) % gridDim.x) * per_wave;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base), static_cast<short>(0),
                                                                      static_cast<int>(per_wave), 0x00020000);
    const uint32_t lane = threadIdx.x;
    const uint32_t rows = static_cast<uint32_t>(per_wave >> 10);
    constexpr int D = 16;
    u32x4 v[D];
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < D; ++j)
        v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (static_cast<uint32_t>(j) << 10) + lane * 16u, 0, 2);
    for (uint32_t k0 = 0; k0 < rows; k0 += D) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            acc += v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
            const uint32_t k = k0 + j + D;
            const uint32_t o = k < rows ? (k << 10) + lane * 16u : 0xFFFFF000u;
            v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 2);
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        rec[3 * blockIdx.x] = t0;
        rec[3 * blockIdx.x + 1] = t1;
        rec[3 * blockIdx.x + 2] = xcc;
    }
    if (acc == 0x12345678u)
        sink[lane] = acc;
}

int main(int argc, char **argv)
{
    const uint32_t waves = argc > 1 ? static_cast<uint32_t>(std::atoi(argv[1])) : 4096u;
    const uint64_t per_wave = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 576ull << 10;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 5;
    const uint32_t shift = argc > 4 ? static_cast<uint32_t>(std::atoi(argv[4])) : 0u;
    const uint64_t bytes = per_wave * waves;
    uint8_t *arena;
    uint64_t *rec;
    uint32_t *sink;
    CHECK(hipMalloc(&arena, bytes));
    CHECK(hipMemset(arena, 0x5a, bytes));
    CHECK(hipMalloc(&rec, 3 * 8ull * waves));
    CHECK(hipMalloc(&sink, 256));
    std::vector<uint64_t> h(3ull * waves);
    for (int r = 0; r < reps + 2; ++r) {  // two warmups
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(stream_probe, dim3(waves), dim3(64), 0, 0, arena, per_wave, rec, sink, shift);
        CHECK(hipGetLastError());
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        CHECK(hipMemcpy(h.data(), rec, h.size() * 8, hipMemcpyDeviceToHost));
        if (r < 2)
            continue;
        uint64_t tmin = ~0ull, tmax = 0;
        for (uint32_t w = 0; w < waves; ++w) {
            tmin = std::min(tmin, h[3 * w]);
            tmax = std::max(tmax, h[3 * w + 1]);
        }
        double cnt[16] = {}, s0[16] = {}, s1[16] = {}, m1[16] = {};
        for (uint32_t w = 0; w < waves; ++w) {
            const uint32_t x = static_cast<uint32_t>(h[3 * w + 2]) & 15u;
            const double a = (h[3 * w] - tmin) / 100.0, b = (h[3 * w + 1] - tmin) / 100.0;  // 100 MHz -> us
            cnt[x] += 1;
            s0[x] += a;
            s1[x] += b;
            m1[x] = std::max(m1[x], b);
        }
        std::printf("{\"shift\": %u, \"waves\": %u, \"bytes_per_wave\": %llu, \"event_us\": %.2f, \"span_us\": %.2f, \"GBps\": %.1f, \"xcd\": [",
                    shift, waves, static_cast<unsigned long long>(per_wave), ms * 1e3, (tmax - tmin) / 100.0, bytes / (ms * 1e6));
        bool first = true;
        for (int x = 0; x < 16; ++x) {
            if (cnt[x] == 0)
                continue;
            std::printf("%s{\"id\": %d, \"waves\": %.0f, \"start_mean\": %.2f, \"end_mean\": %.2f, \"end_max\": %.2f}",
                        first ? "" : ", ", x, cnt[x], s0[x] / cnt[x], s1[x] / cnt[x], m1[x]);
            first = false;
        }
        std::printf("]}\n");
        CHECK(hipEventDestroy(e0));
        CHECK(hipEventDestroy(e1));
    }
    CHECK(hipFree(arena));
    CHECK(hipFree(rec));
    CHECK(hipFree(sink));
    return 0;
}
