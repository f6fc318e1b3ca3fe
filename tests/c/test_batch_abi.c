/*
 * A plain C caller of the batch C ABI, bound the way the reference's Rust would bind
 * it (extern "C" + raw pointers, netif.rs:24-37): no torch, no Python, the HIP runtime
 * only for device memory.  Every result is checked against the oracle
 * (oracle/csum_oracle.c, linked here as test infrastructure only).
 *
 *   gcc -std=gnu11 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include tests/c/test_batch_abi.c \
 *       oracle/csum_oracle.c -L rustnetworkstack_amd -lrns_checksum -L /opt/rocm/lib -lamdhip64 -lpthread
 *
 * Prints "all checks passed" and exits 0 on success.
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rns_checksum.h"

int32_t oracle_compute_ones_comp(uint16_t in_checksum, const uint8_t *slice, size_t len);

static uint64_t rng_state = 0x5EEDC0DEull;
static uint64_t next_u64(void)
{
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int failures = 0;
#define CHECK(cond, ...)                                                                           \
    do {                                                                                           \
        if (!(cond)) {                                                                             \
            if (failures++ < 10) {                                                                 \
                fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);                               \
                fprintf(stderr, __VA_ARGS__);                                                      \
                fprintf(stderr, "\n");                                                             \
            }                                                                                      \
        }                                                                                          \
    } while (0)
#define HIP_OK(x)                                                                                  \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
            return 2;                                                                              \
        }                                                                                          \
    } while (0)

int main(void)
{
    const uint32_t n = 40000;
    uint64_t *off = malloc(n * sizeof *off);
    uint32_t *len = malloc(n * sizeof *len);
    uint16_t *seed = malloc(n * sizeof *seed), *want = malloc(n * sizeof *want), *got = malloc(n * sizeof *got);
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t r = next_u64();
        pos += r % 17;                                  /* gaps: starts at every alignment, odd included */
        len[i] = (i % 997 == 0) ? 9000u : 1u + (uint32_t)((r >> 8) % 2000u);
        off[i] = pos;
        pos += len[i];
        seed[i] = (uint16_t)(r >> 40);
    }
    const uint64_t bytes = pos + 64;
    uint8_t *arena = NULL;
    if (rns_host_alloc(bytes, (void **)&arena) != RNS_OK) {  /* pinned, as the header recommends */
        fprintf(stderr, "rns_host_alloc failed\n");
        return 2;
    }
    for (uint64_t b = 0; b < bytes; b += 8) {
        const uint64_t w = next_u64();
        memcpy(arena + b, &w, bytes - b < 8 ? bytes - b : 8);
    }
    for (uint32_t i = 0; i < n; ++i)
        want[i] = (uint16_t)(0xffffu ^ (uint32_t)oracle_compute_ones_comp(seed[i], arena + off[i], len[i]));

    /* 1. host-resident batch through a staging context (chunked copies, 3 streams) */
    rns_host_ctx *ctx = NULL;
    CHECK(rns_host_ctx_create(0, 8u << 20, 3, &ctx) == RNS_OK, "rns_host_ctx_create");
    memset(got, 0, n * sizeof *got);
    CHECK(rns_csum_batch_host(ctx, arena, bytes, off, len, seed, got, n, RNS_FLAG_COMPLEMENT) == RNS_OK,
          "rns_csum_batch_host");
    for (uint32_t i = 0; i < n; ++i)
        CHECK(got[i] == want[i], "host batch packet %u (len %u off %llu): %04x != %04x", i, len[i],
              (unsigned long long)off[i], got[i], want[i]);
    CHECK(rns_host_ctx_destroy(ctx) == RNS_OK, "rns_host_ctx_destroy");

    /* 2. device-resident batch: the caller owns the HBM buffers and the stream */
    uint8_t *d_arena;
    uint64_t *d_off;
    uint32_t *d_len, *d_bad;
    uint16_t *d_seed, *d_out;
    hipStream_t st;
    HIP_OK(hipMalloc((void **)&d_arena, bytes));
    HIP_OK(hipMalloc((void **)&d_off, n * sizeof *off));
    HIP_OK(hipMalloc((void **)&d_len, n * sizeof *len));
    HIP_OK(hipMalloc((void **)&d_seed, n * sizeof *seed));
    HIP_OK(hipMalloc((void **)&d_out, n * sizeof *got));
    HIP_OK(hipMalloc((void **)&d_bad, sizeof *d_bad));
    HIP_OK(hipStreamCreate(&st));
    HIP_OK(hipMemcpy(d_arena, arena, bytes, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_off, off, n * sizeof *off, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_len, len, n * sizeof *len, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_seed, seed, n * sizeof *seed, hipMemcpyHostToDevice));
    HIP_OK(hipMemset(d_bad, 0, sizeof *d_bad));
    const uint32_t hints[3] = {0u, 64u, 1000u};     /* auto, tiny-packet and mixed shapes */
    for (int h = 0; h < 3; ++h) {
        HIP_OK(hipMemset(d_out, 0, n * sizeof *got));
        CHECK(rns_csum_batch_dev(d_arena, bytes, d_off, d_len, d_seed, d_out, n, RNS_FLAG_COMPLEMENT, hints[h], d_bad,
                                 st) == RNS_OK,
              "rns_csum_batch_dev hint %u", hints[h]);
        HIP_OK(hipStreamSynchronize(st));
        HIP_OK(hipMemcpy(got, d_out, n * sizeof *got, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < n; ++i)
            CHECK(got[i] == want[i], "device batch (hint %u) packet %u: %04x != %04x", hints[h], i, got[i], want[i]);
    }
    /* compact descriptors: the same batch with 32-bit offsets */
    {
        uint32_t *off32 = malloc(n * sizeof *off32), *d_off32 = NULL;
        for (uint32_t i = 0; i < n; ++i)
            off32[i] = (uint32_t)off[i];
        HIP_OK(hipMalloc((void **)&d_off32, n * sizeof *off32));
        HIP_OK(hipMemcpy(d_off32, off32, n * sizeof *off32, hipMemcpyHostToDevice));
        for (int h = 0; h < 3; ++h) {
            HIP_OK(hipMemset(d_out, 0, n * sizeof *got));
            CHECK(rns_csum_batch_dev_off32(d_arena, bytes, d_off32, d_len, d_seed, d_out, n, RNS_FLAG_COMPLEMENT,
                                           hints[h], d_bad, st) == RNS_OK,
                  "rns_csum_batch_dev_off32 hint %u", hints[h]);
            HIP_OK(hipStreamSynchronize(st));
            HIP_OK(hipMemcpy(got, d_out, n * sizeof *got, hipMemcpyDeviceToHost));
            for (uint32_t i = 0; i < n; ++i)
                CHECK(got[i] == want[i], "compact batch (hint %u) packet %u: %04x != %04x", hints[h], i, got[i],
                      want[i]);
        }
        CHECK(rns_csum_batch_dev_off32(d_arena, bytes, NULL, d_len, d_seed, d_out, n, 0, 0, NULL, st) ==
                  RNS_E_INVALID,
              "NULL compact offsets");
        hipFree(d_off32);
        free(off32);
    }
    uint32_t bad = 1;
    HIP_OK(hipMemcpy(&bad, d_bad, sizeof bad, hipMemcpyDeviceToHost));
    CHECK(bad == 0, "d_bad = %u", bad);

    /* 3. errors come back as status codes, never as aborts */
    CHECK(rns_csum_batch_dev(NULL, bytes, d_off, d_len, d_seed, d_out, n, 0, 0, NULL, st) == RNS_E_INVALID,
          "NULL arena");
    CHECK(rns_csum_batch_dev(d_arena, bytes, d_off, d_len, d_seed, d_out, 0, 0, 0, NULL, st) == RNS_OK, "n = 0");
    CHECK(rns_compute_ones_comp(0, arena, 0) < 0, "empty slice reports the reference's panic");

    hipFree(d_arena);
    hipFree(d_off);
    hipFree(d_len);
    hipFree(d_seed);
    hipFree(d_out);
    hipFree(d_bad);
    hipStreamDestroy(st);
    rns_host_free(arena);
    free(off);
    free(len);
    free(seed);
    free(want);
    free(got);
    if (failures) {
        fprintf(stderr, "%d failures\n", failures);
        return 1;
    }
    printf("all checks passed (%u packets)\n", n);
    return 0;
}
