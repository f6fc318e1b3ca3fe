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
int32_t oracle_compute_checksum(const uint8_t *slice, size_t len);
int32_t oracle_compute_pseudo_header_checksum(const uint8_t *src, size_t src_len, const uint8_t *dst, size_t dst_len,
                                              uint64_t length, uint8_t protocol);
void oracle_chain_batch(const uint8_t *arena, const uint64_t *frag_off, const uint32_t *frag_len, const uint32_t *first,
                        const uint16_t *seed, uint16_t *out, size_t npkts, int complement);

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

static void fill_random(uint8_t *p, uint64_t bytes)
{
    for (uint64_t b = 0; b < bytes; b += 8) {
        const uint64_t w = next_u64();
        memcpy(p + b, &w, bytes - b < 8 ? bytes - b : 8);
    }
}

/* rns_csum_batch_packed_dev (util.rs:88-110 per packet, offsets implied by the lengths):
 * lengths 1..1600 plus some jumbo ones, packed at 16-byte alignment by rns_packed_layout,
 * 7 (non-multiple-of-64) packets past a whole number of blocks. */
static int test_packed(hipStream_t st)
{
    const uint32_t n = 64 * 300 + 7;
    uint16_t *len16 = malloc(n * sizeof *len16), *seed = malloc(n * sizeof *seed);
    uint16_t *want = malloc(n * sizeof *want), *got = malloc(n * sizeof *got);
    uint64_t *off = malloc(n * sizeof *off), *blk = malloc(((n + 63) / 64) * sizeof *blk), end = 0;
    uint32_t *len32 = malloc(n * sizeof *len32);
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t r = next_u64();
        len16[i] = (uint16_t)((i % 101 == 0) ? 9000u : 1u + (uint32_t)(r % 1600u));
        len32[i] = len16[i];
        seed[i] = (uint16_t)(r >> 32);
    }
    CHECK(rns_packed_layout(len16, n, 4, 48, blk, off, &end) == RNS_OK, "rns_packed_layout");
    const uint64_t bytes = end + 16;
    uint8_t *arena = malloc(bytes);
    fill_random(arena, bytes);
    for (uint32_t i = 0; i < n; ++i) {
        CHECK(off[i] % 16 == 0 && (i == 0 || off[i] >= off[i - 1] + len16[i - 1]), "packed layout packet %u", i);
        want[i] = (uint16_t)(0xffffu ^ (uint32_t)oracle_compute_ones_comp(seed[i], arena + off[i], len16[i]));
    }
    uint8_t *d_arena;
    uint64_t *d_blk;
    uint16_t *d_len16, *d_seed, *d_out;
    uint32_t *d_bad, bad = 1;
    HIP_OK(hipMalloc((void **)&d_arena, bytes));
    HIP_OK(hipMalloc((void **)&d_blk, ((n + 63) / 64) * sizeof *blk));
    HIP_OK(hipMalloc((void **)&d_len16, n * sizeof *len16));
    HIP_OK(hipMalloc((void **)&d_seed, n * sizeof *seed));
    HIP_OK(hipMalloc((void **)&d_out, n * sizeof *got));
    HIP_OK(hipMalloc((void **)&d_bad, sizeof *d_bad));
    HIP_OK(hipMemcpy(d_arena, arena, bytes, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_blk, blk, ((n + 63) / 64) * sizeof *blk, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_len16, len16, n * sizeof *len16, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_seed, seed, n * sizeof *seed, hipMemcpyHostToDevice));
    HIP_OK(hipMemset(d_bad, 0, sizeof *d_bad));
    const uint32_t hints[3] = {64u, 340u, 1500u};  /* tiny-packet rounds kernel, mixed, mixed nt */
    for (int h = 0; h < 3; ++h) {
        HIP_OK(hipMemset(d_out, 0, n * sizeof *got));
        CHECK(rns_csum_batch_packed_dev(d_arena, bytes, d_blk, d_len16, 4, d_seed, d_out, n, RNS_FLAG_COMPLEMENT,
                                        hints[h], d_bad, st) == RNS_OK,
              "rns_csum_batch_packed_dev hint %u", hints[h]);
        HIP_OK(hipStreamSynchronize(st));
        HIP_OK(hipMemcpy(got, d_out, n * sizeof *got, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < n; ++i)
            CHECK(got[i] == want[i], "packed batch (hint %u) packet %u (len %u): %04x != %04x", hints[h], i, len16[i],
                  got[i], want[i]);
    }
    /* a cut-short arena: the packets past it are rejected (0) and counted */
    const uint64_t cut = off[n - 5];
    HIP_OK(hipMemset(d_out, 0xff, n * sizeof *got));
    CHECK(rns_csum_batch_packed_dev(d_arena, cut, d_blk, d_len16, 4, d_seed, d_out, n, RNS_FLAG_COMPLEMENT, 340u,
                                    d_bad, st) == RNS_OK, "packed, short arena");
    HIP_OK(hipStreamSynchronize(st));
    HIP_OK(hipMemcpy(got, d_out, n * sizeof *got, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(&bad, d_bad, sizeof bad, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i)
        CHECK(got[i] == (i < n - 5 ? want[i] : 0u), "short arena packet %u: %04x", i, got[i]);
    CHECK(bad == 5, "short arena: d_bad = %u (want 5)", bad);
    /* rns_csum_fill_packed_dev: the TCP field [16..18] counted as zero and the result stored
     * big-endian into it (tcp.rs:957-973); packets shorter than 18 bytes rejected, untouched */
    uint32_t short_pkts = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (len16[i] < 18) {
            want[i] = 0;
            ++short_pkts;
            continue;
        }
        uint8_t *f = arena + off[i] + 16;
        const uint8_t f0 = f[0], f1 = f[1];
        f[0] = f[1] = 0;
        want[i] = (uint16_t)(0xffffu ^ (uint32_t)oracle_compute_ones_comp(seed[i], arena + off[i], len16[i]));
        f[0] = f0;
        f[1] = f1;
    }
    HIP_OK(hipMemset(d_bad, 0, sizeof *d_bad));
    CHECK(rns_csum_fill_packed_dev(d_arena, bytes, d_blk, d_len16, 4, d_seed, NULL, 16, d_out, n, RNS_FLAG_COMPLEMENT,
                                   340u, d_bad, st) == RNS_OK, "rns_csum_fill_packed_dev");
    HIP_OK(hipStreamSynchronize(st));
    HIP_OK(hipMemcpy(got, d_out, n * sizeof *got, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(&bad, d_bad, sizeof bad, hipMemcpyDeviceToHost));
    uint8_t *back = malloc(bytes);
    HIP_OK(hipMemcpy(back, d_arena, bytes, hipMemcpyDeviceToHost));
    uint64_t changed = 0;
    for (uint32_t i = 0; i < n; ++i) {
        CHECK(got[i] == want[i], "packed fill packet %u (len %u): %04x != %04x", i, len16[i], got[i], want[i]);
        if (len16[i] >= 18) {
            const uint8_t *f = back + off[i] + 16;
            CHECK(f[0] == (want[i] >> 8) && f[1] == (want[i] & 0xff), "packed fill packet %u: field %02x%02x", i,
                  f[0], f[1]);
            arena[off[i] + 16] = f[0];
            arena[off[i] + 17] = f[1];
        }
    }
    for (uint64_t b = 0; b < bytes; ++b)
        changed += back[b] != arena[b];
    CHECK(changed == 0, "packed fill: %llu bytes outside the fields changed", (unsigned long long)changed);
    CHECK(bad == short_pkts, "packed fill: d_bad = %u (want %u)", bad, short_pkts);
    free(back);
    hipFree(d_arena); hipFree(d_blk); hipFree(d_len16); hipFree(d_seed); hipFree(d_out); hipFree(d_bad);
    free(len16); free(seed); free(want); free(got); free(off); free(blk); free(len32); free(arena);
    return 0;
}

/* rns_csum_batch_strided_dev (util.rs:88-110 per packet, fixed-size slots): 64-byte packets
 * at a 64-byte stride (the bench's c2 form) and 40-byte packets at an odd start and stride. */
static int test_strided(hipStream_t st)
{
    const uint32_t n = 64 * 500 + 3;
    const struct { uint64_t first, stride; uint32_t len; } cases[2] = {{0, 64, 64}, {7, 41, 40}};
    uint16_t *seed = malloc(n * sizeof *seed), *want = malloc(n * sizeof *want), *got = malloc(n * sizeof *got);
    for (uint32_t i = 0; i < n; ++i)
        seed[i] = (uint16_t)next_u64();
    for (int c = 0; c < 2; ++c) {
        const uint64_t bytes = cases[c].first + (uint64_t)cases[c].stride * n + 16;
        uint8_t *arena = malloc(bytes);
        fill_random(arena, bytes);
        for (uint32_t i = 0; i < n; ++i)
            want[i] = (uint16_t)(0xffffu ^ (uint32_t)oracle_compute_ones_comp(
                                               seed[i], arena + cases[c].first + (uint64_t)i * cases[c].stride,
                                               cases[c].len));
        uint8_t *d_arena;
        uint16_t *d_seed, *d_out;
        HIP_OK(hipMalloc((void **)&d_arena, bytes));
        HIP_OK(hipMalloc((void **)&d_seed, n * sizeof *seed));
        HIP_OK(hipMalloc((void **)&d_out, n * sizeof *got));
        HIP_OK(hipMemcpy(d_arena, arena, bytes, hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(d_seed, seed, n * sizeof *seed, hipMemcpyHostToDevice));
        HIP_OK(hipMemset(d_out, 0, n * sizeof *got));
        CHECK(rns_csum_batch_strided_dev(d_arena, bytes, cases[c].first, cases[c].stride, cases[c].len, d_seed, d_out,
                                         n, RNS_FLAG_COMPLEMENT, NULL, st) == RNS_OK,
              "rns_csum_batch_strided_dev case %d", c);
        HIP_OK(hipStreamSynchronize(st));
        HIP_OK(hipMemcpy(got, d_out, n * sizeof *got, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < n; ++i)
            CHECK(got[i] == want[i], "strided case %d packet %u: %04x != %04x", c, i, got[i], want[i]);
        hipFree(d_arena); hipFree(d_seed); hipFree(d_out);
        free(arena);
    }
    free(seed); free(want); free(got);
    return 0;
}

/* rns_csum_chain_dev (util.rs:112-119 over NetBuffer fragments, buf.rs:466-487): packets of
 * 0..6 fragments of 1..700 bytes at scattered offsets, odd non-final fragments included,
 * with and without the runs hint; half the packets' fragments are adjacent views. */
static int test_chains(hipStream_t st)
{
    const uint32_t npk = 5000;
    uint32_t *first = malloc((npk + 1) * sizeof *first);
    uint64_t *foff = malloc(npk * 6 * sizeof *foff);
    uint32_t *flen = malloc(npk * 6 * sizeof *flen);
    uint16_t *seed = malloc(npk * sizeof *seed), *want = malloc(npk * sizeof *want), *got = malloc(npk * sizeof *got);
    uint64_t pos = 0;
    uint32_t nf = 0;
    for (uint32_t i = 0; i < npk; ++i) {
        const uint64_t r = next_u64();
        const uint32_t k = (uint32_t)(r % 7);
        const int adjacent = (r >> 8) & 1;
        first[i] = nf;
        seed[i] = (uint16_t)(r >> 16);
        for (uint32_t j = 0; j < k; ++j) {
            const uint64_t q = next_u64();
            if (!adjacent)
                pos += q % 29;                               /* scattered: any alignment */
            flen[nf] = 1u + (uint32_t)((q >> 8) % 700u);
            if (adjacent && j + 1 < k)
                flen[nf] &= ~1u, flen[nf] += flen[nf] ? 0u : 2u;  /* even non-final fragments form a run */
            foff[nf] = pos;
            pos += flen[nf];
            ++nf;
        }
    }
    first[npk] = nf;
    const uint64_t bytes = pos + 32;
    uint8_t *arena = malloc(bytes);
    fill_random(arena, bytes);
    oracle_chain_batch(arena, foff, flen, first, seed, want, npk, 1);
    uint8_t *d_arena;
    uint64_t *d_foff;
    uint32_t *d_flen, *d_first, *d_bad, bad = 1;
    uint16_t *d_seed, *d_out;
    HIP_OK(hipMalloc((void **)&d_arena, bytes));
    HIP_OK(hipMalloc((void **)&d_foff, nf * sizeof *foff));
    HIP_OK(hipMalloc((void **)&d_flen, nf * sizeof *flen));
    HIP_OK(hipMalloc((void **)&d_first, (npk + 1) * sizeof *first));
    HIP_OK(hipMalloc((void **)&d_seed, npk * sizeof *seed));
    HIP_OK(hipMalloc((void **)&d_out, npk * sizeof *got));
    HIP_OK(hipMalloc((void **)&d_bad, sizeof *d_bad));
    HIP_OK(hipMemcpy(d_arena, arena, bytes, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_foff, foff, nf * sizeof *foff, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_flen, flen, nf * sizeof *flen, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_first, first, (npk + 1) * sizeof *first, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_seed, seed, npk * sizeof *seed, hipMemcpyHostToDevice));
    HIP_OK(hipMemset(d_bad, 0, sizeof *d_bad));
    const uint32_t flags[2] = {RNS_FLAG_COMPLEMENT, RNS_FLAG_COMPLEMENT | RNS_FLAG_CHAIN_RUNS};
    for (int f = 0; f < 2; ++f) {
        HIP_OK(hipMemset(d_out, 0, npk * sizeof *got));
        CHECK(rns_csum_chain_dev(d_arena, bytes, d_foff, d_flen, nf, d_first, d_seed, d_out, npk, flags[f], 350u, NULL,
                                 d_bad, st) == RNS_OK,
              "rns_csum_chain_dev flags %u", flags[f]);
        HIP_OK(hipStreamSynchronize(st));
        HIP_OK(hipMemcpy(got, d_out, npk * sizeof *got, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < npk; ++i)
            CHECK(got[i] == want[i], "chain (flags %u) packet %u (%u fragments): %04x != %04x", flags[f], i,
                  first[i + 1] - first[i], got[i], want[i]);
    }
    HIP_OK(hipMemcpy(&bad, d_bad, sizeof bad, hipMemcpyDeviceToHost));
    CHECK(bad == 0, "chains: d_bad = %u", bad);
    hipFree(d_arena); hipFree(d_foff); hipFree(d_flen); hipFree(d_first); hipFree(d_seed); hipFree(d_out);
    hipFree(d_bad);
    free(first); free(foff); free(flen); free(seed); free(want); free(got); free(arena);
    return 0;
}

/* rns_csum_chain_fill_dev, the tcp_output shape (tcp.rs:938-973): a 20-byte head fragment
 * (alloc_header, buf.rs:262-291; its field [16..18] holds garbage, the reference's is zero)
 * in a header region, then 0..4 payload fragments of 1..700 bytes at scattered offsets.  The
 * oracle: zero the field, compute_buffer_ones_comp ^ 0xffff, set_be16; every arena byte is
 * compared. */
static int test_chain_fill(hipStream_t st)
{
    const uint32_t npk = 4000, hl = 20, fo = 16;
    uint32_t *first = malloc((npk + 1) * sizeof *first);
    uint64_t *foff = malloc(npk * 5 * sizeof *foff);
    uint32_t *flen = malloc(npk * 5 * sizeof *flen);
    uint16_t *seed = malloc(npk * sizeof *seed), *want = malloc(npk * sizeof *want), *got = malloc(npk * sizeof *got);
    uint64_t pos = (uint64_t)npk * hl + 64;
    uint32_t nf = 0;
    for (uint32_t i = 0; i < npk; ++i) {
        const uint64_t r = next_u64();
        const uint32_t k = (uint32_t)(r % 5);
        first[i] = nf;
        seed[i] = (uint16_t)(r >> 16);
        foff[nf] = (uint64_t)i * hl + 1;                     /* heads back to back, odd start */
        flen[nf++] = hl;
        for (uint32_t j = 0; j < k; ++j) {
            const uint64_t q = next_u64();
            pos += q % 29;
            flen[nf] = 1u + (uint32_t)((q >> 8) % 700u);
            foff[nf++] = pos;
            pos += flen[nf - 1];
        }
    }
    first[npk] = nf;
    const uint64_t bytes = pos + 32;
    uint8_t *arena = malloc(bytes), *expect = malloc(bytes), *after = malloc(bytes);
    fill_random(arena, bytes);
    memcpy(expect, arena, bytes);
    for (uint32_t i = 0; i < npk; ++i)
        expect[foff[first[i]] + fo] = expect[foff[first[i]] + fo + 1] = 0;
    oracle_chain_batch(expect, foff, flen, first, seed, want, npk, 1);
    for (uint32_t i = 0; i < npk; ++i) {
        expect[foff[first[i]] + fo] = (uint8_t)(want[i] >> 8);
        expect[foff[first[i]] + fo + 1] = (uint8_t)want[i];
    }
    uint8_t *d_arena;
    uint64_t *d_foff;
    uint32_t *d_flen, *d_first, *d_bad, bad = 1;
    uint16_t *d_seed, *d_out;
    HIP_OK(hipMalloc((void **)&d_arena, bytes));
    HIP_OK(hipMalloc((void **)&d_foff, nf * sizeof *foff));
    HIP_OK(hipMalloc((void **)&d_flen, nf * sizeof *flen));
    HIP_OK(hipMalloc((void **)&d_first, (npk + 1) * sizeof *first));
    HIP_OK(hipMalloc((void **)&d_seed, npk * sizeof *seed));
    HIP_OK(hipMalloc((void **)&d_out, npk * sizeof *got));
    HIP_OK(hipMalloc((void **)&d_bad, sizeof *d_bad));
    HIP_OK(hipMemcpy(d_foff, foff, nf * sizeof *foff, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_flen, flen, nf * sizeof *flen, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_first, first, (npk + 1) * sizeof *first, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_seed, seed, npk * sizeof *seed, hipMemcpyHostToDevice));
    /* the chain kernel at two hints, then the transmit-rows kernel (RNS_FLAG_CHAIN_TX_PACKED:
     * these scattered payloads take its exact per-packet loop) */
    const uint32_t hints[3] = {512u, 100u, 512u};
    const uint32_t flags[3] = {RNS_FLAG_COMPLEMENT, RNS_FLAG_COMPLEMENT, RNS_FLAG_COMPLEMENT | RNS_FLAG_CHAIN_TX_PACKED};
    for (int h = 0; h < 3; ++h) {
        HIP_OK(hipMemcpy(d_arena, arena, bytes, hipMemcpyHostToDevice));
        HIP_OK(hipMemset(d_bad, 0, sizeof *d_bad));
        CHECK(rns_csum_chain_fill_dev(d_arena, bytes, d_foff, d_flen, nf, d_first, d_seed, NULL, fo, d_out, npk,
                                      flags[h], hints[h], d_bad, st) == RNS_OK,
              "rns_csum_chain_fill_dev hint %u flags %x", hints[h], flags[h]);
        HIP_OK(hipStreamSynchronize(st));
        HIP_OK(hipMemcpy(got, d_out, npk * sizeof *got, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(after, d_arena, bytes, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(&bad, d_bad, sizeof bad, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < npk; ++i)
            CHECK(got[i] == want[i], "chain fill (hint %u) packet %u: %04x != %04x", hints[h], i, got[i], want[i]);
        uint64_t diff = 0;
        for (uint64_t b = 0; b < bytes; ++b)
            diff += after[b] != expect[b];
        CHECK(diff == 0, "chain fill (hint %u): %llu arena bytes differ", hints[h], (unsigned long long)diff);
        CHECK(bad == 0, "chain fill: d_bad = %u", bad);
    }
    hipFree(d_arena); hipFree(d_foff); hipFree(d_flen); hipFree(d_first); hipFree(d_seed); hipFree(d_out);
    hipFree(d_bad);
    free(first); free(foff); free(flen); free(seed); free(want); free(got); free(arena); free(expect); free(after);
    return 0;
}

/* rns_csum_chain_fill_dev with RNS_FLAG_CHAIN_TX_PACKED on the layout it streams: 20-byte
 * heads back to back in a header region, each packet's payload (0..1480 bytes) one fragment,
 * the payloads back to back at 16-byte-aligned starts after the header region (the
 * transmit-rows kernel's row path). */
static int test_chain_fill_txpacked(hipStream_t st)
{
    const uint32_t npk = 3000, hl = 20, fo = 16;
    uint32_t *first = malloc((npk + 1) * sizeof *first);
    uint64_t *foff = malloc(npk * 2 * sizeof *foff);
    uint32_t *flen = malloc(npk * 2 * sizeof *flen);
    uint16_t *seed = malloc(npk * sizeof *seed), *want = malloc(npk * sizeof *want), *got = malloc(npk * sizeof *got);
    uint64_t pos = (((uint64_t)npk * hl + 4095) & ~4095ull);
    uint32_t nf = 0;
    for (uint32_t i = 0; i < npk; ++i) {
        const uint64_t r = next_u64();
        const uint32_t pl = (r % 7 == 0) ? 0u : (uint32_t)((r >> 8) % 1481u);
        first[i] = nf;
        seed[i] = (uint16_t)(r >> 32);
        foff[nf] = (uint64_t)i * hl;
        flen[nf++] = hl;
        if (pl) {
            foff[nf] = pos;
            flen[nf++] = pl;
            pos += (pl + 15u) & ~15u;
        }
    }
    first[npk] = nf;
    const uint64_t bytes = pos + 64;
    uint8_t *arena = malloc(bytes), *expect = malloc(bytes), *after = malloc(bytes);
    fill_random(arena, bytes);
    memcpy(expect, arena, bytes);
    for (uint32_t i = 0; i < npk; ++i)
        expect[foff[first[i]] + fo] = expect[foff[first[i]] + fo + 1] = 0;
    oracle_chain_batch(expect, foff, flen, first, seed, want, npk, 1);
    for (uint32_t i = 0; i < npk; ++i) {
        expect[foff[first[i]] + fo] = (uint8_t)(want[i] >> 8);
        expect[foff[first[i]] + fo + 1] = (uint8_t)want[i];
    }
    uint8_t *d_arena;
    uint64_t *d_foff;
    uint32_t *d_flen, *d_first, *d_bad, bad = 1;
    uint16_t *d_seed, *d_out;
    HIP_OK(hipMalloc((void **)&d_arena, bytes));
    HIP_OK(hipMalloc((void **)&d_foff, nf * sizeof *foff));
    HIP_OK(hipMalloc((void **)&d_flen, nf * sizeof *flen));
    HIP_OK(hipMalloc((void **)&d_first, (npk + 1) * sizeof *first));
    HIP_OK(hipMalloc((void **)&d_seed, npk * sizeof *seed));
    HIP_OK(hipMalloc((void **)&d_out, npk * sizeof *got));
    HIP_OK(hipMalloc((void **)&d_bad, sizeof *d_bad));
    HIP_OK(hipMemcpy(d_arena, arena, bytes, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_foff, foff, nf * sizeof *foff, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_flen, flen, nf * sizeof *flen, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_first, first, (npk + 1) * sizeof *first, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_seed, seed, npk * sizeof *seed, hipMemcpyHostToDevice));
    HIP_OK(hipMemset(d_bad, 0, sizeof *d_bad));
    CHECK(rns_csum_chain_fill_dev(d_arena, bytes, d_foff, d_flen, nf, d_first, d_seed, NULL, fo, d_out, npk,
                                  RNS_FLAG_COMPLEMENT | RNS_FLAG_CHAIN_TX_PACKED, 750u, d_bad, st) == RNS_OK,
          "rns_csum_chain_fill_dev (transmit-packed)");
    HIP_OK(hipStreamSynchronize(st));
    HIP_OK(hipMemcpy(got, d_out, npk * sizeof *got, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(after, d_arena, bytes, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(&bad, d_bad, sizeof bad, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < npk; ++i)
        CHECK(got[i] == want[i], "transmit-packed chain fill packet %u: %04x != %04x", i, got[i], want[i]);
    uint64_t diff = 0;
    for (uint64_t b = 0; b < bytes; ++b)
        diff += after[b] != expect[b];
    CHECK(diff == 0, "transmit-packed chain fill: %llu arena bytes differ", (unsigned long long)diff);
    CHECK(bad == 0, "transmit-packed chain fill: d_bad = %u", bad);
    hipFree(d_arena); hipFree(d_foff); hipFree(d_flen); hipFree(d_first); hipFree(d_seed); hipFree(d_out);
    hipFree(d_bad);
    free(first); free(foff); free(flen); free(seed); free(want); free(got); free(arena); free(expect); free(after);
    return 0;
}

/* rns_tx_fill_dev then rns_rx_verify_dev on IPv4 TCP / UDP / ICMP datagrams with garbage in
 * the checksum fields: every field must hold what the transmit call sites store (ip.rs:158-159,
 * tcp.rs:957-973, udp.rs:158-171, icmp.rs:91-94: the oracle's util.rs functions over the
 * datagram with the field zeroed), every other byte unchanged; the receiver (local address =
 * the destination) accepts them all; a flipped payload byte (TCP / ICMP) or header byte is
 * rejected as ip.rs:76-80 / tcp.rs:544-547 / icmp.rs:46-50 drop it. */
static int test_tx_rx(hipStream_t st)
{
    const uint32_t n = 3000;
    const uint8_t src[4] = {10, 0, 0, 1}, dst[4] = {10, 0, 0, 2}, dst6[16] = {0xfd, [15] = 2};
    uint64_t *off = malloc(n * sizeof *off);
    uint32_t *len = malloc(n * sizeof *len);
    uint8_t *proto = malloc(n), *status = malloc(n), *want_st = malloc(n);
    uint64_t pos = 5;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t r = next_u64();
        pos += r % 13;
        len[i] = 40u + (uint32_t)((r >> 8) % 1461u);
        off[i] = pos;
        pos += len[i];
        proto[i] = (i % 3 == 0) ? 6 : (i % 3 == 1) ? 17 : 1;
    }
    const uint64_t bytes = pos + 16;
    uint8_t *arena = malloc(bytes), *ref = malloc(bytes), *back = malloc(bytes);
    fill_random(arena, bytes);
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t *h = arena + off[i];
        h[0] = 0x45; h[1] = 0; h[2] = (uint8_t)(len[i] >> 8); h[3] = (uint8_t)len[i];
        h[6] = 0x40; h[7] = 0; h[8] = 64; h[9] = proto[i];
        memcpy(h + 12, src, 4);
        memcpy(h + 16, dst, 4);                      /* header checksum and L4 field keep their garbage */
    }
    /* expected bytes: the fields zeroed, then filled as the reference's output paths fill them */
    memcpy(ref, arena, bytes);
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t *h = ref + off[i], *seg = h + 20;
        const uint32_t seglen = len[i] - 20, field = proto[i] == 6 ? 16u : proto[i] == 17 ? 6u : 2u;
        h[10] = h[11] = 0;
        const uint32_t ipc = (uint32_t)oracle_compute_checksum(h, 20);
        h[10] = (uint8_t)(ipc >> 8); h[11] = (uint8_t)ipc;
        seg[field] = seg[field + 1] = 0;
        const int32_t ph = proto[i] == 1 ? 0 : oracle_compute_pseudo_header_checksum(src, 4, dst, 4, seglen, proto[i]);
        const uint32_t l4 = 0xffffu ^ (uint32_t)oracle_compute_ones_comp((uint16_t)ph, seg, seglen);
        seg[field] = (uint8_t)(l4 >> 8); seg[field + 1] = (uint8_t)l4;
        want_st[i] = RNS_TX_IP_FILLED | RNS_TX_L4_FILLED;
    }
    uint8_t *d_arena, *d_status;
    uint64_t *d_off;
    uint32_t *d_len;
    uint16_t *d_l4;
    HIP_OK(hipMalloc((void **)&d_arena, bytes));
    HIP_OK(hipMalloc((void **)&d_off, n * sizeof *off));
    HIP_OK(hipMalloc((void **)&d_len, n * sizeof *len));
    HIP_OK(hipMalloc((void **)&d_status, n));
    HIP_OK(hipMalloc((void **)&d_l4, n * sizeof *d_l4));
    HIP_OK(hipMemcpy(d_arena, arena, bytes, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_off, off, n * sizeof *off, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_len, len, n * sizeof *len, hipMemcpyHostToDevice));
    CHECK(rns_tx_fill_dev(d_arena, bytes, d_off, d_len, n, d_status, st) == RNS_OK, "rns_tx_fill_dev");
    HIP_OK(hipStreamSynchronize(st));
    HIP_OK(hipMemcpy(back, d_arena, bytes, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(status, d_status, n, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i)
        CHECK(status[i] == want_st[i], "tx status %u: %02x != %02x", i, status[i], want_st[i]);
    uint64_t diff = 0;
    for (uint64_t b = 0; b < bytes; ++b)
        diff += back[b] != ref[b];
    CHECK(diff == 0, "tx fill: %llu arena bytes differ from the oracle's", (unsigned long long)diff);

    /* receive side: corrupt a payload byte of every 7th datagram, the TTL of every 11th */
    for (uint32_t i = 0; i < n; ++i) {
        const int payload = i % 7 == 3, header = i % 11 == 5;
        if (payload)
            back[off[i] + 20 + (len[i] - 20) / 2] ^= 0x5A;
        if (header)
            back[off[i] + 8] ^= 0x01;
        uint8_t s_ = 0;
        if (!header)
            s_ |= RNS_RX_IP_OK;
        if (proto[i] == 17)
            s_ |= RNS_RX_L4_UNCHECKED;               /* udp.rs:126-148 never verifies */
        else if (!payload)
            s_ |= RNS_RX_L4_OK;
        if ((s_ & RNS_RX_IP_OK) && (s_ & (RNS_RX_L4_OK | RNS_RX_L4_UNCHECKED)))
            s_ |= RNS_RX_ACCEPT;
        want_st[i] = s_;
    }
    HIP_OK(hipMemcpy(d_arena, back, bytes, hipMemcpyHostToDevice));
    CHECK(rns_rx_verify_dev(d_arena, bytes, d_off, d_len, n, dst, dst6, d_status, d_l4, st) == RNS_OK,
          "rns_rx_verify_dev");
    HIP_OK(hipStreamSynchronize(st));
    HIP_OK(hipMemcpy(status, d_status, n, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i)
        CHECK(status[i] == want_st[i], "rx status %u (proto %u): %02x != %02x", i, proto[i], status[i], want_st[i]);
    hipFree(d_arena); hipFree(d_off); hipFree(d_len); hipFree(d_status); hipFree(d_l4);
    free(off); free(len); free(proto); free(status); free(want_st); free(arena); free(ref); free(back);
    return 0;
}

/* The packed transmit arena (rns_tx_fill_packed_dev: the rows transmit kernel) and its packed
 * receive (rns_rx_verify_packed_dev), then the same datagrams in 2048-byte receive slots
 * (rns_rx_verify_strided_dev): IPv4 TCP / UDP / ICMP with garbage in the checksum fields;
 * every field must hold what the transmit call sites store (the oracle's util.rs functions
 * over the datagram with the field zeroed), every other byte — the padding between datagrams
 * included — unchanged, and the receiver accepts them all. */
static int test_tx_rx_packed(hipStream_t st)
{
    const uint32_t n = 2500;
    const uint8_t src[4] = {10, 0, 0, 1}, dst[4] = {10, 0, 0, 2}, dst6[16] = {0xfd, [15] = 2};
    uint16_t *len16 = malloc(n * sizeof *len16);
    uint64_t *off = malloc(n * sizeof *off), *blk = malloc(((n + 63) / 64) * sizeof *blk), end = 0;
    uint8_t *proto = malloc(n), *status = malloc(n);
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t r = next_u64();
        len16[i] = (uint16_t)(40u + (uint32_t)((r >> 8) % 1461u));
        proto[i] = (i % 3 == 0) ? 6 : (i % 3 == 1) ? 17 : 1;
    }
    CHECK(rns_packed_layout(len16, n, 4, 0, blk, off, &end) == RNS_OK, "rns_packed_layout");
    const uint64_t bytes = end + 16;
    uint8_t *arena = malloc(bytes), *ref = malloc(bytes), *back = malloc(bytes);
    fill_random(arena, bytes);
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t *h = arena + off[i];
        h[0] = 0x45; h[1] = 0; h[2] = (uint8_t)(len16[i] >> 8); h[3] = (uint8_t)len16[i];
        h[6] = 0x40; h[7] = 0; h[8] = 64; h[9] = proto[i];
        memcpy(h + 12, src, 4);
        memcpy(h + 16, dst, 4);
    }
    memcpy(ref, arena, bytes);
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t *h = ref + off[i], *seg = h + 20;
        const uint32_t seglen = len16[i] - 20u, field = proto[i] == 6 ? 16u : proto[i] == 17 ? 6u : 2u;
        h[10] = h[11] = 0;
        const uint32_t ipc = (uint32_t)oracle_compute_checksum(h, 20);
        h[10] = (uint8_t)(ipc >> 8); h[11] = (uint8_t)ipc;
        seg[field] = seg[field + 1] = 0;
        const int32_t ph = proto[i] == 1 ? 0 : oracle_compute_pseudo_header_checksum(src, 4, dst, 4, seglen, proto[i]);
        const uint32_t l4 = 0xffffu ^ (uint32_t)oracle_compute_ones_comp((uint16_t)ph, seg, seglen);
        seg[field] = (uint8_t)(l4 >> 8); seg[field + 1] = (uint8_t)l4;
    }
    uint8_t *d_arena, *d_status, *d_slots;
    uint64_t *d_blk;
    uint16_t *d_len16;
    HIP_OK(hipMalloc((void **)&d_arena, bytes));
    HIP_OK(hipMalloc((void **)&d_blk, ((n + 63) / 64) * sizeof *blk));
    HIP_OK(hipMalloc((void **)&d_len16, n * sizeof *len16));
    HIP_OK(hipMalloc((void **)&d_status, n));
    HIP_OK(hipMalloc((void **)&d_slots, (uint64_t)n * 2048));
    HIP_OK(hipMemcpy(d_arena, arena, bytes, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_blk, blk, ((n + 63) / 64) * sizeof *blk, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_len16, len16, n * sizeof *len16, hipMemcpyHostToDevice));
    const uint32_t hints[2] = {0, 1500};
    for (int h = 0; h < 2; ++h) {
        HIP_OK(hipMemcpy(d_arena, arena, bytes, hipMemcpyHostToDevice));
        CHECK(rns_tx_fill_packed_dev(d_arena, bytes, d_blk, d_len16, 4, n, d_status, hints[h], st) == RNS_OK,
              "rns_tx_fill_packed_dev");
        HIP_OK(hipStreamSynchronize(st));
        HIP_OK(hipMemcpy(back, d_arena, bytes, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(status, d_status, n, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < n; ++i)
            CHECK(status[i] == (RNS_TX_IP_FILLED | RNS_TX_L4_FILLED), "packed tx (hint %u) status %u: %02x", hints[h],
                  i, status[i]);
        uint64_t diff = 0;
        for (uint64_t b = 0; b < bytes; ++b)
            diff += back[b] != ref[b];
        CHECK(diff == 0, "packed tx (hint %u): %llu arena bytes differ from the oracle's", hints[h],
              (unsigned long long)diff);
    }
    CHECK(rns_tx_fill_packed_dev(d_arena, bytes, d_blk, d_len16, 3, n, d_status, 0, st) == RNS_E_INVALID,
          "align_log2 < 4 is invalid");
    /* receive: the packed arena, then the datagrams in 2048-byte slots */
    CHECK(rns_rx_verify_packed_dev(d_arena, bytes, d_blk, d_len16, 4, n, dst, dst6, d_status, NULL, st) == RNS_OK,
          "rns_rx_verify_packed_dev");
    HIP_OK(hipStreamSynchronize(st));
    HIP_OK(hipMemcpy(status, d_status, n, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t want = RNS_RX_IP_OK | RNS_RX_ACCEPT | (proto[i] == 17 ? RNS_RX_L4_UNCHECKED : RNS_RX_L4_OK);
        CHECK(status[i] == want, "packed rx status %u: %02x != %02x", i, status[i], want);
    }
    for (uint32_t i = 0; i < n; ++i)
        HIP_OK(hipMemcpy(d_slots + (uint64_t)i * 2048, d_arena + off[i], len16[i], hipMemcpyDeviceToDevice));
    CHECK(rns_rx_verify_strided_dev(d_slots, (uint64_t)n * 2048, 0, 2048, d_len16, n, dst, dst6, d_status, NULL, st) ==
              RNS_OK, "rns_rx_verify_strided_dev");
    HIP_OK(hipStreamSynchronize(st));
    HIP_OK(hipMemcpy(status, d_status, n, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t want = RNS_RX_IP_OK | RNS_RX_ACCEPT | (proto[i] == 17 ? RNS_RX_L4_UNCHECKED : RNS_RX_L4_OK);
        CHECK(status[i] == want, "strided rx status %u: %02x != %02x", i, status[i], want);
    }
    hipFree(d_arena); hipFree(d_blk); hipFree(d_len16); hipFree(d_status); hipFree(d_slots);
    free(len16); free(off); free(blk); free(proto); free(status); free(arena); free(ref); free(back);
    return 0;
}

/* Transmit finalize of NetBuffer chains (rns_tx_fill_chain_dev): heads holding the IPv4 header
 * and the L4 header (TCP 20 B, UDP 8 B, ICMP 9 B: an odd head part) back to back from an odd
 * offset, payloads as 512-byte NetBuffer fragments packed at 16-byte starts.  Expected: the IPv4
 * header checksum (ip.rs:158-159) and the L4 checksum folded per fragment over [L4 header,
 * payload fragments] (util.rs:112-119 as tcp.rs:957-973 / udp.rs:158-171 / icmp.rs:91-94 call
 * it) with the fields zeroed; every other byte unchanged. */
static int test_tx_chain(hipStream_t st)
{
    const uint32_t n = 2000;
    const uint8_t src[4] = {10, 0, 0, 1}, dst[4] = {10, 0, 0, 2};
    uint32_t *first = malloc((n + 1) * sizeof *first), *hl = malloc(n * sizeof *hl), *pl = malloc(n * sizeof *pl);
    uint8_t *proto = malloc(n), *status = malloc(n);
    uint32_t nf = 0;
    uint64_t hpos = 3, ppos = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t r = next_u64();
        proto[i] = (i % 3 == 0) ? 6 : (i % 3 == 1) ? 17 : 1;
        hl[i] = 20u + (proto[i] == 6 ? 20u : proto[i] == 17 ? 8u : 9u);
        pl[i] = (uint32_t)((r >> 8) % 1461u);
        nf += 1u + (pl[i] + 511u) / 512u;
        hpos += hl[i];
    }
    uint64_t *off = malloc(nf * sizeof *off);
    uint32_t *len = malloc(nf * sizeof *len);
    ppos = (hpos + 4095) & ~4095ull;
    hpos = 3;
    nf = 0;
    for (uint32_t i = 0; i < n; ++i) {
        first[i] = nf;
        off[nf] = hpos;
        len[nf++] = hl[i];
        hpos += hl[i];
        for (uint32_t k = 0; k * 512u < pl[i]; ++k) {
            off[nf] = ppos + 512u * k;
            len[nf++] = pl[i] - 512u * k < 512u ? pl[i] - 512u * k : 512u;
        }
        ppos = (ppos + pl[i] + 15) & ~15ull;
    }
    first[n] = nf;
    const uint64_t bytes = ppos + 16;
    uint8_t *arena = malloc(bytes), *ref = malloc(bytes), *back = malloc(bytes);
    fill_random(arena, bytes);
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t *h = arena + off[first[i]];
        const uint32_t tot = hl[i] + pl[i];
        h[0] = 0x45; h[1] = 0; h[2] = (uint8_t)(tot >> 8); h[3] = (uint8_t)tot;
        h[6] = 0x40; h[7] = 0; h[8] = 64; h[9] = proto[i];
        memcpy(h + 12, src, 4);
        memcpy(h + 16, dst, 4);                      /* both checksum fields keep their garbage */
    }
    memcpy(ref, arena, bytes);
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t *h = ref + off[first[i]], *seg = h + 20;
        const uint32_t field = proto[i] == 6 ? 16u : proto[i] == 17 ? 6u : 2u;
        h[10] = h[11] = 0;
        const uint32_t ipc = (uint32_t)oracle_compute_checksum(h, 20);
        h[10] = (uint8_t)(ipc >> 8); h[11] = (uint8_t)ipc;
        seg[field] = seg[field + 1] = 0;
        int32_t acc = proto[i] == 1 ? 0 : oracle_compute_pseudo_header_checksum(src, 4, dst, 4, hl[i] - 20u + pl[i], proto[i]);
        acc = oracle_compute_ones_comp((uint16_t)acc, seg, hl[i] - 20u);
        for (uint32_t f = first[i] + 1; f < first[i + 1]; ++f)
            acc = oracle_compute_ones_comp((uint16_t)acc, ref + off[f], len[f]);
        const uint32_t l4 = 0xffffu ^ (uint32_t)acc;
        seg[field] = (uint8_t)(l4 >> 8); seg[field + 1] = (uint8_t)l4;
    }
    uint8_t *d_arena, *d_status;
    uint64_t *d_off;
    uint32_t *d_len, *d_first;
    HIP_OK(hipMalloc((void **)&d_arena, bytes));
    HIP_OK(hipMalloc((void **)&d_off, nf * sizeof *off));
    HIP_OK(hipMalloc((void **)&d_len, nf * sizeof *len));
    HIP_OK(hipMalloc((void **)&d_first, (n + 1) * sizeof *first));
    HIP_OK(hipMalloc((void **)&d_status, n));
    HIP_OK(hipMemcpy(d_arena, arena, bytes, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_off, off, nf * sizeof *off, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_len, len, nf * sizeof *len, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_first, first, (n + 1) * sizeof *first, hipMemcpyHostToDevice));
    CHECK(rns_tx_fill_chain_dev(d_arena, bytes, d_off, d_len, nf, d_first, n, d_status, st) == RNS_OK,
          "rns_tx_fill_chain_dev");
    HIP_OK(hipStreamSynchronize(st));
    HIP_OK(hipMemcpy(back, d_arena, bytes, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(status, d_status, n, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i)
        CHECK(status[i] == (RNS_TX_IP_FILLED | RNS_TX_L4_FILLED), "chain tx status %u: %02x", i, status[i]);
    uint64_t diff = 0;
    for (uint64_t b = 0; b < bytes; ++b)
        diff += back[b] != ref[b];
    CHECK(diff == 0, "chain tx: %llu arena bytes differ from the oracle's", (unsigned long long)diff);
    CHECK(rns_tx_fill_chain_dev(d_arena, bytes, d_off, d_len, nf, NULL, n, d_status, st) == RNS_E_INVALID,
          "NULL first");
    hipFree(d_arena); hipFree(d_off); hipFree(d_len); hipFree(d_first); hipFree(d_status);
    free(first); free(hl); free(pl); free(proto); free(status); free(off); free(len); free(arena); free(ref);
    free(back);
    return 0;
}

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

    /* 2b. the packed entry bench.py times, the fragment-chain entry, transmit finalize and
     *     receive verify: each against the oracle's util.rs restatement */
    if (test_packed(st) || test_strided(st) || test_chains(st) || test_chain_fill(st) || test_chain_fill_txpacked(st) || test_tx_rx(st) ||
        test_tx_rx_packed(st) || test_tx_chain(st))
        return 2;

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
