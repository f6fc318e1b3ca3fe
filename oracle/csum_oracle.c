/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the Internet (RFC 1071) one's-complement checksum path of
 * jbush001/RustNetworkStack (src/stack/util.rs).  It is the checker the parity
 * tests compare the HIP path against, and the "port" CPU baseline bench.py
 * times.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it; the product library (rustnetworkstack_amd/csrc) never links it.
 *
 * Parity pinning: every function below is checked by tests/test_oracle_golden.py
 * against the reference's own known-answer tests (util.rs:277-317, 436-457)
 * and the RFC 1071 / IPv4-header vectors (tests/golden/reference_kats.json).
 * The reference itself (Rust) cannot be compiled in this image (no cargo/rustc),
 * so there is no oracle/_ref build; see DESIGN.md "Oracle".
 *
 * The restatement is deliberately literal: u32 accumulator that wraps like a
 * Rust release build, big-endian 16-bit words, odd final byte added as b<<8,
 * end-around fold in a while loop.  No vectorisation, no byte-order tricks.
 *
 * Panics in the reference are reported as -1 (RNS_ORACLE_PANIC).
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

#define RNS_ORACLE_PANIC (-1)

/* util.rs:88-106  pub fn compute_ones_comp(in_checksum: u16, slice: &[u8]) -> u16 */
int32_t oracle_compute_ones_comp(uint16_t in_checksum, const uint8_t *slice, size_t len)
{
    uint32_t checksum = in_checksum;               /* util.rs:89 */
    size_t i = 0;

    if (len == 0)                                   /* util.rs:92: slice.len() - 1 underflows */
        return RNS_ORACLE_PANIC;

    while (i < len - 1) {                           /* util.rs:92-95 */
        checksum += (uint32_t)(((uint32_t)slice[i] << 8) | slice[i + 1]);
        i += 2;
    }
    if (i < len)                                    /* util.rs:97-99 */
        checksum += (uint32_t)slice[i] << 8;

    while (checksum > 0xffff)                       /* util.rs:101-103 */
        checksum = (checksum & 0xffff) + (checksum >> 16);

    return (int32_t)(uint16_t)checksum;             /* util.rs:105 */
}

/* util.rs:108-110  pub fn compute_checksum(slice: &[u8]) -> u16 */
int32_t oracle_compute_checksum(const uint8_t *slice, size_t len)
{
    int32_t s = oracle_compute_ones_comp(0, slice, len);
    return s < 0 ? s : (int32_t)(0xffff ^ (uint32_t)s);
}

/*
 * util.rs:112-119  pub fn compute_buffer_ones_comp(initial_sum, &NetBuffer) -> u16
 * The NetBuffer's fragments are passed as (pointer, length) pairs in the order
 * buf.rs:466-487 BufferIterator::next yields them.  Each fragment is folded on
 * its own (an odd non-final fragment is zero-padded: util.rs:97-99).
 */
int32_t oracle_compute_buffer_ones_comp(uint16_t initial_sum, const uint8_t *const *frag_base,
                                        const size_t *frag_len, size_t nfrags)
{
    int32_t sum = initial_sum;                      /* util.rs:113 */
    for (size_t f = 0; f < nfrags; f++) {           /* util.rs:114-116 */
        sum = oracle_compute_ones_comp((uint16_t)sum, frag_base[f], frag_len[f]);
        if (sum < 0)
            return sum;
    }
    return sum;
}

/* util.rs:132-142 set_be16 / set_be32 */
static void set_be16(uint8_t *b, uint16_t v) { b[0] = (uint8_t)(v >> 8); b[1] = (uint8_t)v; }
static void set_be32(uint8_t *b, uint32_t v)
{
    b[0] = (uint8_t)(v >> 24); b[1] = (uint8_t)(v >> 16); b[2] = (uint8_t)(v >> 8); b[3] = (uint8_t)v;
}

/*
 * util.rs:180-207  pub fn compute_pseudo_header_checksum(source_ip, dest_ip, length, protocol)
 * Addresses are 4 (IPAddr::V4) or 16 (IPAddr::V6) bytes; the layout follows
 * the DEST variant (util.rs:186).  IPAddr::copy_to (util.rs:51-56) panics if
 * the source variant's length differs (copy_from_slice length mismatch).
 */
int32_t oracle_compute_pseudo_header_checksum(const uint8_t *src, size_t src_len, const uint8_t *dst,
                                              size_t dst_len, uint64_t length, uint8_t protocol)
{
    uint8_t ph[40];
    if ((src_len != 4 && src_len != 16) || (dst_len != 4 && dst_len != 16))
        return RNS_ORACLE_PANIC;                    /* IPAddr::new_from util.rs:41-48 */
    if (src_len != dst_len)
        return RNS_ORACLE_PANIC;                    /* copy_to into a slot of the dest's size */
    memset(ph, 0, sizeof(ph));
    if (dst_len == 4) {                             /* util.rs:187-195 */
        memcpy(ph + 0, src, 4);
        memcpy(ph + 4, dst, 4);
        ph[9] = protocol;
        set_be16(ph + 10, (uint16_t)length);        /* `length as u16` truncates */
        return oracle_compute_ones_comp(0, ph, 12);
    }
    memcpy(ph + 0, src, 16);                        /* util.rs:197-205 */
    memcpy(ph + 16, dst, 16);
    set_be32(ph + 32, (uint32_t)length);            /* `length as u32` truncates */
    ph[39] = protocol;
    return oracle_compute_ones_comp(0, ph, 40);
}

/*
 * Batch restatement: one compute_ones_comp per packet (the per-packet loop the
 * stack runs on its receive / transmit threads), optionally
 * complemented like every call site does (tcp.rs:848,970; udp.rs:168;
 * icmp.rs:46,91; ip.rs:76,158 via compute_checksum).
 *
 * len == 0 has no reference answer (it panics).  The product API defines it as
 * "seed unchanged"; the oracle reports the same so batch comparisons stay
 * total, and tests/ mark that case "parity unpinned".
 */
void oracle_batch(const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                  const uint16_t *seed, uint16_t *out, size_t n, int complement)
{
    for (size_t i = 0; i < n; i++) {
        uint16_t s = seed ? seed[i] : 0;
        int32_t r = len[i] ? oracle_compute_ones_comp(s, arena + off[i], len[i]) : (int32_t)s;
        out[i] = (uint16_t)(complement ? (0xffff ^ (uint32_t)r) : (uint32_t)r);
    }
}

/* The same loop partitioned by packet index over host threads (cpu_baseline, all cores). */
struct batch_job {
    const uint8_t *arena; const uint64_t *off; const uint32_t *len; const uint16_t *seed;
    uint16_t *out; size_t lo, hi; int complement;
};

static void *batch_worker(void *arg)
{
    struct batch_job *j = (struct batch_job *)arg;
    oracle_batch(j->arena, j->off + j->lo, j->len + j->lo, j->seed ? j->seed + j->lo : NULL,
                 j->out + j->lo, j->hi - j->lo, j->complement);
    return NULL;
}

int oracle_batch_mt(const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                    const uint16_t *seed, uint16_t *out, size_t n, int complement, int nthreads)
{
    pthread_t tid[256];
    struct batch_job job[256];
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; t++) {
        job[t] = (struct batch_job){arena, off, len, seed, out, n * t / nthreads,
                                    n * (t + 1) / nthreads, complement};
        if (pthread_create(&tid[t], NULL, batch_worker, &job[t]) != 0) {
            for (int u = 0; u < t; u++)
                pthread_join(tid[u], NULL);
            return -1;
        }
    }
    for (int t = 0; t < nthreads; t++)
        pthread_join(tid[t], NULL);
    return 0;
}

/*
 * benches/util_bench.rs:20-45 equivalent: time `iters` calls of
 * compute_ones_comp(0, buf[0..len]) in a tight loop (criterion's b.iter with
 * black_box), returning nanoseconds per call.
 */
double oracle_time_ones_comp(const uint8_t *buf, size_t len, uint64_t iters)
{
    struct timespec t0, t1;
    volatile int32_t sink = 0;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (uint64_t i = 0; i < iters; i++) {
        __asm__ volatile("" : : "r"(buf) : "memory");   /* black_box(&buf) */
        sink = oracle_compute_ones_comp(0, buf, len);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    (void)sink;
    return ((double)(t1.tv_sec - t0.tv_sec) * 1e9 + (double)(t1.tv_nsec - t0.tv_nsec)) / (double)(iters ? iters : 1);
}

/*
 * Batch of fragment chains: packet i = fragments [first[i], first[i+1]) of
 * (frag_off, frag_len) in `arena`, folded one after another from seed[i]
 * (util.rs:112-119 over BufferIterator's slices, buf.rs:466-487).  An empty
 * fragment would panic in the reference; here it leaves the sum unchanged, the
 * behaviour the product API defines (tests mark it "parity unpinned").
 */
void oracle_chain_batch(const uint8_t *arena, const uint64_t *frag_off, const uint32_t *frag_len,
                        const uint32_t *first, const uint16_t *seed, uint16_t *out, size_t npkts, int complement)
{
    for (size_t i = 0; i < npkts; i++) {
        int32_t sum = seed ? seed[i] : 0;
        for (uint32_t f = first[i]; f < first[i + 1]; f++)
            if (frag_len[f])
                sum = oracle_compute_ones_comp((uint16_t)sum, arena + frag_off[f], frag_len[f]);
        out[i] = (uint16_t)(complement ? (0xffff ^ (uint32_t)sum) : (uint32_t)sum);
    }
}

/*
 * Transmit finalize of NetBuffer chains (oracle.tx_chain_fill_ref in C; bench.py --op finalize's
 * CPU baseline).  Datagram i = fragments [first[i], first[i+1]): fragment first[i] is the head
 * alloc_header built (buf.rs:262-291: the IP header, then the L4 header), the rest the payload.
 * tcp_output / udp_output / icmp_output_* (tcp.rs:957-973, udp.rs:151-171, icmp.rs:87-112):
 * pseudo-header from the head's addresses and the chain's length, compute_buffer_ones_comp over
 * [head[hdr..], payload...] with the field zeroed, set_be16 of 0xffff ^ it; ip_output_v4
 * (ip.rs:140-160): compute_checksum(head[..IHL*4]) with [10..12] zeroed.  status[i] = TX bits
 * (1 IP filled, 2 L4 filled, 0x80 malformed: no fragments, a fragment outside the arena, a head
 * that does not hold the IP header, a bad version — left unchanged).  Empty pieces add nothing.
 */
static uint8_t tx_chain_fill_one(uint8_t *arena, uint64_t arena_bytes, const uint64_t *fo, const uint32_t *fl,
                                 uint32_t f0, uint32_t f1)
{
    if (f1 <= f0)
        return 0x80;
    uint64_t L = 0;
    for (uint32_t f = f0; f < f1; f++) {
        if (fo[f] > arena_bytes || fl[f] > arena_bytes - fo[f])
            return 0x80;
        L += fl[f];
    }
    uint8_t *h = arena + fo[f0];
    const uint32_t hl = fl[f0];
    if (hl == 0)
        return 0x80;
    const uint32_t version = h[0] >> 4;
    uint32_t hdr, proto;
    const uint8_t *src, *dst;
    size_t alen;
    if (version == 4) {
        hdr = (h[0] & 15u) * 4u;
        if (hdr < 20 || hdr > hl)
            return 0x80;
        proto = h[9]; src = h + 12; dst = h + 16; alen = 4;
    } else if (version == 6) {
        hdr = 40;
        if (hl < 40)
            return 0x80;
        proto = h[6]; src = h + 8; dst = h + 24; alen = 16;
    } else {
        return 0x80;
    }
    const uint64_t seg = L - hdr;
    int field = -1;
    int32_t seed = 0;
    if (proto == 6 || proto == 17) {
        field = proto == 6 ? 16 : 6;
        seed = oracle_compute_pseudo_header_checksum(src, alen, dst, alen, seg & 0xffff, (uint8_t)proto);
    } else if (proto == 1 && version == 4) {
        field = 2;
    } else if (proto == 58 && version == 6) {
        field = 2;
        seed = oracle_compute_pseudo_header_checksum(src, alen, dst, alen, seg, 58);
    }
    uint8_t st = 0;
    if (field >= 0 && seg >= (uint64_t)field + 2 && hdr + (uint32_t)field + 2 <= hl) {
        uint8_t *fp = h + hdr + field;
        fp[0] = fp[1] = 0;
        int32_t acc = seed;
        if (hl > hdr)
            acc = oracle_compute_ones_comp((uint16_t)acc, h + hdr, hl - hdr);
        for (uint32_t f = f0 + 1; f < f1; f++)
            if (fl[f])
                acc = oracle_compute_ones_comp((uint16_t)acc, arena + fo[f], fl[f]);
        set_be16(fp, (uint16_t)(0xffff ^ (uint32_t)acc));
        st |= 2;
    }
    if (version == 4) {
        h[10] = h[11] = 0;
        set_be16(h + 10, (uint16_t)oracle_compute_checksum(h, hdr));
        st |= 1;
    }
    return st;
}

void oracle_tx_chain_fill(uint8_t *arena, uint64_t arena_bytes, const uint64_t *frag_off, const uint32_t *frag_len,
                          const uint32_t *first, uint32_t n_frags, size_t n, uint8_t *status)
{
    for (size_t i = 0; i < n; i++) {
        const uint32_t f0 = first[i], f1 = first[i + 1];
        status[i] = (f0 <= f1 && f1 <= n_frags) ? tx_chain_fill_one(arena, arena_bytes, frag_off, frag_len, f0, f1)
                                                : 0x80;
    }
}

struct txc_job {
    uint8_t *arena; uint64_t arena_bytes; const uint64_t *fo; const uint32_t *fl; const uint32_t *first;
    uint32_t n_frags; uint8_t *status; size_t lo, hi;
};

static void *txc_worker(void *arg)
{
    struct txc_job *j = (struct txc_job *)arg;
    oracle_tx_chain_fill(j->arena, j->arena_bytes, j->fo, j->fl, j->first + j->lo, j->n_frags, j->hi - j->lo,
                         j->status + j->lo);
    return NULL;
}

/* The same partitioned by datagram index over host threads (datagrams must not share heads). */
int oracle_tx_chain_fill_mt(uint8_t *arena, uint64_t arena_bytes, const uint64_t *frag_off, const uint32_t *frag_len,
                            const uint32_t *first, uint32_t n_frags, size_t n, uint8_t *status, int nthreads)
{
    pthread_t tid[256];
    struct txc_job job[256];
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; t++) {
        job[t] = (struct txc_job){arena, arena_bytes, frag_off, frag_len, first, n_frags, status,
                                  n * t / nthreads, n * (t + 1) / nthreads};
        if (pthread_create(&tid[t], NULL, txc_worker, &job[t]) != 0) {
            for (int u = 0; u < t; u++)
                pthread_join(tid[u], NULL);
            return -1;
        }
    }
    for (int t = 0; t < nthreads; t++)
        pthread_join(tid[t], NULL);
    return 0;
}
