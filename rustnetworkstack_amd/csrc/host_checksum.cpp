// Per-packet host entry points of the C ABI (include/rns_checksum.h, group 1).
//
// These are the calls util.rs's four public functions forward to
// (src/stack/util.rs:88, 108, 112, 180).  One packet is ~100 ns of CPU work and
// a GPU launch is microseconds, so single-packet calls stay on the calling
// thread; batches go to the gfx950 kernels (rns_checksum.hip).
//
// Arithmetic: the reference keeps a u32 accumulator `in_checksum + sum of BE
// words` that wraps mod 2^32 (util.rs:89-99) and folds it end-around
// (util.rs:101-103).  Here the word sum is formed exactly in 64 bits from
// 8-byte little-endian loads, split into the bytes that are the high half of
// a BE word (even offsets) and the low half (odd offsets):
//     sum_words = 256 * sum(even bytes) + sum(odd bytes)
// then reduced mod 2^32 and folded the same way, so the result equals the
// reference's for every length, including the wrap beyond 131072 bytes.
#include <cstdint>
#include <cstring>

#include "rns_checksum.h"

namespace {

constexpr uint64_t kByteLanes = 0x00ff00ff00ff00ffull;

// Sum of the four 16-bit fields of x.
inline uint64_t hsum16(uint64_t x)
{
    return (x & 0xffff) + ((x >> 16) & 0xffff) + ((x >> 32) & 0xffff) + (x >> 48);
}

// Exact sum of the big-endian 16-bit words of p[0..len), the odd final byte as byte << 8.
uint64_t be_word_sum(const uint8_t *p, size_t len)
{
    uint64_t even_total = 0, odd_total = 0;
    size_t i = 0;
    while (len - i >= 8) {
        // Each 16-bit field gains at most 0xff per step: 256 steps cannot carry across fields.
        size_t steps = (len - i) / 8;
        if (steps > 256)
            steps = 256;
        uint64_t even = 0, odd = 0;
        for (size_t k = 0; k < steps; k++, i += 8) {
            uint64_t w;
            std::memcpy(&w, p + i, 8);
            even += w & kByteLanes;          // bytes at offsets 0,2,4,6: BE high halves
            odd += (w >> 8) & kByteLanes;    // bytes at offsets 1,3,5,7: BE low halves
        }
        even_total += hsum16(even);
        odd_total += hsum16(odd);
    }
    if (i < len) {  // tail, zero-padded: an odd final byte lands in a high half (util.rs:97-99)
        uint64_t w = 0;
        std::memcpy(&w, p + i, len - i);
        even_total += hsum16(w & kByteLanes);
        odd_total += hsum16((w >> 8) & kByteLanes);
    }
    return (even_total << 8) + odd_total;
}

inline uint16_t fold_u32(uint32_t checksum)
{
    while (checksum > 0xffff)  // util.rs:101-103
        checksum = (checksum & 0xffff) + (checksum >> 16);
    return static_cast<uint16_t>(checksum);
}

inline uint16_t ones_comp(uint16_t seed, const uint8_t *p, size_t len)
{
    uint32_t acc = static_cast<uint32_t>(seed + be_word_sum(p, len));  // mod 2^32 like util.rs:89-99
    return fold_u32(acc);
}

}  // namespace

extern "C" {

int32_t rns_compute_ones_comp(uint16_t in_checksum, const uint8_t *slice, size_t len)
{
    if (len == 0)
        return RNS_E_EMPTY;
    if (slice == nullptr)
        return RNS_E_INVALID;
    return ones_comp(in_checksum, slice, len);
}

int32_t rns_compute_checksum(const uint8_t *slice, size_t len)
{
    int32_t s = rns_compute_ones_comp(0, slice, len);
    return s < 0 ? s : (0xffff ^ s);  // util.rs:108-110
}

int32_t rns_compute_buffer_ones_comp(uint16_t initial_sum, const rns_iovec *frags, size_t nfrags)
{
    if (nfrags != 0 && frags == nullptr)
        return RNS_E_INVALID;
    uint16_t sum = initial_sum;  // util.rs:113-118: fold after every fragment
    for (size_t f = 0; f < nfrags; f++) {
        int32_t r = rns_compute_ones_comp(sum, frags[f].base, frags[f].len);
        if (r < 0)
            return r;
        sum = static_cast<uint16_t>(r);
    }
    return sum;
}

int32_t rns_compute_pseudo_header_checksum(const rns_ipaddr *source_ip, const rns_ipaddr *dest_ip,
                                           uint64_t length, uint8_t protocol)
{
    if (source_ip == nullptr || dest_ip == nullptr)
        return RNS_E_INVALID;
    if ((dest_ip->version != 4 && dest_ip->version != 6) || source_ip->version != dest_ip->version)
        return RNS_E_INVALID;  // reference: copy_to length mismatch panics (util.rs:51-56)
    uint8_t ph[40] = {0};
    if (dest_ip->version == 4) {  // util.rs:187-195: src4 dst4 00 proto len16
        std::memcpy(ph, source_ip->bytes, 4);
        std::memcpy(ph + 4, dest_ip->bytes, 4);
        ph[9] = protocol;
        ph[10] = static_cast<uint8_t>(length >> 8);
        ph[11] = static_cast<uint8_t>(length);
        return ones_comp(0, ph, 12);
    }
    // util.rs:197-205: src16 dst16 len32 00 00 00 proto
    std::memcpy(ph, source_ip->bytes, 16);
    std::memcpy(ph + 16, dest_ip->bytes, 16);
    ph[32] = static_cast<uint8_t>(length >> 24);
    ph[33] = static_cast<uint8_t>(length >> 16);
    ph[34] = static_cast<uint8_t>(length >> 8);
    ph[35] = static_cast<uint8_t>(length);
    ph[39] = protocol;
    return ones_comp(0, ph, 40);
}

int rns_packed_layout(const uint16_t *len16, uint64_t n, uint32_t align_log2, uint64_t first_off, uint64_t *blk_off,
                      uint64_t *off, uint64_t *end)
{
    if ((n && (!len16 || !blk_off)) || !end || align_log2 > 12)
        return RNS_E_INVALID;
    const uint64_t m = (1ull << align_log2) - 1;
    uint64_t at = first_off;
    for (uint64_t i = 0; i < n; ++i) {
        if ((i & 63) == 0)
            blk_off[i >> 6] = at;
        if (off)
            off[i] = at;
        at += (static_cast<uint64_t>(len16[i]) + m) & ~m;  // the kernels' padded length
    }
    *end = at;
    return RNS_OK;
}

int rns_abi_version(void) { return RNS_ABI_VERSION; }

const char *rns_strerror(int status)
{
    switch (status) {
    case RNS_OK: return "ok";
    case RNS_E_INVALID: return "invalid argument";
    case RNS_E_EMPTY: return "empty slice (the reference panics: util.rs:92)";
    case RNS_E_BOUNDS: return "packet descriptor outside its arena";
    case RNS_E_NODEVICE: return "no usable gfx950 device";
    case RNS_E_ORDER: return "packet offsets are not ascending";
    case RNS_E_TOOLARGE: return "packet larger than the staging chunk";
    case RNS_E_IO: return "datagram I/O failed (errno)";
    default: return status <= RNS_E_HIP_BASE ? "HIP runtime error" : "unknown status";
    }
}

}  // extern "C"
