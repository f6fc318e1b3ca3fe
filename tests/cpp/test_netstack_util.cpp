// C++ parity checks of the netstack::util mirror (include/netstack_util.hpp),
// in the shape of the reference's own unit tests (src/stack/util.rs:275-457):
// one function per reference test, the same inputs and expected values.
// Built and run by tests/test_cpp_mirror.py (CPU only; no GPU call).
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "netstack_util.hpp"

using namespace netstack::util;

static int failures = 0;
#define EXPECT_EQ(a, b)                                                                         \
    do {                                                                                        \
        auto _a = (a);                                                                          \
        auto _b = (b);                                                                          \
        if (!(_a == _b)) {                                                                      \
            std::fprintf(stderr, "%s:%d: %s == %s failed (0x%llx vs 0x%llx)\n", __FILE__, __LINE__, \
                         #a, #b, (unsigned long long)_a, (unsigned long long)_b);              \
            ++failures;                                                                         \
        }                                                                                       \
    } while (0)

template <class F>
static bool panics(F f)
{
    try {
        f();
    } catch (const ReferencePanic &) {
        return true;
    }
    return false;
}

static void test_compute_ones_comp()  // util.rs:277-285
{
    EXPECT_EQ(compute_ones_comp(0, {0x00, 0x00}), 0);
    EXPECT_EQ(compute_ones_comp(0, {0x00, 0x01}), 0x1);
    EXPECT_EQ(compute_ones_comp(0, {0x00, 0xff}), 0xff);
    EXPECT_EQ(compute_ones_comp(0, {0xff, 0x23, 0xef, 0x55}), 0xee79);
}

static void test_compute_checksum()  // util.rs:288-293
{
    EXPECT_EQ(compute_checksum({0x00, 0x00}), 0xffff);
    EXPECT_EQ(compute_checksum({0x00, 0x01}), 0xfffe);
    EXPECT_EQ(compute_checksum({0x00, 0xff}), 0xff00);
    EXPECT_EQ(compute_checksum({0xff, 0x23, 0xef, 0x55}), 0x1186);
}

static void test_compute_packet_ones_comp()  // util.rs:296-300
{
    std::vector<uint8_t> frag = {0x12, 0x34};
    EXPECT_EQ(compute_buffer_ones_comp(0, {Slice(frag)}), 0x1234);
}

static void test_compute_packet_ones_comp_multiple_fragments()  // util.rs:303-312
{
    // 512 appends of 12 34 fill two 512-byte fragments (buf.rs:50)
    std::vector<uint8_t> frag;
    for (int i = 0; i < 256; i++) {
        frag.push_back(0x12);
        frag.push_back(0x34);
    }
    EXPECT_EQ(compute_buffer_ones_comp(0, {Slice(frag), Slice(frag)}), 0x6824);
}

static void test_compute_ones_comp_odd_length()  // util.rs:315-317
{
    EXPECT_EQ(compute_ones_comp(0, {0x12, 0x34, 0x56}), 0x6834);
}

static void test_compute_pseudo_header_checksum_v4()  // util.rs:436-443
{
    auto s = IPAddr::new_from({192, 168, 1, 1});
    auto d = IPAddr::new_from({192, 168, 1, 2});
    EXPECT_EQ(compute_pseudo_header_checksum(s, d, 20, 6), 0x836e);
}

static void test_compute_pseudo_header_checksum_v6()  // util.rs:446-457
{
    auto s = IPAddr::new_from({0x20, 0x01, 0x0d, 0xb8, 0xac, 0x10, 0xfe, 0x01, 0, 0, 0, 0, 0, 0, 0, 0});
    auto d = IPAddr::new_from({0x20, 0x01, 0x0d, 0xb8, 0xac, 0x10, 0xfe, 0x02, 0, 0, 0, 0, 0, 0, 0, 0});
    EXPECT_EQ(compute_pseudo_header_checksum(s, d, 20, 6), 0xafb2);
}

static void test_set_get_be()  // util.rs:320-371 (store convention of every checksum call site)
{
    uint8_t b[4] = {0};
    set_be16(b, 0x1234);
    EXPECT_EQ(get_be16(b), 0x1234);
    set_be32(b, 0xdeadbeef);
    EXPECT_EQ(get_be32(b), 0xdeadbeefu);
}

static void test_panics()  // where the reference panics, the mirror throws
{
    std::vector<uint8_t> empty;
    EXPECT_EQ(panics([&] { compute_ones_comp(0, Slice(empty)); }), true);       // util.rs:92
    EXPECT_EQ(panics([&] { compute_checksum(Slice(empty)); }), true);
    EXPECT_EQ(panics([&] { IPAddr::new_from({1, 2, 3}); }), true);              // util.rs:47
    auto v4 = IPAddr::new_from({10, 0, 0, 2});
    auto v6 = IPAddr::V6({0xfe, 0x80, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2});
    EXPECT_EQ(panics([&] { compute_pseudo_header_checksum(v6, v4, 20, 6); }), true);  // copy_to mismatch
}

static void test_ipv4_header_roundtrip()  // ip.rs:158-159 generate, ip.rs:76-80 verify
{
    uint8_t h[20] = {0x45, 0x00, 0x00, 0x73, 0x00, 0x00, 0x40, 0x00, 0x40, 0x11,
                     0x00, 0x00, 0xc0, 0xa8, 0x00, 0x01, 0xc0, 0xa8, 0x00, 0xc7};
    uint16_t c = compute_checksum(Slice(h, 20));
    EXPECT_EQ(c, 0xb861);
    set_be16(h + 10, c);
    EXPECT_EQ(compute_checksum(Slice(h, 20)), 0);
}

static void test_batch_without_device_fails_loudly()
{
    if (rns_device_count() > 0)
        return;  // only meaningful on a GPU-less host
    uint16_t out = 0;
    EXPECT_EQ(rns_csum_batch_dev(reinterpret_cast<const uint8_t *>(16), 16, reinterpret_cast<const uint64_t *>(16),
                                 reinterpret_cast<const uint32_t *>(16), nullptr, &out, 1, 0, 0, nullptr, nullptr),
              RNS_E_NODEVICE);
}

int main()
{
    test_compute_ones_comp();
    test_compute_checksum();
    test_compute_packet_ones_comp();
    test_compute_packet_ones_comp_multiple_fragments();
    test_compute_ones_comp_odd_length();
    test_compute_pseudo_header_checksum_v4();
    test_compute_pseudo_header_checksum_v6();
    test_set_get_be();
    test_panics();
    test_ipv4_header_roundtrip();
    test_batch_without_device_fails_loudly();
    if (failures) {
        std::fprintf(stderr, "%d failure(s)\n", failures);
        return 1;
    }
    std::printf("netstack_util mirror: all checks passed\n");
    return 0;
}
