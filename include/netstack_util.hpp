// netstack_util.hpp — C++ mirror of the reference's checksum surface
// `netstack::util` (jbush001/RustNetworkStack src/stack/util.rs), built on the
// C ABI in rns_checksum.h.  Same names, argument meaning and error behaviour:
// where the Rust code panics this throws netstack::util::ReferencePanic.
//
//   util.rs:22-57    enum IPAddr            -> class IPAddr (V4 / V6 / new_from / copy_to)
//   util.rs:88-106   compute_ones_comp      -> compute_ones_comp(in_checksum, slice)
//   util.rs:108-110  compute_checksum       -> compute_checksum(slice)
//   util.rs:112-119  compute_buffer_ones_comp(initial_sum, &NetBuffer)
//                                           -> compute_buffer_ones_comp(initial_sum, fragments)
//   util.rs:180-207  compute_pseudo_header_checksum(src, dst, length, protocol)
//   util.rs:121-142  get_be16/get_be32/set_be16/set_be32
//
// Batches of packets go through the GPU entry points of rns_checksum.h
// (rns_csum_batch_dev / rns_csum_batch_host); this header is the per-packet
// surface the stack's IP/TCP/UDP/ICMP call sites use.
#ifndef NETSTACK_UTIL_HPP
#define NETSTACK_UTIL_HPP

#include <array>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <initializer_list>
#include <stdexcept>
#include <string>
#include <vector>

#include "rns_checksum.h"

namespace netstack {
namespace util {

struct ReferencePanic : std::logic_error {
    explicit ReferencePanic(const std::string &what) : std::logic_error(what) {}
};

// Borrowed byte slice: the `&[u8]` of the Rust signatures.
struct Slice {
    const uint8_t *ptr;
    size_t len;
    Slice(const uint8_t *p, size_t n) : ptr(p), len(n) {}
    template <class C>
    Slice(const C &c) : ptr(reinterpret_cast<const uint8_t *>(c.data())), len(c.size() * sizeof(*c.data())) {}
    // A braced literal lives until the end of the full expression: long enough for every call below.
#if defined(__GNUC__) && !defined(__clang__)
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Winit-list-lifetime"
#endif
    Slice(std::initializer_list<uint8_t> il) : ptr(il.begin()), len(il.size()) {}
#if defined(__GNUC__) && !defined(__clang__)
#pragma GCC diagnostic pop
#endif
};

inline uint16_t checked(int32_t r, const char *what)
{
    if (r == RNS_E_EMPTY)
        throw ReferencePanic(std::string(what) + ": empty slice (util.rs:92 panics)");
    if (r < 0)
        throw ReferencePanic(std::string(what) + ": " + rns_strerror(r));
    return static_cast<uint16_t>(r);
}

// util.rs:88
inline uint16_t compute_ones_comp(uint16_t in_checksum, Slice slice)
{
    return checked(rns_compute_ones_comp(in_checksum, slice.ptr, slice.len), "compute_ones_comp");
}

// util.rs:108
inline uint16_t compute_checksum(Slice slice)
{
    return checked(rns_compute_checksum(slice.ptr, slice.len), "compute_checksum");
}

// util.rs:112 — `buffer` is the fragment sequence NetBuffer::iter yields (buf.rs:466-487).
inline uint16_t compute_buffer_ones_comp(uint16_t initial_sum, const std::vector<Slice> &buffer)
{
    std::vector<rns_iovec> v;
    v.reserve(buffer.size());
    for (const Slice &s : buffer)
        v.push_back(rns_iovec{s.ptr, s.len});
    return checked(rns_compute_buffer_ones_comp(initial_sum, v.data(), v.size()), "compute_buffer_ones_comp");
}

// util.rs:22-57
class IPAddr {
public:
    IPAddr() : c_{4, {0}} {}  // IPAddr::new() = V4(0.0.0.0)
    static IPAddr V4(const std::array<uint8_t, 4> &a) { return IPAddr(4, a.data(), 4); }
    static IPAddr V6(const std::array<uint8_t, 16> &a) { return IPAddr(6, a.data(), 16); }
    static IPAddr new_from(Slice addr)
    {
        if (addr.len == 4)
            return IPAddr(4, addr.ptr, 4);
        if (addr.len == 16)
            return IPAddr(6, addr.ptr, 16);
        throw ReferencePanic("Invalid IP address length");  // util.rs:47
    }
    bool is_v4() const { return c_.version == 4; }
    size_t len() const { return is_v4() ? 4 : 16; }
    void copy_to(uint8_t *buffer, size_t buffer_len) const
    {
        if (buffer_len != len())
            throw ReferencePanic("copy_from_slice length mismatch");  // util.rs:51-56
        std::memcpy(buffer, c_.bytes, len());
    }
    const rns_ipaddr &c() const { return c_; }
    bool operator==(const IPAddr &o) const
    {
        return c_.version == o.c_.version && std::memcmp(c_.bytes, o.c_.bytes, len()) == 0;
    }

private:
    IPAddr(uint32_t v, const uint8_t *p, size_t n) : c_{v, {0}} { std::memcpy(c_.bytes, p, n); }
    rns_ipaddr c_;
};

// util.rs:180
inline uint16_t compute_pseudo_header_checksum(const IPAddr &source_ip, const IPAddr &dest_ip, size_t length,
                                               uint8_t protocol)
{
    return checked(rns_compute_pseudo_header_checksum(&source_ip.c(), &dest_ip.c(), length, protocol),
                   "compute_pseudo_header_checksum");
}

// util.rs:121-142
inline uint16_t get_be16(const uint8_t *b) { return static_cast<uint16_t>((b[0] << 8) | b[1]); }
inline uint32_t get_be32(const uint8_t *b)
{
    return (uint32_t(b[0]) << 24) | (uint32_t(b[1]) << 16) | (uint32_t(b[2]) << 8) | uint32_t(b[3]);
}
inline void set_be16(uint8_t *b, uint16_t v)
{
    b[0] = static_cast<uint8_t>(v >> 8);
    b[1] = static_cast<uint8_t>(v);
}
inline void set_be32(uint8_t *b, uint32_t v)
{
    b[0] = static_cast<uint8_t>(v >> 24);
    b[1] = static_cast<uint8_t>(v >> 16);
    b[2] = static_cast<uint8_t>(v >> 8);
    b[3] = static_cast<uint8_t>(v);
}

}  // namespace util
}  // namespace netstack

#endif  // NETSTACK_UTIL_HPP
