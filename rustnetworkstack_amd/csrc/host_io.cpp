// Batched datagram I/O for the receive / transmit ends of the checksum path
// (SURVEY §8f row 3).  The reference moves one packet per call: recv_packet
// (netif.rs:65-83) readv()s one datagram from the TUN fd into a 2048-byte MRU
// NetBuffer (tun.c:84-86), send_packet (netif.rs:85-98) writev()s one (tun.c:88-90).
// These entry points move a whole batch between such an fd (TUN, or any datagram
// fd: SOCK_SEQPACKET / SOCK_DGRAM) and an arena of fixed-size slots, so the batch
// can go to the GPU in one copy (rns_csum_batch_host / rns_rx_verify_dev).
#include <cerrno>
#include <cstdint>
#include <fcntl.h>
#include <climits>
#include <poll.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include "rns_checksum.h"

extern "C" {

int rns_io_recv_batch(int fd, uint8_t *h_arena, uint64_t slot_bytes, uint32_t max_pkts, uint64_t *h_off,
                      uint32_t *h_len, int timeout_ms)
{
    if (fd < 0 || !h_arena || !h_off || !h_len || slot_bytes == 0 || max_pkts == 0)
        return RNS_E_INVALID;
    if (max_pkts > static_cast<uint32_t>(INT_MAX))  // the count is returned as an int
        max_pkts = static_cast<uint32_t>(INT_MAX);
    struct pollfd pfd = {fd, POLLIN, 0};
    int pr;
    do {
        pr = poll(&pfd, 1, timeout_ms);  // wait for the first datagram only
    } while (pr < 0 && errno == EINTR);
    if (pr < 0)
        return RNS_E_IO;
    if (pr == 0)
        return 0;
    const int flags = fcntl(fd, F_GETFL);
    if (flags < 0)
        return RNS_E_IO;
    const bool was_blocking = !(flags & O_NONBLOCK);
    if (was_blocking && fcntl(fd, F_SETFL, flags | O_NONBLOCK) < 0)
        return RNS_E_IO;
    uint32_t n = 0;
    int status = 0;
    bool sock = true;  // socket fds: recv(MSG_TRUNC) reports a datagram's full length
    while (n < max_pkts) {
        uint8_t *slot = h_arena + static_cast<uint64_t>(n) * slot_bytes;
        ssize_t r;
        if (sock) {
            r = recv(fd, slot, slot_bytes, MSG_TRUNC);
            if (r < 0 && errno == ENOTSOCK) {
                sock = false;
                continue;
            }
        } else {
            r = read(fd, slot, slot_bytes);  // one datagram per read, like tun_recv
        }
        if (r < 0) {
            if (errno == EINTR)
                continue;
            if (errno != EAGAIN && errno != EWOULDBLOCK)
                status = RNS_E_IO;
            break;
        }
        if (r == 0)  // peer closed (socket fds)
            break;
        if (static_cast<uint64_t>(r) > slot_bytes)  // longer than its slot: dropped, never
            continue;                               // handed on truncated (its slot is reused)
        h_off[n] = static_cast<uint64_t>(n) * slot_bytes;
        h_len[n] = static_cast<uint32_t>(r);
        ++n;
    }
    if (was_blocking)
        (void)fcntl(fd, F_SETFL, flags);
    return (n == 0 && status) ? status : static_cast<int>(n);
}

int rns_io_send_batch(int fd, const uint8_t *h_arena, const uint64_t *h_off, const uint32_t *h_len, uint32_t n)
{
    if (fd < 0 || (n && (!h_arena || !h_off || !h_len)))
        return RNS_E_INVALID;
    for (uint32_t i = 0; i < n; ++i) {
        struct iovec v = {const_cast<uint8_t *>(h_arena + h_off[i]), h_len[i]};
        ssize_t w;
        do {
            w = writev(fd, &v, 1);  // one datagram per writev, like tun_send
        } while (w < 0 && errno == EINTR);
        if (w < 0)
            return i ? static_cast<int>(i) : RNS_E_IO;
    }
    return static_cast<int>(n);
}

}  // extern "C"
