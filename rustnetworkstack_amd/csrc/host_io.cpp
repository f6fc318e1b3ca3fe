// Batched datagram I/O for the receive / transmit ends of the checksum path
// (SURVEY §8f row 3).  The reference moves one packet per call: recv_packet
// (netif.rs:65-83) readv()s one datagram from the TUN fd into a 2048-byte MRU
// NetBuffer (tun.c:84-86), send_packet (netif.rs:85-98) writev()s one (tun.c:88-90).
// These entry points move a whole batch between such an fd (TUN, or any datagram
// fd: SOCK_SEQPACKET / SOCK_DGRAM) and an arena, so the batch can go to the GPU in
// one copy (rns_rx_verify_packed_dev / rns_rx_verify_dev / rns_tx_fill_packed_dev).
// On a socket fd a batch takes recvmmsg / sendmmsg: up to kMmsg datagrams per system
// call; a TUN fd moves one datagram per read / writev (its driver has no batched call).
// rns_io_send_batch_chain sends NetBuffer chains as send_packet does — each datagram's
// fragments as one gather write (to_iovec + tun_send's writev, netif.rs:51-63, 85-98).
#include <cerrno>
#include <climits>
#include <cstdint>
#include <cstring>
#include <fcntl.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include "rns_checksum.h"

namespace {

constexpr unsigned kMmsg = 64;  // datagrams per recvmmsg / sendmmsg call
constexpr uint32_t kChainIov = RNS_IO_MAX_FRAGS;  // fragments per datagram (netif.rs:22 MAX_VECS)

// Waits up to timeout_ms for the first datagram; 1 = readable, 0 = timeout, < 0 = error.
int wait_first(int fd, int timeout_ms)
{
    struct pollfd pfd = {fd, POLLIN, 0};
    int pr;
    do {
        pr = poll(&pfd, 1, timeout_ms);  // wait for the first datagram only
    } while (pr < 0 && errno == EINTR);
    return pr < 0 ? RNS_E_IO : pr;
}

// The fd in non-blocking mode for the duration of one batch (TUN reads), restored after.
struct NonBlocking {
    int fd, flags = -1;
    bool changed = false;
    explicit NonBlocking(int f) : fd(f)
    {
        flags = fcntl(fd, F_GETFL);
        if (flags >= 0 && !(flags & O_NONBLOCK))
            changed = fcntl(fd, F_SETFL, flags | O_NONBLOCK) == 0;
    }
    bool ok() const { return flags >= 0 && ((flags & O_NONBLOCK) || changed); }
    ~NonBlocking()
    {
        if (changed)
            (void)fcntl(fd, F_SETFL, flags);
    }
};

// One recvmmsg round into k buffers of cap bytes at bufs[i]: the number of messages
// (their lengths in len[], each flagged in trunc[] if it did not fit), 0 when nothing
// is queued, RNS_E_IO on an error, -ENOTSOCK when the fd is not a socket.
int recv_round(int fd, uint8_t *const *bufs, uint64_t cap, unsigned k, uint32_t *len, bool *trunc)
{
    struct mmsghdr mh[kMmsg];
    struct iovec iov[kMmsg];
    std::memset(mh, 0, sizeof(mh));
    for (unsigned i = 0; i < k; ++i) {
        iov[i].iov_base = bufs[i];
        iov[i].iov_len = cap;
        mh[i].msg_hdr.msg_iov = &iov[i];
        mh[i].msg_hdr.msg_iovlen = 1;
    }
    int r;
    do {
        r = recvmmsg(fd, mh, k, MSG_DONTWAIT | MSG_TRUNC, nullptr);
    } while (r < 0 && errno == EINTR);
    if (r < 0) {
        if (errno == ENOTSOCK)
            return -ENOTSOCK;
        return (errno == EAGAIN || errno == EWOULDBLOCK) ? 0 : RNS_E_IO;
    }
    for (int i = 0; i < r; ++i) {
        len[i] = mh[i].msg_len;
        trunc[i] = (mh[i].msg_hdr.msg_flags & MSG_TRUNC) || mh[i].msg_len > cap;
    }
    return r;
}

}  // namespace

extern "C" {

int rns_io_recv_batch(int fd, uint8_t *h_arena, uint64_t slot_bytes, uint32_t max_pkts, uint64_t *h_off,
                      uint32_t *h_len, int timeout_ms)
{
    if (fd < 0 || !h_arena || !h_off || !h_len || slot_bytes == 0 || max_pkts == 0)
        return RNS_E_INVALID;
    if (max_pkts > static_cast<uint32_t>(INT_MAX))  // the count is returned as an int
        max_pkts = static_cast<uint32_t>(INT_MAX);
    const int pr = wait_first(fd, timeout_ms);
    if (pr <= 0)
        return pr;
    uint32_t n = 0;
    int status = 0;
    bool sock = true;
    while (sock && n < max_pkts) {  // sockets: recvmmsg straight into the next slots
        const unsigned k = max_pkts - n < kMmsg ? max_pkts - n : kMmsg;
        uint8_t *bufs[kMmsg];
        for (unsigned i = 0; i < k; ++i)
            bufs[i] = h_arena + static_cast<uint64_t>(n + i) * slot_bytes;
        uint32_t len[kMmsg];
        bool trunc[kMmsg];
        const int r = recv_round(fd, bufs, slot_bytes, k, len, trunc);
        if (r == -ENOTSOCK) {
            sock = false;
            break;
        }
        if (r < 0)
            status = r;
        if (r <= 0)
            return (n == 0 && status) ? status : static_cast<int>(n);
        int eof = 0;
        uint32_t kept = 0;
        for (int i = 0; i < r; ++i) {
            if (len[i] == 0) {  // peer closed (a zero-length datagram cannot be told from it)
                eof = 1;
                break;
            }
            if (trunc[i])  // longer than its slot: dropped, never handed on truncated
                continue;
            const uint32_t d = n + kept;
            if (d != n + static_cast<uint32_t>(i))  // close the gap a dropped datagram left
                std::memmove(h_arena + static_cast<uint64_t>(d) * slot_bytes, bufs[i], len[i]);
            h_off[d] = static_cast<uint64_t>(d) * slot_bytes;
            h_len[d] = len[i];
            ++kept;
        }
        n += kept;
        if (eof || static_cast<unsigned>(r) < k)
            return static_cast<int>(n);
    }
    if (sock)
        return static_cast<int>(n);
    NonBlocking nb(fd);  // a TUN fd: one datagram per read, like tun_recv
    if (!nb.ok())
        return RNS_E_IO;
    while (n < max_pkts) {
        uint8_t *slot = h_arena + static_cast<uint64_t>(n) * slot_bytes;
        const ssize_t r = read(fd, slot, slot_bytes);
        if (r < 0) {
            if (errno == EINTR)
                continue;
            if (errno != EAGAIN && errno != EWOULDBLOCK)
                status = RNS_E_IO;
            break;
        }
        if (r == 0)
            break;
        if (static_cast<uint64_t>(r) > slot_bytes)
            continue;
        h_off[n] = static_cast<uint64_t>(n) * slot_bytes;
        h_len[n] = static_cast<uint32_t>(r);
        ++n;
    }
    return (n == 0 && status) ? status : static_cast<int>(n);
}

int rns_io_recv_batch_packed(int fd, uint8_t *h_arena, uint64_t arena_bytes, uint32_t mru, uint32_t max_pkts,
                             uint16_t *h_len16, uint64_t *h_blk_off, uint64_t *h_end, int timeout_ms)
{
    if (fd < 0 || !h_arena || !h_len16 || !h_blk_off || !h_end || mru == 0 || mru > 0xFFFFu || max_pkts == 0)
        return RNS_E_INVALID;
    if (max_pkts > static_cast<uint32_t>(INT_MAX))
        max_pkts = static_cast<uint32_t>(INT_MAX);
    *h_end = 0;
    const int pr = wait_first(fd, timeout_ms);
    if (pr <= 0)
        return pr;
    const uint64_t step = (static_cast<uint64_t>(mru) + 15) & ~15ull;  // >= any padded datagram
    uint64_t pos = 0;  // where the next datagram goes (16-byte aligned)
    uint32_t n = 0;
    int status = 0;
    auto take = [&](uint32_t len) {  // datagram n of len bytes now lies at pos
        if ((n & 63u) == 0)
            h_blk_off[n >> 6] = pos;
        h_len16[n] = static_cast<uint16_t>(len);
        ++n;
        pos = (pos + len + 15) & ~15ull;
    };
    bool sock = true;
    while (sock && n < max_pkts) {
        // recvmmsg into MRU-sized buffers (16-byte steps) from pos on, then each datagram moves
        // down to its packed place (at or below its buffer: one memmove of its own bytes)
        const uint64_t room = arena_bytes > pos ? (arena_bytes - pos) / step : 0;
        unsigned k = max_pkts - n < kMmsg ? max_pkts - n : kMmsg;
        if (room < k)
            k = static_cast<unsigned>(room);
        if (k == 0)
            break;
        uint8_t *bufs[kMmsg];
        for (unsigned i = 0; i < k; ++i)
            bufs[i] = h_arena + pos + static_cast<uint64_t>(i) * step;
        uint32_t len[kMmsg];
        bool trunc[kMmsg];
        const int r = recv_round(fd, bufs, mru, k, len, trunc);
        if (r == -ENOTSOCK) {
            sock = false;
            break;
        }
        if (r < 0)
            status = r;
        if (r <= 0)
            break;
        bool eof = false;
        for (int i = 0; i < r; ++i) {
            if (len[i] == 0) {
                eof = true;
                break;
            }
            if (trunc[i])
                continue;
            if (h_arena + pos != bufs[i])
                std::memmove(h_arena + pos, bufs[i], len[i]);
            take(len[i]);
        }
        if (eof || static_cast<unsigned>(r) < k) {
            *h_end = pos;
            return static_cast<int>(n);
        }
    }
    if (!sock) {
        NonBlocking nb(fd);
        if (!nb.ok())
            return RNS_E_IO;
        while (n < max_pkts && arena_bytes > pos && arena_bytes - pos >= mru) {
            const ssize_t r = read(fd, h_arena + pos, mru);
            if (r < 0) {
                if (errno == EINTR)
                    continue;
                if (errno != EAGAIN && errno != EWOULDBLOCK)
                    status = RNS_E_IO;
                break;
            }
            if (r == 0)
                break;
            if (static_cast<uint64_t>(r) > mru)
                continue;
            take(static_cast<uint32_t>(r));
        }
    }
    *h_end = pos;
    return (n == 0 && status) ? status : static_cast<int>(n);
}

int rns_io_send_batch(int fd, const uint8_t *h_arena, const uint64_t *h_off, const uint32_t *h_len, uint32_t n)
{
    if (fd < 0 || (n && (!h_arena || !h_off || !h_len)))
        return RNS_E_INVALID;
    if (n > static_cast<uint32_t>(INT_MAX))
        n = static_cast<uint32_t>(INT_MAX);
    uint32_t i = 0;
    bool sock = true;
    while (sock && i < n) {  // sockets: sendmmsg, kMmsg datagrams per call
        const unsigned k = n - i < kMmsg ? n - i : kMmsg;
        struct mmsghdr mh[kMmsg];
        struct iovec iov[kMmsg];
        std::memset(mh, 0, sizeof(mh));
        for (unsigned j = 0; j < k; ++j) {
            iov[j].iov_base = const_cast<uint8_t *>(h_arena + h_off[i + j]);
            iov[j].iov_len = h_len[i + j];
            mh[j].msg_hdr.msg_iov = &iov[j];
            mh[j].msg_hdr.msg_iovlen = 1;
        }
        int w;
        do {
            w = sendmmsg(fd, mh, k, 0);
        } while (w < 0 && errno == EINTR);
        if (w < 0) {
            if (errno == ENOTSOCK && i == 0) {
                sock = false;
                break;
            }
            return i ? static_cast<int>(i) : RNS_E_IO;
        }
        i += static_cast<uint32_t>(w);
    }
    for (; i < n; ++i) {  // a TUN fd: one datagram per writev, like tun_send
        struct iovec v = {const_cast<uint8_t *>(h_arena + h_off[i]), h_len[i]};
        ssize_t w;
        do {
            w = writev(fd, &v, 1);
        } while (w < 0 && errno == EINTR);
        if (w < 0)
            return i ? static_cast<int>(i) : RNS_E_IO;
    }
    return static_cast<int>(n);
}

int rns_io_send_batch_chain(int fd, const uint8_t *h_arena, const uint64_t *h_frag_off, const uint32_t *h_frag_len,
                            const uint32_t *h_first, uint32_t n_pkts)
{
    if (fd < 0 || (n_pkts && (!h_arena || !h_first)))
        return RNS_E_INVALID;
    if (n_pkts > static_cast<uint32_t>(INT_MAX))
        n_pkts = static_cast<uint32_t>(INT_MAX);
    // every datagram's fragment range first (1..kChainIov fragments; an empty datagram would read
    // as end-of-stream on a SOCK_SEQPACKET peer): a malformed one sends nothing
    for (uint32_t i = 0; i < n_pkts; ++i) {
        const uint32_t f0 = h_first[i], f1 = h_first[i + 1];
        if (f1 <= f0 || f1 - f0 > kChainIov || !h_frag_off || !h_frag_len)
            return RNS_E_INVALID;
    }
    uint32_t i = 0;
    bool sock = true;
    while (sock && i < n_pkts) {  // sockets: sendmmsg, each message one datagram's fragments
        const unsigned k = n_pkts - i < kMmsg ? n_pkts - i : kMmsg;
        struct mmsghdr mh[kMmsg];
        struct iovec iov[kMmsg * kChainIov];
        std::memset(mh, 0, sizeof(mh));
        for (unsigned j = 0; j < k; ++j) {
            const uint32_t f0 = h_first[i + j], nf = h_first[i + j + 1] - f0;
            struct iovec *v = iov + j * kChainIov;
            for (uint32_t f = 0; f < nf; ++f) {
                v[f].iov_base = const_cast<uint8_t *>(h_arena + h_frag_off[f0 + f]);
                v[f].iov_len = h_frag_len[f0 + f];
            }
            mh[j].msg_hdr.msg_iov = v;
            mh[j].msg_hdr.msg_iovlen = nf;
        }
        int w;
        do {
            w = sendmmsg(fd, mh, k, 0);
        } while (w < 0 && errno == EINTR);
        if (w < 0) {
            if (errno == ENOTSOCK && i == 0) {
                sock = false;
                break;
            }
            return i ? static_cast<int>(i) : RNS_E_IO;
        }
        i += static_cast<uint32_t>(w);
    }
    for (; i < n_pkts; ++i) {  // a TUN fd: one writev per datagram over its fragments, like tun_send
        const uint32_t f0 = h_first[i], nf = h_first[i + 1] - f0;
        struct iovec v[kChainIov];
        for (uint32_t f = 0; f < nf; ++f) {
            v[f].iov_base = const_cast<uint8_t *>(h_arena + h_frag_off[f0 + f]);
            v[f].iov_len = h_frag_len[f0 + f];
        }
        ssize_t w;
        do {
            w = writev(fd, v, static_cast<int>(nf));
        } while (w < 0 && errno == EINTR);
        if (w < 0)
            return i ? static_cast<int>(i) : RNS_E_IO;
    }
    return static_cast<int>(n_pkts);
}

}  // extern "C"
