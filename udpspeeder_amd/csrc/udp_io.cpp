// udp_io.cpp -- batched UDP I/O between sockets and slot slabs (include/rsmi_io.h,
// SURVEY §8f f4).  recvmmsg / sendmmsg replace the reference's one recvfrom /
// recv / sendto per datagram (tunnel_client.cpp:47,119; packet.cpp:149-231).
#include <hip/hip_runtime.h>

#include <errno.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/uio.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rsmi.h"
#include "../../include/rsmi_io.h"

namespace rsmi {
void set_error(const std::string &m);
}

namespace {

constexpr int kChunk = 1024;  // UIO_MAXIOV: the most messages one call takes

int fail(int code, const std::string &m) {
    rsmi::set_error(m);
    return code;
}

int io_fail(const char *what) { return fail(RSMI_ERR_IO, std::string(what) + ": " + std::strerror(errno)); }

// sendmmsg errors that belong to one datagram (its destination or its size),
// after which the next datagram may still go out
// errnos that say the socket itself is unusable: every later datagram would
// fail the same way.  Anything else (ECONNREFUSED after an ICMP
// port-unreachable, EMSGSIZE, an unreachable or filtered destination, EINVAL
// or EAFNOSUPPORT for one bad address, ...) is taken as that datagram's own
// failure, as the reference's per-packet sendto / send treats every error
// (packet.cpp:143-162 logs and carries on).
bool socket_error(int en) {
    return en == EBADF || en == ENOTSOCK || en == EFAULT || en == EDESTADDRREQ || en == EOPNOTSUPP ||
           en == EPIPE;
}

}  // namespace

extern "C" {

int rsmi_host_alloc(int64_t bytes, void **out) {
    if (!out || bytes < 0) return fail(RSMI_ERR_INVALID, "bad rsmi_host_alloc args");
    *out = nullptr;
    if (bytes == 0) return RSMI_OK;
    void *p = nullptr;
    if (hipHostMalloc(&p, (size_t)bytes, hipHostMallocDefault) == hipSuccess) {
        *out = p;
        return RSMI_OK;
    }
    // no usable GPU: plain memory (tagged so rsmi_host_free knows), as the
    // socket side works without a device
    uint8_t *q = static_cast<uint8_t *>(std::malloc((size_t)bytes + 64));
    if (!q) return fail(RSMI_ERR_NOMEM, "rsmi_host_alloc: out of memory");
    std::memcpy(q, "rsmi-plain", 10);
    *out = q + 64;
    return RSMI_OK;
}

void rsmi_host_free(void *p) {
    if (!p) return;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost) {
        (void)hipHostFree(p);
        return;
    }
    (void)hipGetLastError();  // not a HIP allocation
    uint8_t *q = static_cast<uint8_t *>(p) - 64;
    if (std::memcmp(q, "rsmi-plain", 10) == 0) std::free(q);
}

int rsmi_udp_recv_batch(int fd, uint8_t *slab, int64_t slot_stride, int64_t slot_off,
                        int32_t max_len, int32_t max_pkts, int32_t timeout_ms, int32_t *len,
                        rsmi_udp_addr *from) {
    if (fd < 0 || !slab || !len || max_len < 0 || max_pkts < 0 || slot_off < 0 ||
        slot_stride < slot_off + max_len + 1)
        return fail(RSMI_ERR_INVALID, "bad rsmi_udp_recv_batch args (slot needs max_len + 1 bytes)");
    if (max_pkts == 0) return 0;
    if (timeout_ms != 0) {
        struct pollfd p = {fd, POLLIN, 0};
        int r;
        do {
            r = poll(&p, 1, timeout_ms);
        } while (r < 0 && errno == EINTR);
        if (r < 0) return io_fail("poll");
        if (r == 0) return 0;
    }
    std::vector<mmsghdr> msgs((size_t)std::min(max_pkts, kChunk));
    std::vector<iovec> iov(msgs.size());
    int got = 0;
    while (got < max_pkts) {
        const int c = std::min(max_pkts - got, kChunk);
        for (int i = 0; i < c; ++i) {
            // one byte more than max_len: a longer datagram shows as MSG_TRUNC
            iov[(size_t)i].iov_base = slab + (int64_t)(got + i) * slot_stride + slot_off;
            iov[(size_t)i].iov_len = (size_t)max_len + 1;
            std::memset(&msgs[(size_t)i], 0, sizeof(mmsghdr));
            msgs[(size_t)i].msg_hdr.msg_iov = &iov[(size_t)i];
            msgs[(size_t)i].msg_hdr.msg_iovlen = 1;
            if (from) {
                msgs[(size_t)i].msg_hdr.msg_name = from[got + i].storage;
                msgs[(size_t)i].msg_hdr.msg_namelen = sizeof(from[got + i].storage);
            }
        }
        int r;
        do {
            r = recvmmsg(fd, msgs.data(), (unsigned)c, MSG_DONTWAIT, nullptr);
        } while (r < 0 && errno == EINTR);
        if (r < 0) {
            if (errno == EAGAIN || errno == EWOULDBLOCK) break;
            if (got) break;  // report what arrived; the error shows on the next call
            return io_fail("recvmmsg");
        }
        for (int i = 0; i < r; ++i) {
            const mmsghdr &m = msgs[(size_t)i];
            const bool huge = (m.msg_hdr.msg_flags & MSG_TRUNC) || m.msg_len > (unsigned)max_len;
            len[got + i] = huge ? -1 : (int32_t)m.msg_len;
            if (from) {
                from[got + i].len = m.msg_hdr.msg_namelen;
                from[got + i].reserved = 0;
            }
        }
        got += r;
        if (r < c) break;  // the queue is empty
    }
    return got;
}

}  // extern "C"

namespace {

// Sends n datagrams; addr(i) gives datagram i's bytes (nullptr: skip it).
template <class Addr>
int send_all(int fd, int32_t n, const int32_t *len, Addr addr, const rsmi_udp_addr *to) {
    std::vector<mmsghdr> msgs;
    std::vector<iovec> iov;
    msgs.reserve((size_t)std::min(n, kChunk));
    iov.reserve(msgs.capacity());
    int sent = 0, failed = 0, err = 0;
    int i = 0;
    while (i < n) {
        msgs.clear();
        iov.clear();
        for (; i < n && (int)iov.size() < kChunk; ++i) {
            const uint8_t *p = addr(i);
            if (len[i] < 0 || !p) continue;
            iov.push_back(iovec{const_cast<uint8_t *>(p), (size_t)len[i]});
        }
        msgs.resize(iov.size());
        for (size_t j = 0; j < iov.size(); ++j) {
            std::memset(&msgs[j], 0, sizeof(mmsghdr));
            msgs[j].msg_hdr.msg_iov = &iov[j];
            msgs[j].msg_hdr.msg_iovlen = 1;
            if (to) {
                msgs[j].msg_hdr.msg_name = const_cast<uint8_t *>(to->storage);
                msgs[j].msg_hdr.msg_namelen = to->len;
            }
        }
        size_t done = 0;
        while (done < msgs.size()) {
            const int r = sendmmsg(fd, msgs.data() + done, (unsigned)(msgs.size() - done), 0);
            if (r < 0) {
                if (errno == EINTR) continue;
                if (errno == EAGAIN || errno == EWOULDBLOCK || errno == ENOBUFS) {
                    struct pollfd p = {fd, POLLOUT, 0};
                    (void)poll(&p, 1, 10);
                    continue;
                }
                // msgs[done] failed on its own: drop that one datagram and go
                // on.  A broken socket stops the batch; what went out before
                // it is still reported (the error text is kept for
                // rsmi_last_error).
                const int en = errno;
                if (socket_error(en)) {
                    errno = en;
                    const int rc = io_fail("sendmmsg");
                    return sent > 0 ? sent : rc;
                }
                if (!failed) err = en;
                ++failed;
                ++done;
                continue;
            }
            done += (size_t)r;
            sent += r;
        }
    }
    if (failed && sent == 0) {
        errno = err;
        return io_fail("sendmmsg");
    }
    return sent;
}

bool bad_to(const rsmi_udp_addr *to) { return to && (to->len == 0 || to->len > sizeof(to->storage)); }

}  // namespace

extern "C" {

int rsmi_udp_send_batch(int fd, const uint8_t *slab, int64_t slot_stride, int64_t slot_off,
                        const int64_t *slot, const int32_t *len, int32_t n, const rsmi_udp_addr *to) {
    if (fd < 0 || n < 0 || (n && (!slab || !len)) || slot_off < 0 || slot_stride < 0 || bad_to(to))
        return fail(RSMI_ERR_INVALID, "bad rsmi_udp_send_batch args");
    return send_all(fd, n, len, [&](int i) {
        return slab + (slot ? slot[i] : (int64_t)i) * slot_stride + slot_off;
    }, to);
}

int rsmi_udp_send_ptrs(int fd, const uint8_t *const *ptr, const int32_t *len, int32_t n,
                       const rsmi_udp_addr *to) {
    if (fd < 0 || n < 0 || (n && (!ptr || !len)) || bad_to(to))
        return fail(RSMI_ERR_INVALID, "bad rsmi_udp_send_ptrs args");
    return send_all(fd, n, len, [&](int i) { return ptr[i]; }, to);
}

}  // extern "C"
