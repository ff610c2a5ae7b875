/*
 * rsmi_io.h -- batched UDP socket I/O into slot slabs.
 *
 * UDPspeeder moves one datagram per system call: recvfrom on the local
 * listen socket (tunnel_client.cpp:47) and recv on the remote socket
 * (tunnel_client.cpp:119; tunnel_server.cpp is symmetric), and sendto / send
 * per packet in my_send (packet.cpp:149-231).  These entry points move a whole
 * batch per call (recvmmsg / sendmmsg) between a socket and a slab of
 * fixed-size slots -- the layout the FEC managers (rsmi_fec.h) and cook
 * (rsmi_cook.h) work on -- so a batch goes to and from the GPU in one DMA each
 * when the slab is pinned (rsmi_host_alloc).
 *
 * Slot i of a slab starts at slab + i*slot_stride; its datagram sits at
 * slot_off inside the slot.  Lengths follow the reference's receive checks: a
 * datagram longer than max_len is dropped the way the callbacks drop a
 * `data_len == max_data_len + 1` read (tunnel_client.cpp:50-53, :121-124) --
 * here its len is -1 and the slot holds max_len bytes of it.
 */
#ifndef RSMI_IO_H_
#define RSMI_IO_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* A socket address (struct sockaddr_storage bytes + its length): the peer a
 * datagram came from, or the destination of a batch (address_t, common.h). */
typedef struct rsmi_udp_addr {
    uint8_t storage[128];
    uint32_t len;
    uint32_t reserved;
} rsmi_udp_addr;

/* Pinned host memory for slabs (hipHostMalloc; plain memory without a GPU). */
int rsmi_host_alloc(int64_t bytes, void **out);
void rsmi_host_free(void *p);

/* Receive up to max_pkts datagrams from fd into slots 0, 1, ...: waits up to
 * timeout_ms (-1: forever, 0: no wait) for the first, then takes whatever else
 * is queued without waiting.  len[i] = datagram length, or -1 if it exceeded
 * max_len (at most max_len bytes are stored; the slot needs max_len + 1 bytes
 * after slot_off).  from (may be NULL) gets each sender.  Returns the number
 * of datagrams (0 on timeout), or RSMI_ERR_INVALID / RSMI_ERR_IO. */
int rsmi_udp_recv_batch(int fd, uint8_t *slab, int64_t slot_stride, int64_t slot_off,
                        int32_t max_len, int32_t max_pkts, int32_t timeout_ms, int32_t *len,
                        rsmi_udp_addr *from);

/* Send n datagrams: datagram i is len[i] bytes at slab + slot[i]*slot_stride
 * + slot_off (slot NULL: slot i).  Entries with len < 0 are skipped (a packet
 * cook rejected).  to: destination (NULL for a connected socket).  Blocks
 * until the kernel took every datagram (retrying on EAGAIN / ENOBUFS).  A
 * datagram the kernel rejects on its own (ECONNREFUSED after an ICMP
 * port-unreachable, EMSGSIZE, EINVAL, ...) is dropped and the rest still go
 * out, as the reference's per-packet sendto does (packet.cpp:143-162).  A
 * broken socket (EBADF, ENOTSOCK, EFAULT, EDESTADDRREQ, EOPNOTSUPP, EPIPE)
 * ends the batch.  Returns the number sent (also when a broken socket ended
 * the batch after some went out: rsmi_last_error then names the errno), or
 * RSMI_ERR_INVALID, or RSMI_ERR_IO when datagrams were to be sent and none
 * could be. */
int rsmi_udp_send_batch(int fd, const uint8_t *slab, int64_t slot_stride, int64_t slot_off,
                        const int64_t *slot, const int32_t *len, int32_t n,
                        const rsmi_udp_addr *to);

/* As rsmi_udp_send_batch, datagram i being len[i] bytes at ptr[i] (host):
 * the FEC decoder's outputs (rsmi_fdec_output_list) go out without a copy. */
int rsmi_udp_send_ptrs(int fd, const uint8_t *const *ptr, const int32_t *len, int32_t n,
                       const rsmi_udp_addr *to);

#define RSMI_ERR_IO (-5) /* socket error (rsmi_last_error has errno text) */

#ifdef __cplusplus
}
#endif
#endif /* RSMI_IO_H_ */
