/*
 * rsmi_cook.h -- batched GPU packet "cook" / "de_cook" for MI355X (gfx950).
 *
 * SURVEY §8f row f2.  UDPspeeder transforms every packet it sends with
 * do_cook (packet.cpp:303-308) and every packet it receives with de_cook
 * (packet.cpp:310-326):
 *
 *   do_cook:  put_crc32  (packet.cpp:327-336)  append crc32h(data) big-endian
 *             do_obscure (packet.cpp:77-91)    append iv[iv_len] and the byte iv_len;
 *                                              data[i] ^= iv[i % iv_len] over data+crc
 *             encrypt_0  (packet.cpp:32-39)    data[i] ^= key[i % strlen(key)]
 *   de_cook:  decrypt_0 -> de_obscure (packet.cpp:93-106) -> rm_crc32 (:337-346)
 *
 * Each stage is switched off by the reference's globals disable_checksum
 * (misc.cpp:16), disable_obscure, disable_xor (packet.cpp:23-24) -- here the
 * RSMI_COOK_NO_* flags of a context.  These entry points replace the per-packet
 * do_cook call in my_send (packet.cpp:165-168) and the de_cook calls in the
 * receive callbacks (tunnel_client.cpp:139, tunnel_server.cpp:154) with one
 * launch per batch of packets.  Results are byte-identical to the reference's, including
 * the buffer contents it leaves behind when de_cook fails.
 *
 * The reference draws each packet's IV itself (random_between(iv_min=4,
 * iv_max=32), get_fake_random_chars, common.cpp:387-411) from a non-
 * cryptographic PRNG.  Callers either pass the IVs (iv/iv_len below; any
 * values are valid on the wire, the receiver reads iv_len from the packet) or
 * let the kernel draw them from a SplitMix64 stream keyed by (seed, packet
 * index), with iv_len in [4, 32] as the reference draws it.
 *
 * Layout: packet i starts at base + offset[i] (or base + i*stride when offset
 * is NULL), 4-byte aligned, and owns `cap` bytes from there.  The kernels read
 * and write whole 16-byte pieces from the packet start, so cap must be at least
 * the output length rounded up to 16; bytes past the output length inside the
 * last piece are written back unchanged.  Packets are transformed in place.
 *
 * All pointers inside rsmi_packet_batch are device pointers; calls are
 * asynchronous on `stream` (a hipStream_t, NULL = default stream) and
 * graph-capturable once the context exists.
 */
#ifndef RSMI_COOK_H_
#define RSMI_COOK_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSMI_COOK_NO_CHECKSUM 1 /* disable_checksum (misc.cpp:16)   */
#define RSMI_COOK_NO_OBSCURE 2  /* disable_obscure (packet.cpp:23)  */
#define RSMI_COOK_NO_XOR 4      /* disable_xor (packet.cpp:24)      */

#define RSMI_COOK_IV_MAX 32      /* iv_max (packet.cpp:14): stride of the iv array */
#define RSMI_COOK_MAX_LEN 65535  /* largest packet length accepted  */

typedef struct rsmi_cook_ctx rsmi_cook_ctx;

/* key: the reference's key_string (misc.cpp:628), a C string; NULL or "" means
 * no XOR stage, exactly as encrypt_0 returns early on an empty key.
 * flags: RSMI_COOK_NO_* bits.  Builds the CRC tables and the key stream on the
 * current device. */
int rsmi_cook_ctx_create(const char *key, int flags, rsmi_cook_ctx **out);
void rsmi_cook_ctx_destroy(rsmi_cook_ctx *ctx);

typedef struct rsmi_packet_batch {
    uint8_t *base;          /* device */
    const uint64_t *offset; /* device [count] packet start offsets, or NULL      */
    int64_t stride;         /* packet i at base + i*stride when offset is NULL   */
    int64_t count;          /* packets in the batch                              */
    int32_t cap;            /* bytes each packet may use from its start          */
    int32_t reserved;       /* must be 0                                         */
    const int32_t *len;     /* device [count] input lengths                      */
    int32_t *out_len;       /* device [count] output lengths; -1 = rejected /
                               de_cook failed (may alias len)                    */
} rsmi_packet_batch;

/* do_cook over a batch.  iv: device [count][RSMI_COOK_IV_MAX] and iv_len:
 * device [count] (each <= 32), or both NULL to draw them on the device from
 * `seed`.  A packet whose cooked form would not fit `cap`, or with len outside
 * [0, RSMI_COOK_MAX_LEN], is left untouched with out_len -1. */
int rsmi_cook_dev(const rsmi_cook_ctx *ctx, const rsmi_packet_batch *batch,
                  const uint8_t *iv, const uint8_t *iv_len, uint64_t seed, void *stream);

/* de_cook over a batch: out_len = recovered payload length, or -1 where the
 * reference's de_cook returns -1 (the buffer then holds what it leaves). */
int rsmi_decook_dev(const rsmi_cook_ctx *ctx, const rsmi_packet_batch *batch, void *stream);

/* Out of place: packet i is read at batch->base + offset_i and its output
 * written at out + offset_i (same offsets, cap and alignment; out 16-aligned).
 * out may be device memory or pinned host memory mapped for the device
 * (hipHostMalloc, or hipHostRegister'd): the kernel's own stores then carry
 * the cooked packets over PCIe, so the transform and the D2H copy are one
 * pass (the send side: cooked packets land where sendmmsg reads them).  For
 * rsmi_decook_to, batch->base may likewise be pinned host memory read over
 * PCIe (the receive side: the H2D copy and de_cook are one pass). */
int rsmi_cook_to(const rsmi_cook_ctx *ctx, const rsmi_packet_batch *batch, uint8_t *out,
                 const uint8_t *iv, const uint8_t *iv_len, uint64_t seed, void *stream);
int rsmi_decook_to(const rsmi_cook_ctx *ctx, const rsmi_packet_batch *batch, uint8_t *out,
                   void *stream);

/* rsmi_decook_dev (in place in the batch), with every packet's de-cooked
 * bytes (whole 16-byte pieces up to round_up(len, 16)) also stored at the same
 * offset of mirror: pinned host memory, typically the receive buffer the
 * batch was copied from.  The receive side: the device keeps the de-cooked
 * packets for the FEC gather, the host gets them for the decode planner and
 * the outputs, and only packet bytes cross PCIe -- no whole-batch D2H copy. */
int rsmi_decook_mirror(const rsmi_cook_ctx *ctx, const rsmi_packet_batch *batch, uint8_t *mirror,
                       void *stream);

/* Synchronous host-memory forms (one H2D, one launch, one D2H; packet i at
 * host + i*stride): the per-packet mirror of do_cook/de_cook for callers that
 * have not moved to device batches. */
int rsmi_cook_host(const rsmi_cook_ctx *ctx, uint8_t *host, int64_t stride, int64_t count,
                   int32_t cap, const int32_t *len, int32_t *out_len, const uint8_t *iv,
                   const uint8_t *iv_len, uint64_t seed);
int rsmi_decook_host(const rsmi_cook_ctx *ctx, uint8_t *host, int64_t stride, int64_t count,
                     int32_t cap, const int32_t *len, int32_t *out_len);

#ifdef __cplusplus
}
#endif
#endif /* RSMI_COOK_H_ */
