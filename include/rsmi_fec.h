/*
 * rsmi_fec.h -- batched FEC framing on MI355X.
 *
 * UDPspeeder's fec_encode_manager_t (fec_manager.h:271-365,
 * fec_manager.cpp:174-447) turns the packets a connection sends into FEC
 * groups: it collects them (mode 0: a length-prefixed "blob" split into k
 * equal shards, fec_manager.cpp:35-75; mode 1: one packet per data shard,
 * zero-padded to the longest), picks (k, m) (short_packet_optimize,
 * fec_manager.cpp:267-288), prefixes every shard with the 8-byte header
 *     seq (u32 big-endian) | mode | k | m | index      (fec_manager.cpp:318-333)
 * and calls rs_encode2 once per group (fec_manager.cpp:364).
 *
 * Here one rsmi_fenc object holds one manager's state.  A batch of input()
 * calls is planned on the host -- the exact decisions of
 * fec_encode_manager_t::input/output, which need only packet lengths -- and
 * the byte work (blob assembly, padding, headers, the RS encode of every
 * group) runs on the GPU in a few launches over a slot array:
 *
 *   slot s occupies [s*slot_stride, (s+1)*slot_stride) of slots_base;
 *   its packet starts at +RSMI_FEC_SLOT_PACKET (120: the 8-byte header) and
 *   its shard at +RSMI_FEC_SLOT_SHARD (128), so with a slot_stride that is a
 *   multiple of 128 every shard row is cache-line aligned for the encoder.
 *
 * Every packet the reference's output() would return is listed, in the
 * reference's order, as (slot, length); packet bytes are slots_base +
 * slot*slot_stride + RSMI_FEC_SLOT_PACKET .. + length.  Results are byte-identical to the
 * reference's packets, including mode 0's bytes of the last data shard past
 * the blob's end: the reference sends whatever its blob buffer held there
 * (stale bytes of earlier groups, fec_manager.cpp:67-75), and so does this
 * (the encoder keeps a device copy of that buffer).
 *
 * Packets still waiting for their group at the end of a batch (the
 * reference's pending input_buf / blob) are copied into a device carry area
 * owned by the encoder, so the caller may reuse its input buffer once the
 * batch's work on the stream has completed.
 */
#ifndef RSMI_FEC_H_
#define RSMI_FEC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSMI_FEC_MAX_PACKETS 255 /* max_fec_packet_num (fec_manager.h:18) */
#define RSMI_FEC_HEADER 8        /* u32 seq + mode + k + m + index        */
#define RSMI_FEC_SLOT_PACKET 120 /* packet offset in a slot                */
#define RSMI_FEC_SLOT_SHARD 128  /* shard offset in a slot                 */

/* fec_parameter_t (fec_manager.h:26-180) without the timer fields. */
typedef struct rsmi_fec_config {
    int32_t mode;      /* 0 or 1 (-f mode, fec_parameter_t::mode)          */
    int32_t mtu;       /* fec_parameter_t::mtu, default 1250 (common.h:105) */
    int32_t queue_len; /* fec_parameter_t::queue_len, default 200          */
    int32_t short_packet_optimize; /* the global of fec_manager.cpp:30 (1) */
    int32_t header_overhead;       /* the global of fec_manager.cpp:31 (40) */
    int32_t rs_cnt;    /* x of the last -f point (get_tail().x)            */
    uint8_t rs_y[RSMI_FEC_MAX_PACKETS + 1]; /* rs_par[x-1].y, x = 1..rs_cnt  */
} rsmi_fec_config;

/* fec_parameter_t::rs_from_str (fec_manager.h:40-136) plus the defaults
 * above: "20:10" or "1:3,2:4,10:6,20:10".  Returns RSMI_OK, or
 * RSMI_ERR_INVALID where the reference returns -1. */
int rsmi_fec_config_init(rsmi_fec_config *cfg, const char *rs_str, int mode, int mtu,
                         int queue_len);

typedef struct rsmi_fenc rsmi_fenc;

/* A manager with the given config whose first group gets sequence number
 * seq0 (the reference draws it, get_fake_random_number, fec_manager.h:327). */
int rsmi_fenc_create(const rsmi_fec_config *cfg, uint32_t seq0, rsmi_fenc **out);
void rsmi_fenc_destroy(rsmi_fenc *enc);

/* New parameters, taken up when the next group starts -- the reference's
 * fec_par.clone(g_fec_par) at counter == 0 (fec_manager.cpp:207-209). */
int rsmi_fenc_next_config(rsmi_fenc *enc, const rsmi_fec_config *cfg);

/* One emitted packet: output() after input() call `event` returned it. */
typedef struct rsmi_fenc_packet {
    int64_t slot;   /* slot index in the batch's slot array                */
    int32_t len;    /* packet bytes from the slot start + RSMI_FEC_SLOT_PACKET, header included */
    int32_t event;  /* index of the input() call in the batch              */
} rsmi_fenc_packet;

/* Plan a batch of input() calls on the host.  len[i] >= 0 is input(s, len[i])
 * with the packet at in_base + in_off[i] (device memory; the buffer needs 16
 * readable bytes past every packet); len[i] < 0 is input(0, 0), the timer
 * flush (tunnel_client.cpp:41).  ret[i] (host, may be NULL) receives input()'s
 * return value (0, or -1 where the reference logs and drops the packet).
 * Afterwards *n_slots, *n_packets give the sizes of the batch and
 * *slot_stride_min the least slot_stride rsmi_fenc_run_dev accepts.
 * The plan replaces the previous one; state advances as if input() had been
 * called for every event.  Run every plan (its carry copies keep open groups)
 * before the next.  in_base NULL plans decisions only: such an encoder never
 * runs on a device. */
int rsmi_fenc_plan(rsmi_fenc *enc, int64_t n_events, const int32_t *len, const uint64_t *in_off,
                   const uint8_t *in_base, int32_t *ret, int64_t *n_slots, int64_t *n_packets,
                   int32_t *slot_stride_min);
/* slot_stride_min = RSMI_FEC_SLOT_SHARD + round_up(fec_len, 128) over the
 * batch's groups (the encoders may touch a parity row's padding up to the
 * next 128-byte line, rsmi.h).  A caller that cooks packets in place
 * (rsmi_cook.h) adds room for do_cook's tail: 37 bytes, whole 16-byte pieces. */

/* Copy the planned packet list (n_packets entries, host). */
int rsmi_fenc_packets(const rsmi_fenc *enc, rsmi_fenc_packet *out);

/* Per-group view of the plan (host arrays of n_groups entries, any may be
 * NULL): first slot, k, m, shard length (fec_len) and sequence number. */
int rsmi_fenc_groups(const rsmi_fenc *enc, int64_t *n_groups, int64_t *slot0, int32_t *k,
                     int32_t *m, int32_t *fec_len, uint32_t *seq);

/* Run the planned batch on `stream`: frame every group (headers, blob or
 * padded shards) and the mode-1 packets sent ahead of their group, RS-encode
 * every group's parity slots, and move still-pending packets into the carry
 * area.  slots_base: device, 16-aligned, n_slots * slot_stride bytes;
 * slot_stride: a multiple of 16, >= slot_stride_min (a multiple of 128 keeps
 * the shard rows line-aligned).  Asynchronous. */
int rsmi_fenc_run_dev(rsmi_fenc *enc, uint8_t *slots_base, int64_t slot_stride, void *stream);

/* rsmi_fenc_run_dev, then do_cook on every planned packet in the same stream
 * of work -- what the reference does to each packet output() returns before
 * it goes to the socket (fec_manager.cpp:364-460 -> my_send -> do_cook,
 * packet.cpp:165-168, 303-308).  Packet p (rsmi_fenc_packets order) is read
 * from its slot and written cooked at out + slot * slot_stride +
 * RSMI_FEC_SLOT_PACKET; out_len[p] (device int32, n_packets entries) receives
 * its cooked length (-1: it did not fit).  IVs are drawn on the device from
 * (seed, p), iv_len in [4, 32] as the reference draws it.  out: device memory
 * or pinned host memory (n_slots * slot_stride bytes, 16-aligned): with pinned
 * host memory the cook's stores are the D2H transfer.  NULL cooks in place in
 * slots_base.  A packet whose cooked form (up to 37 bytes longer, whole
 * 16-byte pieces) does not fit its slot from RSMI_FEC_SLOT_PACKET gets
 * out_len -1: size slot_stride for the tail (fec.py slot_stride_for).  ctx is
 * an rsmi_cook.h context. */
struct rsmi_cook_ctx;
int rsmi_fenc_run_cooked_dev(rsmi_fenc *enc, uint8_t *slots_base, int64_t slot_stride,
                             const struct rsmi_cook_ctx *ctx, uint64_t seed, uint8_t *out,
                             int32_t *out_len, void *stream);

/* Encoder runs (groups of one code, length and consecutive slots) of the
 * last cooked run that cooked their parity packets in the encoder's epilogue
 * (RSMI_OPT_PARITY_COOK, include/rsmi.h): their parity slots were not
 * written, the output holds the cooked packets as always. */
int64_t rsmi_fenc_last_parity_cooked(const rsmi_fenc *enc);

/* The last plan's packet list as runs (diagnostics and tests): packets first
 * .. first + count - 1 sit in slots slot .. slot + count - 1 of framing job
 * `job`, len bytes each; the first ndata are data packets of clean shards
 * (framed and cooked in one pass by a fused cooked run), at afirst.. of that
 * cook list, the rest at bfirst.. of the other.  Cooked runs upload these
 * instead of the per-packet list and expand them on the device.  out0 is
 * filled in by packed cooked runs.  n receives the run count; out (NULL:
 * count only) n entries. */
typedef struct rsmi_fenc_packet_run {
    int64_t slot, out0;
    int32_t first, afirst, bfirst, len, job;
    uint16_t count, ndata; /* the fused run cooks [0, ndata) from list A, the rest from B */
    uint16_t nfr, pad;     /* list A holds [0, nfr): framed there */
} rsmi_fenc_packet_run;
int rsmi_fenc_packet_runs(const rsmi_fenc *enc, int64_t *n, rsmi_fenc_packet_run *out);

/* A packet's place in a packed cooked output: a 16-aligned span of
 * RSMI_FEC_COOK_LEAD scratch bytes, then the packet, whose cooked form (crc 4
 * + iv <= 32 + iv_len 1 more) fits the rest.  The lead puts every packet at the
 * offset within a 16-byte piece it has in its slot (RSMI_FEC_SLOT_PACKET mod
 * 16), so the cook works on whole aligned pieces. */
#define RSMI_FEC_COOK_LEAD (RSMI_FEC_SLOT_PACKET % 16)
#define RSMI_FEC_COOK_SPAN(len) ((((int64_t)(len)) + 37 + RSMI_FEC_COOK_LEAD + 15) & ~(int64_t)15)

/* rsmi_fenc_run_cooked_dev with the cooked packets packed back to back, so the
 * buffer handed to the socket (or copied to the host for sendmmsg) holds
 * little more than packet bytes: packet p's span starts at out + sum over
 * q < p of RSMI_FEC_COOK_SPAN(len_q) (len from rsmi_fenc_packets), the packet
 * RSMI_FEC_COOK_LEAD bytes into it, out_len[p] cooked bytes.  out: device or
 * pinned host memory, 16-aligned, out_cap >= the sum over all packets
 * (RSMI_ERR_INVALID otherwise).  Every packet fits (out_len >= 0).  The bytes
 * of a span around its packet are unspecified. */
int rsmi_fenc_run_cooked_packed_dev(rsmi_fenc *enc, uint8_t *slots_base, int64_t slot_stride,
                                    const struct rsmi_cook_ctx *ctx, uint64_t seed, uint8_t *out,
                                    int64_t out_cap, int32_t *out_len, void *stream);

/* ---- the collector: many connections' managers in one launch set -----------
 *
 * A server keeps one manager per connection (connection.h:244-245), up to
 * max_conn_num = 200 (common.h:112), each flushing on its own 8 ms timer
 * (fec_manager.h:30), so a flush is a handful of groups per connection.
 * rsmi_fenc_run_many runs n planned encoders' batches (each planned with
 * rsmi_fenc_plan on its own state, unchanged) as one launch set: one framing
 * launch over all their jobs, one encode launch per (k, n) code over all
 * their groups of that code, one carry pass and, with a cook context, one
 * do_cook over all their packets.  The encoders' slots share one slot array:
 * slots_base holds sum(n_slots) slots of slot_stride bytes (slot_stride >=
 * every encoder's slot_stride_min).  Groups are laid out bucketed by code, so
 * afterwards rsmi_fenc_packets / rsmi_fenc_groups / rsmi_fenc_packet_runs of
 * each encoder report slots of the shared array.  Once the slot layout is
 * built every listed encoder's plan is consumed, also when a later step
 * fails: re-plan before running it again (an error before that point --
 * argument checks, a device mismatch -- leaves the plans intact).  With ctx,
 * out_len receives the cooked length of every
 * packet, the encoders' packet lists concatenated in the order of enc[]; IVs
 * are drawn from (seed, that concatenated index).  An encoder may appear once
 * per call.  The collector keeps the combined plan's staging (two sets, so a
 * call may be planned while the previous one runs). */
typedef struct rsmi_fcol rsmi_fcol;
int rsmi_fcol_create(rsmi_fcol **out);
/* Plan n encoders at once: encoder i takes events ev0[i] .. ev0[i+1]-1 of the
 * concatenated len / in_off / ret arrays (offsets into the one in_base), as
 * rsmi_fenc_plan would, on up to nthreads host threads (0: 8); n_slots,
 * n_packets and slot_stride_min (may be NULL) receive each encoder's values.
 * Every encoder is planned; the first failure is returned. */
int rsmi_fenc_plan_many(rsmi_fenc *const *enc, int32_t n, const int64_t *ev0, const int32_t *len,
                        const uint64_t *in_off, const uint8_t *in_base, int32_t *ret,
                        int64_t *n_slots, int64_t *n_packets, int32_t *slot_stride_min,
                        int32_t nthreads);
void rsmi_fcol_destroy(rsmi_fcol *col);
int rsmi_fenc_run_many(rsmi_fcol *col, rsmi_fenc *const *enc, int32_t n, uint8_t *slots_base,
                       int64_t slot_stride, const struct rsmi_cook_ctx *ctx, uint64_t seed,
                       uint8_t *out, int32_t *out_len, void *stream);
/* Test hook: on != 0 makes every rsmi_fenc_run_many fail right after it has
 * consumed its encoders' plans (tests/test_fec_frame.py); returns the
 * previous setting. */
int rsmi_debug_fcol_fail(int on);

/* ---- receive side: fec_decode_manager_t ------------------
 *
 * fec_decode_manager_t::input / output (fec_manager.cpp:469-797) take every
 * received packet (after de_cook): header checks, the anti-replay window of
 * anti_replay_t (fec_manager.h:187-235), the per-seq group map, the ring of
 * fec_buff_num packet buffers whose reuse evicts old groups (:554-576), and --
 * once a group has enough shards -- rs_decode2 plus blob_decode (mode 0) or
 * the length-prefixed data shards (mode 1), with mode-1 data packets passed
 * straight through (decode_fast_send, :760-776).
 *
 * rsmi_fdec_plan replays those decisions for a batch of packets on the host
 * (they need only headers, lengths and the mode-1 length prefixes).
 * rsmi_fdec_run_dev gathers every completed group's first k shards into
 * per-(k,n) staging batches on the device, decodes them with rsmi_decode_dev,
 * packs each group's k data rows contiguously and copies them to pinned host
 * memory.  rsmi_fdec_outputs then lists, per input event and in the
 * reference's order, the packets output() would return.  Received shards of
 * groups still open at the end of a batch are kept in a device carry area
 * indexed like the reference's ring, so groups straddle batches.
 *
 * Differences from the reference: a group whose shard indices include one
 * >= k + m makes the reference abort (assert on rs_decode2, :632 and :710);
 * here that group is dropped like a failed decode (no output, anti-replay
 * marked).  A malformed mode-1 row whose u16 length exceeds the row makes the
 * reference return bytes past the row from its ring buffer's stale contents
 * (:715-717); the output has the same length here with those bytes zero.
 * Nothing else differs. */
typedef struct rsmi_fdec rsmi_fdec;

/* buff_num: fec_buff_num (fec_manager.cpp:33), 0 for the default 2000. */
int rsmi_fdec_create(int32_t buff_num, rsmi_fdec **out);
void rsmi_fdec_destroy(rsmi_fdec *dec);

/* Plan input() for n received packets: packet i is len[i] bytes at
 * host_base + off[i] (host memory, read for headers and mode-1 length
 * prefixes) and at dev_base + off[i] (the same bytes on the device, 16
 * readable bytes after every packet).  now_ms is get_current_time() for the
 * anti-replay timeout (anti_replay_timeout = 120 s, fec_manager.h:185).
 * ret[i] (may be NULL) receives input()'s return value.  *n_decodes: groups
 * this batch decodes.  Run every plan before the next.  dev_base NULL plans
 * decisions only (return codes): such a decoder never runs on a device. */
int rsmi_fdec_plan(rsmi_fdec *dec, int64_t n, const int32_t *len, const uint64_t *off,
                   const uint8_t *host_base, const uint8_t *dev_base, int64_t now_ms,
                   int32_t *ret, int64_t *n_decodes);

/* rsmi_fdec_plan for n decoders at once, on up to nthreads host threads (a
 * server's per-connection managers share nothing).  Decoder i takes packets
 * pk0[i] .. pk0[i+1]-1 of len / off, relative to host_base[i] and (dev_base
 * NULL or dev_base[i] NULL: plan-only) dev_base[i]; ret[pk0[i] + j] and
 * n_decodes[i] (may be NULL) as rsmi_fdec_plan's.  Every decoder is planned;
 * the first failure is returned. */
int rsmi_fdec_plan_many(rsmi_fdec *const *dec, int32_t n, const int64_t *pk0, const int32_t *len,
                        const uint64_t *off, const uint8_t *const *host_base,
                        const uint8_t *const *dev_base, int64_t now_ms, int32_t *ret,
                        int64_t *n_decodes, int32_t nthreads);

/* Gather, decode, pack and copy back the planned groups on `stream`
 * (asynchronous; dev_base must stay valid until it completes). */
int rsmi_fdec_run_dev(rsmi_fdec *dec, void *stream);

/* The receive-side collector (see rsmi_fenc_run_many): n planned decoders'
 * batches in one launch set -- one gather into a staging area shared across
 * decoders and bucketed by (k, n), one decode per code, one pass packing
 * every decoder's rows back to back, one moving their carries -- then one
 * copy of all the rows into the collector's pinned buffer.  Afterwards each
 * decoder's rsmi_fdec_outputs works as after rsmi_fdec_run_dev; the output
 * pointers into decoded rows point into that buffer, which the collector
 * keeps per set of two (calls alternate): they stay valid until the
 * decoder's next plan, the collector's second-next call or its destruction,
 * whichever comes first.  The collector keeps the shared staging; a call
 * waits for its previous call. */
typedef struct rsmi_fdcol rsmi_fdcol;
int rsmi_fdcol_create(rsmi_fdcol **out);
void rsmi_fdcol_destroy(rsmi_fdcol *col);
int rsmi_fdec_run_many(rsmi_fdcol *col, rsmi_fdec *const *dec, int32_t n, void *stream);

/* Wait for the run and resolve the output list: *n_out packets. */
int rsmi_fdec_outputs(rsmi_fdec *dec, int64_t *n_out);

/* The resolved outputs (arrays of n_out entries, any may be NULL): host
 * pointer and length of each packet and the index of the input() call whose
 * output() returned it.  Pointers stay valid until the next plan; a
 * pass-through packet points into host_base. */
int rsmi_fdec_output_list(const rsmi_fdec *dec, const uint8_t **ptr, int32_t *len, int32_t *event);

#ifdef __cplusplus
}
#endif
#endif /* RSMI_FEC_H_ */
