/*
 * rsmi.h -- C ABI of the MI355X-native Reed-Solomon engine (librsmi.so).
 *
 * The code is bit-exact with UDPspeeder's lib/rs.cpp + lib/fec.cpp (Rizzo's
 * systematic Vandermonde code over GF(2^8), polynomial 0x11D).  Two surfaces:
 *
 *  1. The drop-in per-group surface with the reference's own C++ names and
 *     mangling (rs_encode2/rs_decode2/...): declared in rs_compat.h.
 *  2. This extern "C" batched surface: many independent FEC groups per call,
 *     device-resident buffers, plain pointers and sizes, hipStream_t passed
 *     as void*.  It replaces the per-group calls fec_manager makes at
 *     fec_manager.cpp:364 (encode), :632 and :710 (decode); see INTEGRATION.md.
 *
 * Shard layout (uniform batches): group g, shard j (0 <= j < n) lives at
 *     base + g*group_stride + j*shard_stride
 * Data shards are j < k, parity shards k <= j < n (same order as the char*
 * data[] array of rs_encode2, lib/rs.h:41).  Each shard holds len payload
 * bytes.  shard_stride must be a multiple of 16 and >= len; group_stride a
 * multiple of 16.  Slot padding: the kernels may read the bytes
 * [len, pad_end) of any shard slot and overwrite them in the slots they write
 * (parity slots for encode, rebuilt data slots for decode), where
 * pad_end = min(shard_stride, round_up(len, 128)) -- whole cache lines when
 * the stride has room -- and never touch anything at or beyond pad_end.
 *
 * Every call is asynchronous on `stream` (NULL = the default stream) of the
 * current HIP device, and graph-capturable once the (k,n) code is resident
 * (rsmi_prepare_code) and the workspace is large enough (rsmi_reserve).
 * Return values: RSMI_OK or a negative RSMI_ERR_*; rsmi_last_error() gives
 * text.  No call ever exit()s or falls back to the CPU: a missing or failing
 * GPU is reported as RSMI_ERR_HIP.
 */
#ifndef RSMI_H_
#define RSMI_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSMI_OK 0
#define RSMI_ERR_INVALID (-2) /* bad k/n/len/stride/alignment argument        */
#define RSMI_ERR_HIP (-3)     /* HIP runtime error (no device, launch failure) */
#define RSMI_ERR_NOMEM (-4)   /* device or pinned allocation failed            */

/* Per-group decode status written by rsmi_decode_dev (same codes as
 * rs_decode2, lib/rs.cpp:31-32 and lib/fec.cpp:851-856). */
#define RSMI_DEC_OK 0
#define RSMI_DEC_TOO_FEW (-1) /* fewer than k shards present        */
#define RSMI_DEC_SINGULAR 1   /* decode matrix singular (never for valid codes) */
#define RSMI_DEC_UNSUPPORTED 2 /* ragged decode only: invalid descriptor, or its (k,n)
                                  code is not resident (rsmi_prepare_code)        */

/* Library version, e.g. 0x000100 = 0.1.0. */
int rsmi_version(void);

/* Initialise tables on the current device (idempotent, thread-safe). */
int rsmi_init(void);

/* Text of the last error on this thread ("" if none). */
const char *rsmi_last_error(void);

/* Engine options (process-wide).  RSMI_OPT_BITSLICE: 1 (default) uses the
 * bit-sliced encoders (build-time or run-time compiled, rsmi_code_encoder)
 * where available, 0 forces the generic table kernel for uniform encodes (for
 * A/B tests).  Returns the previous value. */
#define RSMI_OPT_BITSLICE 1
/* RSMI_OPT_FUSED_DECODE: 1 (default) builds decode matrices and rebuilds the
 * rows in one fused kernel where the code fits it, 0 forces the two-kernel
 * path (plan kernel + apply kernel). */
#define RSMI_OPT_FUSED_DECODE 2
/* RSMI_OPT_ONE_GROUP: 1 (default) runs single-group host calls (the level-1
 * drop-in rs_encode2 / rs_decode2 / fec_*) as ONE kernel that reads pinned
 * staging over PCIe and raises a completion flag (oneshot.hip); 0 takes the
 * staged copy path (H2D, kernel, D2H). */
#define RSMI_OPT_ONE_GROUP 3
/* RSMI_OPT_CLS_REC_CAP: 0 (default) sizes each ragged plan's decode workgroups
 * to the LDS budget of the class kernels' occupancy; n > 0 caps the group
 * records one workgroup stages at n (tests force small caps to exercise plans
 * of many workgroup rounds).  Read when a plan is created. */
#define RSMI_OPT_CLS_REC_CAP 4
/* RSMI_OPT_ONE_SERVER: idle timeout in microseconds of the resident
 * one-group server (default 20000, or RSMI_ONE_SERVER_IDLE_US; 0 turns it off
 * and stops a running one).  With it on, a single-group host call
 * (RSMI_OPT_ONE_GROUP) posts its group to a 16-workgroup kernel that stays
 * resident on the device between calls and polls a doorbell in pinned host
 * memory -- no kernel launch on the per-call path (UDPspeeder calls
 * rs_decode2 once per group, synchronously, fec_manager.cpp:632,710).  The
 * server ends after that long without a call, or after its lifetime
 * (RSMI_OPT_ONE_SERVER_LIFE) under steady traffic, and is relaunched by the
 * next call.  While it runs it holds 16 CUs' worth of workgroups and its
 * stream's hardware queue: device-wide synchronisation (hipDeviceSynchronize,
 * torch.cuda.synchronize) waits for it to end -- at most one lifetime -- and
 * work on a stream that shares that hardware queue waits as well.  A process
 * that mixes drop-in calls with its own GPU work calls rsmi_quiesce() before
 * a device-wide sync (no wait at all), or sets 0. */
#define RSMI_OPT_ONE_SERVER 5
/* RSMI_OPT_ONE_SERVER_LIFE: the resident server's lifetime cap in
 * milliseconds (default 8, the reference's per-group latency budget
 * fec_manager.h:30, or RSMI_ONE_SERVER_LIFE_MS; >= 1).  Bounds how long a
 * device-wide synchronisation can wait for it under steady traffic; each
 * relaunch costs the call that makes it one kernel launch. */
#define RSMI_OPT_ONE_SERVER_LIFE 6
/* RSMI_OPT_PARITY_COOK: 1 cooks the parity packets of a fused cooked FEC run
 * (rsmi_fenc_run_cooked_dev into device memory) in the encoder's epilogue:
 * the encoder stores their payload already obscured and keyed into the
 * output, and the cook pass adds only the header, the CRC and the tail --
 * the parity is never written plain to the slots, nor written twice.  Taken
 * when every encoder run of the batch has a build-time split-k network;
 * otherwise (and with 0, the default, or RSMI_PARITY_COOK=0 in the
 * environment) the parity is written into the slots and cooked after the
 * encoder.  The cooked bytes are the same either way. */
#define RSMI_OPT_PARITY_COOK 7

int rsmi_option(int option, int value);

/* Stop the resident one-group server on every device and wait for it to end
 * (the next drop-in call relaunches it).  Call before a device-wide
 * synchronisation, or before work that must not share the server's hardware
 * queue, from any thread. */
int rsmi_quiesce(void);

/* Median wall time in microseconds of one drop-in rs_encode2 (decode 0) or
 * rs_decode2 (decode 1; rows with present[j] == 0 erased) call on host
 * buffers, k / n / len, over `calls` calls after 20 untimed ones, timed in C
 * (the harness the reference's per-call figure is timed with). */
int rsmi_dropin_latency(int decode, int k, int n, int len, const uint8_t *present, int calls,
                        double *median_us);

/* Host copy of fec_new(k,n)'s n x k systematic encoding matrix (row-major),
 * lib/fec.cpp:665-720.  Valid: 1 <= k <= n <= 256. */
int rsmi_get_matrix(int k, int n, uint8_t *out_nk);

/* Host-side decode coefficients for one group: the rows fec_decode derives
 * (lib/fec.cpp:795-825, 861-868) under rs_decode's survivor selection
 * (lib/rs.cpp:24-39).  present[n] (nonzero = received).  Writes sel[k] (the
 * k survivor slots used, ascending), miss[e] (missing data rows, ascending)
 * and coef[e*k] (d[miss[r]] = sum_c coef[r*k+c] * shard[sel[c]]); buffers
 * for miss/coef must hold k and k*k bytes.  Returns e >= 0, -1 if fewer than
 * k shards are present, RSMI_ERR_INVALID for bad arguments. */
int rsmi_decode_matrix(int k, int n, const uint8_t *present, uint8_t *sel,
                       uint8_t *miss, uint8_t *coef);

/* Make the (k,n) code resident on the current device (get_code's role,
 * lib/rs.cpp:42-55).  Called implicitly by the entry points below; call it
 * up front to keep later calls free of host<->device traffic. */
int rsmi_prepare_code(int k, int n);

/* Encoder kinds (rsmi_code_encoder).  Build-time bit-sliced XOR networks
 * exist for the (x, x+10) codes and the rs_from_str("1:3,2:4,10:6,20:10")
 * table; every other code that rs_from_str admits (fec_manager.h:40-136) gets
 * its network compiled at run time with hipRTC, in a background thread started
 * by rsmi_prepare_code (or the first call that makes the code resident).
 * Until it is ready that code's encodes run the generic table kernel -- the
 * output is the same bytes either way.  Knobs: RSMI_RTC=0 disables run-time
 * compilation; RSMI_RTC_MAX_COEFS (default 2048) caps k*(n-k);
 * RSMI_RTC_CACHE=<dir>|0 sets or disables the code-object cache
 * (default $XDG_CACHE_HOME/rsmi, else ~/.cache/rsmi). */
#define RSMI_ENC_NONE 0          /* n == k: no parity                          */
#define RSMI_ENC_GENERIC 1       /* v_perm table kernel                        */
#define RSMI_ENC_BITSLICE 2      /* build-time bit-sliced network              */
#define RSMI_ENC_BITSLICE_RTC 3  /* run-time compiled bit-sliced network       */
#define RSMI_ENC_COMPILING 4     /* generic now; network compiling             */
int rsmi_code_encoder(int k, int n);

/* The encoder kind this thread's last uniform encode launched (RSMI_ENC_*;
 * RSMI_ENC_NONE before the first, or when it had nothing to compute). */
int rsmi_last_encoder(void);

/* rsmi_prepare_code, then block until the (k,n) run-time network (if the code
 * gets one) has compiled or failed, and load it on the current device (do
 * this before capturing encodes of the code in a graph). */
int rsmi_wait_code(int k, int n);

/* Compile (or fetch from the disk cache) the run-time network of (k,n)
 * synchronously, without touching any GPU: warms the code-object cache ahead
 * of deployment, and makes later rsmi_prepare_code calls instant.  Returns
 * RSMI_ERR_INVALID when the code gets no run-time network (built-in, n == k,
 * over RSMI_RTC_MAX_COEFS, RSMI_RTC=0), RSMI_ERR_HIP when hipRTC fails. */
int rsmi_precompile_code(int k, int n);

/* Queue the run-time networks of count codes (k[i], n[i]) for the background
 * compile pool and return at once, without touching any GPU (codes with no
 * run-time network are skipped).  Returns how many of the codes get one. */
int rsmi_precompile_codes_async(const int32_t *k, const int32_t *n, int count);

/* Stop run-time compilation: queued compiles are dropped (their codes stay on
 * the generic kernel), and the call returns once every compile already inside
 * hipRTC has finished (one code each, at most 4 pool threads plus waiting
 * callers).  Later requests compile nothing.  The library calls it itself at
 * process exit, from the main thread's exit path before any atexit handler,
 * so comgr/LLVM is never torn down under a running compile; a host that exits
 * some other way (or wants a bounded exit) calls it first.  The Python binding
 * registers it with Python's atexit. */
void rsmi_rtc_shutdown(void);

/* The bit-sliced XOR network source of (k,n) (n > k) as emitted for hipRTC
 * (identical to the build-time generator's text).  Copies at most cap-1 bytes
 * plus a NUL into buf (may be NULL); returns the full length, or
 * RSMI_ERR_INVALID. */
int64_t rsmi_bitslice_source(int k, int n, char *buf, int64_t cap);

/* The two-wave split-k form of the same network (bs_split_<k>_<n>, codes with
 * k >= 10 and 2 <= n-k <= 10; identical to gen_bitslice.emit_split's text),
 * same buffer convention; RSMI_ERR_INVALID for codes without one. */
int64_t rsmi_bitslice_split_source(int k, int n, char *buf, int64_t cap);

/* Make (k,n) resident and pre-size the decode workspace that calls on
 * `stream` use, for up to `ngroups` groups (needed before graph capture). */
int rsmi_reserve(int k, int n, int64_t ngroups, void *stream);

/* ---- uniform batches (all groups share k, n, len) ------------------------ */

/* rs_encode2(k, n, data, len) for every group: writes parity shards k..n-1. */
int rsmi_encode_dev(int k, int n, uint8_t *base, int64_t group_stride,
                    int64_t shard_stride, int len, int64_t ngroups, void *stream);

/* rs_decode2(k, n, data, len) for every group.  present[g*n + j] != 0 marks
 * shard j of group g as received (device array, ngroups*n bytes).  Missing
 * data shards j < k are reconstructed IN THEIR OWN SLOT from the first k
 * present shards in ascending index order (the selection of lib/rs.cpp:24-39);
 * erased slots are never read.  Parity slots are left untouched.
 * status (device int32[ngroups], may be NULL) receives RSMI_DEC_*. */
int rsmi_decode_dev(int k, int n, uint8_t *base, int64_t group_stride,
                    int64_t shard_stride, int len, int64_t ngroups,
                    const uint8_t *present, int32_t *status, void *stream);

/* rs_decode2 with the reference's placement (lib/fec.cpp:838-882): each
 * rebuilt data row i is written over the parity survivor that fec_decode's
 * shuffle (fec.cpp:755-788) leaves in data[i] -- the buffer rs_decode2's
 * caller finds behind data[i] afterwards (fec.cpp:872-877, lib/rs.h:36-38).
 * Data survivors stay in place.  slot_map (DEVICE uint8[ngroups*k], may be
 * NULL) receives per group the slot now holding data row i, i.e. the pointer
 * permutation rs_decode leaves in data[0..k-1] (0xFF for an erased row of a
 * group with fewer than k shards).  Erased data slots are scratch (the
 * fused kernel writes them only for groups rebuilding more than 5 rows, the
 * two-kernel path always).  Same arguments, stream
 * semantics and status codes as rsmi_decode_dev.  The parity survivors are
 * read before they are overwritten, so a repeat call on the same buffer
 * decodes different input. */
int rsmi_decode_dev_ref(int k, int n, uint8_t *base, int64_t group_stride,
                        int64_t shard_stride, int len, int64_t ngroups,
                        const uint8_t *present, int32_t *status, uint8_t *slot_map,
                        void *stream);

/* Host computation of one group's reference slot map (as rsmi_decode_dev_ref
 * writes it) from present[n]; slot_map receives k entries.  Returns the
 * number of missing data rows, -1 for too few shards, RSMI_ERR_INVALID. */
int rsmi_ref_slot_map(int k, int n, const uint8_t *present, uint8_t *slot_map);

/* ---- ragged batches (mode 0 mix: each group its own k, n, len) ---------- */

typedef struct rsmi_group {
    uint64_t offset;       /* byte offset of shard 0 from base (multiple of 16) */
    uint32_t shard_stride; /* multiple of 16, >= len                            */
    uint32_t len;          /* payload bytes per shard                           */
    uint16_t k;            /* data shards                                       */
    uint16_t n;            /* total shards                                      */
    uint32_t reserved;     /* must be 0                                         */
} rsmi_group;              /* 24 bytes */

/* Encode ngroups groups described by groups[] (HOST array): builds a ragged
 * plan (below), launches it on `stream` and returns once it has completed. */
int rsmi_encode_ragged(const rsmi_group *groups, int64_t ngroups, uint8_t *base,
                       void *stream);

/* Same, with a DEVICE descriptor array (graph-capturable).  Every (k,n) used
 * must already be resident (rsmi_prepare_code); groups whose code is not
 * resident, or whose descriptor is invalid, are left untouched. */
int rsmi_encode_ragged_dev(const rsmi_group *dev_groups, int64_t ngroups,
                           uint8_t *base, void *stream);

/* Ragged plans (like FFT plans): built once on the host from the group
 * descriptors, kept on the device, reused by every launch over the same
 * layout (graph-capturable).  When every (k,n) in the batch has a
 * specialised bit-sliced network the plan buckets groups by code and one
 * launch covers all buckets; otherwise the generic kernel runs.  Destroy a
 * plan only after the launches that use it have completed. */
typedef struct rsmi_ragged_plan rsmi_ragged_plan;
int rsmi_ragged_plan_create(const rsmi_group *groups, int64_t ngroups,
                            rsmi_ragged_plan **plan);
int rsmi_encode_ragged_plan(const rsmi_ragged_plan *plan, uint8_t *base, void *stream);
int rsmi_ragged_plan_uses_bitslice(const rsmi_ragged_plan *plan);

/* Ragged decode: rs_decode2(k, n, data, len) on every group of a ragged
 * batch (fec_manager.cpp:632 once per mode-0 group, each with its own k, n
 * and length).  present_bits (DEVICE uint32[ngroups * 8]): bit (j % 32) of
 * word g*8 + j/32 set = shard j of group g received (bits >= n ignored).
 * Missing data shards are rebuilt in their own slots from the first k
 * present shards in ascending order, as rsmi_decode_dev does; the slot
 * padding rule above applies.  status (DEVICE int32[ngroups], required)
 * receives RSMI_DEC_*.  One launch for groups with min(k, n-k) <= 10 and
 * k <= 64 (all of -f's default and C3 tables), a second, workgroup-per-group
 * launch for the rest.  Codes must be resident; a plan makes them so. */
int rsmi_decode_ragged_plan(const rsmi_ragged_plan *plan, uint8_t *base,
                            const uint32_t *present_bits, int32_t *status, void *stream);
/* Same with a DEVICE descriptor array (graph-capturable): kmax = the largest k
 * in the batch (sizes the one-wave kernel's LDS); groups whose code is not
 * resident get RSMI_DEC_UNSUPPORTED. */
int rsmi_decode_ragged_dev(const rsmi_group *dev_groups, int64_t ngroups, uint8_t *base,
                           const uint32_t *present_bits, int32_t *status, int kmax,
                           void *stream);
/* Same with a HOST descriptor array: builds a plan, launches it on `stream`
 * and returns once it has completed. */
int rsmi_decode_ragged(const rsmi_group *groups, int64_t ngroups, uint8_t *base,
                       const uint32_t *present_bits, int32_t *status, void *stream);
/* The ragged decodes with the reference's placement (as rsmi_decode_dev_ref):
 * rebuilt data rows over the parity survivors fec_decode's shuffle leaves in
 * data[i]; slot_map (DEVICE, may be NULL) receives group g's k entries at
 * slot_map + g * map_stride (entries i >= map_stride are not written), 0xFF
 * for an erased row of a group not decoded; groups with status
 * RSMI_DEC_UNSUPPORTED get no map.  Erased data slots are scratch. */
int rsmi_decode_ragged_plan_ref(const rsmi_ragged_plan *plan, uint8_t *base,
                                const uint32_t *present_bits, int32_t *status,
                                uint8_t *slot_map, int32_t map_stride, void *stream);
int rsmi_decode_ragged_dev_ref(const rsmi_group *dev_groups, int64_t ngroups, uint8_t *base,
                               const uint32_t *present_bits, int32_t *status, int kmax,
                               uint8_t *slot_map, int32_t map_stride, void *stream);
void rsmi_ragged_plan_destroy(rsmi_ragged_plan *plan);

/* ---- host-memory convenience (pinned staging + H2D/D2H on an internal
 * stream; synchronous).  Same layout contract, host pointers. --------------- */
int rsmi_encode_host(int k, int n, uint8_t *base, int64_t group_stride,
                     int64_t shard_stride, int len, int64_t ngroups);
int rsmi_decode_host(int k, int n, uint8_t *base, int64_t group_stride,
                     int64_t shard_stride, int len, int64_t ngroups,
                     const uint8_t *present, int32_t *status);

/* Pipelined end-to-end encode from host memory (the UDP-socket side of the
 * path): data shards of group g at host_data + g*data_gs + j*shard_stride
 * (j < k), parity written to host_parity + g*parity_gs + (j-k)*shard_stride.
 * Chunks of `chunk_groups` groups flow H2D -> encode -> D2H on three HIP
 * streams so the two copy directions and the kernels overlap.  Host buffers
 * should be pinned (hipHostMalloc / torch pin_memory) for the copies to run
 * asynchronously.  Synchronous: returns when all parity is in host memory. */
int rsmi_encode_pinned(int k, int n, const uint8_t *host_data, int64_t data_gs,
                       uint8_t *host_parity, int64_t parity_gs, int64_t shard_stride,
                       int len, int64_t ngroups, int64_t chunk_groups);

/* End-to-end decode from host memory: group g's n shard slots at
 * host_shards + g*shards_gs + j*shard_stride (erased slots may hold junk),
 * present flags [ngroups][n]; missing data rows are written back into their
 * own host slots (the slot padding rule above applies to them), status[g]
 * receives RSMI_DEC_*.  Synchronous.
 *
 * Pinned, device-mapped shards (hipHostMalloc, torch pin_memory,
 * hipHostRegister) take the zero-copy path: the decode kernel reads only the
 * k survivors it selects (the first k present, lib/rs.cpp:24-39) straight
 * from host memory over PCIe and writes only the rebuilt rows back -- no
 * staging copy.  Any other memory, or a code the fused kernel does not take,
 * goes through the staged pipeline: chunks of chunk_groups groups H2D ->
 * decode -> D2H of the data rows on three streams. */
int rsmi_decode_pinned(int k, int n, uint8_t *host_shards, int64_t shards_gs,
                       int64_t shard_stride, int len, int64_t ngroups,
                       const uint8_t *present, int32_t *status, int64_t chunk_groups);

/* Which path this thread's last rsmi_decode_pinned took (with several
 * devices: the OR of the paths the ranges took). */
#define RSMI_PINNED_ZERO_COPY 1
#define RSMI_PINNED_STAGED 2
int rsmi_last_decode_pinned_path(void);

/* Ragged batches in host memory (the mode-0 mix as it leaves the sockets):
 * groups[] (HOST) describe the batch at host_base (offsets relative to it,
 * ascending and non-overlapping, 16-aligned); chunks of chunk_groups groups
 * flow H2D (their contiguous byte span) -> ragged encode (parity rows
 * written) or decode (rebuilt data rows in their own slots; present_bits HOST
 * uint32[ngroups * 8] as rsmi_decode_ragged_plan's, status HOST int32[ngroups],
 * may be NULL) -> span D2H on three streams.  Host memory should be pinned.
 * With a device list (rsmi_use_devices) the groups split into contiguous
 * ranges of near-equal summed n * len, one per listed device.  Synchronous. */
int rsmi_encode_ragged_pinned(const rsmi_group *groups, int64_t ngroups, uint8_t *host_base,
                              int64_t chunk_groups);
int rsmi_decode_ragged_pinned(const rsmi_group *groups, int64_t ngroups, uint8_t *host_base,
                              const uint32_t *present_bits, int32_t *status, int64_t chunk_groups);

/* ---- several GPUs behind the host-memory batch entry points --
 *
 * UDPspeeder serves up to max_conn_num = 200 connections from one libev
 * thread (common.h:112, tunnel_server.cpp:159-196), one FEC manager pair each
 * (connection.h:244-245).  FEC groups are independent, so a host batch splits
 * into contiguous group ranges, one per listed device, with no exchange
 * between them.  After rsmi_use_devices(devs, n) (n >= 1; a device may be
 * listed more than once), rsmi_encode_pinned and rsmi_decode_pinned run range
 * i = [G*i/n, G*(i+1)/n) on devs[i] (the ragged host entries: ranges of
 * near-equal summed n * len), each on its own host thread with its own
 * HIP streams and pipeline buffers; results land in that range's part of the
 * caller's host arrays, and the call returns when every range is done (the
 * first failing range's error is reported, prefixed with its device).  One
 * such call runs at a time.  n = 0 restores the default: the calling thread's
 * current device.  rsmi_get_devices returns the list's length and copies up
 * to cap entries into out (may be NULL).
 *
 * For the device-resident collectors (rsmi_fenc_run_many / rsmi_fdec_run_many)
 * the unit of sharding is the connection: keep one collector per device and
 * give each the managers of a contiguous range of connections;
 * rsmi_split_ranges computes such ranges.  bounds[0..parts] receives the cuts
 * of n items into `parts` contiguous ranges: near-equal counts (cost NULL), or
 * near-equal summed cost (the cut before part i is the first item whose prefix
 * sum reaches i/parts of the total), as udpspeeder_amd.shard.balanced_ranges. */
int rsmi_use_devices(const int32_t *devices, int32_t n);
int rsmi_get_devices(int32_t *out, int32_t cap);
int rsmi_split_ranges(int64_t n, const int64_t *cost, int32_t parts, int64_t *bounds);

/* ---- synthetic inputs (bench / tests) ----------------------------------- */

/* Fill data shards (j < k) of every group with the SplitMix64 stream:
 * byte q of group g's k*len data bytes (shard-major) is byte q%8 of
 * mix((seed ^ g) + (q/8 + 1) * 0x9E3779B97F4A7C15).  Groups g0..g0+ngroups-1
 * are written at base + (g-g0)*group_stride. */
int rsmi_fill_data(int k, int len, uint8_t *base, int64_t group_stride,
                   int64_t shard_stride, int64_t g0, int64_t ngroups,
                   uint64_t seed, void *stream);

/* Same stream definition for a ragged batch: data rows of group i (device
 * descriptor array) get the stream of group id g0 + i. */
int rsmi_fill_ragged(const rsmi_group *dev_groups, int64_t ngroups, uint8_t *base,
                     int64_t g0, uint64_t seed, void *stream);

/* ---- measurement ---------------------------------------------------------
 * Device-to-device copy of nbytes (a multiple of 16; both pointers 16-byte
 * aligned, not overlapping): bench.py's measured HBM copy peak, the line the
 * codec kernels' achieved rates are read against besides the 8 TB/s spec.
 * variant: 0 / 1 = 4 / 8 16-byte words per thread, 2 / 3 = the same with
 * nontemporal loads and stores.  Variants 4-6 are read:write mixes that read
 * nbytes (a multiple of 16 * 256 * 24) from src and write a share of it to
 * dst: 4 = read only (nothing written), 5 = 2:1 (the encoders' mix: nbytes / 2
 * written), 6 = 6:1 (the decode's mix: nbytes / 6 written).  No reference
 * counterpart. */
int rsmi_copy_peak(uint8_t *dst, const uint8_t *src, int64_t nbytes, int variant, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* RSMI_H_ */
