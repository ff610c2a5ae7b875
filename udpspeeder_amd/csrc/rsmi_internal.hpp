// rsmi_internal.hpp -- shared declarations between the host runtime (api.cpp)
// and the HIP kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <memory>

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "../../include/rsmi.h"
#include "../../include/rsmi_fec.h"
#include "../../include/rsmi_cook.h"

namespace rsmi {

// Decode plan record (one per group, written by k_decode_plan, read by the
// decode apply kernel).  Layout for a batch with parameters (k, emax):
//   +0  int32 status (RSMI_DEC_*)       +4 uint8 e (missing data rows)
//   +8  uint8 sel[k]   survivors used (ascending slot indices)
//   +8+k uint8 miss[emax]  missing data rows
//   +coef_off uint8 coef[emax][k]  (coef_off 16-aligned)
struct PlanLayout {
    int k, emax, coef_off, stride;
    __host__ __device__ PlanLayout(int k_, int emax_) : k(k_), emax(emax_) {
        coef_off = (8 + k + emax + 15) & ~15;
        stride = (coef_off + emax * k + 15) & ~15;
    }
};

// Launch descriptors (plain structs passed by value to kernels).
struct UniformArgs {
    uint8_t *base;
    int64_t group_stride, shard_stride;
    int len, k, n, tiles;   // tiles per group (of 256*W bytes)
    int64_t ngroups;
};

// Ragged decodes with the reference's placement (rsmi_decode_ragged_*_ref):
// on = 1 writes rebuilt rows over the parity survivors fec_decode's shuffle
// picks (ref_slot_of); map (device, may be null) receives group g's slot map
// at map + g * stride (entries i < min(k, stride)).
struct RefOut {
    uint8_t *map;
    int32_t stride;
    int32_t on;
};

// Host-side launchers implemented in kernels.hip; return hipError_t.
hipError_t launch_encode_generic(const UniformArgs &a, int W, const uint8_t *parity_rows,
                                 const uint32_t *ptab, hipStream_t s);
hipError_t launch_decode_plan(const UniformArgs &a, const uint8_t *present,
                              const uint8_t *parity_rows, uint8_t *plans, int32_t *status,
                              const uint8_t *gftab, hipStream_t s);
hipError_t launch_decode_apply(const UniformArgs &a, int W, const uint8_t *plans,
                               const uint32_t *ptab, hipStream_t s);
hipError_t launch_encode_ragged(const rsmi_group *groups, int64_t ngroups, uint8_t *base,
                                const uint64_t *code_dir, const uint32_t *ptab, hipStream_t s);
// After plan + apply: rebuilt rows to the reference's slots, and the slot map
// (rsmi_decode_dev_ref); present is the call's [ngroups][n] flags.
hipError_t launch_decode_ref_move(const UniformArgs &a, const uint8_t *plans, const uint8_t *present,
                                  uint8_t *slot_map, hipStream_t s);
hipError_t launch_copy_peak(uint8_t *dst, const uint8_t *src, int64_t nbytes, int variant, hipStream_t s);
hipError_t launch_fill_data(int k, int len, uint8_t *base, int64_t group_stride,
                            int64_t shard_stride, int64_t g0, int64_t ngroups, uint64_t seed,
                            hipStream_t s);

hipError_t launch_fill_ragged(const rsmi_group *groups, int64_t ngroups, uint8_t *base,
                              int64_t g0, uint64_t seed, hipStream_t s);

// Fused decode (plan + reconstruction in one wave per group, decode.hip).
bool decode_fused_ok(int k, int n, int64_t group_stride, int64_t shard_stride, int len);
// host_shards: a.base is pinned host memory the kernel reads and writes over
// PCIe (system-scope loads and stores)
hipError_t launch_decode_fused(const UniformArgs &a, const uint8_t *present,
                               const uint8_t *parity_rows, int32_t *status,
                               const uint32_t *ptab, const uint8_t *gftab, hipStream_t s,
                               bool host_shards = false, bool ref = false,
                               uint8_t *slot_map = nullptr);
// The reference's placement of a group's rebuilt rows (fec.cpp:755-788,
// 872-877): slot of the parity survivor that ends in data[i] for each missing
// data row i, given sel (the k survivors, ascending) and the missing rows.
__host__ __device__ inline int ref_slot_of(int k, int e, const uint8_t *sel, int miss_row) {
    int x = miss_row;
    while (x < k - e) x = sel[x];
    return sel[x];
}

// Ragged decode (decode.hip): one-wave-per-group kernel, then the
// workgroup-per-group kernel for the groups it defers.
hipError_t launch_decode_ragged(const rsmi_group *groups, int64_t ngroups, uint8_t *base,
                                const uint32_t *present_bits, int32_t *status, int kmax,
                                const uint64_t *code_dir, const uint32_t *ptab,
                                const uint8_t *gftab, hipStream_t s, RefOut ro = RefOut{nullptr, 0, 0});
// Tile width of a ragged group (lane dwords: 1, 2, 4 or 5): the narrowest
// that covers its padded length in one pass, else 1280-byte tiles.  Lane
// pieces of 4, 8 or 16 bytes divide the padded length (a multiple of 16).
__host__ __device__ inline int rag_lpad(uint32_t len, uint32_t ss) {
    const uint32_t l128 = (len + 127) / 128 * 128;  // whole lines where the slot has room
    return (int)(l128 < ss ? l128 : ss);
}
__host__ __device__ inline int rag_width(int lpad) {
    const int nw = (lpad + 255) / 256;
    return nw <= 1 ? 1 : (nw == 2 ? 2 : (nw <= 4 ? 4 : 5));
}
__host__ __device__ inline int rag_width_class(int w) { return w == 1 ? 0 : (w == 2 ? 1 : (w == 4 ? 2 : 3)); }
// Plans: the groups sorted into the four width classes, one register-cut
// kernel per class.  Within class c the groups are dealt to nw[c] workgroups
// of kClsWaves waves (about one resident round: decode_cls_occupancy) by
// longest-processing-time first on an estimated cost; workgroup b holds
// records rec[wst[c][b] .. wst[c][b+1]) (at most maxb[c]) and its waves take
// them one at a time.
#ifndef DEC_CLS_WAVES
#define DEC_CLS_WAVES 4
#endif
constexpr int kClsWaves = DEC_CLS_WAVES;  // waves per class workgroup (they share its groups)
struct ClsLaunch {
    const uint32_t *rec;     // device: 8-dword group records (decode.hip), workgroup-major per class
    const uint32_t *wst[4];  // device: per class, nw[c] + 1 offsets into rec (in records)
    int nw[4];               // workgroups of class c
    int maxb[4];             // most records one workgroup of class c holds
    uint32_t *defer;         // device word: set to epoch when a group is left for the big kernel
    uint32_t epoch;          // this call's mark (plans count calls)
    int need_big;            // the plan holds groups the class kernels defer (k > 32, or
                             // slots spanning >= 2 GiB): launch the big kernel after them
    RefOut ref;              // placement of this call's rows (set per call)
};
// The (k,n) code's parity rows on the current device (nullptr: not resident).
const uint8_t *device_code_rows(int k, int n);
int decode_cls_occupancy(int c);  // waves per SIMD class c's kernel is cut for
size_t cls_lds_bytes(int kmax, int maxb);  // LDS of a class workgroup holding maxb records
// Class c runs on cs[c]; the caller orders cs[] against s and then runs
// launch_decode_ragged_big on s.
hipError_t launch_decode_ragged_cls(const rsmi_group *groups, const ClsLaunch &L, uint8_t *base,
                                    const uint32_t *present_bits, int32_t *status, int kmax,
                                    const uint64_t *code_dir, const uint32_t *ptab,
                                    const uint8_t *gftab, hipStream_t s, const hipStream_t cs[4]);
// The workgroup-per-group kernel for the groups the one-wave kernels deferred
// (defer_word: skip everything unless *defer_word == epoch; nullptr: scan).
hipError_t launch_decode_ragged_big(const rsmi_group *groups, int64_t ngroups, uint8_t *base,
                                    const uint32_t *present_bits, int32_t *status,
                                    const uint64_t *code_dir, const uint32_t *ptab,
                                    const uint8_t *gftab, hipStream_t s,
                                    const uint32_t *defer_word = nullptr, uint32_t epoch = 0,
                                    RefOut ro = RefOut{nullptr, 0, 0});

// Bit-sliced encode kernels specialised at build time for hot (k,n) codes
// (gen_bitslice.py -> gen/bitslice_codes.inc), or compiled at run time
// (bitslice_rtc.cpp).  Returns hipErrorNotSupported when (k,n) has neither
// (yet).
hipError_t launch_encode_bitslice(const UniformArgs &a, hipStream_t s);
bool has_bitslice(int k, int n);
int bitslice_code_index(int k, int n);  // position in the generated code list, -1 if none
int bitslice_code_k(int idx);  // (k, n) of generated code idx
int bitslice_code_n(int idx);
// Ragged bucketed launch over a host-built plan (ragged.cpp): colmap entries
// (group << 12) | piece, waves = {code index, first column} pairs.
hipError_t launch_encode_bitslice_ragged(const rsmi_group *groups, const uint32_t *colmap,
                                         const uint32_t *waves, uint32_t nwaves, uint8_t *base,
                                         uint32_t bytes, hipStream_t s);

// Codes without a build-time network (bitslice_rtc.cpp): emitted and compiled
// with hipRTC in the background when first made resident.
int bitslice_builtin_count();
bool bitslice_emit(int k, int n, std::string &src, int *nxor);  // gen_bitslice.emit_code's text
bool bitslice_rtc_eligible(int k, int n);
void bitslice_rtc_request(const std::vector<std::pair<int, int>> &codes);  // async
void bitslice_rtc_wait(const std::vector<std::pair<int, int>> &codes);
int bitslice_rtc_state(int k, int n);  // 0 idle, 1 compiling, 2 ready, 3 failed
enum RtcKind { kRtcUniform = 0, kRtcRagged = 1, kRtcSplit = 2 };
hipFunction_t bitslice_rtc_function(int k, int n, RtcKind kind);  // nullptr unless ready
bool bitslice_split_ok(int k, int n);                                // gen_bitslice.split_ok
bool bitslice_emit_split(int k, int n, std::string &src);           // gen_bitslice.emit_split's text
hipError_t launch_encode_bitslice_ragged_rtc(int k, int n, const rsmi_group *groups,
                                             const uint32_t *colmap, const uint32_t *waves,
                                             uint32_t nwaves, uint8_t *base, uint32_t bytes,
                                             hipStream_t s);

constexpr int kPtabDwords = 8;  // per coefficient: T0lo T0hi T1lo T1hi | T2 pad pad pad
// The device GF table blob (gftab): exp[512] | log[256] | pad, then at
// kGfLtabOff the ragged decode's Lagrange tables (decode.hip LTables image).
constexpr int kGfLtabOff = 1024;
constexpr int kGfLtabBytes = 5632;

// ---- one group per call, latency path (oneshot.hip) ------------------------------
constexpr int kOneAug = 16384;  // LDS bytes for [A | M] (e * (e + k)) or the encode coefficients
struct OneArgs {
    const uint8_t *in;      // device address of pinned staging: slot j at in + j * ss
    uint8_t *out;           // device address of pinned rows: output row r at out + r * ss
    const uint8_t *rows;    // the code's (n-k) x k parity rows (device)
    const uint32_t *ptab;   // v_perm split tables (device)
    const uint8_t *gftab;   // exp[512] | log[256] (device)
    int32_t *status;        // device address of a pinned word: RSMI_DEC_*
    uint32_t *flag;         // device address of a pinned word: set to seq when done
    uint32_t seq;
    int k, n, len, ss;
    int encode;             // 1: out rows = parity rows k..n-1; 0: rebuilt data rows, miss order
    uint32_t present[8];    // decode: bit j = shard j received
};
bool one_group_ok(int k, int n, int len, int ss, bool encode);
hipError_t launch_one_group(const OneArgs &a, hipStream_t s);
// The multi-workgroup one-group kernels (oneshot.hip): kOneSrvWgs workgroups
// split the group's 16-byte pieces; each raises its own completion word.
constexpr int kOneSrvWgs = 16;
bool one_multi_ok(int k, int n, int len, int ss, int rows);  // rows: output rows of the call
hipError_t launch_one_multi(const OneArgs &a, hipStream_t s);  // a.flag: kOneSrvWgs words
// The resident server's control block (pinned, device-mapped).  job[i]:
// dword i of the job's OneArgs in the low half, the job's seq in the high
// half -- one aligned 8-byte store each, written after the job's inputs, so a
// wave whose every lane reads the new seq has read the whole job and its
// inputs are visible; quit stops the server; the kernel writes its generation
// to exit_gen when it ends and flags[wg] = seq when workgroup wg has finished
// a job.
constexpr int kOneJobWords = 30;
struct OneSrvCtl {
    uint64_t job[32];
    uint32_t quit, exit_gen, pad[14];
    uint32_t flags[kOneSrvWgs];
};
struct OneSrvDev {  // device memory: workgroup 0's stop decision, the exit count
    uint32_t stop, exited, pad[2];
};
hipError_t launch_one_server(OneSrvCtl *ctl_dev, OneSrvDev *dv, const uint32_t *ptab, const uint8_t *gftab,
                             uint32_t gen, uint32_t done0, uint32_t idle_us, uint32_t life_ms, hipStream_t s);

// ---- packet cook / de_cook (cook.hip, cook_host.cpp) -------------------------------
// A packet is walked by kCookLpp lanes of a wave (8: eight packets per wave;
// 16: four; 32: two), each holding every kCookLpp-th 16-byte piece.
#ifndef COOK_LPP
#define COOK_LPP 8
#endif
constexpr int kCookLpp = COOK_LPP;
// CRC table blob (u32 words), built on the host by cook_host.cpp:
//   [0, 2048)        slicing-by-8 tables T_k[256], k = 0..7
//   kCookLane + 128k nibble map of Z_{16k}, k = 0..kCookLpp-1 (k = 0: identity)
//   kCookZH          byte map of Z_{16 kCookLpp}, a lane's Horner step (4 x 256 words)
//   kCookUns + 128i  nibble maps of Z_{-c}, c = 1..3, then Z_{-4c}, c = 1..3
//   kCookNib + 16i   raw CRC of a 16-byte piece holding nibble i alone, i = 0..31
//   kCookZN          nibble map of Z_{16 kCookLpp}
//   kCookS16 + 256k  (COOK_S16) T_{8+k}, k = 0..7: slicing-by-16 with T_0..T_7
//   kCookZH2         (COOK_2CH) byte map of Z_{32 kCookLpp}, the two-chain step (4 x 256)
// COOK_NIB selects the nibble forms for the per-piece work: 16-entry tables sit in
// distinct LDS banks, so a wave's lookups into one never conflict.
// COOK_S16: a piece's raw CRC as 16 independent byte lookups (one level)
// instead of two chained slicing-by-8 steps.
#ifndef COOK_NIB
#define COOK_NIB 0
#endif
#ifndef COOK_S16
#define COOK_S16 1
#endif
constexpr int kCookLane = 2048;
constexpr int kCookZH = kCookLane + kCookLpp * 128;
constexpr int kCookUns = kCookZH + 1024;
constexpr int kCookNib = kCookUns + 6 * 128;
constexpr int kCookZN = kCookNib + 512;
constexpr int kCookS16 = kCookNib;  // COOK_S16 and COOK_NIB exclude each other
// COOK_2CH: k_cook folds a lane's pieces as two interleaved Horner chains
// (even and odd piece slots, step Z_{32 kCookLpp}: byte tables at kCookZH2),
// half the dependent LDS round trips per round.  k_decook keeps one chain and
// copies only the tables before kCookZH2 (its per-packet scratch is larger).
#ifndef COOK_2CH
#define COOK_2CH 1
#endif
constexpr int kCookZH2 = COOK_NIB ? kCookZN + 128 : (COOK_S16 ? kCookS16 + 2048 : kCookNib);
constexpr int kCookTabDecook = kCookZH2;                            // k_decook's LDS tables
constexpr int kCookTabWords = kCookZH2 + (COOK_2CH ? 1024 : 0);     // the blob, k_cook's tables
static_assert(!(COOK_NIB && COOK_S16), "COOK_NIB and COOK_S16 are alternatives");
constexpr int kCookKsBytes = 65536 + 128;  // key stream covers every byte position used
constexpr int kCookKsLead = 16;            // ... and 16 bytes before position 0 (phase pieces)

struct CookArgs {
    uint8_t *base;
    uint8_t *dst;                // out of place: packet i's output at dst + its offset (NULL: in place);
                                 // may be pinned host memory (the transfer is fused into the kernel)
    const uint64_t *offset;
    const rsmi_fenc_packet *pk;  // or an FEC packet list: packet i at pk[i].slot * stride + pk_off,
    int32_t pk_off;              // pk[i].len bytes (len unused)
    int32_t pk_idx;              // 1: pk[i].event is packet i's index in the batch (IV draw, out_len,
                                 // dst_off), a cook list of k_expand_packets
    int32_t phase;               // 1: the bytes of a packet's first 16-byte piece before it (source and
                                 // output alike) are scratch, so k_cook works on whole aligned pieces
    uint8_t *mirror;             // de_cook only: the output also at mirror + its offset (pinned host)
    const int64_t *dst_off;      // packed output: packet i's output at dst + dst_off[i], room for
                                 // RSMI_FEC_COOK_SPAN(len) bytes (NULL: dst + its own offset)
    int64_t stride, count;
    int32_t cap, flags;
    const int32_t *len;
    int32_t *out_len;
    const uint8_t *iv, *iv_len;  // cook only; NULL -> device-drawn from seed
    uint64_t seed;
    const uint32_t *tabs;        // device CRC blob
    const uint8_t *ks;           // device key stream, NULL when there is no XOR stage
    int32_t prex;                // cook only: entries with kPrexFlag were cooked by the encoder
};
size_t cook_lds_bytes(bool decook);
// do_cook over an FEC packet list (rsmi_fenc_run_cooked_dev): packet p at
// slots + pk[p].slot * S + RSMI_FEC_SLOT_PACKET, pk[p].len bytes (a device
// cook list of k_expand_packets: pk[p].event = the packet's index i in the
// batch); output at the same offset of dst (NULL: in place) or at dst +
// dst_off[i], out_len[i], IVs drawn on the device from (seed, i) (cook_host.cpp).
int cook_ctx_flags(const rsmi_cook_ctx *ctx);
const uint8_t *cook_ctx_ks(const rsmi_cook_ctx *ctx);  // key stream at packet offset 0 (zeros: no XOR)
// prex: list entries flagged kPrexFlag had their body cooked by the encoder's
// epilogue into dst (EpiRec above).
int cook_packets(const rsmi_cook_ctx *ctx, uint8_t *slots, int64_t S, const rsmi_fenc_packet *pk,
                 int64_t npk, int32_t *out_len, uint8_t *dst, const int64_t *dst_off, uint64_t seed,
                 hipStream_t s, bool prex = false);
hipError_t launch_cook(const CookArgs &a, bool decook, int max_blocks, hipStream_t s);



// ---- FEC framing (frame.hip, fec_enc.cpp) --------------------------------------
constexpr int kSlotHeader = RSMI_FEC_SLOT_PACKET;  // packet (8-byte header) offset in a slot
constexpr int kSlotShard = RSMI_FEC_SLOT_SHARD;    // shard offset: 128-byte aligned rows
// One framing job: a completed FEC group (nslots = k + m slots, nframe = k data
// shards) or a mode-1 packet sent ahead of its group (nslots = nframe = 1).
struct FrameGroup {
    uint64_t slot0;     // first slot
    uint32_t seq;
    uint32_t fec_len;   // shard bytes
    uint32_t src0;      // first FrameSrc of the job
    uint32_t nsrc;      // mode 0: blob records (the blob's u32 count); mode 1: = nframe
    uint32_t blob_len;  // mode 0: blob bytes (blob_encode_t::current_len)
    uint16_t nslots, nframe;
    uint8_t mode, k, m, idx0;  // header bytes; idx0 = index of slot 0
    // the fused framing cook (k_cook_frame) frames data shards cfirst..nfr-1
    // (packets emitted in this batch, at most kFuseRecs source records each)
    // and cooks cfirst..nclean-1 (no stale blob bytes: final once framed)
    uint16_t cfirst, nclean, nfr;
    uint16_t pad[3];    // the planner's: [0..1] its encoder run, [2] that run cooks parity in its epilogue
};
// A payload address in a plan: a device address, or (kCarryTag set) an offset
// into carry buffer 0 or 1 (kCarryBuf1), resolved by the kernels.
constexpr uint64_t kCarryTag = 1ull << 63, kCarryBuf1 = 1ull << 62, kCarryOff = kCarryBuf1 - 1;
struct CarryBase {
    const uint8_t *buf[2];
    __host__ __device__ const uint8_t *resolve(uint64_t a) const {
        // a mask select, not buf[i]: an indexed member (which LLVM makes of a
        // plain ?: as well) sends the struct to scratch in k_frame
        const uint64_t b0 = (uint64_t)(uintptr_t)buf[0], b1 = (uint64_t)(uintptr_t)buf[1];
        const uint8_t *b = reinterpret_cast<const uint8_t *>(
            (uintptr_t)(b0 ^ ((b0 ^ b1) & (0 - ((a >> 62) & 1)))));
        return (a & kCarryTag) ? b + (a & kCarryOff) : reinterpret_cast<const uint8_t *>(a);
    }
};
#ifndef FRAME_LDS_SRC
#define FRAME_LDS_SRC 1024
#endif
constexpr uint32_t kFrameLdsSrc = FRAME_LDS_SRC;  // k_frame stages a job's records in LDS up to this many
struct FrameSrc {
    uint64_t addr;      // payload address (carry-tagged or device)
    uint32_t len;
    uint32_t off;       // mode 0: blob offset of the record's u16 length; mode 1: 0
};
struct CarryCopy {
    uint64_t src, dst;  // carry-tagged or device addresses; dst 16-aligned, room for round_up(len, 16)
    uint32_t len, pad;
};
// Receive side (fec_dec.cpp): copy a received shard into decode staging,
// zero-filled to dst_len (a multiple of 16, dst 16-aligned).
struct GatherCopy {
    uint64_t src;       // carry-tagged or device address
    uint64_t dst;
    uint32_t len, dst_len;
};
hipError_t launch_gather(const GatherCopy *jobs, int64_t njobs, CarryBase carry, hipStream_t s);
// Receive side, rows copied back: rows src, src + stride, ... (k of them, len
// bytes each) joined back to back at dst (16-aligned, room for
// round_up(k * len, 16)).  A mode-0 group's k data rows become its blob in one
// piece, so no record straddles two rows on the host; k = 1 copies one row.
struct JoinCopy {
    uint64_t src, dst;  // device addresses
    uint32_t len, k, stride, pad;
};
hipError_t launch_join(const JoinCopy *jobs, int64_t njobs, hipStream_t s);
// Mode-0 stale bytes (fec_enc.cpp): a byte run between shard rows of the
// batch's slots and the encoder's device copy of blob_encode_t's buffer.  A
// location is a slot index (byte slots + slot*stride + kSlotShard + off) or,
// with kShadowLoc, the buffer itself (byte shadow + off).
constexpr uint64_t kShadowLoc = 1ull << 63;
// ... or, with kAbsLoc, an absolute device address (the collector's runs over
// many encoders, each with its own blob buffer: rsmi_fenc_run_many).
constexpr uint64_t kAbsLoc = 1ull << 62;
constexpr int kBlobBufBytes = (255 + 5) * 3800;  // blob_encode_t::input_buf, fec_manager.h:257
struct ByteRun {
    uint64_t dst, src;
    uint32_t dst_off, src_off, len, pad;
};
hipError_t launch_byte_runs(const ByteRun *runs, int64_t nruns, uint8_t *slots, int64_t slot_stride,
                            uint8_t *shadow, hipStream_t s);
// skip_clean: leave data shards cfirst..nclean-1 (and their headers) to k_cook_frame.
hipError_t launch_frame(const FrameGroup *groups, int64_t ngroups, const FrameSrc *srcs,
                        CarryBase carry, uint8_t *slots, int64_t slot_stride, hipStream_t s,
                        bool skip_clean = false);
hipError_t launch_carry(const CarryCopy *jobs, int64_t njobs, CarryBase carry, hipStream_t s);
// A run of a batch's packet list (what output() returned): packets first ..
// first + count - 1 sit in slots slot .. slot + count - 1, len bytes each (a
// mode-0 group is one run; fec_enc.cpp).  Cooked runs upload the runs and
// expand them on the device (k_expand_packets) into two cook lists: A, the
// data packets of clean shards (FrameGroup.nclean: framed and cooked in one
// pass by k_cook_frame in a fused run), and B, every other packet.  A list
// entry's `event` is the packet's index in the batch (its IV draw, out_len and
// packed place).  Packed cooked output (rsmi_fenc_run_cooked_packed_dev): the
// run's packets go to out0, out0 + span, ... with span = RSMI_FEC_COOK_SPAN(len).
struct PacketRun {
    int64_t slot, out0;
    int32_t first;           // index of the run's first packet in the batch
    int32_t afirst, bfirst;  // where its list-A packets start in list A, its others in B
    int32_t len;
    int32_t job;             // the FrameGroup (job) its slots belong to
    uint16_t count, ndata;   // packets [0, ndata) are cooked from list A, [ndata, count) from B
    uint16_t nfr, pad;       // packets [0, nfr) are in list A (framed there; nfr >= ndata)
};
// job_a (optional, the fused run): list A's entries' jobs; then the parity
// packets' headers are written too (groups: the plan's; slots, slot_stride).
// ---- the parity packets cooked in the encoder's epilogue (RSMI_OPT_PARITY_COOK) ----
// A fused cooked run normally has the encoder write the parity shards plain
// into their slots and k_cook read them back.  With the epilogue, the encoder
// (k_bs2c_<k>_<n>) stores every whole 16-byte payload piece of a parity packet
// already obscured and keyed (the piece XOR its IV and key-stream windows)
// into the output, and the rest of the packet's pieces (the partial last one
// and any line padding) plain into the output; k_cook's PREX form then reads
// the packet back from the output, recovers the plain bytes for the CRC, and
// writes only the header piece and the tail (crc / IV / iv_len).  The parity
// slots are never written.  k_expand_packets fills one record per parity slot
// with what the encoder needs, and flags those packets' list-B entries
// (kPrexFlag in len).
struct EpiRec {
    uint32_t tag;    // the run's tag: records of other runs (or never written) do not match
    uint32_t meta;   // packet length (header included) | iv_len << 16 (0: no obscure stage)
    uint32_t magic;  // 0xFFFFFFFF / iv_len (mod by multiply-high, as k_cook)
    uint32_t pad;
    uint32_t iv[12]; // the IV repeated: byte t = iv[t % iv_len], t < 48
};
static_assert(sizeof(EpiRec) == 64, "EpiRec is one 64-byte record per slot");
constexpr int32_t kPrexFlag = 1 << 30;  // list-B entry len: the encoder cooked its body
struct EpiArgs {     // k_expand_packets' side (rec == nullptr: no epilogue)
    EpiRec *rec;     // indexed by slot
    uint8_t *out;    // the cooked output (slot geometry): parity headers go there too
    uint64_t seed;   // the run's IV seed (the draw k_cook would make)
    uint32_t tag;
    int32_t obs;     // the obscure stage is on
};
struct CookEpi {     // the encoder's side, per encoder run
    uint8_t *out;    // the run's shard base in the output (the slots' base + (out - slots))
    const EpiRec *rec;  // records of the run's first slot
    const uint8_t *ks;  // key stream at packet offset 0 (zeros without an XOR stage; never NULL)
    uint32_t tag, n;    // slots per group
};
hipError_t launch_expand_packets(const PacketRun *runs, int64_t nruns, rsmi_fenc_packet *pk_a,
                                 rsmi_fenc_packet *pk_b, int64_t *dst_off, int32_t *job_a, hipStream_t s,
                                 const FrameGroup *groups = nullptr, uint8_t *slots = nullptr,
                                 int64_t slot_stride = 0, EpiArgs epi = EpiArgs{nullptr, nullptr, 0, 0, 0});
// The cooking split-k encoder exists for (k, n) and this geometry (the
// checks launch_encode_bitslice_cooked makes).
bool bitslice_cooked_ok(const UniformArgs &a);
hipError_t launch_encode_bitslice_cooked(const UniformArgs &a, const CookEpi &e, hipStream_t s);
// encode_dev's checks and code setup, then the cooking encoder (api.cpp).
bool encode_cooked_ok(int k, int n, int64_t gs, int64_t ss, int len, int64_t ngroups);
int encode_dev_cooked(int k, int n, uint8_t *base, int64_t gs, int64_t ss, int len, int64_t ngroups,
                      const CookEpi &e, hipStream_t s);
bool parity_cook_enabled();
// The fused framing cook (k_cook_frame): list A's packets are data packets of
// clean shards (FrameGroup.nclean), framed from their source records into
// their slots (for the encoder) and cooked into the output in the same pass.
constexpr int kFuseRecs = 8;  // source records one fused shard may overlap
struct FuseArgs {
    const FrameGroup *groups;
    const FrameSrc *srcs;
    CarryBase carry;
    const int32_t *job;  // per list entry: its group's FrameGroup index
    const uint32_t *rec; // per list entry: (first record << 8) | records its shard overlaps
};
int cook_frame_packets(const rsmi_cook_ctx *ctx, uint8_t *slots, int64_t S, const rsmi_fenc_packet *pk,
                       int64_t npk, int32_t *out_len, uint8_t *dst, const int64_t *dst_off, uint64_t seed,
                       const FuseArgs &f, hipStream_t s);
hipError_t launch_cook_frame(const CookArgs &a, const FuseArgs &f, int max_blocks, hipStream_t s);

// host_pool.cpp: fn(0..n-1) over up to nthreads host threads (the caller
// included); returns when every item is done.
void host_parallel_for(int n, int nthreads, const std::function<void(int)> &fn);

// An event several plan sets / batches may wait on: a collector's
// (rsmi_fenc_run_many, rsmi_fdec_run_many), which every manager it ran holds
// until its own next run -- one record per flush instead of one per manager.
struct SharedEv {
    hipEvent_t ev = nullptr;
    ~SharedEv() {
        if (ev) (void)hipEventDestroy(ev);
    }
};

}  // namespace rsmi
