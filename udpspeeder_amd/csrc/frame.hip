// frame.hip -- FEC framing kernels for gfx950 (include/rsmi_fec.h).
//
// fec_encode_manager_t builds each FEC packet on the CPU with memcpy: mode 0
// appends [u16 len][payload] records behind a u32 count (blob_encode_t::input,
// fec_manager.cpp:55-65) and cuts the blob into k shards of fec_len bytes
// (blob_encode_t::output, :67-75); mode 1 puts [u16 len][payload] in shard i
// and zero-pads it to fec_len (:190-198, :341-344); every packet gets the
// 8-byte header of :318-333.  Here one workgroup frames one group: it stages
// the group's source records in LDS and writes every shard as whole 16-byte
// pieces.  A piece is read from the "stream" it belongs to (the blob in mode 0,
// the shard's own [u16 len][payload] in mode 1) as a run of segments -- the
// 4-byte count, a 2-byte length prefix, a payload range, the zero tail -- so a
// piece inside one payload (the common case) is one 16-byte load (dwordx4 +
// dword, funnel-shifted with v_alignbyte) and one 16-byte store.
//
// k_carry copies packets still pending at the end of a batch into the
// encoder's carry area with the same unaligned-window loads.  k_byte_runs
// fills mode 0's stale bytes past the blob's end and keeps the encoder's copy
// of the blob buffer (fec_enc.cpp).
#include "rsmi_internal.hpp"

namespace rsmi {
#include "frame_piece.hpp"
namespace {

constexpr int kThreads = 256;
#ifndef FRAME_THREADS
#define FRAME_THREADS 256  // k_frame's threads per group (one workgroup frames one group)
#endif
constexpr int kFThreads = FRAME_THREADS;
constexpr int kLdsSrc = (int)kFrameLdsSrc;  // source records staged in LDS per group

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
using namespace fpiece;

// Source records of the job being framed, staged in LDS (structure of arrays).
struct LdsSrc {
    uint64_t addr[kLdsSrc];
    uint32_t off[kLdsSrc];
    uint32_t len[kLdsSrc];
};

// Read access to a job's source records: from LDS, or straight from global
// memory for the rare job with more than kLdsSrc records (tiny packets, long
// queue_len), so that the LDS path holds no global loads a wait could join.
template <bool kGlobal>
struct View {
    const FrameSrc *g;
    const LdsSrc *l;
    CarryBase carry;
    __device__ __forceinline__ uint32_t off(uint32_t j) const { return kGlobal ? g[j].off : l->off[j]; }
    __device__ __forceinline__ uint32_t len(uint32_t j) const { return kGlobal ? g[j].len : l->len[j]; }
    __device__ __forceinline__ const uint8_t *addr(uint32_t j) const {
        return kGlobal ? carry.resolve(g[j].addr) : reinterpret_cast<const uint8_t *>(l->addr[j]);
    }
};

#ifndef FRAME_BATCH
#define FRAME_BATCH 4
#endif
constexpr int kBatch = FRAME_BATCH;     // pieces per thread per step: their loads are in flight together
#ifndef FRAME_SLOW_MAX
#define FRAME_SLOW_MAX 1024
#endif
constexpr int kSlowMax = FRAME_SLOW_MAX;  // boundary pieces queued per job (more are assembled in place)

struct Piece {
    uint32_t i, q, j;
    int64_t b;
};

// Piece t = shard i * pps + piece q, its stream position b, and (mode 0) the
// record j holding stream byte max(b, 4) is found by the caller.
__device__ __forceinline__ Piece piece_at(const FrameGroup &G, uint32_t t, uint32_t pps,
                                          uint32_t magic) {
    uint32_t i = pps == 1 ? t : __umulhi(t, magic);  // t / pps, corrected below
    if (i * pps > t) --i;
    if ((i + 1) * pps <= t) ++i;
    Piece P;
    P.i = i;
    P.q = t - i * pps;
    P.b = G.mode == 0 ? (int64_t)i * G.fec_len + 16 * (int64_t)P.q : 16 * (int64_t)P.q;
    P.j = G.mode == 0 ? 0u : i;
    return P;
}

template <class V>
__device__ __forceinline__ uint32_t find_record(const V &src, uint32_t n, int64_t b) {
    uint32_t j = 0;
    const int64_t pos = max(b, (int64_t)4);
    while (n > 1) {
        const uint32_t h = n >> 1;
        j = (int64_t)src.off(j + h) <= pos ? j + h : j;
        n -= h;
    }
    return j;
}

template <class V>
__device__ __forceinline__ u32x4 slow_piece(const FrameGroup &G, const V &src, uint32_t nsrc,
                                            const Piece &P) {
    if (G.mode == 0) return stream_piece(src, P.j, nsrc, P.b, G.blob_len, true, G.nsrc);
    return stream_piece(src, P.j, P.j + 1, P.b, (int64_t)src.len(P.j) + 2, false, 0);
}

__device__ __forceinline__ void put_piece(uint8_t *s0, int64_t slot_stride, const Piece &P, u32x4 v) {
    *reinterpret_cast<u32x4 *>(s0 + (int64_t)P.i * slot_stride + kSlotShard + 16 * (int64_t)P.q) = v;
}

// Frame one job with kThreads threads.  Phase 1 takes kBatch pieces per thread
// per step: the record searches run interleaved and the 16-byte loads of the
// pieces that lie inside one payload are issued together (straight-line, every
// lane loads: the others read a dummy address) and stored.  Pieces that cross
// a record or stream boundary (a few per record) are queued in LDS; phase 2
// assembles them segment by segment, one per lane, so no wave runs the segment
// loop for a single lane of its 64.
template <bool kGlobal>
__device__ __forceinline__ void frame_job(const FrameGroup &G, const View<kGlobal> &src,
                                          uint8_t *s0, int64_t slot_stride, const uint8_t *dummy,
                                          uint32_t *slow, uint32_t *nslow, uint32_t c0, uint32_t c1) {
    const uint32_t nsrc = G.mode == 0 ? G.nsrc : G.nframe;
    const uint32_t pps = (G.fec_len + 15) >> 4;
    // shards c0..c1-1 are framed elsewhere: piece index v of the others is
    // piece t = v, or v + (c1 - c0) pps past shard c0
    const uint32_t n1 = pps * c0, gap = pps * (c1 - c0);
    const uint32_t total = pps * G.nframe - gap;
    auto tof = [&](uint32_t v) { return v < n1 ? v : v + gap; };
    const uint32_t magic = pps == 1 ? 0u : (uint32_t)(0xFFFFFFFFu / pps) + 1u;
    for (uint32_t t0 = threadIdx.x; t0 < total; t0 += kBatch * kFThreads) {
        Piece P[kBatch];
#pragma unroll
        for (int u = 0; u < kBatch; ++u) P[u] = piece_at(G, tof(min(t0 + u * kFThreads, total - 1)), pps, magic);
        if (G.mode == 0) {  // kBatch interleaved searches (same trip count)
            uint32_t n = nsrc;
            while (n > 1) {
                const uint32_t h = n >> 1;
#pragma unroll
                for (int u = 0; u < kBatch; ++u)
                    P[u].j = (int64_t)src.off(P[u].j + h) <= max(P[u].b, (int64_t)4) ? P[u].j + h : P[u].j;
                n -= h;
            }
        }
        const uint8_t *A[kBatch];
        bool fast[kBatch];
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {
            const int64_t q0 = G.mode == 0 ? (int64_t)src.off(P[u].j) + 2 : 2;
            const int64_t q1 = q0 + src.len(P[u].j);
            fast[u] = P[u].b >= q0 && P[u].b + 16 <= q1;
            A[u] = fast[u] ? src.addr(P[u].j) + (P[u].b - q0) : dummy;
        }
        u32x4 v[kBatch];
#pragma unroll
        for (int u = 0; u < kBatch; ++u) v[u] = window(A[u], 0, 16);
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {
            const uint32_t t = t0 + u * kFThreads;
            if (t >= total) continue;
            if (fast[u]) {
                put_piece(s0, slot_stride, P[u], v[u]);
            } else {
                const uint32_t k = atomicAdd(nslow, 1u);
                if (k < (uint32_t)kSlowMax) slow[k] = tof(t);
            }
        }
    }
    __syncthreads();
    const uint32_t nq = *nslow;
    if (nq <= (uint32_t)kSlowMax) {
        for (uint32_t k = threadIdx.x; k < nq; k += kFThreads) {
            Piece Q = piece_at(G, slow[k], pps, magic);
            if (G.mode == 0) Q.j = find_record(src, nsrc, Q.b);
            put_piece(s0, slot_stride, Q, slow_piece(G, src, nsrc, Q));
        }
    } else {  // queue overflow (thousands of tiny records): every boundary piece in place
        for (uint32_t v = threadIdx.x; v < total; v += kFThreads) {
            Piece Q = piece_at(G, tof(v), pps, magic);
            if (G.mode == 0) Q.j = find_record(src, nsrc, Q.b);
            const int64_t q0 = G.mode == 0 ? (int64_t)src.off(Q.j) + 2 : 2;
            if (Q.b >= q0 && Q.b + 16 <= q0 + src.len(Q.j)) continue;
            put_piece(s0, slot_stride, Q, slow_piece(G, src, nsrc, Q));
        }
    }
}

__global__ __launch_bounds__(kFThreads) void k_frame(const FrameGroup *groups, int64_t ngroups,
                                                     const FrameSrc *srcs, CarryBase carry,
                                                     uint8_t *slots, int64_t slot_stride, int skip_clean) {
    __shared__ LdsSrc lsrc;
    __shared__ uint32_t slow[kSlowMax];
    __shared__ uint32_t nslow;
    const uint8_t *dummy = reinterpret_cast<const uint8_t *>(groups);  // >= 20 readable bytes
    for (int64_t gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {
        const FrameGroup G = groups[gi];
        const FrameSrc *gs = srcs + G.src0;
        const uint32_t nsrc = G.mode == 0 ? G.nsrc : G.nframe;
        const bool in_lds = nsrc <= (uint32_t)kLdsSrc;
        if (in_lds)
            for (uint32_t t = threadIdx.x; t < nsrc; t += kFThreads) {
                const FrameSrc f = gs[t];
                lsrc.addr[t] = (uint64_t)(uintptr_t)carry.resolve(f.addr);
                lsrc.off[t] = f.off;
                lsrc.len[t] = f.len;
            }
        if (threadIdx.x == 0) nslow = 0;
        __syncthreads();
        uint8_t *s0 = slots + (int64_t)G.slot0 * slot_stride;
        // headers: seq | mode | k | m | index (fec_manager.cpp:318-333); mode-1
        // data packets carry k = m = 0 (:321-323)
        const uint32_t c0 = skip_clean ? (uint32_t)G.cfirst : 0u, c1 = skip_clean ? (uint32_t)G.nfr : 0u;
        for (uint32_t j = threadIdx.x; j < G.nslots; j += kFThreads) {
            if (j >= c0 && j < c1) continue;
            const bool zero_km = G.mode == 1 && j < G.nframe;
            const uint32_t w1 = (uint32_t)G.mode |
                                (zero_km ? 0u : ((uint32_t)G.k << 8 | (uint32_t)G.m << 16)) |
                                ((G.idx0 + j) & 0xffu) << 24;
            *reinterpret_cast<u32x2 *>(s0 + (int64_t)j * slot_stride + kSlotHeader) =
                u32x2{bswap32(G.seq), w1};
        }
        if (in_lds)
            frame_job(G, View<false>{gs, &lsrc, carry}, s0, slot_stride, dummy, slow, &nslow, c0, max(c0, c1));
        else
            frame_job(G, View<true>{gs, &lsrc, carry}, s0, slot_stride, dummy, slow, &nslow, c0, max(c0, c1));
        __syncthreads();  // lsrc and the queue are reset for the next group
    }
}

// Pending packets -> carry area: dst (16-aligned) gets len bytes of src, whole
// pieces (bytes past len inside the last piece are zero).
__global__ __launch_bounds__(kThreads) void k_carry(const CarryCopy *jobs, int64_t njobs,
                                                     CarryBase carry) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    for (int64_t w = w0; w < njobs; w += (int64_t)gridDim.x * (kThreads / 64)) {
        const CarryCopy J = jobs[w];
        const uint8_t *src = carry.resolve(J.src);
        uint8_t *dst = const_cast<uint8_t *>(carry.resolve(J.dst));
        for (uint32_t q = lane; 16 * q < J.len; q += 64) {
            const int hi = (int)min(16u, J.len - 16 * q);
            *reinterpret_cast<u32x4 *>(dst + 16 * (int64_t)q) = keep(window(src + 16 * q, 0, hi), 0, hi);
        }
    }
}

// Rows copied back (fec_dec.cpp): one wave per job, a 16-byte output piece
// per lane; a piece that crosses a row end takes the next row's head as a
// second window (a third and more only when len < 16).
__global__ __launch_bounds__(kThreads) void k_join(const JoinCopy *jobs, int64_t njobs) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    for (int64_t w = w0; w < njobs; w += (int64_t)gridDim.x * (kThreads / 64)) {
        const JoinCopy J = jobs[w];
        const uint8_t *src = reinterpret_cast<const uint8_t *>(J.src);
        uint8_t *dst = reinterpret_cast<uint8_t *>(J.dst);
        const uint32_t L = J.len, total = J.k * J.len;
        for (uint32_t b = 16 * lane; b < total; b += 16 * 64) {
            const uint32_t end = min(b + 16, total);
            uint32_t r = b / L, o = b - r * L, pos = b;
            u32x4 acc = {0, 0, 0, 0};
            while (pos < end) {
                const uint32_t n = min(end - pos, L - o);
                const int lo = (int)(pos - b), hi = lo + (int)n;
                acc |= keep(window(src + (int64_t)r * J.stride + o, lo, hi), lo, hi);
                pos += n;
                ++r;
                o = 0;
            }
            *reinterpret_cast<u32x4 *>(dst + b) = acc;
        }
    }
}

// Received shard -> decode staging, zero-filled to dst_len: one wave per shard.
__global__ __launch_bounds__(kThreads) void k_gather(const GatherCopy *jobs, int64_t njobs,
                                                      CarryBase carry) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    for (int64_t w = w0; w < njobs; w += (int64_t)gridDim.x * (kThreads / 64)) {
        const GatherCopy J = jobs[w];
        const uint8_t *src = carry.resolve(J.src);
        uint8_t *dst = reinterpret_cast<uint8_t *>(J.dst);
        for (uint32_t q = lane; 16 * q < J.dst_len; q += 64) {
            u32x4 v = {0, 0, 0, 0};
            if (16 * q < J.len) {
                const int hi = (int)min(16u, J.len - 16 * q);
                v = keep(window(src + 16 * q, 0, hi), 0, hi);
            }
            *reinterpret_cast<u32x4 *>(dst + 16 * (int64_t)q) = v;
        }
    }
}

// Byte runs (mode-0 stale bytes, fec_enc.cpp): one wave per run, a byte per
// lane; runs are short (stale tails) or one shard row (buffer updates).
__global__ __launch_bounds__(kThreads) void k_byte_runs(const ByteRun *runs, int64_t nruns,
                                                         uint8_t *slots, int64_t slot_stride,
                                                         uint8_t *shadow) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    auto at = [&](uint64_t loc, uint32_t off) {
        if (loc & kShadowLoc) return shadow + off;
        if (loc & kAbsLoc) return reinterpret_cast<uint8_t *>((uintptr_t)(loc & ~kAbsLoc)) + off;
        return slots + (int64_t)loc * slot_stride + kSlotShard + off;
    };
    for (int64_t w = w0; w < nruns; w += (int64_t)gridDim.x * (kThreads / 64)) {
        const ByteRun R = runs[w];
        uint8_t *dst = at(R.dst, R.dst_off);
        const uint8_t *src = at(R.src, R.src_off);
        for (uint32_t i = lane; i < R.len; i += 64) dst[i] = src[i];
    }
}

// Packet runs -> the cook list(s): one wave per run.  Unfused (no job_a), one
// list in packet order (pk_a).  Fused, lists A (packets [0, nfr) of a run,
// with their jobs in job_a) and B (packets [ndata, count)), and the parity
// packets' 8-byte headers (fec_manager.cpp:318-333), which k_frame may not be
// run to write.  With dst_off, also each packet's offset in the packed output.
// k_cook's IV draw (cook.hip splitmix): word w of packet i's stream.
__device__ __forceinline__ uint64_t iv_draw(uint64_t seed, uint64_t idx, uint64_t w) {
    uint64_t z = (seed ^ idx) + (w + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// A parity packet cooked in the encoder's epilogue: its record (the IV k_cook
// would draw for batch index gi, repeated to 48 bytes) and its header in the
// output's header piece, where k_cook's PREX form reads the packet.
__device__ void write_epi(const EpiArgs &ep, int64_t slot, int64_t gi, int32_t len, uint8_t *hdr_out,
                          u32x2 hdr) {
    EpiRec *r = ep.rec + slot;
    uint32_t ivl = 0, magic = 0;
    uint64_t z[4] = {0, 0, 0, 0};
    if (ep.obs) {
        ivl = 4u + (uint32_t)(iv_draw(ep.seed, (uint64_t)gi, 0) % 29u);
        magic = 0xFFFFFFFFu / ivl;
#pragma unroll
        for (int w = 0; w < 4; ++w) z[w] = 8 * w < (int)ivl ? iv_draw(ep.seed, (uint64_t)gi, 1 + (uint64_t)w) : 0;
    }
    uint32_t iv[12];
    uint32_t t8 = 0;  // t % ivl
#pragma unroll
    for (int d = 0; d < 12; ++d) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t w = t8 >> 3;
            const uint64_t zw = w == 0 ? z[0] : w == 1 ? z[1] : w == 2 ? z[2] : z[3];
            v |= (uint32_t)((zw >> (8 * (t8 & 7))) & 0xffu) << (8 * b);
            t8 = (ivl && t8 + 1 >= ivl) ? 0 : t8 + 1;
        }
        iv[d] = v;
    }
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    v4 *rv = reinterpret_cast<v4 *>(r);
    rv[0] = v4{ep.tag, (uint32_t)len | ivl << 16, magic, 0u};
    rv[1] = v4{iv[0], iv[1], iv[2], iv[3]};
    rv[2] = v4{iv[4], iv[5], iv[6], iv[7]};
    rv[3] = v4{iv[8], iv[9], iv[10], iv[11]};
    *reinterpret_cast<u32x2 *>(hdr_out) = hdr;
}

__global__ __launch_bounds__(kThreads) void k_expand_packets(const PacketRun *runs, int64_t nruns,
                                                              rsmi_fenc_packet *pk_a, rsmi_fenc_packet *pk_b,
                                                              int64_t *dst_off, int32_t *job_a,
                                                              const FrameGroup *groups, uint8_t *slots,
                                                              int64_t slot_stride, EpiArgs ep) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    for (int64_t w = w0; w < nruns; w += (int64_t)gridDim.x * (kThreads / 64)) {
        const PacketRun R = runs[w];
        for (int c = lane; c < (int)R.count; c += 64) {
            const rsmi_fenc_packet p{R.slot + c, R.len, R.first + c};
            if (!job_a) {
                pk_a[R.first + c] = p;
            } else {
                if (c < (int)R.nfr) {
                    pk_a[R.afirst + c] = p;
                    job_a[R.afirst + c] = R.job;
                }
                if (c >= (int)R.ndata) pk_b[R.bfirst + c - (int)R.ndata] = p;  // (flagged below)
            }
            if (dst_off) dst_off[R.first + c] = R.out0 + (int64_t)c * RSMI_FEC_COOK_SPAN(R.len);
            if (job_a) {
                const FrameGroup G = groups[R.job];
                const uint32_t j = (uint32_t)(R.slot + c - (int64_t)G.slot0);
                if (j >= G.nframe) {  // a parity packet: seq | mode | k | m | index
                    const uint32_t w1 = (uint32_t)G.mode | ((uint32_t)G.k << 8 | (uint32_t)G.m << 16) |
                                        ((G.idx0 + j) & 0xffu) << 24;
                    const u32x2 hdr{bswap32(G.seq), w1};
                    if (ep.rec && G.pad[2] && c >= (int)R.ndata) {  // cooked by the encoder: header to the output
                        write_epi(ep, R.slot + c, p.event, p.len,
                                  ep.out + (R.slot + c) * slot_stride + kSlotHeader, hdr);
                        pk_b[R.bfirst + c - (int)R.ndata].len = p.len | kPrexFlag;
                    } else {
                        *reinterpret_cast<u32x2 *>(slots + (R.slot + c) * slot_stride + kSlotHeader) = hdr;
                    }
                }
            }
        }
    }
}

}  // namespace

hipError_t launch_expand_packets(const PacketRun *runs, int64_t nruns, rsmi_fenc_packet *pk_a,
                                 rsmi_fenc_packet *pk_b, int64_t *dst_off, int32_t *job_a, hipStream_t s,
                                 const FrameGroup *groups, uint8_t *slots, int64_t slot_stride, EpiArgs epi) {
    if (nruns <= 0) return hipSuccess;
    int64_t blocks = (nruns + kThreads / 64 - 1) / (kThreads / 64);
    if (blocks > 8192) blocks = 8192;
    k_expand_packets<<<(unsigned)blocks, kThreads, 0, s>>>(runs, nruns, pk_a, pk_b, dst_off, job_a, groups,
                                                           slots, slot_stride, epi);
    return hipGetLastError();
}

hipError_t launch_byte_runs(const ByteRun *runs, int64_t nruns, uint8_t *slots, int64_t slot_stride,
                            uint8_t *shadow, hipStream_t s) {
    if (nruns <= 0) return hipSuccess;
    int64_t blocks = (nruns + kThreads / 64 - 1) / (kThreads / 64);
    if (blocks > 8192) blocks = 8192;
    k_byte_runs<<<(unsigned)blocks, kThreads, 0, s>>>(runs, nruns, slots, slot_stride, shadow);
    return hipGetLastError();
}

hipError_t launch_gather(const GatherCopy *jobs, int64_t njobs, CarryBase carry, hipStream_t s) {
    if (njobs <= 0) return hipSuccess;
    int64_t blocks = (njobs + kThreads / 64 - 1) / (kThreads / 64);
    if (blocks > 16384) blocks = 16384;
    k_gather<<<(unsigned)blocks, kThreads, 0, s>>>(jobs, njobs, carry);
    return hipGetLastError();
}

hipError_t launch_frame(const FrameGroup *groups, int64_t ngroups, const FrameSrc *srcs,
                        CarryBase carry, uint8_t *slots, int64_t slot_stride, hipStream_t s,
                        bool skip_clean) {
    if (ngroups <= 0) return hipSuccess;
    const int64_t blocks = ngroups < 65536 ? ngroups : 65536;
    k_frame<<<(unsigned)blocks, kFThreads, 0, s>>>(groups, ngroups, srcs, carry, slots, slot_stride,
                                                   skip_clean ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_join(const JoinCopy *jobs, int64_t njobs, hipStream_t s) {
    if (njobs <= 0) return hipSuccess;
    int64_t blocks = (njobs + kThreads / 64 - 1) / (kThreads / 64);
    if (blocks > 8192) blocks = 8192;
    k_join<<<(unsigned)blocks, kThreads, 0, s>>>(jobs, njobs);
    return hipGetLastError();
}

hipError_t launch_carry(const CarryCopy *jobs, int64_t njobs, CarryBase carry, hipStream_t s) {
    if (njobs <= 0) return hipSuccess;
    int64_t blocks = (njobs + kThreads / 64 - 1) / (kThreads / 64);
    if (blocks > 8192) blocks = 8192;
    k_carry<<<(unsigned)blocks, kThreads, 0, s>>>(jobs, njobs, carry);
    return hipGetLastError();
}

}  // namespace rsmi
