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
// encoder's carry area with the same unaligned-window loads.
#include "rsmi_internal.hpp"

namespace rsmi {
namespace {

constexpr int kThreads = 256;
constexpr int kLdsSrc = 1024;  // source records staged in LDS per group

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

// Bytes [lo, hi) of a 16-byte piece taken from src[a .. a + hi - lo): piece
// byte p = src[a - lo + p].  Only the aligned dwords that hold wanted bytes are
// read, so nothing outside the source range's own dwords is touched.
__device__ __forceinline__ u32x4 window(const uint8_t *a, int lo, int hi) {
    const uint8_t *w = a - lo;                      // address of piece byte 0
    const uintptr_t wa = (uintptr_t)w;
    const uint32_t *d = reinterpret_cast<const uint32_t *>(wa & ~uintptr_t(3));
    const uint32_t sh = (uint32_t)(wa & 3);
    // dword e covers piece bytes [4e - sh, 4e - sh + 4); wanted if it meets [lo, hi)
    uint32_t e[5];
    if (lo == 0 && hi == 16) {
        const u32x4 v = *reinterpret_cast<const u32x4_a4 *>(d);
        e[0] = v.x; e[1] = v.y; e[2] = v.z; e[3] = v.w;
        e[4] = sh ? d[4] : 0u;
    } else {
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int b0 = 4 * i - (int)sh;
            e[i] = (b0 < hi && b0 + 4 > lo) ? d[i] : 0u;
        }
    }
    u32x4 r;
    r.x = __builtin_amdgcn_alignbyte(e[1], e[0], sh);
    r.y = __builtin_amdgcn_alignbyte(e[2], e[1], sh);
    r.z = __builtin_amdgcn_alignbyte(e[3], e[2], sh);
    r.w = __builtin_amdgcn_alignbyte(e[4], e[3], sh);
    return r;
}

// Keep bytes [lo, hi) of a piece.
__device__ __forceinline__ u32x4 keep(u32x4 v, int lo, int hi) {
    u32x4 m;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int a = max(lo - 4 * d, 0), b = min(hi - 4 * d, 4);
        const uint32_t hm = b >= 4 ? ~0u : (b <= 0 ? 0u : ((1u << (8 * b)) - 1u));
        const uint32_t lm = a >= 4 ? ~0u : (a <= 0 ? 0u : ((1u << (8 * a)) - 1u));
        m[d] = hm & ~lm;
    }
    return v & m;
}

// Big-endian constant c (nb <= 4 bytes) at stream position s0, placed into the
// piece that starts at stream position b.
__device__ __forceinline__ u32x4 konst(uint32_t c, int nb, int64_t s0, int64_t b) {
    // the nb bytes in memory order as a little-endian integer, placed at piece
    // byte p = s0 - b (-3 <= p <= 15) by per-dword shifts (no indexed writes)
    const uint64_t v = nb == 4 ? (uint64_t)__builtin_bswap32(c)
                               : (uint64_t)(((c & 0xffu) << 8) | ((c >> 8) & 0xffu));
    const int p = (int)(s0 - b);
    u32x4 r;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int sh = 8 * (p - 4 * d);  // bit position of the constant in dword d
        uint32_t w = 0;
        if (sh >= 0 && sh < 32) w = (uint32_t)(v << sh);
        else if (sh < 0 && sh > -8 * nb) w = (uint32_t)(v >> -sh);
        r[d] = w;
    }
    return r;
}

struct Src {
    const uint8_t *addr;
    uint32_t len, off;
};

__device__ __forceinline__ Src get_src(const FrameSrc *g, const FrameSrc *lds, uint32_t j,
                                       uint32_t nlds) {
    const FrameSrc &s = j < nlds ? lds[j] : g[j];
    return Src{reinterpret_cast<const uint8_t *>(s.addr), s.len, s.off};
}

// Largest j in [0, n) with off_j <= pos (off_0 <= pos is guaranteed).
__device__ __forceinline__ uint32_t find_src(const FrameSrc *g, const FrameSrc *lds, uint32_t n,
                                             uint32_t nlds, int64_t pos) {
    uint32_t lo = 0, hi = n;  // invariant: off_lo <= pos, answer < hi
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint32_t o = mid < nlds ? lds[mid].off : g[mid].off;
        if ((int64_t)o <= pos) lo = mid;
        else hi = mid;
    }
    return lo;
}

// The 16 stream bytes at [b, b+16) of a stream made of: an optional 4-byte
// big-endian count at [0, 4), then source records [u16 len BE][payload] at
// their offsets, then zeros from stream_len on.
__device__ u32x4 stream_piece(const FrameSrc *g, const FrameSrc *lds, uint32_t j0, uint32_t n,
                              uint32_t nlds, int64_t b, int64_t stream_len, bool count_hdr,
                              uint32_t count) {
    u32x4 acc = {0, 0, 0, 0};
    const int64_t end = min(b + 16, stream_len);
    int64_t pos = b;
    if (pos >= end) return acc;
    if (count_hdr && pos < 4) {
        acc |= konst(count, 4, 0, b);
        pos = 4;
    }
    if (pos >= end || n == 0) return acc;
    uint32_t j = j0 + find_src(g + j0, lds + j0, n, nlds > j0 ? nlds - j0 : 0, pos);
    const uint32_t jend = j0 + n;
    while (pos < end && j < jend) {
        const Src s = get_src(g, lds, j, nlds);
        const int64_t p0 = s.off, q0 = p0 + 2, q1 = q0 + s.len;
        if (pos < q0) {
            acc |= konst(s.len & 0xffffu, 2, p0, b);
            pos = min(q0, end);
        }
        if (pos < end && pos < q1) {
            const int64_t e = min(q1, end);
            const int lo = (int)(pos - b), hi = (int)(e - b);
            acc |= keep(window(s.addr + (pos - q0), lo, hi), lo, hi);
            pos = e;
        }
        if (pos >= q1) ++j;
    }
    return acc;
}

__global__ __launch_bounds__(kThreads) void k_frame(const FrameGroup *groups, int64_t ngroups,
                                                     const FrameSrc *srcs, uint8_t *slots,
                                                     int64_t slot_stride) {
    __shared__ FrameSrc lsrc[kLdsSrc];
    for (int64_t gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {
        const FrameGroup G = groups[gi];
        const FrameSrc *gs = srcs + G.src0;
        const uint32_t nsrc = G.mode == 0 ? G.nsrc : G.nframe;
        const uint32_t nl = min(nsrc, (uint32_t)kLdsSrc);
        for (uint32_t t = threadIdx.x; t < nl; t += kThreads) lsrc[t] = gs[t];
        __syncthreads();
        uint8_t *s0 = slots + (int64_t)G.slot0 * slot_stride;
        // headers: seq | mode | k | m | index (fec_manager.cpp:318-333); mode-1
        // data packets carry k = m = 0 (:321-323)
        for (uint32_t j = threadIdx.x; j < G.nslots; j += kThreads) {
            const bool zero_km = G.mode == 1 && j < G.nframe;
            const uint32_t w1 = (uint32_t)G.mode | (zero_km ? 0u : ((uint32_t)G.k << 8 | (uint32_t)G.m << 16)) |
                                ((G.idx0 + j) & 0xffu) << 24;
            *reinterpret_cast<u32x2 *>(s0 + (int64_t)j * slot_stride + 8) = u32x2{bswap32(G.seq), w1};
        }
        // data shards, whole 16-byte pieces
        const uint32_t pps = (G.fec_len + 15) >> 4;
        const uint32_t total = pps * G.nframe;
        for (uint32_t t = threadIdx.x; t < total; t += kThreads) {
            const uint32_t i = t / pps, q = t - i * pps;
            u32x4 v;
            if (G.mode == 0) {
                const int64_t b = (int64_t)i * G.fec_len + 16 * (int64_t)q;
                v = stream_piece(gs, lsrc, 0, nsrc, nl, b, G.blob_len, true, G.nsrc);
            } else {
                const Src s = get_src(gs, lsrc, i, nl);
                v = stream_piece(gs, lsrc, i, 1, nl, 16 * (int64_t)q, (int64_t)s.len + 2, false, 0);
            }
            *reinterpret_cast<u32x4 *>(s0 + (int64_t)i * slot_stride + 16 + 16 * (int64_t)q) = v;
        }
        __syncthreads();  // lsrc is restaged for the next group
    }
}

// Pending packets -> carry area: dst (16-aligned) gets len bytes of src, whole
// pieces (bytes past len inside the last piece are zero).
__global__ __launch_bounds__(kThreads) void k_carry(const CarryCopy *jobs, int64_t njobs) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    for (int64_t w = w0; w < njobs; w += (int64_t)gridDim.x * (kThreads / 64)) {
        const CarryCopy J = jobs[w];
        const uint8_t *src = reinterpret_cast<const uint8_t *>(J.src);
        uint8_t *dst = reinterpret_cast<uint8_t *>(J.dst);
        for (uint32_t q = lane; 16 * q < J.len; q += 64) {
            const int hi = (int)min(16u, J.len - 16 * q);
            *reinterpret_cast<u32x4 *>(dst + 16 * (int64_t)q) = keep(window(src + 16 * q, 0, hi), 0, hi);
        }
    }
}

}  // namespace

hipError_t launch_frame(const FrameGroup *groups, int64_t ngroups, const FrameSrc *srcs,
                        uint8_t *slots, int64_t slot_stride, hipStream_t s) {
    if (ngroups <= 0) return hipSuccess;
    const int64_t blocks = ngroups < 65536 ? ngroups : 65536;
    k_frame<<<(unsigned)blocks, kThreads, 0, s>>>(groups, ngroups, srcs, slots, slot_stride);
    return hipGetLastError();
}

hipError_t launch_carry(const CarryCopy *jobs, int64_t njobs, hipStream_t s) {
    if (njobs <= 0) return hipSuccess;
    int64_t blocks = (njobs + kThreads / 64 - 1) / (kThreads / 64);
    if (blocks > 8192) blocks = 8192;
    k_carry<<<(unsigned)blocks, kThreads, 0, s>>>(jobs, njobs);
    return hipGetLastError();
}

}  // namespace rsmi
