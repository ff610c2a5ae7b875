// frame_piece.hpp -- 16-byte pieces of the FEC framing streams, shared by
// k_frame (frame.hip) and the fused framing cook (cook.hip k_cook_frame).
//
// A piece is read from the "stream" it belongs to (the blob in mode 0, the
// shard's own [u16 len][payload] in mode 1) as a run of segments -- the 4-byte
// count, a 2-byte length prefix, a payload range, the zero tail -- so a piece
// inside one payload (the common case) is one 16-byte load (dwordx4 + dword,
// funnel-shifted with v_alignbyte).  Device code only; the includer provides
// namespace rsmi.
#pragma once

namespace fpiece {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));

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

// The 16 stream bytes at [b, b+16) of a stream made of: an optional 4-byte
// big-endian count at [0, 4), then records j0.. [u16 len BE][payload] at their
// offsets, then zeros from stream_len on.  j is a record with off_j <= max(b, 4)
// whose successor starts beyond it (the search result).
template <class V>
__device__ u32x4 stream_piece(const V &src, uint32_t j, uint32_t jend, int64_t b, int64_t stream_len,
                              bool count_hdr, uint32_t count) {
    u32x4 acc = {0, 0, 0, 0};
    const int64_t end = min(b + 16, stream_len);
    int64_t pos = b;
    if (pos >= end) return acc;
    if (count_hdr && pos < 4) {
        acc |= konst(count, 4, 0, b);
        pos = 4;
    }
    while (pos < end && j < jend) {
        const int64_t p0 = src.off(j), q0 = p0 + 2, q1 = q0 + src.len(j);
        if (pos < q0) {
            acc |= konst(src.len(j) & 0xffffu, 2, p0, b);
            pos = min(q0, end);
        }
        if (pos < end && pos < q1) {
            const int64_t e = min(q1, end);
            const int lo = (int)(pos - b), hi = (int)(e - b);
            acc |= keep(window(src.addr(j) + (pos - q0), lo, hi), lo, hi);
            pos = e;
        }
        if (pos >= q1) ++j;
    }
    return acc;
}

}  // namespace fpiece
