// bitslice_cook.hip -- the split-k bit-sliced encoders with the parity cook in
// their epilogue (RSMI_OPT_PARITY_COOK; rsmi_internal.hpp EpiRec): the same
// generated networks as bitslice.hip's k_bs2_<k>_<n>, with a store stage that
// writes the parity packets' payload pieces obscured and keyed into the cooked
// output.  A file of its own so the plain encoders' sources (and the counter
// passes pinned to them, bench.py KERNEL_SOURCES) stay as they are.
#include "rsmi_internal.hpp"

#include "bitslice_core.hpp"
#include "bitslice_kern.hpp"

#ifndef BS_SPLIT
#define BS_SPLIT 1
#endif
#ifndef BS_COOK_EPI
#define BS_COOK_EPI 1  // build the cooking split-k encoders (k_bs2c_*)
#endif
#ifndef BS_COOK_OCC
#define BS_COOK_OCC BS_OCC  // waves per SIMD of the cooking encoders
#endif
#ifdef BS_INC
#include BS_INC
#else
#include "gen/bitslice_codes.inc"
#endif

namespace rsmi {
namespace {

// ---- the same split-k networks with the parity cook in the epilogue ----------
// (rsmi_internal.hpp EpiRec; RSMI_OPT_PARITY_COOK).  Row j's two pieces of a
// lane belong to packet slot g*n + j of the run (g: the piece's group).  A
// piece wholly inside its packet's payload is stored into the output XOR its
// IV window and key stream at its packet offset x = 8 + 16 col (do_obscure +
// encrypt_0, packet.cpp:77-91, 32-39; the CRC and tail are k_cook's), the
// other pieces plain into the output.  The parity slots are not written.
typedef uint32_t bs_u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
struct CookIO {
    DevIO io;
    __amdgpu_buffer_rsrc_t orsrc;  // the output, same geometry as io.rsrc
    const EpiRec *rbase;           // records of the wave's first group's first slot (uniform)
    uint32_t u0, u1;               // the pieces' (group - first group) << 16 | column
    const uint8_t *ks;
    uint32_t tag, n;
    __device__ __forceinline__ void load(int j, uint32_t (&p)[8]) const { io.load(j, p); }
    // Branch-free (a branch here, even a uniform one, splits the store phase
    // and the network spills 200+ VGPRs at 3 waves/SIMD): a record of another run
    // (a parity slot no packet of this run sends) reads as a plain piece into
    // the output, where nothing reads it; its window index is clamped into
    // the record.
    __device__ __forceinline__ void piece(uint32_t u, uint32_t voff, int j, bs_u32x4 v) const {
        BS_SCHED_BARRIER();  // (the record loads stay at their row)
        const EpiRec *r = rbase + (u >> 16) * n + j;
        const uint32_t x = 8u + 16u * (u & 0xFFFFu);
        const bs_u32x4 h = *reinterpret_cast<const bs_u32x4 *>(r);
        const uint32_t len = h.y & 0xFFFFu, ivl = h.y >> 16;
        uint32_t rr = x - __umulhi(x, h.z) * ivl;
        rr = (rr >= ivl ? rr - ivl : rr) & 31u;
        const uint32_t *w = r->iv + (rr >> 2);
        const bs_u32x4 a = *reinterpret_cast<const bs_u32x4_a4 *>(w);
        const uint32_t a4 = w[4], sh = rr & 3u;
        const bool whole = h.x == tag && x + 16u <= len;
        const uint32_t wm = (whole && ivl) ? ~0u : 0u;  // (iv_len 0: no obscure stage)
        bs_u32x4 m = bs_u32x4{__builtin_amdgcn_alignbyte(a.y, a.x, sh), __builtin_amdgcn_alignbyte(a.z, a.y, sh),
                              __builtin_amdgcn_alignbyte(a.w, a.z, sh), __builtin_amdgcn_alignbyte(a4, a.w, sh)} &
                     bs_u32x4{wm, wm, wm, wm};
        {  // (ks: the key stream, or zeros without an XOR stage -- no branch here)
            const uint32_t km = whole ? ~0u : 0u;
            m ^= *reinterpret_cast<const bs_u32x4_a4 *>(ks + (whole ? x : 8u)) & bs_u32x4{km, km, km, km};
        }
        __builtin_amdgcn_raw_buffer_store_b128(v ^ m, orsrc, voff + j * io.ss, 0, BS_ST_AUX);
    }
    __device__ __forceinline__ void store(int j, const uint32_t (&q)[8]) const {
        piece(u0, io.v0, j, bs_u32x4{q[0], q[1], q[2], q[3]});
        piece(u1, io.v1, j, bs_u32x4{q[4], q[5], q[6], q[7]});
    }
};

__device__ __forceinline__ CookIO bs_make_cook_io(uint8_t *base0, int64_t group_stride, int64_t shard_stride,
                                                  uint32_t cols, uint32_t P, uint32_t wave, const CookEpi &e) {
    CookIO c;
    c.io = bs_make_io(base0, group_stride, shard_stride, cols, P, wave);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t cfirst = wave * 128u;
    const uint32_t clast = (cfirst + 127u < cols) ? cfirst + 127u : cols - 1u;
    const uint32_t gfirst = cfirst / P, glast = clast / P;
    c.orsrc = __builtin_amdgcn_make_buffer_rsrc(e.out + (int64_t)gfirst * group_stride, 0,
                                                (int)((glast - gfirst + 1u) * (uint32_t)group_stride), 0x00020000);
    const uint32_t c0 = cfirst + lane, c1 = c0 + 64u;
    const uint32_t g0 = c0 / P, g1 = c1 / P;
    // (a lane past the last column reads the first group's records, and its
    // column 0xFFFF makes no piece whole; its stores are dropped by the range
    // check)
    c.rbase = e.rec + (int64_t)gfirst * e.n;
    c.u0 = c0 < cols ? (g0 - gfirst) << 16 | (c0 - g0 * P) : 0xFFFFu;
    c.u1 = c1 < cols ? (g1 - gfirst) << 16 | (c1 - g1 * P) : 0xFFFFu;
    c.n = e.n;
    c.ks = e.ks;
    c.tag = e.tag;
    return c;
}

#if BS_COOK_EPI
#define BS_SPLIT_COOK_KERNEL(K, N)                                                                  \
    __global__ __launch_bounds__(128, BS_COOK_OCC) void k_bs2c_##K##_##N(                           \
        uint8_t *base, int64_t group_stride, int64_t shard_stride, uint32_t cols, uint32_t P,       \
        CookEpi e) {                                                                                \
        __shared__ bs_u32x4 xch[2][2 * 5][64];                                                      \
        const uint32_t bid = BS_XCD ? (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)      \
                                    : blockIdx.x;                                                   \
        if (bid * 128u >= cols) return;                                                             \
        const uint32_t h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);                        \
        CookIO io = bs_make_cook_io(base, group_stride, shard_stride, cols, P, bid, e);             \
        BsXch x{xch[h], xch[h ^ 1u]};                                                               \
        bs_split_##K##_##N(io, h, x);                                                               \
    }
BS_FOR_EACH_SPLIT(BS_SPLIT_COOK_KERNEL)
#undef BS_SPLIT_COOK_KERNEL
#endif

}  // namespace

namespace {
// Columns per group and the batch's columns of a uniform launch (false: the
// descriptor geometry does not fit): the rule of bitslice.hip's
// launch_encode_bitslice, which the plain split-k encoders use -- whole
// 128-B lines when the slot has room (rsmi.h padding rule).
bool bs_geometry(const UniformArgs &a, int64_t &P, int64_t &cols) {
    P = (a.len + 15) / 16;
    const int64_t P128 = (a.len + 127) / 128 * 8;
    if (P128 * 16 <= a.shard_stride) P = P128;
    cols = a.ngroups * P;
    if (P == 0 || cols == 0) return true;
    // a wave spans <= 128/P + 2 groups, all 32-bit offsets
    const int64_t span = (128 / P + 2) * a.group_stride;
    return !(cols >= (int64_t(1) << 31) || a.shard_stride < P * 16 || span >= (int64_t(1) << 31) ||
             a.group_stride < a.n * a.shard_stride);
}

bool has_split(int k, int n) {
    switch (k * 257 + n) {
#define BS_CASE(K, N) case K * 257 + N: return true;
        BS_FOR_EACH_SPLIT(BS_CASE)
#undef BS_CASE
        default: return false;
    }
}
}  // namespace

bool bitslice_cooked_ok(const UniformArgs &a) {
    int64_t P, cols;
    return BS_COOK_EPI && BS_SPLIT && has_split(a.k, a.n) && bs_geometry(a, P, cols) &&
           (cols + 127) / 128 + 7 <= 0x7fffffff;
}

hipError_t launch_encode_bitslice_cooked(const UniformArgs &a, const CookEpi &e, hipStream_t s) {
    int64_t P, cols;
    if (!bitslice_cooked_ok(a) || !bs_geometry(a, P, cols)) return hipErrorNotSupported;
    if (P == 0 || cols == 0) return hipSuccess;
    int64_t sblocks = (cols + 127) / 128;
    if (BS_XCD) sblocks = (sblocks + 7) & ~int64_t(7);
    uint8_t *base = a.base;
    int64_t gs = a.group_stride, ss = a.shard_stride;
    uint32_t ucols = (uint32_t)cols, uP = (uint32_t)P;
    switch (a.k * 257 + a.n) {
#if BS_COOK_EPI
#define BS_LAUNCH2C(K, N)                                                                  \
    case K * 257 + N:                                                                      \
        k_bs2c_##K##_##N<<<(unsigned)sblocks, 128, 0, s>>>(base, gs, ss, ucols, uP, e);    \
        return hipGetLastError();
        BS_FOR_EACH_SPLIT(BS_LAUNCH2C)
#undef BS_LAUNCH2C
#endif
        default: return hipErrorNotSupported;
    }
}

}  // namespace rsmi
