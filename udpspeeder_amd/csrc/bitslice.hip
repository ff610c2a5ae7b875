// bitslice.hip -- bit-sliced RS encode kernels, specialised at build time for
// the hot (k,n) codes (gen_bitslice.py -> gen/bitslice_codes.inc).
//
// Layout: a "column" is one 16-byte piece of a shard row, P = ceil(len/16)
// columns per group; the batch is a flat space of G*P columns.  Wave w owns
// columns [128w, 128w+128): lane l loads piece c0 = 128w+l and c1 = c0+64 of
// every data shard (two fully coalesced 1 KiB dwordx4 wave-loads per shard),
// i.e. 32 bytes -> 8 dwords -> 8 bit-planes.  Lanes of one wave may belong
// to different groups: the network is the same for every group of the code.
// The XOR network replaces k*m GF multiply-accumulates per byte with ~3 XOR
// ops per input byte (v_bitop3_b32), bit-exact by construction.
#include "rsmi_internal.hpp"

#include "bitslice_core.hpp"

// Accumulator updates go through the v_bitop3 builtin.  Plain `acc ^= a ^ b`
// chains get reassociated by LLVM into one tree per accumulator at the end of
// the kernel (every intermediate combination stays live: hundreds of spilled
// VGPRs); the builtin keeps each update in its shard block.  (Inline-asm
// accumulators were tried and produced intermittently wrong parity under
// load -- the compiler's hazard/wait bookkeeping does not see inside asm.)
#ifndef BS_OCC
#define BS_OCC 3
#endif
#ifndef BS_PERSIST
#define BS_PERSIST 0  // 1: balanced persistent grid (measured 5 % slower than one wave per chunk)
#endif
#ifndef BS_FENCE
#define BS_FENCE 0  // agent-scope release at the end of every wave
#endif
#ifndef BS_LD_AUX
#define BS_LD_AUX 2  // cache-policy bits of the streaming loads (2 = nt: read once)
#endif
#ifndef BS_ST_AUX
#define BS_ST_AUX 2  // cache-policy bits of the parity stores (2 = nt)
#endif
#ifndef BS_ST_SGPR
#define BS_ST_SGPR 0  // 1: shard offset of the parity stores in soffset (the round-1 form: wrong
                      // parity dwords under co-resident load, see DevIO::store)
#endif
#define BS_ACC3(acc, a, b) ((acc) = __builtin_amdgcn_bitop3_b32((acc), (a), (b), 0x96))
#define BS_ACC2(acc, a) ((acc) ^= (a))
// keep the generated shard blocks in order so the raw-load ring bounds the
// registers in flight (the scheduler would otherwise hoist every load)
#define BS_SCHED_BARRIER() __builtin_amdgcn_sched_barrier(0)
#ifdef BS_INC
#include BS_INC
#else
#include "gen/bitslice_codes.inc"
#endif

namespace rsmi {
namespace {

// Buffer-descriptor IO: one wave-uniform descriptor per wave covering the
// (at most a few) groups its 128 columns touch; per lane only two 32-bit
// voffsets, the shard offset j*shard_stride goes in the scalar soffset.
// Lanes past the last column get an out-of-range voffset: their loads
// return 0 and their stores are dropped by the hardware range check.
struct DevIO {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t v0, v1;
    uint32_t ss;
    __device__ __forceinline__ void load(int j, uint32_t (&p)[8]) const {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v0, j * ss, BS_LD_AUX);
        const u32x4 y = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v1, j * ss, BS_LD_AUX);
        p[0] = x.x; p[1] = x.y; p[2] = x.z; p[3] = x.w;
        p[4] = y.x; p[5] = y.y; p[6] = y.z; p[7] = y.w;
    }
    // Stores keep the whole offset in the VGPR (soffset 0).  LLVM's hazard
    // recognizer (GCNHazardRecognizer::createsVALUHazard) exempts MUBUF stores
    // with a register soffset from the "store of > 64 bits, then a VALU write
    // of its data VGPRs" wait state, and the register allocator reuses the
    // first data VGPR of the second store in the very next VALU instruction.
    // On gfx950 the store then sometimes sent the NEW value of that VGPR for
    // lanes 12-15 of each 16 (wrong first dwords of 16-B pieces at 192..255
    // mod 256) once another kernel's waves shared the CU: DESIGN.md §4.
    __device__ __forceinline__ void store(int j, const uint32_t (&q)[8]) const {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 x = {q[0], q[1], q[2], q[3]};
        const u32x4 y = {q[4], q[5], q[6], q[7]};
#if BS_ST_SGPR
        __builtin_amdgcn_raw_buffer_store_b128(x, rsrc, v0, j * ss, BS_ST_AUX);
        __builtin_amdgcn_raw_buffer_store_b128(y, rsrc, v1, j * ss, BS_ST_AUX);
#else
        __builtin_amdgcn_raw_buffer_store_b128(x, rsrc, v0 + j * ss, 0, BS_ST_AUX);
        __builtin_amdgcn_raw_buffer_store_b128(y, rsrc, v1 + j * ss, 0, BS_ST_AUX);
#endif
    }
};

__device__ __forceinline__ DevIO make_io(const UniformArgs &a, uint32_t cols, uint32_t P,
                                         uint32_t wave) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t cfirst = wave * 128u;
    const uint32_t clast = (cfirst + 127u < cols) ? cfirst + 127u : cols - 1u;
    const uint32_t gfirst = cfirst / P, glast = clast / P;
    const uint32_t gs = (uint32_t)a.group_stride;
    const uint8_t *base = a.base + (int64_t)gfirst * a.group_stride;
    const uint32_t bytes = (glast - gfirst + 1u) * gs;
    DevIO io;
    io.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base), 0, (int)bytes,
                                                0x00020000);
    const uint32_t c0 = cfirst + lane, c1 = c0 + 64u;
    const uint32_t g0 = c0 / P, g1 = c1 / P;
    io.v0 = c0 < cols ? (g0 - gfirst) * gs + (c0 - g0 * P) * 16u : 0x80000000u;
    io.v1 = c1 < cols ? (g1 - gfirst) * gs + (c1 - g1 * P) * 16u : 0x80000000u;
    io.ss = (uint32_t)a.shard_stride;
    return io;
}

// A wave encodes 128-column chunks w, w + wstep, ...: the launch sizes the grid
// so every resident wave gets the same number of chunks (no partly filled last
// round of waves).  Waves past the end exit before touching memory.
#define BS_KERNEL(K, N)                                                                   \
    __global__ __launch_bounds__(256, BS_OCC) void k_bs_##K##_##N(UniformArgs a, uint32_t cols,     \
                                                          uint32_t P, uint32_t wstep) {    \
        for (uint32_t wave = blockIdx.x * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); \
             wave * 128u < cols; wave += wstep) {                                          \
            DevIO io = make_io(a, cols, P, wave);                                         \
            bs_code_##K##_##N(io);                                                        \
        }                                                                                 \
        if (BS_FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");                  \
    }
BS_FOR_EACH_CODE(BS_KERNEL)
#undef BS_KERNEL

// ---- ragged batches: one launch over (k,n) buckets -------------------------
// The host plan (ragged.cpp) sorts groups into buckets by code and lays each
// bucket's 16-B columns out consecutively, padded to whole waves.  colmap[c]
// = (group << 12) | piece for a real column, ~0u for padding; every wave's
// 128 columns belong to one bucket (waves[w] = {code index, first column}).
// Lanes resolve their own group's offset and shard stride, so one wave can
// mix groups of different lengths; the shard stride varies per lane and goes
// into the per-lane voffset instead of soffset.
struct RagIO {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t o0, o1, ss0, ss1;
    __device__ __forceinline__ void load(int j, uint32_t (&p)[8]) const {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o0 + j * ss0, 0, 0);
        const u32x4 y = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o1 + j * ss1, 0, 0);
        p[0] = x.x; p[1] = x.y; p[2] = x.z; p[3] = x.w;
        p[4] = y.x; p[5] = y.y; p[6] = y.z; p[7] = y.w;
    }
    __device__ __forceinline__ void store(int j, const uint32_t (&q)[8]) const {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 x = {q[0], q[1], q[2], q[3]};
        const u32x4 y = {q[4], q[5], q[6], q[7]};
        __builtin_amdgcn_raw_buffer_store_b128(x, rsrc, o0 + j * ss0, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(y, rsrc, o1 + j * ss1, 0, 0);
    }
};

__device__ __forceinline__ void rag_lane(const rsmi_group *groups, uint32_t m, uint32_t &off,
                                         uint32_t &ss) {
    if (m == 0xFFFFFFFFu) {
        off = 0x80000000u;  // out of range: loads read 0, stores dropped
        ss = 0;
        return;
    }
    const rsmi_group d = groups[m >> 12];
    off = (uint32_t)d.offset + (m & 4095u) * 16u;
    ss = d.shard_stride;
}

__global__ __launch_bounds__(256, BS_OCC) void k_bs_ragged(const rsmi_group *groups,
                                                           const uint32_t *colmap,
                                                           const uint2 *waves, uint32_t nwaves,
                                                           uint8_t *base, uint32_t bytes) {
    const uint32_t w = blockIdx.x * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (w >= nwaves) return;
    const uint2 wr = waves[w];  // {code index, first column}
    const uint32_t code = __builtin_amdgcn_readfirstlane(wr.x);
    const uint32_t c0 = __builtin_amdgcn_readfirstlane(wr.y) + (threadIdx.x & 63u);
    RagIO io;
    io.rsrc = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
    rag_lane(groups, colmap[c0], io.o0, io.ss0);
    rag_lane(groups, colmap[c0 + 64], io.o1, io.ss1);
    int idx = 0;
#define BS_RAG_CASE(K, N)              \
    if (code == (uint32_t)idx) {       \
        bs_code_##K##_##N(io);         \
        return;                        \
    }                                  \
    ++idx;
    BS_FOR_EACH_CODE(BS_RAG_CASE)
#undef BS_RAG_CASE
}

}  // namespace

int bitslice_code_index(int k, int n) {
    int idx = 0;
#define BS_IDX(K, N)                    \
    if (k == K && n == N) return idx;   \
    ++idx;
    BS_FOR_EACH_CODE(BS_IDX)
#undef BS_IDX
    return -1;
}

hipError_t launch_encode_bitslice_ragged(const rsmi_group *groups, const uint32_t *colmap,
                                         const uint32_t *waves, uint32_t nwaves, uint8_t *base,
                                         uint32_t bytes, hipStream_t s) {
    if (nwaves == 0) return hipSuccess;
    const uint32_t blocks = (nwaves + 3) / 4;
    k_bs_ragged<<<blocks, 256, 0, s>>>(groups, colmap, reinterpret_cast<const uint2 *>(waves),
                                       nwaves, base, bytes);
    return hipGetLastError();
}

bool has_bitslice(int k, int n) {
    switch (k * 257 + n) {
#define BS_CASE(K, N) case K * 257 + N: return true;
        BS_FOR_EACH_CODE(BS_CASE)
#undef BS_CASE
        default: return false;
    }
}

hipError_t launch_encode_bitslice(const UniformArgs &a, hipStream_t s) {
    // Columns per group: whole 128-B lines when the slot has room (measured
    // ~10 % faster than stopping at the last 16-B piece: rows and wave
    // boundaries then fall on cache-line boundaries); see rsmi.h padding rule.
    int64_t P = (a.len + 15) / 16;
    const int64_t P128 = (a.len + 127) / 128 * 8;
    if (P128 * 16 <= a.shard_stride) P = P128;
    const int64_t cols = a.ngroups * P;
    if (P == 0 || cols == 0) return hipSuccess;
    // descriptor geometry: a wave spans <= 128/P + 2 groups, all 32-bit offsets
    const int64_t span = (128 / P + 2) * a.group_stride;
    if (cols >= (int64_t(1) << 31) || a.shard_stride < P * 16 || span >= (int64_t(1) << 31) ||
        a.group_stride < a.n * a.shard_stride)
        return hipErrorNotSupported;
    const int64_t chunks = (cols + 127) / 128;
    int64_t waves = chunks;
#if BS_PERSIST
    // balanced persistent grid: every resident wave slot takes ceil(chunks /
    // slots) chunks, and only as many waves run as that needs
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
    }
    const int64_t slots = (int64_t)cus * 4 * BS_OCC;
    const int64_t per = (chunks + slots - 1) / slots;
    waves = (chunks + per - 1) / per;
#endif
    const int64_t blocks = (waves + 3) / 4;
    if (blocks > 0x7fffffff) return hipErrorNotSupported;
    const uint32_t wstep = (uint32_t)(blocks * 4);
    switch (a.k * 257 + a.n) {
#define BS_LAUNCH(K, N)                                                                 \
    case K * 257 + N:                                                                   \
        k_bs_##K##_##N<<<(unsigned)blocks, 256, 0, s>>>(a, (uint32_t)cols, (uint32_t)P, wstep); \
        return hipGetLastError();
        BS_FOR_EACH_CODE(BS_LAUNCH)
#undef BS_LAUNCH
        default: return hipErrorNotSupported;
    }
}

}  // namespace rsmi
