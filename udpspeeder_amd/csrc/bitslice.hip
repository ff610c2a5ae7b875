// bitslice.hip -- bit-sliced RS encode kernels, specialised at build time for
// the hot (k,n) codes (gen_bitslice.py -> gen/bitslice_codes.inc), and the
// launchers that also serve the codes compiled at run time (bitslice_rtc.cpp).
//
// The XOR network replaces k*m GF multiply-accumulates per byte with ~3 XOR
// ops per input byte (v_bitop3_b32), bit-exact by construction.  Device IO and
// the kernel bodies live in bitslice_kern.hpp (shared with hipRTC).
#include "rsmi_internal.hpp"

#include "bitslice_core.hpp"
#include "bitslice_kern.hpp"

#ifndef BS_SPLIT
#define BS_SPLIT 1  // uniform launches of codes with a split-k network use the 2-wave form
#endif
#ifndef BS_PERSIST
#define BS_PERSIST 0  // 1: balanced persistent grid (measured 5 % slower than one wave per chunk)
#endif
#ifndef BS_RAG_PERSIST
#define BS_RAG_PERSIST 0  // k_bs_ragged: persistent waves (blocks per CU) that load the next chunk's
                          // wave record and column map during this chunk's network.  Round 6
                          // (profiles/r06/c3_persist_ab.txt): 3 blocks/CU 0.175-0.178 ms, 6 blocks/CU
                          // 0.175-0.176, against 0.166-0.167 one wave per chunk (the carried words
                          // spill 20 VGPRs at 3 waves/SIMD)
#endif
#ifdef BS_INC
#include BS_INC
#else
#include "gen/bitslice_codes.inc"
#endif

static_assert(sizeof(BsGroup) == sizeof(rsmi_group) &&
                  offsetof(BsGroup, shard_stride) == offsetof(rsmi_group, shard_stride) &&
                  offsetof(BsGroup, len) == offsetof(rsmi_group, len) &&
                  offsetof(BsGroup, k) == offsetof(rsmi_group, k),
              "BsGroup must mirror rsmi_group");

namespace rsmi {
namespace {

#define BS_KERNEL(K, N) BS_DEFINE_UNIFORM(k_bs_##K##_##N, bs_code_##K##_##N, BS_OCC)
BS_FOR_EACH_CODE(BS_KERNEL)
#undef BS_KERNEL

// ---- split-k form: BsXch and BS_DEFINE_SPLIT in bitslice_kern.hpp ----------
#define BS_SPLIT_KERNEL(K, N) BS_DEFINE_SPLIT(k_bs2_##K##_##N, bs_split_##K##_##N, BS_OCC)
BS_FOR_EACH_SPLIT(BS_SPLIT_KERNEL)
#undef BS_SPLIT_KERNEL

// One launch over every bucket of the built-in codes (code = index in the
// generated list).
__global__ __launch_bounds__(256, BS_OCC) void k_bs_ragged(const BsGroup *groups,
                                                           const uint32_t *colmap,
                                                           const uint32_t *waves, uint32_t nwaves,
                                                           uint8_t *base, uint32_t bytes) {
#if BS_RAG_PERSIST
    // wave w's chunks w, w + wstep, ...: the next chunk's wave record and
    // column-map words load while this chunk's network runs, so only the
    // group-record load stays in front of each chunk
    const uint32_t wstep = gridDim.x * 4u;
    uint32_t w = blockIdx.x * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (w >= nwaves) return;
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t code = __builtin_amdgcn_readfirstlane(waves[2 * w]);
    uint32_t c0 = __builtin_amdgcn_readfirstlane(waves[2 * w + 1]) + lane;
    uint32_t m0 = colmap[c0], m1 = colmap[c0 + 64];
    for (;;) {
        RagIO io;
        io.rsrc = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
        bs_rag_lane(groups, m0, io.o0, io.ss0);
        bs_rag_lane(groups, m1, io.o1, io.ss1);
        const uint32_t wn = w + wstep;
        const bool more = wn < nwaves;
        uint32_t coden = 0, m0n = 0xFFFFFFFFu, m1n = 0xFFFFFFFFu;
        if (more) {
            coden = __builtin_amdgcn_readfirstlane(waves[2 * wn]);
            const uint32_t cn = __builtin_amdgcn_readfirstlane(waves[2 * wn + 1]) + lane;
            m0n = colmap[cn];
            m1n = colmap[cn + 64];
        }
        int idx = 0;
#define BS_RAG_CASE(K, N)              \
    if (code == (uint32_t)idx) bs_code_##K##_##N(io); \
    ++idx;
        BS_FOR_EACH_CODE(BS_RAG_CASE)
#undef BS_RAG_CASE
        if (!more) break;
        w = wn;
        code = coden;
        m0 = m0n;
        m1 = m1n;
    }
#else
    RagIO io;
    uint32_t code;
    if (!bs_rag_setup(groups, colmap, waves, nwaves, base, bytes, io, code)) return;
    int idx = 0;
#define BS_RAG_CASE(K, N)              \
    if (code == (uint32_t)idx) {       \
        bs_code_##K##_##N(io);         \
        return;                        \
    }                                  \
    ++idx;
    BS_FOR_EACH_CODE(BS_RAG_CASE)
#undef BS_RAG_CASE
#endif
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

int bitslice_builtin_count() { return BS_NUM_CODES; }

int bitslice_code_k(int i) {
    int idx = 0;
#define BS_K(K, N)                   \
    if (i == idx) return K;          \
    ++idx;
    BS_FOR_EACH_CODE(BS_K)
#undef BS_K
    return 0;
}

int bitslice_code_n(int i) {
    int idx = 0;
#define BS_N(K, N)                   \
    if (i == idx) return N;          \
    ++idx;
    BS_FOR_EACH_CODE(BS_N)
#undef BS_N
    return 0;
}

hipError_t launch_encode_bitslice_ragged(const rsmi_group *groups, const uint32_t *colmap,
                                         const uint32_t *waves, uint32_t nwaves, uint8_t *base,
                                         uint32_t bytes, hipStream_t s) {
    if (nwaves == 0) return hipSuccess;
    uint32_t blocks = (nwaves + 3) / 4;
    if (BS_RAG_XCD) blocks = (blocks + 7) & ~7u;  // whole rounds of 8 XCDs (the remap)
    if (BS_RAG_PERSIST && blocks > 256u * BS_RAG_PERSIST) blocks = 256u * BS_RAG_PERSIST;
    k_bs_ragged<<<blocks, 256, 0, s>>>(reinterpret_cast<const BsGroup *>(groups), colmap, waves,
                                       nwaves, base, bytes);
    return hipGetLastError();
}

hipError_t launch_encode_bitslice_ragged_rtc(int k, int n, const rsmi_group *groups,
                                             const uint32_t *colmap, const uint32_t *waves,
                                             uint32_t nwaves, uint8_t *base, uint32_t bytes,
                                             hipStream_t s) {
    if (nwaves == 0) return hipSuccess;
    hipFunction_t f = bitslice_rtc_function(k, n, kRtcRagged);
    if (!f) return hipErrorNotSupported;
    const BsGroup *g = reinterpret_cast<const BsGroup *>(groups);
    void *args[] = {&g, &colmap, &waves, &nwaves, &base, &bytes};
    uint32_t blocks = (nwaves + 3) / 4;
    if (BS_RAG_XCD) blocks = (blocks + 7) & ~7u;
    return hipModuleLaunchKernel(f, blocks, 1, 1, 256, 1, 1, 0, s, args, nullptr);
}

bool has_bitslice(int k, int n) {
    switch (k * 257 + n) {
#define BS_CASE(K, N) case K * 257 + N: return true;
        BS_FOR_EACH_CODE(BS_CASE)
#undef BS_CASE
        default: return false;
    }
}

// Built-in network if the code has one, else the runtime-compiled one once it
// is ready; hipErrorNotSupported otherwise (the caller runs the generic kernel).
hipError_t launch_encode_bitslice(const UniformArgs &a, hipStream_t s) {
    hipFunction_t rtc = nullptr;
    if (!has_bitslice(a.k, a.n)) {
        rtc = bitslice_rtc_function(a.k, a.n, kRtcUniform);
        if (!rtc) return hipErrorNotSupported;
    }
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
#ifdef BS_CPW
    waves = (chunks + BS_CPW - 1) / BS_CPW;  // measurement knob: chunks per wave
#endif
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
    int64_t blocks = (waves + 3) / 4;
    if (BS_XCD) blocks = (blocks + 7) & ~int64_t(7);  // the remap needs whole rounds of 8 XCDs
    if (blocks > 0x7fffffff) return hipErrorNotSupported;
    uint8_t *base = a.base;
    int64_t gs = a.group_stride, ss = a.shard_stride;
    uint32_t ucols = (uint32_t)cols, uP = (uint32_t)P, wstep = (uint32_t)(blocks * 4);
    if (BS_SPLIT && rtc) {
        hipFunction_t f2 = bitslice_rtc_function(a.k, a.n, kRtcSplit);
        if (f2) {
            int64_t sblocks = chunks;
            if (BS_XCD) sblocks = (sblocks + 7) & ~int64_t(7);
            if (sblocks > 0x7fffffff) return hipErrorNotSupported;
            void *args[] = {&base, &gs, &ss, &ucols, &uP};
            return hipModuleLaunchKernel(f2, (unsigned)sblocks, 1, 1, 128, 1, 1, 0, s, args, nullptr);
        }
    }
    if (BS_SPLIT && !rtc) {
        // one 2-wave block per chunk
        int64_t sblocks = chunks;
        if (BS_XCD) sblocks = (sblocks + 7) & ~int64_t(7);
        if (sblocks > 0x7fffffff) return hipErrorNotSupported;
        switch (a.k * 257 + a.n) {
#define BS_LAUNCH2(K, N)                                                                 \
    case K * 257 + N:                                                                    \
        k_bs2_##K##_##N<<<(unsigned)sblocks, 128, 0, s>>>(base, gs, ss, ucols, uP);      \
        return hipGetLastError();
            BS_FOR_EACH_SPLIT(BS_LAUNCH2)
#undef BS_LAUNCH2
            default: break;
        }
    }
    if (rtc) {
        void *args[] = {&base, &gs, &ss, &ucols, &uP, &wstep};
        return hipModuleLaunchKernel(rtc, (unsigned)blocks, 1, 1, 256, 1, 1, 0, s, args, nullptr);
    }
    switch (a.k * 257 + a.n) {
#define BS_LAUNCH(K, N)                                                                  \
    case K * 257 + N:                                                                    \
        k_bs_##K##_##N<<<(unsigned)blocks, 256, 0, s>>>(base, gs, ss, ucols, uP, wstep); \
        return hipGetLastError();
        BS_FOR_EACH_CODE(BS_LAUNCH)
#undef BS_LAUNCH
        default: return hipErrorNotSupported;
    }
}

}  // namespace rsmi
