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
#ifndef BS_RAG_SPLIT
#define BS_RAG_SPLIT 0  // 1: ragged plans run the buckets of split-k codes in the 2-wave form
                        // (k_bs_ragged_split).  Round 6 (profiles/r06/ragsplit/): C3 encode
                        // 0.177 ms against 0.166 one wave per record -- both waves repeat the
                        // record's column-map and group loads, and the exchange adds a barrier
                        // per chunk, which the uniform C1 launch (one descriptor) does not pay
#endif
#ifndef BS_COOK_EPI
#define BS_COOK_EPI 1  // build the cooking split-k encoders (k_bs2c_*, RSMI_OPT_PARITY_COOK)
#endif
#ifndef BS_COOK_OCC
#define BS_COOK_OCC BS_OCC  // waves per SIMD of the cooking encoders
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

// ---- the same split-k networks with the parity cook in the epilogue ----------
// (rsmi_internal.hpp EpiRec; RSMI_OPT_PARITY_COOK).  Row j's two pieces of a
// lane belong to packet slot g*n + j of the run (g: the piece's group).  A
// piece wholly inside its packet's payload is stored into the output XOR its
// IV window and key stream at its packet offset x = 8 + 16 col (do_obscure +
// encrypt_0, packet.cpp:77-91, 32-39; the CRC and tail are k_cook's), the
// other pieces plain into the output; a slot without this run's record keeps
// the plain store into the slot.
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

// Position of (k, n) in the generated code list (compile time).
constexpr int bs_code_idx(int k, int n) {
    int i = 0;
#define BS_IDX_C(K, N)                  \
    if (k == K && n == N) return i;     \
    ++i;
    BS_FOR_EACH_CODE(BS_IDX_C)
#undef BS_IDX_C
    return -1;
}
#define BS_SPLIT_IN_LIST(K, N) static_assert(bs_code_idx(K, N) >= 0, "split code without a one-wave network");
BS_FOR_EACH_SPLIT(BS_SPLIT_IN_LIST)
#undef BS_SPLIT_IN_LIST

#if BS_RAG_SPLIT
// Ragged launch with the split-k form for the buckets that have one (BS_RAG_SPLIT):
// 2-wave blocks; block b < nsplit runs wave record b split-k (the two waves
// share its 128 columns, half the data shards each, as k_bs2_*), the blocks
// after it run two one-wave records each (no barrier there).  The plan lists
// the split buckets' records first.
__global__ __launch_bounds__(128, BS_OCC) void k_bs_ragged_split(const BsGroup *groups, const uint32_t *colmap,
                                                                 const uint32_t *waves, uint32_t nsplit,
                                                                 uint32_t nwaves, uint8_t *base, uint32_t bytes) {
    __shared__ bs_u32x4 xch[2][2 * 5][64];
    const uint32_t b = blockIdx.x;
    const uint32_t h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t w = b < nsplit ? b : nsplit + 2u * (b - nsplit) + h;
    if (w >= nwaves) return;  // (a one-wave block's second wave only: no barrier follows)
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t code = __builtin_amdgcn_readfirstlane(waves[2 * w]);
    const uint32_t c0 = __builtin_amdgcn_readfirstlane(waves[2 * w + 1]) + lane;
    RagIO io;
    io.rsrc = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
    bs_rag_lane(groups, colmap[c0], io.o0, io.ss0);
    bs_rag_lane(groups, colmap[c0 + 64], io.o1, io.ss1);
    if (b < nsplit) {
        BsXch x{xch[h], xch[h ^ 1u]};
        switch (code) {
#define BS_RAG_SPLIT_CASE(K, N)                  \
    case (uint32_t)bs_code_idx(K, N):            \
        bs_split_##K##_##N(io, h, x);            \
        return;
            BS_FOR_EACH_SPLIT(BS_RAG_SPLIT_CASE)
#undef BS_RAG_SPLIT_CASE
            default: return;
        }
    }
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
#endif

}  // namespace

bool bitslice_has_split(int k, int n) {
    switch (k * 257 + n) {
#define BS_CASE(K, N) case K * 257 + N: return BS_RAG_SPLIT != 0;
        BS_FOR_EACH_SPLIT(BS_CASE)
#undef BS_CASE
        default: return false;
    }
}

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
                                         uint32_t bytes, hipStream_t s, uint32_t nsplit) {
    if (nwaves == 0) return hipSuccess;
#if BS_RAG_SPLIT
    if (nsplit > 0) {
        const uint32_t blocks = nsplit + (nwaves - nsplit + 1) / 2;
        k_bs_ragged_split<<<blocks, 128, 0, s>>>(reinterpret_cast<const BsGroup *>(groups), colmap, waves,
                                                 nsplit, nwaves, base, bytes);
        return hipGetLastError();
    }
#else
    (void)nsplit;
#endif
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

namespace {
// Columns per group and the batch's columns of a uniform launch (false: the
// descriptor geometry does not fit).  Whole 128-B lines when the slot has room
// (measured ~10 % faster than stopping at the last 16-B piece: rows and wave
// boundaries then fall on cache-line boundaries); see rsmi.h padding rule.
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

// Built-in network if the code has one, else the runtime-compiled one once it
// is ready; hipErrorNotSupported otherwise (the caller runs the generic kernel).
hipError_t launch_encode_bitslice(const UniformArgs &a, hipStream_t s) {
    hipFunction_t rtc = nullptr;
    if (!has_bitslice(a.k, a.n)) {
        rtc = bitslice_rtc_function(a.k, a.n, kRtcUniform);
        if (!rtc) return hipErrorNotSupported;
    }
    int64_t P, cols;
    const bool fits = bs_geometry(a, P, cols);
    if (P == 0 || cols == 0) return hipSuccess;
    if (!fits) return hipErrorNotSupported;
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
