// bitslice_kern.hpp -- device side of the bit-sliced RS encoders, shared by the
// build-time kernels (bitslice.hip, networks from gen/bitslice_codes.inc) and
// the kernels compiled at run time for every other code (bitslice_rtc.cpp hands
// this text, bitslice_core.hpp and the emitted network to hipRTC).  It has no
// #include of its own: the includer provides uint8_t/uint32_t/uint64_t/int64_t.
//
// Layout: a "column" is one 16-byte piece of a shard row, P = ceil(len/16)
// columns per group (rounded up to whole 128-B lines when the slot has room);
// the batch is a flat space of G*P columns.  Wave w owns columns
// [128w, 128w+128): lane l loads piece c0 = 128w+l and c1 = c0+64 of every
// data shard (two fully coalesced 1 KiB dwordx4 wave-loads per shard), i.e.
// 32 bytes -> 8 dwords -> 8 bit-planes.  Lanes of one wave may belong to
// different groups: the network is the same for every group of the code.
#pragma once

// Accumulator updates go through the v_bitop3 builtin.  Plain `acc ^= a ^ b`
// chains get reassociated by LLVM into one tree per accumulator at the end of
// the kernel (every intermediate combination stays live: hundreds of spilled
// VGPRs); the builtin keeps each update in its shard block.  (Inline-asm
// accumulators were tried and produced intermittently wrong parity under
// load -- the compiler's hazard/wait bookkeeping does not see inside asm.)
#ifndef BS_OCC
#define BS_OCC 3  // waves per SIMD the register budget is sized for (<= 10 parity rows per pass)
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
#ifndef BS_XCD
#define BS_XCD 1  // blocks b, b+8, ... (dispatched to one XCD) take one contiguous range of
                  // chunks (measured 1.5 % faster than the plain order, scripts/archive/gpu_bench_ab.sh)
#endif
#ifndef BS_RAG_XCD
#define BS_RAG_XCD 0  // 1: the same remap for the ragged kernels, so the blocks one CU holds come
                      // from one narrow window of the code-sorted wave list (one code's network
                      // of the ~550 KB in k_bs_ragged).  Measured 10 % slower on C3: each XCD
                      // then owns one slice of the codes and the slice of the largest ones
                      // finishes last (scripts/gpu_ab.sh c3)
#endif
#define BS_ACC3(acc, a, b) ((acc) = __builtin_amdgcn_bitop3_b32((acc), (a), (b), 0x96))
#define BS_ACC2(acc, a) ((acc) ^= (a))
// keep the generated shard blocks in order so the raw-load ring bounds the
// registers in flight (the scheduler would otherwise hoist every load)
#define BS_SCHED_BARRIER() __builtin_amdgcn_sched_barrier(0)

typedef uint32_t bs_u32x4 __attribute__((ext_vector_type(4)));

// Same layout as rsmi_group (include/rsmi.h); bitslice.hip static_asserts it.
struct BsGroup {
    uint64_t offset;
    uint32_t shard_stride, len;
    uint16_t k, n;
    uint32_t reserved;
};

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
        const bs_u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v0, j * ss, BS_LD_AUX);
        const bs_u32x4 y = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v1, j * ss, BS_LD_AUX);
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
        const bs_u32x4 x = {q[0], q[1], q[2], q[3]};
        const bs_u32x4 y = {q[4], q[5], q[6], q[7]};
#if BS_ST_SGPR
        __builtin_amdgcn_raw_buffer_store_b128(x, rsrc, v0, j * ss, BS_ST_AUX);
        __builtin_amdgcn_raw_buffer_store_b128(y, rsrc, v1, j * ss, BS_ST_AUX);
#else
        __builtin_amdgcn_raw_buffer_store_b128(x, rsrc, v0 + j * ss, 0, BS_ST_AUX);
        __builtin_amdgcn_raw_buffer_store_b128(y, rsrc, v1 + j * ss, 0, BS_ST_AUX);
#endif
    }
};

__device__ __forceinline__ DevIO bs_make_io(uint8_t *base0, int64_t group_stride,
                                            int64_t shard_stride, uint32_t cols, uint32_t P,
                                            uint32_t wave) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t cfirst = wave * 128u;
    const uint32_t clast = (cfirst + 127u < cols) ? cfirst + 127u : cols - 1u;
    const uint32_t gfirst = cfirst / P, glast = clast / P;
    const uint32_t gs = (uint32_t)group_stride;
    uint8_t *base = base0 + (int64_t)gfirst * group_stride;
    const uint32_t bytes = (glast - gfirst + 1u) * gs;
    DevIO io;
    io.rsrc = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
    const uint32_t c0 = cfirst + lane, c1 = c0 + 64u;
    const uint32_t g0 = c0 / P, g1 = c1 / P;
    io.v0 = c0 < cols ? (g0 - gfirst) * gs + (c0 - g0 * P) * 16u : 0x80000000u;
    io.v1 = c1 < cols ? (g1 - gfirst) * gs + (c1 - g1 * P) * 16u : 0x80000000u;
    io.ss = (uint32_t)shard_stride;
    return io;
}

// Uniform batch kernel for one network FN.  A wave encodes 128-column chunks
// w, w + wstep, ...: the launch sizes the grid so every resident wave gets the
// same number of chunks.  Waves past the end exit before touching memory.
#define BS_DEFINE_UNIFORM(NAME, FN, OCC)                                                       \
    __global__ __launch_bounds__(256, OCC) void NAME(uint8_t *base, int64_t group_stride,     \
                                                        int64_t shard_stride, uint32_t cols,     \
                                                        uint32_t P, uint32_t wstep) {            \
        const uint32_t bid = BS_XCD ? (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)   \
                                    : blockIdx.x;                                                \
        for (uint32_t wave = bid * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);         \
             wave * 128u < cols; wave += wstep) {                                                \
            DevIO io = bs_make_io(base, group_stride, shard_stride, cols, P, wave);               \
            FN(io);                                                                              \
        }                                                                                        \
        if (BS_FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");                         \
    }

// ---- ragged batches: one launch over (k,n) buckets -------------------------
// The host plan (ragged.cpp) sorts groups into buckets by code and lays each
// bucket's 16-B columns out consecutively, padded to whole waves.  colmap[c]
// = (group << 12) | piece for a real column, ~0u for padding; every wave's
// 128 columns belong to one bucket (waves[2w..2w+1] = {code index, first
// column}).  Lanes resolve their own group's offset and shard stride, so one
// wave can mix groups of different lengths; the shard stride varies per lane
// and goes into the per-lane voffset instead of soffset.
#ifndef BS_RAG_LD_AUX
#define BS_RAG_LD_AUX 2  // cache-policy bits of the ragged kernels' loads: nt (round 5: C3 encode
                         // 0.167-0.169 vs 0.176-0.178 ms default; nt stores as well 0.182-0.183)
#endif
#ifndef BS_RAG_ST_AUX
#define BS_RAG_ST_AUX 0  // ... and of their parity stores
#endif
struct RagIO {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t o0, o1, ss0, ss1;
    __device__ __forceinline__ void load(int j, uint32_t (&p)[8]) const {
        const bs_u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o0 + j * ss0, 0, BS_RAG_LD_AUX);
        const bs_u32x4 y = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o1 + j * ss1, 0, BS_RAG_LD_AUX);
        p[0] = x.x; p[1] = x.y; p[2] = x.z; p[3] = x.w;
        p[4] = y.x; p[5] = y.y; p[6] = y.z; p[7] = y.w;
    }
    __device__ __forceinline__ void store(int j, const uint32_t (&q)[8]) const {
        const bs_u32x4 x = {q[0], q[1], q[2], q[3]};
        const bs_u32x4 y = {q[4], q[5], q[6], q[7]};
        __builtin_amdgcn_raw_buffer_store_b128(x, rsrc, o0 + j * ss0, 0, BS_RAG_ST_AUX);
        __builtin_amdgcn_raw_buffer_store_b128(y, rsrc, o1 + j * ss1, 0, BS_RAG_ST_AUX);
    }
};

__device__ __forceinline__ void bs_rag_lane(const BsGroup *groups, uint32_t m, uint32_t &off,
                                            uint32_t &ss) {
    if (m == 0xFFFFFFFFu) {
        off = 0x80000000u;  // out of range: loads read 0, stores dropped
        ss = 0;
        return;
    }
    const BsGroup d = groups[m >> 12];
    off = (uint32_t)d.offset + (m & 4095u) * 16u;
    ss = d.shard_stride;
}

// Sets up `io` and `code` (the wave's bucket code index) for ragged wave w;
// returns false for waves past the end.
__device__ __forceinline__ bool bs_rag_setup(const BsGroup *groups, const uint32_t *colmap,
                                             const uint32_t *waves, uint32_t nwaves,
                                             uint8_t *base, uint32_t bytes, RagIO &io,
                                             uint32_t &code) {
    const uint32_t bid = BS_RAG_XCD ? (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)
                                    : blockIdx.x;
    const uint32_t w = bid * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (w >= nwaves) return false;
    code = __builtin_amdgcn_readfirstlane(waves[2 * w]);
    const uint32_t c0 = __builtin_amdgcn_readfirstlane(waves[2 * w + 1]) + (threadIdx.x & 63u);
    io.rsrc = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
    bs_rag_lane(groups, colmap[c0], io.o0, io.ss0);
    bs_rag_lane(groups, colmap[c0 + 64], io.o1, io.ss1);
    return true;
}

// Ragged kernel for the waves of ONE code's bucket (runtime-compiled codes:
// the host launches it over that bucket's slice of the wave list).
#define BS_DEFINE_RAGGED_ONE(NAME, FN, OCC)                                                     \
    __global__ __launch_bounds__(256, OCC) void NAME(const BsGroup *groups,                   \
                                                        const uint32_t *colmap,                  \
                                                        const uint32_t *waves, uint32_t nwaves,  \
                                                        uint8_t *base, uint32_t bytes) {         \
        RagIO io;                                                                                \
        uint32_t code;                                                                           \
        if (!bs_rag_setup(groups, colmap, waves, nwaves, base, bytes, io, code)) return;         \
        FN(io);                                                                                  \
    }

#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
// ---- split-k form (gen_bitslice.py emit_split) --------------------------------
// A 2-wave workgroup per 128-column chunk: wave h reads half of the data
// shards, the two waves swap the partial sums of each other's parity rows
// through LDS, and each stores half of the rows.  Partials go out as two
// 16-byte writes per lane per row (a wave writes 1 KiB contiguous per
// instruction: conflict-free).
struct BsXch {
    bs_u32x4 (*out)[64];
    const bs_u32x4 (*in)[64];
    __device__ __forceinline__ void send(int r, uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3,
                                         uint32_t a4, uint32_t a5, uint32_t a6, uint32_t a7) const {
        const uint32_t lane = threadIdx.x & 63u;
        out[2 * r][lane] = bs_u32x4{a0, a1, a2, a3};
        out[2 * r + 1][lane] = bs_u32x4{a4, a5, a6, a7};
    }
    __device__ __forceinline__ void sync() const { __syncthreads(); }
    __device__ __forceinline__ void recv(int r, uint32_t &a0, uint32_t &a1, uint32_t &a2, uint32_t &a3,
                                         uint32_t &a4, uint32_t &a5, uint32_t &a6, uint32_t &a7) const {
        const uint32_t lane = threadIdx.x & 63u;
        const bs_u32x4 x = in[2 * r][lane], y = in[2 * r + 1][lane];
        a0 ^= x.x; a1 ^= x.y; a2 ^= x.z; a3 ^= x.w;
        a4 ^= y.x; a5 ^= y.y; a6 ^= y.z; a7 ^= y.w;
    }
};

// Block b (XCD-contiguous order as BS_DEFINE_UNIFORM) = chunk b; both waves of
// a block leave together past the last chunk, so the barrier always pairs up.
#define BS_DEFINE_SPLIT(NAME, FN, OCC)                                                           \
    __global__ __launch_bounds__(128, OCC) void NAME(uint8_t *base, int64_t group_stride,       \
                                                        int64_t shard_stride, uint32_t cols,     \
                                                        uint32_t P) {                            \
        __shared__ bs_u32x4 xch[2][2 * 5][64];                                                   \
        const uint32_t bid = BS_XCD ? (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)   \
                                    : blockIdx.x;                                                \
        if (bid * 128u >= cols) return;                                                          \
        const uint32_t h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);                     \
        DevIO io = bs_make_io(base, group_stride, shard_stride, cols, P, bid);                  \
        BsXch x{xch[h], xch[h ^ 1u]};                                                            \
        FN(io, h, x);                                                                            \
    }
#endif
