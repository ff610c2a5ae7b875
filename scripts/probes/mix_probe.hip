// mix_probe.hip -- measurement tool: the HBM ceiling of a 2:1 read:write
// stream (the RS(20,10) encode's byte mix) in several shapes, with no
// arithmetic.  Not product code.  Build: hipcc -O3 --offload-arch=gfx950
//
//  flat    : src and dst are separate regions; wave c reads 2U KiB at src+2cU
//            and writes U KiB at dst+cU (one wave per chunk).
//  inplace : the encode's layout, [G][30][1280]; one wave per 128-column chunk
//            reads 20 shard rows and writes 10 (P = 80 pieces per shard),
//            XCD-contiguous block order as k_bs_20_30.
//  split   : data [G][20][1280] and parity [G][10][1280] in two regions,
//            same wave shape as inplace.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, int LD, int ST>
__global__ __launch_bounds__(256) void flat(uint8_t *src, uint8_t *dst, uint32_t chunks) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t c = blockIdx.x * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (c >= chunks) return;
    auto rs = __builtin_amdgcn_make_buffer_rsrc(src + (uint64_t)c * 2 * U * 1024, 0, 2 * U * 1024, 0x00020000);
    auto rd = __builtin_amdgcn_make_buffer_rsrc(dst + (uint64_t)c * U * 1024, 0, U * 1024, 0x00020000);
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, u * 1024, LD) ^
               __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, (U + u) * 1024, LD);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, lane * 16 + u * 1024, 0, ST);
}

// one wave per 128 columns of G*80; rows 0..19 read, 20..29 written.
// PSTRIDE/PGS locate the parity rows: in place (same base, rows 20..29) or split.
template <int RING, int LD, int ST, bool XCD>
__global__ __launch_bounds__(256, 3) void shaped(uint8_t *dbase, uint8_t *pbase, uint32_t cols,
                                                 uint32_t dgs, uint32_t pgs, uint32_t poff, uint32_t wstep) {
    const uint32_t bid = XCD ? (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  for (uint32_t wave = bid * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); wave * 128u < cols; wave += wstep) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t P = 80;
    const uint32_t cfirst = wave * 128u, gfirst = cfirst / P;
    auto rs = __builtin_amdgcn_make_buffer_rsrc(dbase + (uint64_t)gfirst * dgs, 0, 4 * dgs, 0x00020000);
    auto rp = __builtin_amdgcn_make_buffer_rsrc(pbase + (uint64_t)gfirst * pgs, 0, 4 * pgs, 0x00020000);
    uint32_t c0 = cfirst + lane, c1 = c0 + 64;
    uint32_t g0 = c0 / P, g1 = c1 / P;
    uint32_t d0 = c0 < cols ? (g0 - gfirst) * dgs + (c0 - g0 * P) * 16 : 0x80000000u;
    uint32_t d1 = c1 < cols ? (g1 - gfirst) * dgs + (c1 - g1 * P) * 16 : 0x80000000u;
    uint32_t p0 = c0 < cols ? (g0 - gfirst) * pgs + poff + (c0 - g0 * P) * 16 : 0x80000000u;
    uint32_t p1 = c1 < cols ? (g1 - gfirst) * pgs + poff + (c1 - g1 * P) * 16 : 0x80000000u;
    u32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    u32x4 r0[RING], r1[RING];
#pragma unroll
    for (int q = 0; q < RING; ++q) {
        r0[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, d0 + q * 1280, 0, LD);
        r1[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, d1 + q * 1280, 0, LD);
    }
#pragma unroll
    for (int j = 0; j < 20; ++j) {
        const int q = j % RING;
        acc0 ^= r0[q];
        acc1 ^= r1[q];
        if (j + RING < 20) {
            r0[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, d0 + (j + RING) * 1280, 0, LD);
            r1[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, d1 + (j + RING) * 1280, 0, LD);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        __builtin_amdgcn_raw_buffer_store_b128(acc0 + i, rp, p0 + i * 1280, 0, ST);
        __builtin_amdgcn_raw_buffer_store_b128(acc1 + i, rp, p1 + i * 1280, 0, ST);
    }
  }
}


// HALF = 1: one wave per 64 columns (each lane one 16-B piece): half the
// footprint per wave.  SPLITK = 1: two waves per 128 columns, wave h reads data
// rows 10h..10h+9 and writes parity rows 20+5h..20+5h+4.
template <int HALF, int SPLITK, int NS = 2>
__global__ __launch_bounds__(256, 3) void shaped2(uint8_t *dbase, uint32_t cols, uint32_t dgs) {
    const uint32_t bid = (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const uint32_t w = bid * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t cpw = HALF ? 64u : 128u;
    const uint32_t wave = SPLITK ? w / NS : w, h = SPLITK ? (w % NS) : 0u;
    if (wave * cpw >= cols) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t P = 80;
    const uint32_t cfirst = wave * cpw, gfirst = cfirst / P;
    auto rs = __builtin_amdgcn_make_buffer_rsrc(dbase + (uint64_t)gfirst * dgs, 0, 4 * dgs, 0x00020000);
    uint32_t c0 = cfirst + lane, c1 = c0 + 64;
    uint32_t g0 = c0 / P, g1 = c1 / P;
    uint32_t d0 = c0 < cols ? (g0 - gfirst) * dgs + (c0 - g0 * P) * 16 : 0x80000000u;
    uint32_t d1 = (!HALF && c1 < cols) ? (g1 - gfirst) * dgs + (c1 - g1 * P) * 16 : 0x80000000u;
    const int J = SPLITK ? 20 / NS : 20, I = SPLITK ? (NS == 4 ? (h < 2 ? 3 : 2) : 5) : 10;
    const uint32_t jo = h * (20 / NS) * 1280, io = 20 * 1280 + (NS == 4 ? (h < 2 ? 3 * h : 6 + 2 * (h - 2)) : h * 5) * 1280;
    u32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    u32x4 r0[4], r1[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        r0[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, d0 + jo + q * 1280, 0, 2);
        if (!HALF) r1[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, d1 + jo + q * 1280, 0, 2);
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
        const int q = j % 4;
        acc0 ^= r0[q];
        if (!HALF) acc1 ^= r1[q];
        if (j + 4 < J) {
            r0[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, d0 + jo + (j + 4) * 1280, 0, 2);
            if (!HALF) r1[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, d1 + jo + (j + 4) * 1280, 0, 2);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < I; ++i) {
        __builtin_amdgcn_raw_buffer_store_b128(acc0 + i, rs, d0 + io + i * 1280, 0, 2);
        if (!HALF) __builtin_amdgcn_raw_buffer_store_b128(acc1 + i, rs, d1 + io + i * 1280, 0, 2);
    }
}

template <class F>
float time_ms(F f, int reps = 30) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    std::vector<float> v;
    for (int i = 0; i < reps + 5; ++i) {
        hipEventRecord(a);
        f();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (i >= 5) v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    const uint32_t G = 65536;
    const size_t bytes = (size_t)G * 30 * 1280;  // 2.52 GB: the encode's footprint
    uint8_t *buf, *buf2;
    hipMalloc(&buf, bytes);
    hipMalloc(&buf2, bytes);
    hipMemset(buf, 1, bytes);
    hipMemset(buf2, 1, bytes);
    // settle clocks
    for (int i = 0; i < 200; ++i) flat<2, 2, 2><<<(bytes / 3 / 2048 + 3) / 4, 256>>>(buf, buf2, bytes / 3 / 2048);
    hipDeviceSynchronize();
    const double moved = (double)bytes;
    auto report = [&](const char *name, float ms) {
        printf("%-34s %.4f ms  %.0f GB/s moved  (%.3f of 8 TB/s; encode-equivalent alg frac %.3f)\n", name,
               ms, moved / ms / 1e6, moved / ms / 8e9 * 1e3, moved / ms / 8e9 * 1e3 / 1.024);
    };
#define FLAT(U, LD, ST)                                                                      \
    {                                                                                        \
        const uint32_t ch = (uint32_t)(bytes / 3 / (U * 1024));                              \
        float ms = time_ms([&] { flat<U, LD, ST><<<(ch + 3) / 4, 256>>>(buf, buf2, ch); });  \
        report("flat U" #U " ld" #LD " st" #ST, ms);                                         \
    }
    FLAT(2, 2, 2) FLAT(4, 2, 2) FLAT(8, 2, 2) FLAT(2, 0, 0) FLAT(4, 0, 0) FLAT(4, 2, 0) FLAT(4, 0, 2)
    FLAT(4, 3, 3) FLAT(4, 2, 18)
    const uint32_t cols = G * 80, waves = (cols + 127) / 128, blocks = ((waves + 3) / 4 + 7) & ~7u;
#define SHAPEDC(NAME, RING, LD, ST, XCD, PB, PGS, POFF, COLS, CPW)                                \
    {                                                                                              \
        const uint32_t wv = ((COLS) / 128 + (CPW) - 1) / (CPW);                                    \
        const uint32_t bl = ((wv + 3) / 4 + 7) & ~7u;                                              \
        float ms = time_ms([&] {                                                                   \
            shaped<RING, LD, ST, XCD><<<bl, 256>>>(buf, PB, COLS, DGS, PGS, POFF, bl * 4);         \
        });                                                                                        \
        printf("[cols %u cpw %d waves %u] ", (unsigned)(COLS), (int)(CPW), wv);                   \
        report(NAME, ms * (double)cols / (COLS));                                                  \
    }
#define SHAPED(NAME, RING, LD, ST, XCD, PB, PGS, POFF) SHAPEDC(NAME, RING, LD, ST, XCD, PB, PGS, POFF, cols, 1)
    {
        const uint32_t DGS = 30 * 1280;
        SHAPED("inplace ring4 nt xcd", 4, 2, 2, true, buf, 30 * 1280, 20 * 1280)
        SHAPED("inplace ring4 nt", 4, 2, 2, false, buf, 30 * 1280, 20 * 1280)
        SHAPED("inplace ring8 nt xcd", 8, 2, 2, true, buf, 30 * 1280, 20 * 1280)
        SHAPED("inplace ring4 ld-nt st-def xcd", 4, 2, 0, true, buf, 30 * 1280, 20 * 1280)
        // per-wave chunk counts: 2, 4, 14 (persistent: 2926 waves)
        SHAPEDC("inplace cpw2", 4, 2, 2, true, buf, 30 * 1280, 20 * 1280, cols, 2)
        SHAPEDC("inplace cpw4", 4, 2, 2, true, buf, 30 * 1280, 20 * 1280, cols, 4)
        SHAPEDC("inplace cpw14", 4, 2, 2, true, buf, 30 * 1280, 20 * 1280, cols, 14)
        // tail: exactly 13 and 12 rounds of 3072 wave slots (time scaled to 65536 groups);
        // COLS must stay <= G * 80: the buffer holds G groups
        {
            const uint32_t wv = cols / 64, bl = ((wv + 3) / 4 + 7) & ~7u;
            report("inplace half-footprint (64 col)", time_ms([&] { shaped2<1, 0><<<bl, 256>>>(buf, cols, DGS); }));
            const uint32_t wv2 = cols / 128 * 2, bl2 = ((wv2 + 3) / 4 + 7) & ~7u;
            report("inplace split-k (2 waves/128 col)", time_ms([&] { shaped2<0, 1><<<bl2, 256>>>(buf, cols, DGS); }));
            const uint32_t wv4 = cols / 128 * 4, bl4 = ((wv4 + 3) / 4 + 7) & ~7u;
            report("inplace split-4 (4 waves/128 col)", time_ms([&] { shaped2<0, 1, 4><<<bl4, 256>>>(buf, cols, DGS); }));
            report("inplace ring4 nt xcd (again)", time_ms([&] { shaped<4, 2, 2, true><<<blocks, 256>>>(buf, buf, cols, DGS, 30 * 1280, 20 * 1280, blocks * 4); }));
        }
        SHAPEDC("inplace 13 rounds", 4, 2, 2, true, buf, 30 * 1280, 20 * 1280, 3072u * 13 * 128, 1)
        SHAPEDC("inplace 12 rounds", 4, 2, 2, true, buf, 30 * 1280, 20 * 1280, 3072u * 12 * 128, 1)
    }
    {
        const uint32_t DGS = 20 * 1280;
        SHAPED("split ring4 nt xcd", 4, 2, 2, true, buf2, 10 * 1280, 0)
        SHAPED("split ring8 nt xcd", 8, 2, 2, true, buf2, 10 * 1280, 0)
        SHAPED("split ring4 ld-nt st-def xcd", 4, 2, 0, true, buf2, 10 * 1280, 0)
    }
    hipFree(buf);
    hipFree(buf2);
    return 0;
}
