// dec_probe.hip -- measurement tool: access-pattern ceilings for the fused decode
// (one wave per group, 20 survivor rows of a 1280-B slot read, E rows written),
// with no arithmetic.  Variants:
//   dx4+d   per survivor one 1-KiB dwordx4 wave-load + one 256-B dword wave-load
//   packed  per 4 survivors four 1-KiB dwordx4 loads + one dwordx4 load carrying
//           the four 256-B tails (lane l: survivor l/16, bytes 1024 + 16 (l%16))
//   glds    survivors staged into a per-wave LDS ring by buffer_load ... lds
// Build: hipcc --offload-arch=gfx950 -O3 -o dec_probe dec_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t G = 65536, N = 30, S = 1280, K = 20;

template <int RING, int E, int OCC, int AUX>
__global__ __launch_bounds__(256, OCC) void p_dx4d(uint8_t *base) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t g = blockIdx.x * 4u + wid; g < G; g += gridDim.x * 4u) {
        auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base + (uint64_t)g * N * S, 0, (int)(N * S), 0x00020000);
        const uint32_t v16 = lane * 16, v4 = 1024 + lane * 4, o = (g & 7) * S;
        u32x4 rq[RING];
        uint32_t rd[RING];
#pragma unroll
        for (int q = 0; q < RING; ++q) {
            rq[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v16, o + q * S, AUX);
            rd[q] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, v4, o + q * S, AUX);
        }
        u32x4 acc = {0, 0, 0, 0};
        uint32_t accd = 0;
        for (int jb = 0; jb < (int)K; jb += RING) {
#pragma unroll
            for (int q = 0; q < RING; ++q) {
                const int j = jb + q;
                acc ^= rq[q];
                accd ^= rd[q];
                if (j + RING < (int)K) {
                    rq[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v16, o + (j + RING) * S, AUX);
                    rd[q] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, v4, o + (j + RING) * S, AUX);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < E; ++r) {
            __builtin_amdgcn_raw_buffer_store_b128(acc + r, rsrc, v16, r * S, 0);
            __builtin_amdgcn_raw_buffer_store_b32(accd + r, rsrc, v4, r * S, 0);
        }
    }
}

// RING blocks of 4 survivors in flight (5 dwordx4 loads per block)
template <int RING, int E, int OCC, int AUX>
__global__ __launch_bounds__(256, OCC) void p_packed(uint8_t *base) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t g = blockIdx.x * 4u + wid; g < G; g += gridDim.x * 4u) {
        auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base + (uint64_t)g * N * S, 0, (int)(N * S), 0x00020000);
        const uint32_t v16 = lane * 16, o = (g & 7) * S;
        const uint32_t vt = (lane >> 4) * S + 1024 + (lane & 15) * 16;
        u32x4 rq[RING][5];
#pragma unroll
        for (int q = 0; q < RING; ++q) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                rq[q][i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v16, o + (4 * q + i) * S, AUX);
            rq[q][4] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, vt, o + 4 * q * S, AUX);
        }
        u32x4 acc = {0, 0, 0, 0}, acct = {0, 0, 0, 0};
        for (int jb = 0; jb < (int)K / 4; jb += RING) {
#pragma unroll
            for (int q = 0; q < RING; ++q) {
                const int j = jb + q;
                acc ^= rq[q][0] ^ rq[q][1] ^ rq[q][2] ^ rq[q][3];
                acct ^= rq[q][4];
                if (j + RING < (int)K / 4) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        rq[q][i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v16, o + (4 * (j + RING) + i) * S, AUX);
                    rq[q][4] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, vt, o + 4 * (j + RING) * S, AUX);
                }
            }
        }
        const uint32_t vw = 1024 + (lane & 15) * 16;
#pragma unroll
        for (int r = 0; r < E; ++r) {
            __builtin_amdgcn_raw_buffer_store_b128(acc + r, rsrc, v16, r * S, 0);
            if (lane < 16) __builtin_amdgcn_raw_buffer_store_b128(acct + r, rsrc, vw, r * S, 0);
        }
    }
}

// survivors staged in a per-wave LDS ring of RING 1280-B tiles
template <int RING, int E, int AUX>
__global__ __launch_bounds__(256) void p_glds(uint8_t *base) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *ring = smem + wid * RING * S;
    for (uint32_t g = blockIdx.x * 4u + wid; g < G; g += gridDim.x * 4u) {
        auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base + (uint64_t)g * N * S, 0, (int)(N * S), 0x00020000);
        const uint32_t v16 = lane * 16, v4 = 1024 + lane * 4, o = (g & 7) * S;
#pragma unroll
        for (int q = 0; q < RING; ++q) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(ring + q * S), 16, v16, o + q * S, 0, AUX);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(ring + q * S + 1024), 4, v4, o + q * S, 0, AUX);
        }
        u32x4 acc = {0, 0, 0, 0};
        uint32_t accd = 0;
        for (int jb = 0; jb < (int)K; jb += RING) {
#pragma unroll
            for (int q = 0; q < RING; ++q) {
                const int j = jb + q;
                // the oldest tile has landed once at most 2 (RING - 1) DMAs are pending
                __builtin_amdgcn_s_waitcnt(0x3F70 | ((2 * (RING - 1)) & 15) | (((2 * (RING - 1)) >> 4) << 14));
                const u32x4 x = *reinterpret_cast<const u32x4 *>(ring + q * S + lane * 16);
                const uint32_t xd = *reinterpret_cast<const uint32_t *>(ring + q * S + 1024 + lane * 4);
                acc ^= x;
                accd ^= xd;
                __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the tile is read before refill
                if (j + RING < (int)K) {
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(ring + q * S), 16, v16, o + (j + RING) * S, 0, AUX);
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void *)(ring + q * S + 1024), 4, v4, o + (j + RING) * S, 0, AUX);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < E; ++r) {
            __builtin_amdgcn_raw_buffer_store_b128(acc + r, rsrc, v16, r * S, 0);
            __builtin_amdgcn_raw_buffer_store_b32(accd + r, rsrc, v4, r * S, 0);
        }
    }
}

template <class F>
float time_ms(F f, int reps = 20) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    std::vector<float> v;
    for (int i = 0; i < reps + 3; ++i) {
        hipEventRecord(a);
        f();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (i >= 3) v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    const size_t bytes = (size_t)G * N * S;
    uint8_t *buf;
    hipMalloc(&buf, bytes);
    hipMemset(buf, 1, bytes);
    auto run = [&](const char *name, auto kern, int grid, int e, size_t lds = 0) {
        const double alg = (double)G * (K + e) * 1250;
        float ms = time_ms([&] { kern<<<grid, 256, lds>>>(buf); });
        printf("%-34s %.4f ms  %.0f GB/s alg\n", name, ms, alg / ms / 1e6);
    };
    run("dx4d ring4 occ4 g2048 E3", p_dx4d<4, 3, 4, 0>, 2048, 3);
    run("dx4d ring4 occ4 g2048 E3 nt", p_dx4d<4, 3, 4, 2>, 2048, 3);
    run("dx4d ring4 occ4 g4096 E3", p_dx4d<4, 3, 4, 0>, 4096, 3);
    run("dx4d ring4 occ4 g1024 E3", p_dx4d<4, 3, 4, 0>, 1024, 3);
    run("dx4d ring6 occ4 g2048 E3", p_dx4d<6, 3, 4, 0>, 2048, 3);
    run("dx4d ring2 occ8 g4096 E3", p_dx4d<2, 3, 8, 0>, 4096, 3);
    run("packed ring1 occ4 g2048 E3", p_packed<1, 3, 4, 0>, 2048, 3);
    run("packed ring2 occ4 g2048 E3", p_packed<2, 3, 4, 0>, 2048, 3);
    run("packed ring1 occ8 g4096 E3", p_packed<1, 3, 8, 0>, 4096, 3);
    run("dx4d ring6 occ4 g2048 E3 nt", p_dx4d<6, 3, 4, 2>, 2048, 3);
    run("dx4d ring8 occ3 g2048 E3 nt", p_dx4d<8, 3, 3, 2>, 2048, 3);
    run("dx4d ring2 occ8 g4096 E3 nt", p_dx4d<2, 3, 8, 2>, 4096, 3);
    run("packed ring2 occ4 g2048 E3 nt", p_packed<2, 3, 4, 2>, 2048, 3);
    run("packed ring1 occ4 g2048 E3 nt", p_packed<1, 3, 4, 2>, 2048, 3);
    run("glds ring8 g2048 E3 nt", p_glds<8, 3, 2>, 2048, 3, 4 * 8 * S);
    run("glds ring4 g2048 E3", p_glds<4, 3, 0>, 2048, 3, 4 * 4 * S);
    run("glds ring8 g2048 E3", p_glds<8, 3, 0>, 2048, 3, 4 * 8 * S);
    run("glds ring8 g1024 E3", p_glds<8, 3, 0>, 1024, 3, 4 * 8 * S);
    run("glds ring10 g2048 E3", p_glds<10, 3, 0>, 2048, 3, 4 * 10 * S);
    run("glds ring4 g4096 E3", p_glds<4, 3, 0>, 4096, 3, 4 * 4 * S);
    hipFree(buf);
    return 0;
}
