// dec2_probe.hip -- measurement tool: memory-pattern ceilings for decode-shaped
// work (20 of 30 rows of a 1280-B slot group read, E rows written), with no
// arithmetic, in several wave->data mappings.  G = 65536 groups of 30 x 1280 B.
//   row    one wave per group, per survivor a 1-KiB dwordx4 + a 256-B dword
//          wave-load (the round-1 fused decode), RING survivors in flight
//   quad   one wave per group, all loads dwordx4: lane l holds survivor
//          4i + l/16, bytes 256t + 16(l%16) (5 loads per 4 survivors)
//   col    encode-like: a wave owns C 16-B columns of the flat group x piece
//          space (lanes of one wave may hold different groups), reads 20 rows
//          and writes E rows per column (C = 64: 1 load per row, 128: 2)
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/dec2_probe dec2_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t G = 65536, N = 30, S = 1280, K = 20, P = 80;

template <int RING, int E, int OCC, int AUX>
__global__ __launch_bounds__(256, OCC) void p_row(uint8_t *base) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t g = blockIdx.x * 4u + wid; g < G; g += gridDim.x * 4u) {
        auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base + (uint64_t)g * N * S, 0, (int)(N * S),
                                                      0x00020000);
        const uint32_t v16 = lane * 16, v4 = 1024 + lane * 4, o = (g & 7) * S;
        u32x4 rq[RING];
        uint32_t rd[RING];
#pragma unroll
        for (int q = 0; q < RING; ++q) {
            rq[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v16 + o + q * S, 0, AUX);
            rd[q] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, v4 + o + q * S, 0, AUX);
        }
        u32x4 acc = {0, 0, 0, 0};
        uint32_t accd = 0;
        for (int jb = 0; jb < (int)K; jb += RING) {
#pragma unroll
            for (int q = 0; q < RING; ++q) {
                const int j = jb + q;
                if (j < (int)K) {
                    acc ^= rq[q];
                    accd ^= rd[q];
                    if (j + RING < (int)K) {
                        rq[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v16 + o + (j + RING) * S, 0, AUX);
                        rd[q] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, v4 + o + (j + RING) * S, 0, AUX);
                    }
                }
            }
        }
#pragma unroll
        for (int r = 0; r < E; ++r) {
            __builtin_amdgcn_raw_buffer_store_b128(acc + r, rsrc, v16 + r * S, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b32(accd + r, rsrc, v4 + r * S, 0, 0);
        }
    }
}

// quads of survivors: load t of quad q: lane l reads survivor 4q + l/16 at 256t + 16(l%16)
template <int RING, int E, int OCC, int AUX>
__global__ __launch_bounds__(256, OCC) void p_quad(uint8_t *base) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int Q = K / 4;
    for (uint32_t g = blockIdx.x * 4u + wid; g < G; g += gridDim.x * 4u) {
        auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base + (uint64_t)g * N * S, 0, (int)(N * S),
                                                      0x00020000);
        const uint32_t o = (g & 7) * S;
        const uint32_t vl = (lane >> 4) * S + (lane & 15) * 16 + o;
        u32x4 rq[RING][5];
#pragma unroll
        for (int q = 0; q < RING; ++q)
#pragma unroll
            for (int t = 0; t < 5; ++t)
                rq[q][t] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, vl + 4 * q * S + 256 * t, 0, AUX);
        u32x4 acc[5] = {};
        for (int qb = 0; qb < Q; qb += RING) {
#pragma unroll
            for (int q = 0; q < RING; ++q) {
                const int j = qb + q;
                if (j < Q) {
#pragma unroll
                    for (int t = 0; t < 5; ++t) acc[t] ^= rq[q][t];
                    if (j + RING < Q) {
#pragma unroll
                        for (int t = 0; t < 5; ++t)
                            rq[q][t] = __builtin_amdgcn_raw_buffer_load_b128(
                                rsrc, vl + 4 * (j + RING) * S + 256 * t, 0, AUX);
                    }
                }
            }
        }
        // rows r: lanes of group l/16 == r % 4 store their 256-B pieces
#pragma unroll
        for (int r = 0; r < E; ++r)
#pragma unroll
            for (int t = 0; t < 5; ++t)
                if ((int)(lane >> 4) == (r & 3))
                    __builtin_amdgcn_raw_buffer_store_b128(acc[t] + r, rsrc,
                                                           r * S + 256 * t + (lane & 15) * 16, 0, 0);
    }
}

// encode-like column mapping: wave w owns columns [C w, C w + C)
template <int C, int RING, int E, int OCC, int AUX>
__global__ __launch_bounds__(256, OCC) void p_col(uint8_t *base) {
    constexpr int L = C / 64;  // loads per row
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t cols = G * P;
    for (uint32_t wave = blockIdx.x * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
         wave * C < cols; wave += gridDim.x * 4u) {
        const uint32_t cfirst = wave * C, gfirst = cfirst / P, glast = (cfirst + C - 1) / P;
        auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base + (uint64_t)gfirst * N * S, 0,
                                                      (int)((glast - gfirst + 1) * N * S), 0x00020000);
        uint32_t v[L], w[L];
#pragma unroll
        for (int l = 0; l < L; ++l) {
            const uint32_t c = cfirst + lane + 64 * l, g = c / P;
            w[l] = (g - gfirst) * N * S + (c - g * P) * 16;
            v[l] = w[l] + (g & 7) * S;
        }
        u32x4 r[RING][L];
#pragma unroll
        for (int q = 0; q < RING; ++q)
#pragma unroll
            for (int l = 0; l < L; ++l)
                r[q][l] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v[l] + q * S, 0, AUX);
        u32x4 acc[L] = {};
#pragma unroll
        for (int j = 0; j < (int)K; ++j) {
#pragma unroll
            for (int l = 0; l < L; ++l) {
                acc[l] ^= r[j % RING][l];
                if (j + RING < (int)K)
                    r[j % RING][l] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v[l] + (j + RING) * S, 0, AUX);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int e = 0; e < E; ++e)
#pragma unroll
            for (int l = 0; l < L; ++l)
                __builtin_amdgcn_raw_buffer_store_b128(acc[l] + e, rsrc, w[l] + e * S, 0, 0);
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
    if (hipMalloc(&buf, bytes) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    auto run = [&](const char *name, auto kern, int grid, int e) {
        const double alg = (double)G * (K + e) * 1250;  // the decode's algorithmic bytes
        float ms = time_ms([&] { kern<<<grid, 256>>>(buf); });
        printf("%-36s %.4f ms  %6.0f GB/s alg  frac %.3f\n", name, ms, alg / ms / 1e6,
               alg / ms / 1e6 / 8000.0);
    };
    const int gc64 = (G * P / 64 + 3) / 4, gc128 = (G * P / 128 + 3) / 4;
    run("row ring4 occ4 E3", p_row<4, 3, 4, 0>, 2048, 3);
    run("row ring4 occ4 E3 nt", p_row<4, 3, 4, 2>, 2048, 3);
    run("row ring8 occ2 E3 nt", p_row<8, 3, 2, 2>, 2048, 3);
    run("row ring4 occ4 E3 nt g4096", p_row<4, 3, 4, 2>, 4096, 3);
    run("quad ring1 occ4 E3", p_quad<1, 3, 4, 0>, 2048, 3);
    run("quad ring1 occ4 E3 nt", p_quad<1, 3, 4, 2>, 2048, 3);
    run("quad ring2 occ3 E3 nt", p_quad<2, 3, 3, 2>, 2048, 3);
    run("quad ring2 occ2 E3 nt", p_quad<2, 3, 2, 2>, 2048, 3);
    run("col64 ring4 occ4 E3 nt", p_col<64, 4, 3, 4, 2>, gc64, 3);
    run("col64 ring8 occ4 E3 nt", p_col<64, 8, 3, 4, 2>, gc64, 3);
    run("col128 ring4 occ3 E3 nt", p_col<128, 4, 3, 3, 2>, gc128, 3);
    run("col128 ring4 occ3 E3", p_col<128, 4, 3, 3, 0>, gc128, 3);
    run("col128 ring6 occ2 E3 nt", p_col<128, 6, 3, 2, 2>, gc128, 3);
    run("col64 ring8 occ4 E5 nt", p_col<64, 8, 5, 4, 2>, gc64, 5);
    run("row ring4 occ4 E5", p_row<4, 5, 4, 0>, 2048, 5);
    hipFree(buf);
    return 0;
}
