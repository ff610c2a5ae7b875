// bperm_probe.hip -- measurement tool for a decode MAC built on ds_bpermute_b32:
// a survivor byte's 6-bit fields index a 64-entry table held one entry per
// lane (4 rebuilt rows' products packed in a dword), read with bpermute.
//   1. semantics: which address bits ds_bpermute_b32 uses on gfx950;
//   2. throughput of back-to-back bpermutes (wave-instructions per cycle per CU);
//   3. the MAC mix per survivor dword (7 shifts + 8 bpermutes + 4 xor3) in
//      survivor bytes per cycle per CU, against the v_perm MAC mix;
//   4. ds_read_b32 gathers from a 256-entry LDS table (random bytes).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/bperm bperm_probe.hip && /tmp/bperm
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

constexpr int kIters = 2048;

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t bperm(uint32_t addr, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)addr, (int)v);
}

// 1. lane i reads lane (i * 7 + 3) & 63 through an address with junk above
// bit 7 and in bits 0..1
__global__ void sem(uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t src = (lane * 7 + 3) & 63;
    const uint32_t v = 1000 + lane;
    out[threadIdx.x] = bperm(src * 4, v);
    out[64 + threadIdx.x] = bperm(src * 4 + (lane << 8) + 0x5A00 + (lane & 3), v);
    out[128 + threadIdx.x] = bperm((src * 4) | 0xFFFFFF00u | 3u, v);
}

// 2. independent bpermutes
__global__ __launch_bounds__(256) void bp_rate(uint32_t *out, uint32_t seed, uint64_t *clk) {
    uint32_t t = seed * 0x9E3779B9u + threadIdx.x;
    uint32_t x[8], acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        x[i] = (seed + i) * 0x85EBCA6Bu ^ (threadIdx.x * 0x27D4EB2Fu);
        acc[i] = 0;
    }
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] ^= bperm(x[i], t);
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] += acc[(i + 3) & 7];
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s ^= acc[i];
    if (s == 0x12345678u) out[threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = c1 - c0;
        clk[1] = r1 - r0;
    }
}

// 3. the bpermute MAC over 5 survivor dwords per lane (a 1280-B tile): per
// dword 7 shifts, 8 bpermutes, 4 xor3 into 4 position accumulators
__global__ __launch_bounds__(256) void bp_mac(uint32_t *out, uint32_t seed, uint64_t *clk) {
    const uint32_t tlo = seed * 0x9E3779B9u + threadIdx.x, thi = tlo * 0x27D4EB2Fu;
    uint32_t d[5], acc[5][4];
#pragma unroll
    for (int w = 0; w < 5; ++w) {
        d[w] = (seed + w) * 0x85EBCA6Bu ^ (threadIdx.x * 0xC2B2AE35u);
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[w][b] = 0;
    }
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int w = 0; w < 5; ++w) {
            const uint32_t x = d[w];
            acc[w][0] = xor3(acc[w][0], bperm(x << 2, tlo), bperm(x, thi));
            acc[w][1] = xor3(acc[w][1], bperm(x >> 6, tlo), bperm(x >> 8, thi));
            acc[w][2] = xor3(acc[w][2], bperm(x >> 14, tlo), bperm(x >> 16, thi));
            acc[w][3] = xor3(acc[w][3], bperm(x >> 22, tlo), bperm(x >> 24, thi));
        }
#pragma unroll
        for (int w = 0; w < 5; ++w) d[w] = d[w] * 0x01000193u + it;  // next survivor (2 VALU stand-in for a load)
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int w = 0; w < 5; ++w)
#pragma unroll
        for (int b = 0; b < 4; ++b) s ^= acc[w][b];
    if (s == 0x12345678u) out[threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = c1 - c0;
        clk[1] = r1 - r0;
    }
}

// 3b. the v_perm MAC (current decode) over the same 5 dwords, R rows
template <int R>
__global__ __launch_bounds__(256) void vp_mac(uint32_t *out, uint32_t seed, uint64_t *clk) {
    uint32_t t[R][5];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int i = 0; i < 5; ++i) t[r][i] = (seed + 7 * r + i) * 0x9E3779B9u;
    uint32_t d[5], acc[R][5];
#pragma unroll
    for (int w = 0; w < 5; ++w) {
        d[w] = (seed + w) * 0x85EBCA6Bu ^ (threadIdx.x * 0xC2B2AE35u);
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][w] = 0;
    }
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int w = 0; w < 5; ++w) {
            const uint32_t a0 = d[w] & 0x07070707u, a1 = (d[w] >> 3) & 0x07070707u,
                           a2 = (d[w] >> 6) & 0x03030303u;
#pragma unroll
            for (int r = 0; r < R; ++r)
                acc[r][w] ^= xor3(__builtin_amdgcn_perm(t[r][1], t[r][0], a0),
                                  __builtin_amdgcn_perm(t[r][3], t[r][2], a1),
                                  __builtin_amdgcn_perm(t[r][4], t[r][4], a2));
        }
#pragma unroll
        for (int w = 0; w < 5; ++w) d[w] = d[w] * 0x01000193u + it;
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int w = 0; w < 5; ++w)
#pragma unroll
        for (int r = 0; r < R; ++r) s ^= acc[r][w];
    if (s == 0x12345678u) out[threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = c1 - c0;
        clk[1] = r1 - r0;
    }
}

// 4. ds_read_b32 gathers: one 256-entry table per wave in LDS, 4 lookups per dword
__global__ __launch_bounds__(256) void lds_mac(uint32_t *out, uint32_t seed, uint64_t *clk) {
    __shared__ uint32_t tab[4][256];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = lane; i < 256; i += 64) tab[wid][i] = (seed + i) * 0x9E3779B9u;
    __syncthreads();
    const uint32_t *T = tab[wid];
    uint32_t d[5], acc[5][4];
#pragma unroll
    for (int w = 0; w < 5; ++w) {
        d[w] = (seed + w) * 0x85EBCA6Bu ^ (threadIdx.x * 0xC2B2AE35u);
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[w][b] = 0;
    }
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int w = 0; w < 5; ++w) {
            const uint32_t x = d[w];
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[w][b] ^= T[(x >> (8 * b)) & 255];
        }
#pragma unroll
        for (int w = 0; w < 5; ++w) d[w] = d[w] * 0x01000193u + it;
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int w = 0; w < 5; ++w)
#pragma unroll
        for (int b = 0; b < 4; ++b) s ^= acc[w][b];
    if (s == 0x12345678u) out[threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = c1 - c0;
        clk[1] = r1 - r0;
    }
}

typedef void (*Kern)(uint32_t *, uint32_t, uint64_t *);

int run(const char *name, Kern k, int cus, double units_per_wave_iter, const char *unit) {
    uint32_t *out;
    uint64_t *clk;
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMalloc(&clk, 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int wps : {1, 2, 4, 6, 8}) {
        const int blocks = cus * wps;
        k<<<blocks, 256>>>(out, 1, clk);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        k<<<blocks, 256>>>(out, 2, clk);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        uint64_t h[2];
        CK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
        const double ghz = (double)h[0] / ((double)h[1] * 10.0);
        const double waves = blocks * 4.0;
        const double units = waves * kIters * units_per_wave_iter;
        const double cyc = ms * 1e-3 * ghz * 1e9;
        printf("%-10s waves/SIMD %d: %.3f ms, %.2f GHz, %.3f %s per cycle per CU\n", name, wps, ms, ghz,
               units / (cyc * cus), unit);
    }
    return 0;
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *o;
    CK(hipMalloc(&o, 4096));
    sem<<<1, 64>>>(o);
    std::vector<uint32_t> h(192);
    CK(hipMemcpy(h.data(), o, 192 * 4, hipMemcpyDeviceToHost));
    int ok0 = 1, ok1 = 1, ok2 = 1;
    for (int i = 0; i < 64; ++i) {
        const uint32_t want = 1000 + ((i * 7 + 3) & 63);
        ok0 &= h[i] == want;
        ok1 &= h[64 + i] == want;
        ok2 &= h[128 + i] == want;
    }
    printf("bpermute semantics: plain %d, junk above bit 7 and in bits 0..1 ignored %d, all-ones high %d\n",
           ok0, ok1, ok2);
    // 8 bpermute wave-instructions per wave-iteration
    run("bp_rate", bp_rate, cus, 8.0, "bpermute wave-instr");
    // survivor bytes per wave-iteration: 5 dwords x 64 lanes
    run("bp_mac", bp_mac, cus, 1280.0, "survivor B (4 rows)");
    run("vp_mac4", vp_mac<4>, cus, 1280.0, "survivor B (4 rows)");
    run("vp_mac3", vp_mac<3>, cus, 1280.0, "survivor B (3 rows)");
    run("lds_mac", lds_mac, cus, 1280.0, "survivor B (4 rows)");
    return 0;
}
