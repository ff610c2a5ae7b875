// valu_probe.hip -- measurement tool: sustained VALU issue rate per SIMD for
// the decode MAC's instruction mix (v_perm_b32 + v_bitop3_b32), at 1..8 waves
// per SIMD, in wave-instructions per cycle per SIMD (in-kernel clock from
// s_memtime / s_memrealtime).  Tells whether a kernel at X VALU
// wave-instructions per second is issue-bound.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/valu valu_probe.hip && /tmp/valu
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

constexpr int kIters = 4096;

// 8 independent accumulators, each step: 3 v_perm + 1 v_bitop3 (xor3) + 1 xor
// per accumulator = the decode MAC's 5 VALU per dword
__global__ __launch_bounds__(256) void mac_mix(uint32_t *out, uint32_t seed, uint64_t *clk) {
    uint32_t t0 = seed ^ threadIdx.x, t1 = t0 * 3u, t2 = t0 * 5u, t3 = t0 * 7u, t4 = t0 * 11u;
    uint32_t acc[8];
    uint32_t x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        acc[i] = 0;
        x[i] = (seed + i) * 0x9E3779B9u ^ threadIdx.x;
    }
    uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t s0 = x[i] & 0x07070707u;
            const uint32_t p0 = __builtin_amdgcn_perm(t1, t0, s0);
            const uint32_t p1 = __builtin_amdgcn_perm(t3, t2, s0 ^ 0x01010101u);
            const uint32_t p2 = __builtin_amdgcn_perm(t4, t4, s0 ^ 0x02020202u);
            acc[i] ^= __builtin_amdgcn_bitop3_b32(p0, p1, p2, 0x96);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = acc[i] ^ x[(i + 1) & 7];
    }
    uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s ^= acc[i];
    if (s == 0x12345678u) out[threadIdx.x] = s;  // keep the work
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = c1 - c0;
        clk[1] = r1 - r0;
    }
}

int main() {
    uint32_t *out;
    uint64_t *clk;
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMalloc(&clk, 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    // VALU per loop iteration, counted in the compiled loop body (hipcc -S,
    // ROCm 7.2): 72 (24 v_perm, bitop3 / xor / and for the rest), 3 SALU
    const double valu_per_thread_iter = 72.0;
    for (int wps : {1, 2, 4, 6, 8}) {  // waves per SIMD: blocks of 4 waves, wps blocks per CU
        const int blocks = cus * wps;
        mac_mix<<<blocks, 256>>>(out, 1, clk);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        mac_mix<<<blocks, 256>>>(out, 2, clk);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        uint64_t h[2];
        CK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
        const double ghz = (double)h[0] / ((double)h[1] * 10.0);  // memrealtime = 100 MHz
        const double waves = blocks * 4.0;
        const double instr = waves * kIters * valu_per_thread_iter;
        const double cyc = ms * 1e-3 * ghz * 1e9;
        printf("waves/SIMD %d: %.3f ms, clock %.2f GHz, %.3f VALU wave-instr per cycle per SIMD\n", wps,
               ms, ghz, instr / (cyc * cus * 4));
    }
    return 0;
}
