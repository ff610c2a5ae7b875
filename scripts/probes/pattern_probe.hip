// pattern_probe.hip -- measurement tool: the C1 encode's exact memory pattern
// (20 x 2 KiB wave-reads, 10 x 2 KiB wave-writes per wave, 128 16-B columns per
// wave, buffer descriptors, nt) with almost no arithmetic, to find the ceiling
// of the access pattern itself; plus a flat float4 copy for reference.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int RING, int AUX>
__global__ __launch_bounds__(256, 3) void probe(uint8_t *base, uint32_t cols, uint32_t P,
                                                uint32_t gs, uint32_t ss) {
    const uint32_t wave = blockIdx.x * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave * 128u >= cols) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t cfirst = wave * 128u;
    const uint32_t clast = std::min(cfirst + 127u, cols - 1u);
    const uint32_t gfirst = cfirst / P, glast = clast / P;
    auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base + (uint64_t)gfirst * gs, 0,
                                                  (int)((glast - gfirst + 1) * gs), 0x00020000);
    const uint32_t c0 = cfirst + lane, c1 = c0 + 64;
    const uint32_t g0 = c0 / P, g1 = c1 / P;
    const uint32_t v0 = c0 < cols ? (g0 - gfirst) * gs + (c0 - g0 * P) * 16 : 0x80000000u;
    const uint32_t v1 = c1 < cols ? (g1 - gfirst) * gs + (c1 - g1 * P) * 16 : 0x80000000u;
    u32x4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
    u32x4 rx[RING], ry[RING];
#pragma unroll
    for (int r = 0; r < RING; ++r) {
        rx[r] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v0, r * ss, AUX);
        ry[r] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v1, r * ss, AUX);
    }
#pragma unroll
    for (int j = 0; j < 20; ++j) {
        a ^= rx[j % RING];
        b ^= ry[j % RING];
        if (j + RING < 20) {
            rx[j % RING] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v0, (j + RING) * ss, AUX);
            ry[j % RING] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v1, (j + RING) * ss, AUX);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        u32x4 x = a + i, y = b + i;
        __builtin_amdgcn_raw_buffer_store_b128(x, rsrc, v0, (20 + i) * ss, AUX);
        __builtin_amdgcn_raw_buffer_store_b128(y, rsrc, v1, (20 + i) * ss, AUX);
    }
}

__global__ void copy4(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// decode-shaped probe: one wave per group, 20 survivor rows of 1280 B read with a
// ring of RING rows (dwordx4 for bytes 0..1023 + dword for 1024..1279), E rows written
template <int RING, int E, int OCC>
__global__ __launch_bounds__(256, OCC) void dprobe(uint8_t *base, uint32_t G, uint32_t gs, uint32_t ss) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t g = blockIdx.x * 4u + wid; g < G; g += gridDim.x * 4u) {
        auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base + (uint64_t)g * gs, 0, (int)gs, 0x00020000);
        const uint32_t v16 = lane * 16, v4 = 1024 + lane * 4;
        u32x4 rq[RING];
        uint32_t rd[RING];
#pragma unroll
        for (int q = 0; q < RING; ++q) {
            rq[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v16, (q + (g & 7)) * ss, 0);
            rd[q] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, v4, (q + (g & 7)) * ss, 0);
        }
        u32x4 acc = {0, 0, 0, 0};
        uint32_t accd = 0;
        for (int jb = 0; jb < 20; jb += RING) {
#pragma unroll
            for (int q = 0; q < RING; ++q) {
                const int j = jb + q;
                acc ^= rq[q];
                accd ^= rd[q];
                if (j + RING < 20) {
                    rq[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v16, (j + RING + (g & 7)) * ss, 0);
                    rd[q] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, v4, (j + RING + (g & 7)) * ss, 0);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < E; ++r) {
            __builtin_amdgcn_raw_buffer_store_b128(acc + r, rsrc, v16, r * ss, 0);
            __builtin_amdgcn_raw_buffer_store_b32(accd + r, rsrc, v4, r * ss, 0);
        }
    }
}

template <int U, int AUX>
__global__ __launch_bounds__(256) void copy_nt(uint8_t *src, uint8_t *dst, uint32_t chunks) {
    // each wave moves U x 1 KiB per step with buffer ops; grid-stride over chunks of U KiB
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nw = gridDim.x * 4u;
    for (uint32_t c = wave; c < chunks; c += nw) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc(src + (uint64_t)c * U * 1024, 0, U * 1024, 0x00020000);
        auto rd = __builtin_amdgcn_make_buffer_rsrc(dst + (uint64_t)c * U * 1024, 0, U * 1024, 0x00020000);
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, u * 1024, AUX);
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, lane * 16, u * 1024, AUX);
    }
}

template <int U, int AUX>
__global__ __launch_bounds__(256) void read_only(uint8_t *src, uint32_t chunks, uint32_t *sink) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nw = gridDim.x * 4u;
    u32x4 acc = {0, 0, 0, 0};
    for (uint32_t c = wave; c < chunks; c += nw) {
        auto rs = __builtin_amdgcn_make_buffer_rsrc(src + (uint64_t)c * U * 1024, 0, U * 1024, 0x00020000);
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, u * 1024, AUX);
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

template <int U, int AUX>
__global__ __launch_bounds__(256) void write_only(uint8_t *dst, uint32_t chunks) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nw = gridDim.x * 4u;
    u32x4 v = {lane, wave, 1, 2};
    for (uint32_t c = wave; c < chunks; c += nw) {
        auto rd = __builtin_amdgcn_make_buffer_rsrc(dst + (uint64_t)c * U * 1024, 0, U * 1024, 0x00020000);
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(v, rd, lane * 16, u * 1024, AUX);
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
    const uint32_t G = 65536, n = 30, S = 1280, P = 79;
    const size_t bytes = (size_t)G * n * S;
    uint8_t *buf;
    hipMalloc(&buf, bytes);
    hipMemset(buf, 1, bytes);
    const uint32_t cols = G * P, waves = (cols + 127) / 128, blocks = (waves + 3) / 4;
    const double alg = (double)G * 30 * 1250;
    auto run = [&](const char *name, auto kern) {
        float ms = time_ms([&] { kern<<<blocks, 256>>>(buf, cols, P, n * S, S); });
        printf("%-22s %.4f ms  %.0f GB/s alg  %.0f GB/s moved\n", name, ms, alg / ms / 1e6,
               (double)G * 30 * 1280 / ms / 1e6);
    };
    run("pattern ring4", probe<4, 0>);
    run("pattern ring4 nt", probe<4, 2>);
    run("pattern ring8 nt", probe<8, 2>);
    run("pattern ring2 nt", probe<2, 2>);
    {
        const uint32_t P80 = 80, cols80 = G * P80, w80 = (cols80 + 127) / 128, b80 = (w80 + 3) / 4;
        float ms = time_ms([&] { probe<4, 2><<<b80, 256>>>(buf, cols80, P80, n * S, S); });
        printf("%-22s %.4f ms  %.0f GB/s alg  %.0f GB/s moved\n", "pattern P80 ring4 nt", ms,
               alg / ms / 1e6, (double)G * 30 * 1280 / ms / 1e6);
        float ms2 = time_ms([&] { probe<4, 0><<<b80, 256>>>(buf, cols80, P80, n * S, S); });
        printf("%-22s %.4f ms  %.0f GB/s alg  %.0f GB/s moved\n", "pattern P80 ring4", ms2,
               alg / ms2 / 1e6, (double)G * 30 * 1280 / ms2 / 1e6);
    }
    // flat copy of the same byte count: read 2/3, write 1/3 ... plain 1:1 copy
    const size_t n4 = bytes / 2 / 16;
    for (int grid : {1024, 2048, 4096, 8192}) {
        float ms = time_ms([&] {
            copy4<<<grid, 256>>>((const uint4 *)buf, (uint4 *)(buf + bytes / 2), n4);
        });
        printf("copy4 grid %-5d        %.4f ms  %.0f GB/s (read+write)\n", grid, ms,
               2.0 * n4 * 16 / ms / 1e6);
    }
    {
        const double dalg = (double)G * (20 + 3) * 1250;
        auto drun = [&](const char *name, auto kern, int grid) {
            float ms = time_ms([&] { kern<<<grid, 256>>>(buf, G, n * S, S); });
            printf("%-28s %.4f ms  %.0f GB/s alg\n", name, ms, dalg / ms / 1e6);
        };
        drun("dprobe ring4 occ4 grid2048", dprobe<4, 3, 4>, 2048);
        drun("dprobe ring4 occ4 grid4096", dprobe<4, 3, 4>, 4096);
        drun("dprobe ring4 occ4 grid16384", dprobe<4, 3, 4>, 16384);
        drun("dprobe ring8 occ4 grid4096", dprobe<8, 3, 4>, 4096);
        drun("dprobe ring2 occ8 grid8192", dprobe<2, 3, 8>, 8192);
    }
    const uint32_t half = (uint32_t)(bytes / 2);
    uint32_t *sink;
    hipMalloc(&sink, 4);
    for (int grid : {1024, 2048, 4096}) {
        const uint32_t ch8 = half / 8192;
        float ms = time_ms([&] { copy_nt<8, 2><<<grid, 256>>>(buf, buf + half, ch8); });
        printf("copy_nt U8 grid %-5d    %.4f ms  %.0f GB/s (read+write)\n", grid, ms, 2.0 * ch8 * 8192 / ms / 1e6);
        float ms2 = time_ms([&] { copy_nt<8, 0><<<grid, 256>>>(buf, buf + half, ch8); });
        printf("copy    U8 grid %-5d    %.4f ms  %.0f GB/s (read+write)\n", grid, ms2, 2.0 * ch8 * 8192 / ms2 / 1e6);
        const uint32_t chr = (uint32_t)(bytes / 8192);
        float ms3 = time_ms([&] { read_only<8, 2><<<grid, 256>>>(buf, chr, sink); });
        printf("read_nt U8 grid %-5d    %.4f ms  %.0f GB/s (read)\n", grid, ms3, (double)chr * 8192 / ms3 / 1e6);
        float ms4 = time_ms([&] { write_only<8, 2><<<grid, 256>>>(buf, chr); });
        printf("write_nt U8 grid %-5d   %.4f ms  %.0f GB/s (write)\n", grid, ms4, (double)chr * 8192 / ms4 / 1e6);
    }
    hipFree(buf);
    return 0;
}
