// dec3_probe.hip -- measurement tool: does splitting one group's survivors over
// several waves (split-k, as the encode's k_bs2 does) help the C2 decode?
//
// G = 65536 groups of 30 x 1280-B slots, the bench's C2 erasure pattern shape
// (5 of 30 erased per group, seeded here with a plain LCG; the k = 20 lowest
// present shards are read, the erased data rows written).  Per survivor dword
// the kernels run the decode's own VALU work: the 3-bit split (5 ops) and, per
// erased row, 3 v_perm + a 3-input XOR + the accumulate, with stand-in split
// tables (the real kernel's come from LDS; the arithmetic is the same).
//   WPG = 1: one wave per group (the shipped k_decode_fused shape)
//   WPG = 2, 4: WPG waves per group, wave h taking survivors j = h (mod WPG)
//            (MODE 1) or a contiguous range (MODE 0); partial rows summed in
//            LDS, wave h storing rows r = h (mod WPG)
// VALU = 0 runs the same loads and stores with no arithmetic.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/dec3_probe dec3_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t G = 65536, N = 30, S = 1280, K = 20;

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// pat[g] : 20 survivor indices (bytes 0..19), e (byte 20), miss[5] (bytes 24..28)
template <int WPG, int MODE, int RING, int OCC, int VALU>
__global__ __launch_bounds__(256, OCC) void p_split(uint8_t *base, const uint8_t *pat, uint32_t salt) {
    constexpr int GPB = 4 / WPG;  // groups per 4-wave block
    __shared__ uint32_t part[WPG > 1 ? GPB * WPG * 5 * 5 * 64 : 1];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t h = wid % WPG, slot = wid / WPG;
    const uint32_t nb = gridDim.x;
    const uint32_t bid = (nb & 7) == 0 ? (blockIdx.x & 7) * (nb >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    for (uint32_t g0 = bid * GPB; g0 < G; g0 += nb * GPB) {
        const uint32_t g = g0 + slot;  // G is a multiple of GPB
        const uint8_t *pg = pat + (size_t)g * 32;
        const uint32_t pw = lane < 8 ? reinterpret_cast<const uint32_t *>(pg)[lane] : 0u;
        auto byte_at = [&](int i) {
            return (uint32_t)(__builtin_amdgcn_readlane((int)pw, i >> 2) >> ((i & 3) * 8)) & 255u;
        };
        const int e = (int)byte_at(20);
        auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base + (uint64_t)g * N * S, 0, (int)(N * S), 0x00020000);
        const uint32_t v16 = lane * 16, v4 = 1024 + lane * 4;
        constexpr int J = K / WPG;  // survivors per wave
        auto sidx = [&](int t) { return MODE ? t * WPG + (int)h : (int)h * J + t; };
        u32x4 rq[RING];
        uint32_t rd[RING];
#pragma unroll
        for (int q = 0; q < RING; ++q) {
            const uint32_t so = byte_at(sidx(q)) * S;
            rq[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v16, so, 2);
            rd[q] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, v4, so, 2);
            __builtin_amdgcn_sched_barrier(0);
        }
        uint32_t acc[5][5];
#pragma unroll
        for (int r = 0; r < 5; ++r)
#pragma unroll
            for (int w = 0; w < 5; ++w) acc[r][w] = 0;
        int nr = e;
        asm volatile("" : "+s"(nr));
        for (int tb = 0; tb < J; tb += RING) {
#pragma unroll
            for (int q = 0; q < RING; ++q) {
                const int t = tb + q;
                if (t >= J) break;
                const uint32_t x[5] = {rq[q].x, rq[q].y, rq[q].z, rq[q].w, rd[q]};
                uint32_t a0[5], a1[5], a2[5];
#pragma unroll
                for (int w = 0; w < 5; ++w) {
                    a0[w] = x[w] & 0x07070707u;
                    a1[w] = (x[w] >> 3) & 0x07070707u;
                    a2[w] = (x[w] >> 6) & 0x03030303u;
                }
                {
                    const bool ok = t + RING < J;
                    const uint32_t so = byte_at(sidx(ok ? t + RING : 0)) * S;
                    auto r = ok ? rsrc : __builtin_amdgcn_make_buffer_rsrc(base, 0, 0, 0x00020000);
                    rq[q] = __builtin_amdgcn_raw_buffer_load_b128(r, v16, so, 2);
                    rd[q] = __builtin_amdgcn_raw_buffer_load_b32(r, v4, so, 2);
                }
                if (VALU) {
#pragma unroll
                    for (int r = 0; r < 5; ++r) {
                        if (r < nr) {
                            const uint32_t t0 = salt * (t + 1) + r, t1 = t0 * 3u, t2 = t0 ^ 0x5a5a5a5au,
                                           t3 = t1 + 7u, t4 = t0 * 5u;
#pragma unroll
                            for (int w = 0; w < 5; ++w)
                                acc[r][w] ^= xor3(__builtin_amdgcn_perm(t1, t0, a0[w]),
                                                  __builtin_amdgcn_perm(t3, t2, a1[w]),
                                                  __builtin_amdgcn_perm(t4, t4, a2[w]));
                        }
                    }
                } else {
#pragma unroll
                    for (int w = 0; w < 5; ++w) acc[0][w] ^= a0[w] ^ a1[w] ^ a2[w];
                }
            }
        }
        if (!VALU) {
#pragma unroll
            for (int r = 1; r < 5; ++r)
#pragma unroll
                for (int w = 0; w < 5; ++w) acc[r][w] = acc[0][w] + r;
        }
        if (WPG > 1) {
            uint32_t *my = part + (size_t)(slot * WPG + h) * 25 * 64;
#pragma unroll
            for (int r = 0; r < 5; ++r)
                if (r < nr)
#pragma unroll
                    for (int w = 0; w < 5; ++w) my[(r * 5 + w) * 64 + lane] = acc[r][w];
            __syncthreads();
            const uint32_t *grp = part + (size_t)slot * WPG * 25 * 64;
#pragma unroll
            for (int r = 0; r < 5; ++r) {
                if (r < nr && (r % WPG) == (int)h) {
#pragma unroll
                    for (int w = 0; w < 5; ++w) {
                        uint32_t s = 0;
#pragma unroll
                        for (int o = 0; o < WPG; ++o) s ^= grp[((o * 25) + r * 5 + w) * 64 + lane];
                        acc[r][w] = s;
                    }
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (int r = 0; r < 5; ++r) {
            if (r < nr && (r % WPG) == (int)h) {
                const uint32_t so = byte_at(24 + r) * S;
                const u32x4 v = {acc[r][0], acc[r][1], acc[r][2], acc[r][3]};
                __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, v16 + so, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b32(acc[r][4], rsrc, v4 + so, 0, 0);
            }
        }
    }
}

template <class F>
float time_ms(F f, int reps = 30) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    std::vector<float> v;
    for (int i = 0; i < 40; ++i) f();  // clocks up
    (void)hipDeviceSynchronize();
    for (int i = 0; i < reps; ++i) {
        hipEventRecord(a);
        f();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    const size_t bytes = (size_t)G * N * S;
    uint8_t *buf, *dpat;
    if (hipMalloc(&buf, bytes) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    std::vector<uint8_t> pat((size_t)G * 32, 0);
    uint64_t st = 0x5EEDC0DEull;
    double alg = 0;
    for (uint32_t g = 0; g < G; ++g) {
        bool er[N] = {};
        for (int c = 0; c < 5;) {
            st = st * 6364136223846793005ull + 1442695040888963407ull;
            const int i = (int)((st >> 33) % N);
            if (!er[i]) { er[i] = true; ++c; }
        }
        uint8_t *p = &pat[(size_t)g * 32];
        int ns = 0, e = 0;
        for (int i = 0; i < (int)N && ns < (int)K; ++i)
            if (!er[i]) p[ns++] = (uint8_t)i;
        for (int i = 0; i < (int)K; ++i)
            if (er[i]) p[24 + e++] = (uint8_t)i;
        p[20] = (uint8_t)e;
        if (e) alg += (double)(K + e) * 1250;
    }
    if (hipMalloc(&dpat, pat.size()) != hipSuccess) return 1;
    (void)hipMemcpy(dpat, pat.data(), pat.size(), hipMemcpyHostToDevice);
    auto run = [&](const char *name, auto kern, int grid) {
        float ms = time_ms([&] { kern<<<grid, 256>>>(buf, dpat, 0x9E3779B9u); });
        printf("%-40s %.4f ms  frac %.3f\n", name, ms, alg / (ms * 1e-3) / 8e12);
        fflush(stdout);
    };
    const int cu = 256;
    for (int rep = 0; rep < 2; ++rep) {
        run("wpg1 ring2 occ5 valu", p_split<1, 0, 2, 5, 1>, cu * 8);
        run("wpg1 ring2 occ5 novalu", p_split<1, 0, 2, 5, 0>, cu * 8);
        run("wpg2 halves ring2 occ5 valu", p_split<2, 0, 2, 5, 1>, cu * 8);
        run("wpg2 inter ring2 occ5 valu", p_split<2, 1, 2, 5, 1>, cu * 8);
        run("wpg2 inter ring2 occ5 novalu", p_split<2, 1, 2, 5, 0>, cu * 8);
        run("wpg4 inter ring2 occ5 valu", p_split<4, 1, 2, 5, 1>, cu * 8);
        run("wpg4 halves ring2 occ5 valu", p_split<4, 0, 2, 5, 1>, cu * 8);
        run("wpg4 inter ring1 occ5 valu", p_split<4, 1, 1, 5, 1>, cu * 8);
        run("wpg2 inter ring1 occ5 valu", p_split<2, 1, 1, 5, 1>, cu * 8);
        run("wpg1 ring2 occ5 valu g16", p_split<1, 0, 2, 5, 1>, cu * 16);
        run("wpg2 inter ring2 occ5 valu g16", p_split<2, 1, 2, 5, 1>, cu * 16);
    }
    hipFree(buf);
    hipFree(dpat);
    return 0;
}
