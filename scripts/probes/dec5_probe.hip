// dec5_probe.hip -- measurement tool: the C2 decode's access pattern (no
// arithmetic; see dec4_probe.hip) with the rebuilt-row stores of group g
// issued before or after the first survivor loads of the wave's next group.
// On gfx9 vmcnt counts stores too, in order: a wave that stores group g's rows
// and then loads group g + 1's first survivors waits for those stores before
// it can use the first survivor.  XPIPE = 1 issues the next group's ring
// loads first.  STAUX: store cache policy.
// Build: hipcc --offload-arch=gfx950 -O3 -o dec5_probe dec5_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t G = 65536, N = 30, S = 1280, K = 20;

template <int XPIPE, int STAUX, int OCC>
__global__ __launch_bounds__(256, OCC) void p_x(uint8_t *base, const uint8_t *pat, uint32_t *sink) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nb = gridDim.x;
    const uint32_t bid = (nb & 7) == 0 ? (blockIdx.x & 7) * (nb >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    const uint32_t nw = nb * 4;
    uint32_t g = bid * 4 + wid;
    auto patw = [&](uint32_t gg) {
        return (gg < G && lane < 8) ? reinterpret_cast<const uint32_t *>(pat + (size_t)gg * 32)[lane] : 0u;
    };
    auto byte_of = [&](uint32_t pw, int i) {
        return (uint32_t)(__builtin_amdgcn_readlane((int)pw, i >> 2) >> ((i & 3) * 8)) & 255u;
    };
    auto grsrc = [&](uint32_t gg) {
        return __builtin_amdgcn_make_buffer_rsrc(base + (uint64_t)(gg < G ? gg : 0) * N * S, 0,
                                                 gg < G ? (int)(N * S) : 0, 0x00020000);
    };
    const auto rnull = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0, 0x00020000);
    const uint32_t v16 = lane * 16, v4 = 1024 + lane * 4;
    uint32_t pw = patw(g);
    uint32_t pw_next = patw(g + nw);
    uint32_t keep = 0;
    u32x4 rq[2];
    uint32_t rd[2];
    auto first_loads = [&](uint32_t gg, uint32_t p) {
        const auto r = grsrc(gg);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            rq[q] = __builtin_amdgcn_raw_buffer_load_b128(r, v16, byte_of(p, q) * S, 2);
            rd[q] = __builtin_amdgcn_raw_buffer_load_b32(r, v4, byte_of(p, q) * S, 2);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    if (XPIPE) first_loads(g, pw);
    for (; g < G; g += nw) {
        const int e = (int)byte_of(pw, 20);
        const auto rsrc = grsrc(g);
        if (!XPIPE) first_loads(g, pw);
        uint32_t acc[5] = {0, 0, 0, 0, 0};
        for (int jb = 0; jb < (int)K; jb += 2) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int j = jb + q;
                acc[0] ^= rq[q].x; acc[1] ^= rq[q].y; acc[2] ^= rq[q].z; acc[3] ^= rq[q].w; acc[4] ^= rd[q];
                if (j + 2 < (int)K) {
                    const uint32_t so = byte_of(pw, j + 2) * S;
                    rq[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v16, so, 2);
                    rd[q] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, v4, so, 2);
                } else if (XPIPE) {  // the next group's survivor j + 2 - K
                    const uint32_t so = byte_of(pw_next, j + 2 - (int)K) * S;
                    const auto rn = grsrc(g + nw);
                    rq[q] = __builtin_amdgcn_raw_buffer_load_b128(rn, v16, so, 2);
                    rd[q] = __builtin_amdgcn_raw_buffer_load_b32(rn, v4, so, 2);
                } else {
                    rq[q] = __builtin_amdgcn_raw_buffer_load_b128(rnull, v16, 0, 2);
                    rd[q] = __builtin_amdgcn_raw_buffer_load_b32(rnull, v4, 0, 2);
                }
            }
        }
        for (int r = 0; r < e; ++r) {
            const uint32_t so = byte_of(pw, 24 + r) * S;
            const u32x4 v = {acc[0] + r, acc[1], acc[2], acc[3]};
            __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, v16 + so, 0, STAUX);
            __builtin_amdgcn_raw_buffer_store_b32(acc[4], rsrc, v4 + so, 0, STAUX);
        }
        keep ^= acc[0];
        pw = pw_next;
        pw_next = patw(g + 2 * nw);
    }
    if (keep == 0x12345678u) sink[threadIdx.x] = keep;
}

template <class F>
float time_ms(F f, int reps = 30) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    std::vector<float> v;
    for (int i = 0; i < 40; ++i) f();
    (void)hipDeviceSynchronize();
    for (int i = 0; i < reps; ++i) {
        (void)hipEventRecord(a);
        f();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    const size_t bytes = (size_t)G * N * S;
    uint8_t *buf, *dpat;
    uint32_t *sink;
    if (hipMalloc(&buf, bytes) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    (void)hipMalloc(&sink, 4096);
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
        float ms = time_ms([&] { kern<<<grid, 256>>>(buf, dpat, sink); });
        printf("%-40s %.4f ms  alg frac %.3f\n", name, ms, alg / (ms * 1e-3) / 8e12);
        fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep) {
        run("stores then next loads, default", p_x<0, 0, 5>, 2048);
        run("next loads then stores, default", p_x<1, 0, 5>, 2048);
        run("stores then next loads, sc0 sc1", p_x<0, 17, 5>, 2048);
        run("next loads then stores, sc0 sc1", p_x<1, 17, 5>, 2048);
        run("next loads then stores, nt", p_x<1, 2, 5>, 2048);
        run("next loads then stores, default, occ4", p_x<1, 0, 4>, 2048);
    }
    return 0;
}
