// dec4_probe.hip -- measurement tool: what bounds the C2 decode's access
// pattern with no arithmetic?  G = 65536 groups of 30 x 1280-B slots, 5 of 30
// shards erased per group (LCG-seeded), the 20 lowest present read and the
// erased data rows written -- one wave per group, 2 survivors in flight, 5
// waves per SIMD, as k_decode_fused.  Flags:
//   PREF    the group's pattern word loaded one group ahead (else at the group's start)
//   CONTIG  survivors are slots 0..19 and rows 0..e-1 are written (no pattern)
//   STORE   write the erased rows (else reads only)
//   QUAD    all-dwordx4 loads: lane l reads survivor 4q + l/16, bytes 256t + 16(l%16)
//           (5 loads per 4 survivors instead of 8)
//   AUX     cache policy of the loads (2 = nt)
// Build: hipcc --offload-arch=gfx950 -O3 -o dec4_probe dec4_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t G = 65536, N = 30, S = 1280, K = 20;

template <int PREF, int CONTIG, int STORE, int QUAD, int AUX, int STAUX, int WMODE = 0, int REV = 0>
__global__ __launch_bounds__(256, 5) void p_pat(uint8_t *base, const uint8_t *pat, uint32_t *sink) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nb = gridDim.x;
    const uint32_t bid = (nb & 7) == 0 ? (blockIdx.x & 7) * (nb >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    const uint32_t nw = nb * 4;
    uint32_t g = bid * 4 + wid;
    uint32_t pw_next = (PREF && g < G && lane < 8) ? reinterpret_cast<const uint32_t *>(pat + (size_t)g * 32)[lane] : 0u;
    uint32_t keep = 0;
    for (; g < G; g += nw) {
        uint32_t pw;
        if (PREF) {
            pw = pw_next;
            const uint32_t gn = g + nw;
            pw_next = (gn < G && lane < 8) ? reinterpret_cast<const uint32_t *>(pat + (size_t)gn * 32)[lane] : 0u;
        } else {
            pw = lane < 8 ? reinterpret_cast<const uint32_t *>(pat + (size_t)g * 32)[lane] : 0u;
        }
        auto byte_at = [&](int i) {
            return (uint32_t)(__builtin_amdgcn_readlane((int)pw, i >> 2) >> ((i & 3) * 8)) & 255u;
        };
        const int e = (int)byte_at(20);
        auto sl = [&](int j) { if (REV) j = (int)K - 1 - j; return CONTIG ? (uint32_t)j : byte_at(j); };
        auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base + (uint64_t)g * N * S, 0, (int)(N * S), 0x00020000);
        uint32_t acc[5] = {0, 0, 0, 0, 0};
        if (!QUAD) {
            const uint32_t v16 = lane * 16, v4 = 1024 + lane * 4;
            u32x4 rq[2];
            uint32_t rd[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                rq[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v16, sl(q) * S, AUX);
                rd[q] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, v4, sl(q) * S, AUX);
                __builtin_amdgcn_sched_barrier(0);
            }
            for (int jb = 0; jb < (int)K; jb += 2) {
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int j = jb + q;
                    acc[0] ^= rq[q].x; acc[1] ^= rq[q].y; acc[2] ^= rq[q].z; acc[3] ^= rq[q].w; acc[4] ^= rd[q];
                    const bool ok = j + 2 < (int)K;
                    auto r = ok ? rsrc : __builtin_amdgcn_make_buffer_rsrc(base, 0, 0, 0x00020000);
                    const uint32_t so = sl(ok ? j + 2 : 0) * S;
                    rq[q] = __builtin_amdgcn_raw_buffer_load_b128(r, v16, so, AUX);
                    rd[q] = __builtin_amdgcn_raw_buffer_load_b32(r, v4, so, AUX);
                }
            }
            if (STORE) {
                // WMODE 0: the erased data slot; 1: a compact output area past the
                // groups (g * 5 + r); 2: the slot of the r-th last survivor (a
                // parity shard just read, the reference's placement)
                auto wr = WMODE == 1 ? __builtin_amdgcn_make_buffer_rsrc(base + (uint64_t)G * N * S + (uint64_t)g * 5 * S,
                                                                          0, (int)(5 * S), 0x00020000)
                                     : rsrc;
                for (int r = 0; r < e; ++r) {
                    const uint32_t so = WMODE == 1 ? r * S
                                      : WMODE == 2 ? byte_at((int)K - 1 - r) * S
                                                   : (CONTIG ? (uint32_t)r : byte_at(24 + r)) * S;
                    const u32x4 v = {acc[0] + r, acc[1], acc[2], acc[3]};
                    __builtin_amdgcn_raw_buffer_store_b128(v, wr, v16 + so, 0, STAUX);
                    __builtin_amdgcn_raw_buffer_store_b32(acc[4], wr, v4 + so, 0, STAUX);
                }
            }
        } else {
            // quad q: survivors 4q..4q+3, lane l -> survivor 4q + l/16, pieces 256t + 16(l%16)
            const uint32_t vl = (lane & 15) * 16;
            const int sub = (int)(lane >> 4);
            u32x4 rq[5];
            auto so_of = [&](int q) {  // per-lane slot offset of quad q
                const uint32_t s0 = sl(4 * q), s1 = sl(4 * q + 1), s2 = sl(4 * q + 2), s3 = sl(4 * q + 3);
                const uint32_t s = sub == 0 ? s0 : sub == 1 ? s1 : sub == 2 ? s2 : s3;
                return s * S + vl;
            };
            uint32_t vo = so_of(0);
#pragma unroll
            for (int t = 0; t < 5; ++t) rq[t] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, vo + 256 * t, 0, AUX);
            for (int q = 0; q < (int)K / 4; ++q) {
                const bool ok = q + 1 < (int)K / 4;
                const uint32_t vn = so_of(ok ? q + 1 : 0);
                auto r = ok ? rsrc : __builtin_amdgcn_make_buffer_rsrc(base, 0, 0, 0x00020000);
#pragma unroll
                for (int t = 0; t < 5; ++t) {
                    acc[t] ^= rq[t].x ^ rq[t].y ^ rq[t].z ^ rq[t].w;
                    rq[t] = __builtin_amdgcn_raw_buffer_load_b128(r, vn + 256 * t, 0, AUX);
                }
            }
            if (STORE) {  // row r: the 16 lanes of sub r % 4 store its 1280 B
                for (int r = 0; r < e; ++r) {
                    if (sub == (r & 3)) {
                        const uint32_t so = (CONTIG ? (uint32_t)r : byte_at(24 + r)) * S;
#pragma unroll
                        for (int t = 0; t < 5; ++t) {
                            const u32x4 v = {acc[t] + r, acc[t], acc[t], acc[t]};
                            __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, so + vl + 256 * t, 0, STAUX);
                        }
                    }
                }
            }
        }
        keep ^= acc[0] ^ acc[1] ^ acc[2] ^ acc[3] ^ acc[4];
    }
    if (keep == 0x12345678u) sink[threadIdx.x] = keep;  // keeps the loads alive
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
    const size_t bytes = (size_t)G * N * S + (size_t)G * 5 * S;
    uint8_t *buf, *dpat;
    uint32_t *sink;
    if (hipMalloc(&buf, bytes) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    (void)hipMalloc(&sink, 4096);
    std::vector<uint8_t> pat((size_t)G * 32, 0);
    uint64_t st = 0x5EEDC0DEull;
    double alg = 0, moved = 0;
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
        moved += (double)(K + e) * 1280;
    }
    if (hipMalloc(&dpat, pat.size()) != hipSuccess) return 1;
    (void)hipMemcpy(dpat, pat.data(), pat.size(), hipMemcpyHostToDevice);
    auto run = [&](const char *name, auto kern, int grid) {
        float ms = time_ms([&] { kern<<<grid, 256>>>(buf, dpat, sink); });
        printf("%-44s %.4f ms  alg frac %.3f  moved %.2f TB/s\n", name, ms, alg / (ms * 1e-3) / 8e12,
               moved / (ms * 1e-3) / 1e12);
        fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep) {
        run("erased data slot, default", p_pat<1, 0, 1, 0, 2, 0, 0, 0>, 2048);
        run("erased data slot, sc0 sc1", p_pat<1, 0, 1, 0, 2, 17, 0, 0>, 2048);
        run("erased data slot, reversed reads", p_pat<1, 0, 1, 0, 2, 0, 0, 1>, 2048);
        run("compact output area", p_pat<1, 0, 1, 0, 2, 0, 1, 0>, 2048);
        run("compact output area, sc0 sc1", p_pat<1, 0, 1, 0, 2, 17, 1, 0>, 2048);
        run("last survivors' slots", p_pat<1, 0, 1, 0, 2, 0, 2, 0>, 2048);
        run("last survivors' slots, sc0 sc1", p_pat<1, 0, 1, 0, 2, 17, 2, 0>, 2048);
        run("no store", p_pat<1, 0, 0, 0, 2, 0, 0, 0>, 2048);
    }
    return 0;
}
