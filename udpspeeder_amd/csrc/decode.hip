// decode.hip -- fused batched RS decode for gfx950: one wavefront per group
// builds that group's decode matrix in LDS and streams the reconstruction.
//
// Semantics are rs_decode2's (lib/rs.cpp:21-40 -> lib/fec.cpp:838-882): the k
// survivors used are the first k present shards in ascending index order; a
// missing data row d_j is a fixed GF(2^8) combination of them.  With E the
// missing data rows (|E| = e) and R the e parity rows among the survivors,
//     d_E = A^-1 (p_R + B d_P),   A = enc[R][E],  B = enc[R][P]
// Gauss-Jordan on [A | M] (M's column per survivor: a unit vector for a parity
// survivor, enc[R][s] for a data survivor) leaves [I | coef]; the inverse is
// unique, so coef equals the rows fec_decode derives.  Rebuilt rows are
// written into their own (data) slots.
//
// Per wave:
//   1. ballot the group's present flags -> sel[k], miss[e], status;
//   2. issue the first RING survivor loads (they fly during step 3);
//   3. Gauss-Jordan in the wave's LDS slice; expand every coefficient into its
//      v_perm split tables (5 dwords, see kernels.hip) in LDS;
//   4. stream: per survivor, 5 dwords per lane (one 1-KiB dwordx4 wave-load +
//      one 256-B dword wave-load cover a 1280-B tile), GF multiply-accumulate
//      into e row accumulators, prefetch survivor j+RING; store e rows.
// Buffer descriptors with out-of-range offsets handle ragged tails: those
// loads read 0 and those stores are dropped.
#include "rsmi_internal.hpp"

namespace rsmi {
namespace {

constexpr int kWaves = 4;      // waves per block (one group each)
#ifndef DEC_RING
#define DEC_RING 4
#endif
#ifndef DEC_LD_AUX
#define DEC_LD_AUX 0           // cache policy of the survivor loads (2 = nt)
#endif
#ifndef DEC_ST_AUX
#define DEC_ST_AUX 0           // cache policy of the rebuilt-row stores
#endif
constexpr int kRing = DEC_RING;  // survivors in flight per wave
constexpr int kRows = 10;      // max e handled by the fused kernel (emax <= kRows)
constexpr int kPass = 5;       // rows accumulated per pass over the survivors
constexpr int kTile = 1280;    // bytes per lane-tile pass (64 x 16 + 64 x 4)
#ifndef DEC_OCC
#define DEC_OCC 4              // waves per SIMD the register budget is cut for
#endif

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t gmul(const uint8_t *lexp, const uint8_t *llog, uint32_t a,
                                         uint32_t b) {
    return (a && b) ? lexp[llog[a] + llog[b]] : 0u;
}

struct WaveLds {  // per-wave LDS slice
    uint8_t *sel, *miss, *aug;
    uint32_t *tab;  // [k][kRows] entries of 8 dwords (T0lo T0hi T1lo T1hi T2 - - -)
};

__host__ __device__ inline int wave_lds_bytes(int k) {
    // sel[256] miss[256] aug[kRows*(kRows+k)] tab[k*kRows*32]
    const int aug = (kRows * (kRows + k) + 15) & ~15;
    return 512 + aug + k * kRows * 32;
}

__global__ __launch_bounds__(256, DEC_OCC) void k_decode_fused(UniformArgs a, const uint8_t *present,
                                                      const uint8_t *prows, int32_t *status_out,
                                                      const uint32_t *ptab, const uint8_t *gftab) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint4 *s01 = reinterpret_cast<uint4 *>(smem);                  // 256 x 16 B
    uint32_t *s2 = reinterpret_cast<uint32_t *>(smem + 4096);      // 256 x 4 B
    uint8_t *lexp = smem + 5120;                                   // 512
    uint8_t *llog = smem + 5632;                                   // 256
    const int k = a.k, n = a.n;
    const int wbytes = wave_lds_bytes(k);
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int rows_bytes = ((n - k) * k + 15) & ~15;
    uint8_t *lrows = smem + 5888;  // the code's parity rows, (n-k) x k
    uint8_t *wl = smem + 5888 + rows_bytes + wid * wbytes;
    WaveLds L{wl, wl + 256, wl + 512,
              reinterpret_cast<uint32_t *>(wl + 512 + ((kRows * (kRows + k) + 15) & ~15))};

    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        s01[i] = reinterpret_cast<const uint4 *>(ptab + i * kPtabDwords)[0];
        s2[i] = ptab[i * kPtabDwords + 4];
    }
    for (int i = threadIdx.x; i < 768; i += blockDim.x) smem[5120 + i] = gftab[i];
    for (int i = threadIdx.x; i < (n - k) * k; i += blockDim.x) lrows[i] = prows[i];
    __syncthreads();

    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const int64_t nwaves = (int64_t)gridDim.x * kWaves;
    const int64_t g0 = (int64_t)blockIdx.x * kWaves + wid;
    // present flags of the first 64 shards, prefetched one group ahead
    uint32_t pf = (g0 < a.ngroups && lane < n) ? present[g0 * n + lane] : 0u;
    uint32_t pf_next = 0;
    for (int64_t g = g0; g < a.ngroups; g += nwaves, pf = pf_next) {
        {
            const int64_t gn = g + nwaves;
            pf_next = (gn < a.ngroups && lane < n) ? present[gn * n + lane] : 0u;
        }
        // ---- 1. survivor selection (rs.cpp:24-39) ------------------------------
        const uint8_t *pr = present + g * n;
        int cnt = 0, e = 0;
        for (int b = 0; b < n && cnt < k; b += 64) {
            const int idx = b + lane;
            const bool f = idx < n && (b == 0 ? pf : pr[idx]) != 0;
            const uint64_t mk = __ballot(f);
            const int rank = cnt + __popcll(mk & lt);
            if (f && rank < k) L.sel[rank] = (uint8_t)idx;
            cnt += __popcll(mk);
        }
        int st = RSMI_DEC_OK;
        if (cnt < k) {
            st = RSMI_DEC_TOO_FEW;
        } else {
            for (int b = 0; b < k; b += 64) {
                const int idx = b + lane;
                const bool ms = idx < k && (b == 0 ? pf : pr[idx]) == 0;
                const uint64_t mk = __ballot(ms);
                if (ms) L.miss[e + __popcll(mk & lt)] = (uint8_t)idx;
                e += __popcll(mk);
            }
        }
        // values that steer control flow are wave-uniform: say so, or the
        // compiler wraps every buffer op below in a waterfall loop
        cnt = __builtin_amdgcn_readfirstlane(cnt);
        e = __builtin_amdgcn_readfirstlane(e);
        st = __builtin_amdgcn_readfirstlane(st);
        wave_sync();
        if (st != RSMI_DEC_OK || e == 0) {
            if (lane == 0 && status_out) status_out[g] = st;
            continue;
        }

        // ---- 2. descriptor + first loads ---------------------------------------
        // descriptor inputs through readfirstlane (cdna_hip_programming.md T20)
        const uint64_t gb = (uint64_t)(uintptr_t)(a.base + g * a.group_stride);
        const uint64_t gbu = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(gb >> 32)) << 32) |
                             (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)gb);
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<uint8_t *>(gbu), 0, (int)(a.n * a.shard_stride), 0x00020000);
        const uint32_t ss = (uint32_t)a.shard_stride;
        // survivor j's shard offset lives in lane j (k <= 64 on this path):
        // v_readlane gives the scalar soffset without an LDS round trip
        const uint32_t so_lane = (lane < k ? (uint32_t)L.sel[lane] : 0u) * ss;
        const uint32_t mo_lane = (lane < e ? (uint32_t)L.miss[lane] : 0u) * ss;
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        u32x4 rq[kRing];
        uint32_t rd[kRing];
        uint32_t v16, v4;
        // whole cache lines where the slot has room (rsmi.h padding rule)
        const int lpad = (int)((a.len + 127) / 128 * 128 < a.shard_stride
                                   ? (a.len + 127) / 128 * 128 : a.shard_stride);
        auto start_tile = [&](int toff) {
            const int tlen = lpad - toff;
            v16 = (16 * lane < tlen) ? (uint32_t)(toff + 16 * lane) : 0x80000000u;
            v4 = (1024 + 4 * lane < tlen) ? (uint32_t)(toff + 1024 + 4 * lane) : 0x80000000u;
#pragma unroll
            for (int q = 0; q < kRing; ++q) {
                if (q < k) {
                    const uint32_t so = __builtin_amdgcn_readlane(so_lane, q);
                    rq[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v16, so, DEC_LD_AUX);
                    rd[q] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, v4, so, DEC_LD_AUX);
                }
            }
        };
        start_tile(0);  // the first survivors fly while the matrix is inverted

        // ---- 3. Gauss-Jordan: aug = [A | M], e x (e+k) -------------------------
        const int W = e + k;
        for (int t = lane; t < e * W; t += 64) {
            const int r = t / W, c = t - r * W;
            const int R = L.sel[k - e + r];
            const uint8_t *prow = lrows + (R - k) * k;
            uint8_t v;
            if (c < e) {
                v = prow[L.miss[c]];
            } else {
                const int s = L.sel[c - e];
                v = (s >= k) ? (uint8_t)(s == R) : prow[s];
            }
            L.aug[t] = v;
        }
        wave_sync();
        for (int p = 0; p < e && st == RSMI_DEC_OK; ++p) {
            const uint32_t piv = __builtin_amdgcn_readfirstlane(L.aug[p * W + p]);
            if (piv == 0) {
                st = RSMI_DEC_SINGULAR;
                break;
            }
            const uint32_t ipiv = __builtin_amdgcn_readfirstlane(lexp[255 - llog[piv]]);
            for (int c = p + 1 + lane; c < W; c += 64)
                L.aug[p * W + c] = (uint8_t)gmul(lexp, llog, ipiv, L.aug[p * W + c]);
            wave_sync();
            const int cols = W - p - 1;
            for (int t = lane; t < e * cols; t += 64) {
                const int r = t / cols;
                if (r == p) continue;
                const int c = p + 1 + (t - r * cols);
                const uint32_t f = L.aug[r * W + p];
                if (f) L.aug[r * W + c] ^= (uint8_t)gmul(lexp, llog, f, L.aug[p * W + c]);
            }
            wave_sync();
        }
        st = __builtin_amdgcn_readfirstlane(st);
        if (st != RSMI_DEC_OK) {
            if (lane == 0 && status_out) status_out[g] = st;
            continue;
        }
        // expand coef[r][j] = aug[r][e + j] into split tables tab[j][r]
        for (int t = lane; t < e * k; t += 64) {
            const int r = t / k, j = t - r * k;
            const uint32_t c = L.aug[r * W + e + j];
            const uint4 t01 = s01[c];
            uint32_t *dst = L.tab + (j * kRows + r) * 8;
            reinterpret_cast<uint4 *>(dst)[0] = t01;
            dst[4] = s2[c];
        }
        wave_sync();

        // ---- 4. stream the survivors: passes over (tile, block of kPass rows) --
        for (int toff = 0; toff < a.len; toff += kTile) {
            for (int rb = 0; rb < e; rb += kPass) {
                if (toff || rb) start_tile(toff);  // pass 0's loads are already in flight
                uint32_t acc[kPass][5];
#pragma unroll
                for (int r = 0; r < kPass; ++r)
#pragma unroll
                    for (int w = 0; w < 5; ++w) acc[r][w] = 0;
                for (int jb = 0; jb < k; jb += kRing) {
#pragma unroll
                    for (int q = 0; q < kRing; ++q) {
                        const int j = jb + q;
                        if (j < k) {
                            const uint32_t x[5] = {rq[q].x, rq[q].y, rq[q].z, rq[q].w, rd[q]};
                            uint32_t q0[5], q1[5], q2[5];
#pragma unroll
                            for (int w = 0; w < 5; ++w) {
                                q0[w] = x[w] & 0x07070707u;
                                q1[w] = (x[w] >> 3) & 0x07070707u;
                                q2[w] = (x[w] >> 6) & 0x03030303u;
                            }
                            if (j + kRing < k) {
                                const uint32_t so = __builtin_amdgcn_readlane(so_lane, j + kRing);
                                rq[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v16, so, DEC_LD_AUX);
                                rd[q] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, v4, so, DEC_LD_AUX);
                            }
                            const uint32_t *tj = L.tab + (j * kRows + rb) * 8;
#pragma unroll
                            for (int r = 0; r < kPass; ++r) {
                                if (rb + r < e) {
                                    const uint4 t = reinterpret_cast<const uint4 *>(tj + r * 8)[0];
                                    const uint32_t t2 = tj[r * 8 + 4];
#pragma unroll
                                    for (int w = 0; w < 5; ++w) {
                                        const uint32_t p0 = __builtin_amdgcn_perm(t.y, t.x, q0[w]);
                                        const uint32_t p1 = __builtin_amdgcn_perm(t.w, t.z, q1[w]);
                                        const uint32_t p2 = __builtin_amdgcn_perm(t2, t2, q2[w]);
                                        acc[r][w] = acc[r][w] ^ xor3(p0, p1, p2);
                                    }
                                }
                            }
                        }
                    }
                }
#pragma unroll
                for (int r = 0; r < kPass; ++r) {
                    if (rb + r < e) {
                        const uint32_t so = __builtin_amdgcn_readlane(mo_lane, rb + r);
                        const u32x4 v = {acc[r][0], acc[r][1], acc[r][2], acc[r][3]};
                        __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, v16, so, DEC_ST_AUX);
                        __builtin_amdgcn_raw_buffer_store_b32(acc[r][4], rsrc, v4, so, DEC_ST_AUX);
                    }
                }
            }
        }
        if (lane == 0 && status_out) status_out[g] = RSMI_DEC_OK;
        wave_sync();  // the LDS slice is rewritten by the next group
    }
}

}  // namespace

bool decode_fused_ok(int k, int n, int64_t group_stride, int64_t shard_stride, int len) {
    const int m = n - k;
    const int emax = k < m ? k : m;
    return emax <= kRows && k <= 64 && n * shard_stride < (int64_t(1) << 31) && len > 0 &&
           5888 + ((m * k + 15) & ~15) + kWaves * wave_lds_bytes(k) <= 64 * 1024 &&
           group_stride >= n * shard_stride;
}

hipError_t launch_decode_fused(const UniformArgs &a, const uint8_t *present,
                               const uint8_t *parity_rows, int32_t *status,
                               const uint32_t *ptab, const uint8_t *gftab, hipStream_t s) {
    const size_t lds = 5888 + (size_t)(((a.n - a.k) * a.k + 15) & ~15) +
                       (size_t)kWaves * wave_lds_bytes(a.k);
    int64_t blocks = (a.ngroups + kWaves - 1) / kWaves;
    const int64_t cap = 256 * 8;
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    k_decode_fused<<<(unsigned)blocks, 64 * kWaves, lds, s>>>(a, present, parity_rows, status,
                                                             ptab, gftab);
    return hipGetLastError();
}

}  // namespace rsmi
