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
//   3. Gauss-Jordan with column c of [A | M] in lane c (e bytes in registers,
//      W = e + k <= 64; wider systems use the wave's LDS slice); multiplies by
//      a wave-uniform factor go through that factor's v_perm split table;
//      expand every coefficient into its split table (5 dwords, see
//      kernels.hip) in LDS;
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
#define DEC_LD_AUX 0           // cache policy of the survivor loads (2 = nt: 9 % faster alone,
                               // but the next encode is 1.5 % slower: no gain in bench.py)
#endif
#ifndef DEC_ST_AUX
#define DEC_ST_AUX 0           // cache policy of the rebuilt-row stores
#endif
constexpr int kRing = DEC_RING;  // survivors in flight per wave
static_assert(kRing % 2 == 0, "ring slots are consumed in pairs under DEC_PAIR");
constexpr int kRows = 10;      // max e handled by the fused kernel (emax <= kRows)
constexpr int kPass = 5;       // rows accumulated per pass over the survivors
constexpr int kTile = 1280;    // bytes per lane-tile pass (64 x 16 + 64 x 4)
#ifndef DEC_ST_SGPR
#define DEC_ST_SGPR 0          // 1: row offset of the rebuilt-row stores in soffset (see bitslice.hip
                               // DevIO::store: no hazard wait state is inserted for that form)
#endif
#ifndef DEC_PAIR
#define DEC_PAIR 0             // fold survivors in pairs (fewer XORs, more VGPRs)
#endif
#ifndef DEC_FENCE
#define DEC_FENCE 0            // agent-scope release at the end of every wave
#endif
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

constexpr int kRowsAt = 6144;  // smem: s01 | s2 | exp | log | inv | parity rows | wave slices

// c * x for a byte x (upper bits zero), c given by its split table (t, t2)
__device__ __forceinline__ uint32_t gmul_t(uint4 t, uint32_t t2, uint32_t x) {
    return xor3(__builtin_amdgcn_perm(t.y, t.x, x & 7u), __builtin_amdgcn_perm(t.w, t.z, (x >> 3) & 7u),
                __builtin_amdgcn_perm(t2, t2, x >> 6));
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
    uint8_t *linv = smem + 5888;                                   // 256: x^-1
    const int k = a.k, n = a.n;
    const int wbytes = wave_lds_bytes(k);
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int rows_bytes = ((n - k) * k + 15) & ~15;
    uint8_t *lrows = smem + kRowsAt;  // the code's parity rows, (n-k) x k
    uint8_t *wl = smem + kRowsAt + rows_bytes + wid * wbytes;
    WaveLds L{wl, wl + 256, wl + 512,
              reinterpret_cast<uint32_t *>(wl + 512 + ((kRows * (kRows + k) + 15) & ~15))};

    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        s01[i] = reinterpret_cast<const uint4 *>(ptab + i * kPtabDwords)[0];
        s2[i] = ptab[i * kPtabDwords + 4];
    }
    for (int i = threadIdx.x; i < 768; i += blockDim.x) smem[5120 + i] = gftab[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x)
        linv[i] = i ? gftab[255 - gftab[512 + i]] : 0;  // exp[255 - log x]
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
        const uint32_t sel_lane = lane < k ? (uint32_t)L.sel[lane] : 0u;
        const uint32_t so_lane = sel_lane * ss;
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

        // ---- 3. Gauss-Jordan on [A | M], e x (e+k) ------------------------------
        const int W = e + k;
        if (W <= 64) {
            // lane c holds column c: a missing data index (c < e) or survivor c - e
            const uint32_t col = lane < e ? (uint32_t)L.miss[lane]
                                          : (lane < W ? (uint32_t)L.sel[lane - e] : 0u);
            uint32_t a[kRows];
#pragma unroll
            for (int r = 0; r < kRows; ++r) {
                a[r] = 0;
                if (r < e) {
                    const uint32_t R = __builtin_amdgcn_readlane(sel_lane, k - e + r);
                    const uint8_t *prow = lrows + (R - k) * k;
                    const uint32_t v = prow[col < (uint32_t)k ? col : 0u];
                    a[r] = (lane >= e && col >= (uint32_t)k) ? (uint32_t)(col == R) : v;
                }
            }
#pragma unroll
            for (int p = 0; p < kRows; ++p) {
                if (p < e) {
                    const uint32_t piv = __builtin_amdgcn_readlane(a[p], p);
                    if (piv == 0) {
                        st = RSMI_DEC_SINGULAR;
                        break;
                    }
                    const uint32_t ip = __builtin_amdgcn_readfirstlane(linv[piv]);
                    a[p] = gmul_t(s01[ip], s2[ip], a[p]);
#pragma unroll
                    for (int r = 0; r < kRows; ++r) {
                        if (r < e && r != p) {
                            const uint32_t f = __builtin_amdgcn_readlane(a[r], p);
                            a[r] ^= gmul_t(s01[f], s2[f], a[p]);
                        }
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }
            st = __builtin_amdgcn_readfirstlane(st);
            if (st != RSMI_DEC_OK) {
                if (lane == 0 && status_out) status_out[g] = st;
                continue;
            }
            // coef[r][j] sits in lane e + j: expand into split tables tab[j][r]
            if (lane >= e && lane < W) {
                uint32_t *dst = L.tab + (lane - e) * kRows * 8;
#pragma unroll
                for (int r = 0; r < kRows; ++r) {
                    if (r < e) {
                        reinterpret_cast<uint4 *>(dst + r * 8)[0] = s01[a[r]];
                        dst[r * 8 + 4] = s2[a[r]];
                    }
                }
            }
            wave_sync();
        } else {
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
        }

        // ---- 4. stream the survivors: passes over (tile, block of kPass rows) --
        // the 3-bit split selectors of a survivor's 5 dwords
        auto split = [](const u32x4 &v, uint32_t d, uint32_t (&s0)[5], uint32_t (&s1)[5],
                        uint32_t (&s2)[5]) {
            const uint32_t x[5] = {v.x, v.y, v.z, v.w, d};
#pragma unroll
            for (int w = 0; w < 5; ++w) {
                s0[w] = x[w] & 0x07070707u;
                s1[w] = (x[w] >> 3) & 0x07070707u;
                s2[w] = (x[w] >> 6) & 0x03030303u;
            }
        };
        // ring slot q took survivor j: load survivor j + kRing into it
        auto refill = [&](int q, int j) {
            if (j + kRing < k) {
                const uint32_t so = __builtin_amdgcn_readlane(so_lane, j + kRing);
                rq[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v16, so, DEC_LD_AUX);
                rd[q] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, v4, so, DEC_LD_AUX);
            }
        };
        for (int toff = 0; toff < a.len; toff += kTile) {
            for (int rb = 0; rb < e; rb += kPass) {
                if (toff || rb) start_tile(toff);  // pass 0's loads are already in flight
                uint32_t acc[kPass][5];
#pragma unroll
                for (int r = 0; r < kPass; ++r)
#pragma unroll
                    for (int w = 0; w < 5; ++w) acc[r][w] = 0;
                // with DEC_PAIR, survivors go in pairs: the six split products of
                // two survivors fold into a row with three 3-input XORs
                for (int jb = 0; jb < k; jb += kRing) {
#pragma unroll
                    for (int q = 0; q < kRing; q += DEC_PAIR ? 2 : 1) {
                        const int j = jb + q;
                        if (DEC_PAIR && j + 1 < k) {
                            uint32_t a0[5], a1[5], a2[5], b0[5], b1[5], b2[5];
                            split(rq[q], rd[q], a0, a1, a2);
                            split(rq[q + 1], rd[q + 1], b0, b1, b2);
                            refill(q, j);
                            refill(q + 1, j + 1);
                            const uint32_t *ta = L.tab + (j * kRows + rb) * 8;
                            const uint32_t *tb = ta + kRows * 8;
#pragma unroll
                            for (int r = 0; r < kPass; ++r) {
                                if (rb + r < e) {
                                    const uint4 t = reinterpret_cast<const uint4 *>(ta + r * 8)[0];
                                    const uint32_t t2 = ta[r * 8 + 4];
                                    const uint4 u = reinterpret_cast<const uint4 *>(tb + r * 8)[0];
                                    const uint32_t u2 = tb[r * 8 + 4];
#pragma unroll
                                    for (int w = 0; w < 5; ++w) {
                                        uint32_t x = xor3(acc[r][w], __builtin_amdgcn_perm(t.y, t.x, a0[w]),
                                                          __builtin_amdgcn_perm(t.w, t.z, a1[w]));
                                        x = xor3(x, __builtin_amdgcn_perm(t2, t2, a2[w]),
                                                 __builtin_amdgcn_perm(u.y, u.x, b0[w]));
                                        acc[r][w] = xor3(x, __builtin_amdgcn_perm(u.w, u.z, b1[w]),
                                                         __builtin_amdgcn_perm(u2, u2, b2[w]));
                                    }
                                }
                            }
                        } else if (j < k) {
                            uint32_t a0[5], a1[5], a2[5];
                            split(rq[q], rd[q], a0, a1, a2);
                            refill(q, j);
                            const uint32_t *ta = L.tab + (j * kRows + rb) * 8;
#pragma unroll
                            for (int r = 0; r < kPass; ++r) {
                                if (rb + r < e) {
                                    const uint4 t = reinterpret_cast<const uint4 *>(ta + r * 8)[0];
                                    const uint32_t t2 = ta[r * 8 + 4];
#pragma unroll
                                    for (int w = 0; w < 5; ++w)
                                        acc[r][w] ^= xor3(__builtin_amdgcn_perm(t.y, t.x, a0[w]),
                                                          __builtin_amdgcn_perm(t.w, t.z, a1[w]),
                                                          __builtin_amdgcn_perm(t2, t2, a2[w]));
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
#if DEC_ST_SGPR
                        __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, v16, so, DEC_ST_AUX);
                        __builtin_amdgcn_raw_buffer_store_b32(acc[r][4], rsrc, v4, so, DEC_ST_AUX);
#else
                        __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, v16 + so, 0, DEC_ST_AUX);
                        __builtin_amdgcn_raw_buffer_store_b32(acc[r][4], rsrc, v4 + so, 0, DEC_ST_AUX);
#endif
                    }
                }
            }
        }
        if (lane == 0 && status_out) status_out[g] = RSMI_DEC_OK;
        wave_sync();  // the LDS slice is rewritten by the next group
    }
#if DEC_FENCE
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#endif
}

}  // namespace

bool decode_fused_ok(int k, int n, int64_t group_stride, int64_t shard_stride, int len) {
    const int m = n - k;
    const int emax = k < m ? k : m;
    return emax <= kRows && k <= 64 && n * shard_stride < (int64_t(1) << 31) && len > 0 &&
           kRowsAt + ((m * k + 15) & ~15) + kWaves * wave_lds_bytes(k) <= 64 * 1024 &&
           group_stride >= n * shard_stride;
}

hipError_t launch_decode_fused(const UniformArgs &a, const uint8_t *present,
                               const uint8_t *parity_rows, int32_t *status,
                               const uint32_t *ptab, const uint8_t *gftab, hipStream_t s) {
    const size_t lds = kRowsAt + (size_t)(((a.n - a.k) * a.k + 15) & ~15) +
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
