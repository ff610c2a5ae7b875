// oneshot.hip -- one FEC group per call, for the level-1 drop-in
// (rs_encode2 / rs_decode2 / fec_encode / fec_decode, lib/rs.cpp:56-64,
// lib/fec.cpp:727-750, 838-882): latency, not throughput.
//
// The caller's shards sit in pinned, device-mapped staging; ONE kernel reads
// them over PCIe (system-scope loads, all in flight at once), builds the
// coefficients, multiplies, writes the output rows straight back into pinned
// memory and raises a completion flag the host polls.  No hipMemcpy and no
// stream synchronisation on the way: the per-call floor is one kernel launch
// plus one PCIe round trip.
//
// One 1024-thread workgroup (four waves per SIMD, so the multiply is spread
// over the whole CU instead of one wave's issue slots):
//  1. every thread stages the GF tables; wave 0 picks the survivors from the
//     256-bit present mask (the first k present, lib/rs.cpp:24-39);
//  2. the survivors' 16-byte pieces are loaded by all threads at once and
//     parked in LDS; meanwhile wave 0 runs Gauss-Jordan on [A | M] with lane
//     c holding column c (decode.hip's header has the algebra), or, for the
//     encode, the code's parity rows are the coefficients;
//  3. thread t multiplies dword column t % C (C = dword columns of the shard)
//     for the output rows r = t / C, t / C + 1024 / C, ... through the v_perm
//     split tables (kernels.hip), reading the survivors from LDS.
#include "rsmi_internal.hpp"

namespace rsmi {
namespace {

constexpr int kOneThreads = 1024;
constexpr int kSurvLds = 32768;  // survivor bytes parked in LDS: k * lpad
constexpr int kCoefMax = 640;    // output rows x survivors
constexpr int kAugMax = 4096;    // [A | M] bytes for the LDS elimination (W > 64)
constexpr int kRegRows = 10;     // rows of the register elimination
constexpr int kRowsPerThread = 10;
constexpr int kAux = 3;          // sc0 | sc1: system scope, coherent with the host

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t gmul(const uint8_t *lexp, const uint8_t *llog, uint32_t a,
                                         uint32_t b) {
    return (a && b) ? lexp[llog[a] + llog[b]] : 0u;
}

// c * x for a byte x, c given by its split table (t, t2)
__device__ __forceinline__ uint32_t gmul_t(uint4 t, uint32_t t2, uint32_t x) {
    return xor3(__builtin_amdgcn_perm(t.y, t.x, x & 7u), __builtin_amdgcn_perm(t.w, t.z, (x >> 3) & 7u),
                __builtin_amdgcn_perm(t2, t2, x >> 6));
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#include "lagrange.hpp"

// The workgroup's LDS (one group's tables, survivors and coefficients).
struct OneSmem {
    uint4 s01[256];
    uint32_t s2[256];
    uint8_t lexp[512], llog[256], linv[256];
    uint8_t sel[256], miss[256];
    uint4 ct01[kCoefMax];  // coefficient (r, j)'s split table at r * k + j
    uint32_t ct2[kCoefMax];
    uint8_t aug[kAugMax];
    __attribute__((aligned(16))) uint8_t xs[kSurvLds];  // survivor j at j * lpad
    int s_e, s_st;
};

// One group in one workgroup (codes and shapes the multi-workgroup form below
// does not take).
__device__ __forceinline__ void one_body(const OneArgs &a, OneSmem &S) {
    uint4 *s01 = S.s01;
    uint32_t *s2 = S.s2;
    uint8_t *lexp = S.lexp, *llog = S.llog, *linv = S.linv, *sel = S.sel, *miss = S.miss;
    uint4 *ct01 = S.ct01;
    uint32_t *ct2 = S.ct2;
    uint8_t *aug = S.aug, *xs = S.xs;
    int &s_e = S.s_e, &s_st = S.s_st;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int k = a.k, n = a.n, len = a.len;
    const uint32_t ss = (uint32_t)a.ss;
    const int lpad = (len + 15) & ~15;  // whole 16-B pieces, inside the slot
    for (int i = tid; i < 256; i += kOneThreads) {
        s01[i] = reinterpret_cast<const uint4 *>(a.ptab + i * kPtabDwords)[0];
        s2[i] = a.ptab[i * kPtabDwords + 4];
        linv[i] = i ? a.gftab[255 - a.gftab[512 + i]] : 0;  // exp[255 - log x]
    }
    for (int i = tid; i < 768; i += kOneThreads) (i < 512 ? lexp[i] : llog[i - 512]) = a.gftab[i];
    // ---- 1. survivors (decode) / data shards (encode)
    if (tid < 64) {
        const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
        int cnt = 0, e = 0;
        if (a.encode) {
            for (int j = lane; j < k; j += 64) sel[j] = (uint8_t)j;
            cnt = k;
            e = n - k;
        } else {
            for (int b = 0; b < n && cnt < k; b += 64) {
                const int idx = b + lane;
                const bool f = idx < n && ((a.present[idx >> 5] >> (idx & 31)) & 1u);
                const uint64_t mk = __ballot(f);
                const int rank = cnt + __popcll(mk & lt);
                if (f && rank < k) sel[rank] = (uint8_t)idx;
                cnt += __popcll(mk);
            }
            if (cnt >= k)
                for (int b = 0; b < k; b += 64) {
                    const int idx = b + lane;
                    const bool ms = idx < k && !((a.present[idx >> 5] >> (idx & 31)) & 1u);
                    const uint64_t mk = __ballot(ms);
                    if (ms) miss[e + __popcll(mk & lt)] = (uint8_t)idx;
                    e += __popcll(mk);
                }
        }
        if (lane == 0) {
            s_e = e;
            s_st = cnt < k ? RSMI_DEC_TOO_FEW : RSMI_DEC_OK;
        }
    }
    __syncthreads();
    const int e = s_e;
    const int W = e + k;
    const bool work = s_st == RSMI_DEC_OK && e > 0 && len > 0;
    if (work) {
        // ---- 2. every survivor piece in flight at once
        const auto in = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.in), 0, (int)(n * ss),
                                                          0x00020000);
        const int np = lpad >> 4;  // pieces per shard
        constexpr int kMaxPer = (kSurvLds / 16 + kOneThreads - 1) / kOneThreads;
        u32x4 v[kMaxPer];
#pragma unroll
        for (int q = 0; q < kMaxPer; ++q) {
            const int p = tid + q * kOneThreads;
            if (p < k * np) {
                const int j = p / np, c = p - j * np;
                // the shard offset differs per lane: it belongs in voffset
                // (soffset must be wave-uniform, or the compiler wraps the
                // load in a waterfall loop, one pass per distinct value)
                v[q] = __builtin_amdgcn_raw_buffer_load_b128(in, (uint32_t)c * 16u + (uint32_t)sel[j] * ss, 0u,
                                                             kAux);
            }
        }
        // coefficients while the loads fly
        if (a.encode) {
            for (int t = tid; t < e * k; t += kOneThreads) {
                const uint8_t c = a.rows[t];  // parity row r = t / k, column j = t % k
                ct01[t] = s01[c];
                ct2[t] = s2[c];
            }
        } else if (W <= 64 && e <= kRegRows) {
            if (tid < 64) {  // register elimination: lane c holds column c of [A | M]
                const uint32_t col = lane < e ? (uint32_t)miss[lane] : (lane < W ? (uint32_t)sel[lane - e] : 0u);
                uint32_t m_[kRegRows];
#pragma unroll
                for (int r = 0; r < kRegRows; ++r) {
                    m_[r] = 0;
                    if (r < e) {
                        const uint32_t R = sel[k - e + r];
                        const uint32_t pv = a.rows[(R - k) * k + (col < (uint32_t)k ? col : 0u)];
                        m_[r] = (lane >= e && col >= (uint32_t)k) ? (uint32_t)(col == R) : pv;
                    }
                }
                int st = RSMI_DEC_OK;
#pragma unroll
                for (int p = 0; p < kRegRows; ++p) {
                    if (p < e) {
                        const uint32_t piv = __builtin_amdgcn_readlane(m_[p], p);
                        if (piv == 0) {  // never for an MDS code
                            st = RSMI_DEC_SINGULAR;
                            break;
                        }
                        const uint32_t ip = __builtin_amdgcn_readfirstlane(linv[piv]);
                        m_[p] = gmul_t(s01[ip], s2[ip], m_[p]);
#pragma unroll
                        for (int r = 0; r < kRegRows; ++r) {
                            if (r < e && r != p) {
                                const uint32_t f = __builtin_amdgcn_readlane(m_[r], p);
                                m_[r] ^= gmul_t(s01[f], s2[f], m_[p]);
                            }
                        }
                    }
                }
                if (st == RSMI_DEC_OK && lane >= e && lane < W) {
#pragma unroll
                    for (int r = 0; r < kRegRows; ++r)
                        if (r < e) {
                            ct01[r * k + lane - e] = s01[m_[r]];
                            ct2[r * k + lane - e] = s2[m_[r]];
                        }
                }
                if (lane == 0) s_st = st;
            }
        } else {
            // wide systems: elimination in LDS by the whole workgroup
            for (int t = tid; t < e * W; t += kOneThreads) {
                const int r = t / W, c = t - r * W;
                const int R = sel[k - e + r];
                const uint8_t *pr = a.rows + (R - k) * k;
                const int s = c < e ? miss[c] : sel[c - e];
                aug[t] = (c >= e && s >= k) ? (uint8_t)(s == R) : pr[s];
            }
            __syncthreads();
            for (int p = 0; p < e; ++p) {
                const uint32_t piv = aug[p * W + p];
                if (piv == 0) {
                    if (tid == 0) s_st = RSMI_DEC_SINGULAR;
                    break;
                }
                const uint32_t ipiv = linv[piv];
                for (int c = p + 1 + tid; c < W; c += kOneThreads)
                    aug[p * W + c] = (uint8_t)gmul(lexp, llog, ipiv, aug[p * W + c]);
                __syncthreads();
                const int cols = W - p - 1;
                for (int t = tid; t < e * cols; t += kOneThreads) {
                    const int r = t / cols;
                    if (r == p) continue;
                    const int c = p + 1 + (t - r * cols);
                    const uint32_t f = aug[r * W + p];
                    if (f) aug[r * W + c] ^= (uint8_t)gmul(lexp, llog, f, aug[p * W + c]);
                }
                __syncthreads();
            }
            for (int t = tid; t < e * k; t += kOneThreads) {
                const int r = t / k, j = t - r * k;
                const uint8_t c = aug[r * W + e + j];
                ct01[t] = s01[c];
                ct2[t] = s2[c];
            }
        }
        // park the survivors in LDS
#pragma unroll
        for (int q = 0; q < kMaxPer; ++q) {
            const int p = tid + q * kOneThreads;
            if (p < k * np) {
                const int j = p / np, c = p - j * np;
                *reinterpret_cast<u32x4 *>(xs + j * lpad + c * 16) = v[q];
            }
        }
    }
    __syncthreads();
    if (work && s_st == RSMI_DEC_OK) {
        // ---- 3. multiply: dword column c, rows g, g + RG, ...
        const int C = lpad >> 2;
        const int RG = C >= kOneThreads ? 1 : kOneThreads / C;
        const auto out = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, (int)(e * ss), 0x00020000);
        for (int t = tid; t < C * RG; t += kOneThreads) {
            const int c = t % C, g = t / C;
            uint32_t acc[kRowsPerThread];
#pragma unroll
            for (int i = 0; i < kRowsPerThread; ++i) acc[i] = 0;
            for (int rb = g; rb < e; rb += RG * kRowsPerThread) {
                for (int j = 0; j < k; ++j) {
                    const uint32_t x = *reinterpret_cast<const uint32_t *>(xs + j * lpad + c * 4);
                    const uint32_t a0 = x & 0x07070707u, a1 = (x >> 3) & 0x07070707u,
                                   a2 = (x >> 6) & 0x03030303u;
#pragma unroll
                    for (int i = 0; i < kRowsPerThread; ++i) {
                        const int r = rb + i * RG;
                        if (r < e) {
                            const uint4 tt = ct01[r * k + j];
                            const uint32_t t2 = ct2[r * k + j];
                            acc[i] ^= xor3(__builtin_amdgcn_perm(tt.y, tt.x, a0),
                                           __builtin_amdgcn_perm(tt.w, tt.z, a1),
                                           __builtin_amdgcn_perm(t2, t2, a2));
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < kRowsPerThread; ++i) {
                    const int r = rb + i * RG;
                    if (r < e) {
                        __builtin_amdgcn_raw_buffer_store_b32(acc[i], out, (uint32_t)c * 4u + (uint32_t)r * ss, 0,
                                                              kAux);
                        acc[i] = 0;
                    }
                }
            }
        }
    }
    // ---- completion: rows, then status, then the flag the host polls
    // (every storing wave drains its stores before the barrier, then one lane
    // releases at system scope: MI355X_MICROARCH.md, inter-workgroup visibility)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __hip_atomic_store(a.status, (int32_t)s_st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(a.flag, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ __launch_bounds__(kOneThreads) void k_one_group(OneArgs a) {
    __shared__ OneSmem S;
    one_body(a, S);
}

// ---- the multi-workgroup form: per-call launch or resident server --------------
// k_one_group runs a whole group in ONE workgroup: at the clocks a nearly idle
// GPU runs (one group per call), its serial chain -- survivors over PCIe,
// Gauss-Jordan in one wave, a 20-survivor MAC per thread -- took ~15 us of
// the ~19 us call (profiles/r05/dropin).  Here kOneSrvWgs workgroups split the
// group's 16-byte pieces (columns): each one selects the survivors, computes
// the coefficients (Lagrange form, lagrange.hpp; the code's rows for the
// encode), loads only its pieces of the survivors, splits the MAC over its
// four waves by survivor and stores its pieces of the output rows, then raises
// its own completion word (flags[wg] = seq).  No workgroup waits for another.
constexpr int kMwThreads = 256;
constexpr int kMwCoef = 640;     // e x k coefficients (e <= 10, k <= 64)
constexpr int kMwSurv = 16384;   // k x pieces-per-workgroup x 16 bytes
constexpr int kMwOut = 1024;     // e x dwords-per-workgroup outputs

struct MwSmem {
    __attribute__((aligned(16))) uint8_t ltab[kLTabBytes];  // LTables image
    uint4 s01[256];                                         // split tables by value (encode)
    uint32_t s2[256];
    uint4 ct01[kMwCoef];  // coefficient (r, j) at r * k + j
    uint32_t ct2[kMwCoef];
    __attribute__((aligned(16))) uint8_t xs[kMwSurv];  // survivor j's pieces at j * pw * 16
    uint32_t part[4 * kMwOut];                          // per-wave partial sums
    uint8_t sel[64], miss[16];
    uint32_t args[32];
    int e, st;
    uint32_t cmd, seq;
};

__device__ __forceinline__ void mw_tables(MwSmem &S, const uint32_t *ptab, const uint8_t *gftab) {
    const uint4 *src = reinterpret_cast<const uint4 *>(gftab + kGfLtabOff);
    for (int i = threadIdx.x; i < kLTabBytes / 16; i += kMwThreads)
        reinterpret_cast<uint4 *>(S.ltab)[i] = src[i];
    for (int i = threadIdx.x; i < 256; i += kMwThreads) {
        S.s01[i] = reinterpret_cast<const uint4 *>(ptab + i * kPtabDwords)[0];
        S.s2[i] = ptab[i * kPtabDwords + 4];
    }
}

// The pieces [p0, p0 + pw) of workgroup wg (of nwg) among the group's P.
__device__ __forceinline__ void mw_span(int P, int wg, int nwg, int &p0, int &pw) {
    const int per = (P + nwg - 1) / nwg;
    p0 = wg * per;
    pw = p0 >= P ? 0 : (P - p0 < per ? P - p0 : per);
}

// One workgroup's share of one group (a: the job), then flags[wg] = seq.
__device__ __forceinline__ void mw_body(const OneArgs &a, MwSmem &S, int wg, int nwg, uint32_t *flags) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int k = a.k, n = a.n, len = a.len;
    const uint32_t ss = (uint32_t)a.ss;
    const int lpad = (len + 15) & ~15;
    const int P = lpad >> 4;
    int p0, pw;
    mw_span(P, wg, nwg, p0, pw);
    // ---- survivors (the first k present, lib/rs.cpp:24-39) or the data shards
    if (wv == 0) {
        const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
        int cnt = 0, e = 0;
        if (a.encode) {
            if (lane < k) S.sel[lane] = (uint8_t)lane;
            cnt = k;
            e = n - k;
        } else {
            for (int b = 0; b < n && cnt < k; b += 64) {
                const int idx = b + lane;
                const bool f = idx < n && ((a.present[idx >> 5] >> (idx & 31)) & 1u);
                const uint64_t mk = __ballot(f);
                const int rank = cnt + __popcll(mk & lt);
                if (f && rank < k) S.sel[rank] = (uint8_t)idx;
                cnt += __popcll(mk);
            }
            if (cnt >= k) {  // k <= 64: one window of data indices
                const bool ms = lane < k && !((a.present[lane >> 5] >> (lane & 31)) & 1u);
                const uint64_t mk = __ballot(ms);
                if (ms) S.miss[__popcll(mk & lt)] = (uint8_t)lane;
                e = __popcll(mk);
            }
        }
        if (lane == 0) {
            S.e = e;
            S.st = cnt < k ? RSMI_DEC_TOO_FEW : RSMI_DEC_OK;
        }
    }
    __syncthreads();
    const int e = S.e;
    const bool work = S.st == RSMI_DEC_OK && e > 0 && pw > 0;
    if (work) {
        // ---- this workgroup's survivor pieces, all in flight at once
        const auto in = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.in), 0, (int)(n * ss), 0x00020000);
        const int items = k * pw;  // <= kMwSurv / 16 = 1024
        u32x4 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int t = tid + q * kMwThreads;
            if (t < items) {
                const int j = t / pw, c = t - j * pw;
                v[q] = __builtin_amdgcn_raw_buffer_load_b128(in, (uint32_t)(p0 + c) * 16u + (uint32_t)S.sel[j] * ss,
                                                             0u, kAux);
            }
        }
        // ---- coefficients while the loads fly
        if (a.encode) {
            for (int t = tid; t < e * k; t += kMwThreads) {
                const uint8_t c = a.rows[t];  // parity row r = t / k, column j = t % k
                S.ct01[t] = S.s01[c];
                S.ct2[t] = S.s2[c];
            }
        } else if (wv == 0) {
            const LTables LT{reinterpret_cast<const uint4 *>(S.ltab), reinterpret_cast<const uint32_t *>(S.ltab + 4096),
                             S.ltab + 5120, S.ltab + 5376};
            const uint32_t xs = LT.px[lane < k ? S.sel[lane] : 0u];
            const uint32_t B = lagrange_b(k, xs, LT);
            for (int rb = 0; rb < e; rb += 5) {
                const uint32_t xm = lane + rb < e ? (uint32_t)LT.px[S.miss[lane + rb]] : 0u;
                lagrange_rows<5>(k, e - rb < 5 ? e - rb : 5, xs, B, xm, LT, lane, [&](int r, uint32_t lv) {
                    S.ct01[(rb + r) * k + lane] = LT.t01[lv];
                    S.ct2[(rb + r) * k + lane] = LT.t2[lv];
                });
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int t = tid + q * kMwThreads;
            if (t < items) *reinterpret_cast<u32x4 *>(S.xs + t * 16) = v[q];  // survivor j at j * pw pieces
        }
    }
    __syncthreads();
    const int D = 4 * pw;  // output dwords of each row in this workgroup
    const int O = e * D;
    if (work) {
        // ---- MAC: wave wv takes survivors wv, wv + 4, ...; lane o an output (row, dword)
        for (int o = lane; o < O; o += 64) {
            const int r = o / D, d = o - r * D;
            uint32_t acc = 0;
            for (int j = wv; j < k; j += 4) {
                const uint32_t x = *reinterpret_cast<const uint32_t *>(S.xs + (j * pw) * 16 + d * 4);
                const uint4 t = S.ct01[r * k + j];
                const uint32_t t2 = S.ct2[r * k + j];
                acc ^= xor3(__builtin_amdgcn_perm(t.y, t.x, x & 0x07070707u),
                            __builtin_amdgcn_perm(t.w, t.z, (x >> 3) & 0x07070707u),
                            __builtin_amdgcn_perm(t2, t2, (x >> 6) & 0x03030303u));
            }
            S.part[wv * O + o] = acc;
        }
    }
    __syncthreads();
    if (work) {
        const auto out = __builtin_amdgcn_make_buffer_rsrc(a.out, 0, (int)(e * ss), 0x00020000);
        for (int o = tid; o < O; o += kMwThreads) {
            const int r = o / D, d = o - r * D;
            const uint32_t val = S.part[o] ^ S.part[O + o] ^ S.part[2 * O + o] ^ S.part[3 * O + o];
            __builtin_amdgcn_raw_buffer_store_b32(val, out, (uint32_t)r * ss + (uint32_t)(p0 * 16 + d * 4), 0, kAux);
        }
    }
    // ---- completion: this workgroup's rows (and the status), then its flag
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        if (wg == 0) __hip_atomic_store(a.status, (int32_t)S.st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(flags + wg, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ __launch_bounds__(kMwThreads) void k_one_multi(OneArgs a) {
    __shared__ MwSmem S;
    mw_tables(S, a.ptab, a.gftab);
    __syncthreads();
    mw_body(a, S, (int)blockIdx.x, (int)gridDim.x, a.flag);
}

// ---- the resident server: no launch on the per-call path -----------------------
// kOneSrvWgs workgroups stay on the device and poll the job block in pinned
// host memory (OneSrvCtl::job: every dword of the job's OneArgs paired with
// the job's seq in one 8-byte word, written after the job's inputs; a wave
// whose lanes all read the same new seq has read the whole job).  Each
// workgroup runs its pieces of the job (mw_body) and raises flags[wg].
// Workgroup 0 decides when the server ends -- ctl->quit from the host, no job
// for idle_ticks of the 100 MHz s_memrealtime clock, or life_ticks in any case
// -- and tells the others through dv->stop (device memory); the last one out
// writes the generation to ctl->exit_gen, which tells the host to launch a new
// server for the next job (a job that workgroups saw in part before they
// stopped is run again whole by the next server: a job's outputs depend only
// on its inputs).
#ifndef SRV_PIPE
#define SRV_PIPE 1  // k_one_server: 4 = four job polls in flight per wave, 1 = one round trip per poll
#endif
#ifndef SRV_GAP
#define SRV_GAP 4  // s_sleep units (64 clocks each) between two polls
#endif
__device__ __forceinline__ uint32_t sys_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t sys_load64(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kMwThreads) void k_one_server(OneSrvCtl *ctl, OneSrvDev *dv, const uint32_t *ptab,
                                                           const uint8_t *gftab, uint32_t gen, uint32_t done0,
                                                           uint64_t idle_ticks, uint64_t life_ticks) {
    __shared__ MwSmem S;
    static_assert(sizeof(OneArgs) <= 4 * kOneJobWords && sizeof(OneArgs) % 4 == 0, "OneArgs fits the job block");
    const int tid = threadIdx.x, lane = tid & 63, wg = (int)blockIdx.x;
    mw_tables(S, ptab, gftab);
    uint32_t done = done0;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    uint64_t t_last = t_start;
    for (;;) {
        if (tid < 64) {
            uint32_t cmd = 0, seq = 0, w = 0;
#if SRV_PIPE > 1
            // four polls in flight, one issued every SRV_GAP sleep: a job is seen
            // about one PCIe round trip after it lands, not up to two.  Lanes
            // 0..29 read the job words, 30-31 the quit word, 32-63 workgroup 0's
            // stop word (no exec mask and no other load in the loop, so every
            // wait is for one poll and the rest stay in flight)
            const uint64_t *pa = lane < kOneJobWords ? &ctl->job[lane]
                                 : lane < 32       ? reinterpret_cast<const uint64_t *>(&ctl->quit)
                                                   : reinterpret_cast<const uint64_t *>(&dv->stop);
            bool stop = false;
            auto check = [&](uint64_t jw) -> bool {
                w = (uint32_t)jw;
                const uint32_t js = (uint32_t)(jw >> 32);
                const uint32_t s0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)js);
                const bool torn = __ballot(lane < kOneJobWords && js != s0) != 0;  // host mid-write
                if (!torn && s0 != done) {
                    cmd = 1;
                    seq = s0;
                    return true;
                }
                if (wg == 0) {
                    const uint32_t q = (uint32_t)__builtin_amdgcn_readlane((int)w, 30);
                    const uint64_t now = __builtin_amdgcn_s_memrealtime();
                    if (q || now - t_last > idle_ticks || now - t_start > life_ticks) {
                        if (lane == 0) __hip_atomic_store(&dv->stop, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        stop = true;
                        return true;
                    }
                } else if ((uint32_t)__builtin_amdgcn_readlane((int)w, 32) == gen) {
                    stop = true;
                    return true;
                }
                return false;
            };
            uint64_t r0 = sys_load64(pa);
            __builtin_amdgcn_s_sleep(SRV_GAP);
            uint64_t r1 = sys_load64(pa);
            __builtin_amdgcn_s_sleep(SRV_GAP);
            uint64_t r2 = sys_load64(pa);
            __builtin_amdgcn_s_sleep(SRV_GAP);
            uint64_t r3 = sys_load64(pa);
#define SRV_STEP(R)                             \
    if (check(R)) break;                        \
    __builtin_amdgcn_s_sleep(SRV_GAP);          \
    R = sys_load64(pa);
            for (;;) {
                SRV_STEP(r0)
                SRV_STEP(r1)
                SRV_STEP(r2)
                SRV_STEP(r3)
            }
#undef SRV_STEP
            (void)stop;
#else
            for (;;) {
                const uint64_t jw = lane < kOneJobWords ? sys_load64(&ctl->job[lane]) : 0ull;
                w = (uint32_t)jw;
                const uint32_t js = (uint32_t)(jw >> 32);
                const uint32_t s0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)js);
                const bool torn = __ballot(lane < kOneJobWords && js != s0) != 0;  // host mid-write
                if (!torn && s0 != done) { cmd = 1; seq = s0; break; }
                if (wg == 0) {
                    const uint32_t q = sys_load(&ctl->quit);
                    const uint64_t now = __builtin_amdgcn_s_memrealtime();
                    if (q || now - t_last > idle_ticks || now - t_start > life_ticks) {
                        if (lane == 0) __hip_atomic_store(&dv->stop, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                } else if (__hip_atomic_load(&dv->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) {
                    break;
                }
                __builtin_amdgcn_s_sleep(SRV_GAP);
            }
#endif
            if (lane < kOneJobWords) S.args[lane] = w;
            if (lane == 0) {
                S.cmd = cmd;
                S.seq = seq;
            }
        }
        __syncthreads();
        if (S.cmd != 1) break;
        // system-scope acquire (buffer_inv sc0 sc1): without it, survivor loads
        // of staging lines an earlier job read came back stale (a launched
        // kernel gets this invalidate from its dispatch)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        OneArgs a;
        {
            uint32_t w[kOneJobWords];
#pragma unroll
            for (int i = 0; i < kOneJobWords; ++i) w[i] = S.args[i];
            __builtin_memcpy(&a, w, sizeof(OneArgs));
        }
        a.seq = S.seq;
        mw_body(a, S, wg, (int)gridDim.x, ctl->flags);
        done = a.seq;
        t_last = __builtin_amdgcn_s_memrealtime();
        __syncthreads();  // S.args / S.cmd are rewritten by the next poll
    }
    if (tid == 0) {
        const uint32_t out = __hip_atomic_fetch_add(&dv->exited, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (out + 1 == gridDim.x) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            __hip_atomic_store(&ctl->exit_gen, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

}  // namespace

hipError_t launch_one_server(OneSrvCtl *ctl_dev, OneSrvDev *dv, const uint32_t *ptab, const uint8_t *gftab,
                             uint32_t gen, uint32_t done0, uint32_t idle_us, uint32_t life_ms, hipStream_t s) {
    hipError_t e = hipMemsetAsync(dv, 0, sizeof(OneSrvDev), s);
    if (e != hipSuccess) return e;
    k_one_server<<<kOneSrvWgs, kMwThreads, 0, s>>>(ctl_dev, dv, ptab, gftab, gen, done0, (uint64_t)idle_us * 100u,
                                                   (uint64_t)life_ms * 100000u);
    return hipGetLastError();
}

bool one_multi_ok(int k, int n, int len, int ss, int e) {  // e: the output rows of this call
    const int P = ((len + 15) & ~15) >> 4;
    const int pw = (P + kOneSrvWgs - 1) / kOneSrvWgs;
    return k >= 1 && k <= 64 && n > k && n <= 256 && e <= 10 && len >= 0 && ss >= ((len + 15) & ~15) &&
           ss % 16 == 0 && k * pw * 16 <= kMwSurv && e * 4 * pw <= kMwOut && e * k <= kMwCoef &&
           (int64_t)n * ss < (int64_t(1) << 31);
}

hipError_t launch_one_multi(const OneArgs &a, hipStream_t s) {
    k_one_multi<<<kOneSrvWgs, kMwThreads, 0, s>>>(a);
    return hipGetLastError();
}

bool one_group_ok(int k, int n, int len, int ss, bool encode) {
    const int m = n - k;
    const int e = encode ? m : (k < m ? k : m);  // output rows at most
    const int lpad = (len + 15) & ~15;
    const bool elim_ok = encode || (e + k <= 64 && e <= kRegRows) || e * (e + k) <= kAugMax;
    return k >= 1 && n > k && n <= 256 && len >= 0 && ss >= lpad && ss % 16 == 0 &&
           (int64_t)k * lpad <= kSurvLds && e * k <= kCoefMax && elim_ok &&
           (int64_t)n * ss < (int64_t(1) << 31);
}

hipError_t launch_one_group(const OneArgs &a, hipStream_t s) {
    k_one_group<<<1, kOneThreads, 0, s>>>(a);
    return hipGetLastError();
}

}  // namespace rsmi
