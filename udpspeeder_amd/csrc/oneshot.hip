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

__global__ __launch_bounds__(kOneThreads) void k_one_group(OneArgs a) {
    __shared__ uint4 s01[256];
    __shared__ uint32_t s2[256];
    __shared__ uint8_t lexp[512], llog[256], linv[256];
    __shared__ uint8_t sel[256], miss[256];
    __shared__ uint4 ct01[kCoefMax];  // coefficient (r, j)'s split table at r * k + j
    __shared__ uint32_t ct2[kCoefMax];
    __shared__ uint8_t aug[kAugMax];
    __shared__ __attribute__((aligned(16))) uint8_t xs[kSurvLds];  // survivor j at j * lpad
    __shared__ int s_e, s_st;
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

}  // namespace

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
