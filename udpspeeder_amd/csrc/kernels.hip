// kernels.hip -- generic GF(2^8) Reed-Solomon kernels for gfx950 (CDNA4).
//
// The byte arithmetic is the reference's dst ^= c * src (addmul1,
// lib/fec.cpp:336-376), batched over many FEC groups.  A GF multiply by a
// wave-uniform constant c is done 4 bytes at a time with v_perm_b32 on
// 3-bit slices of each byte:
//     c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6]
// (GF multiplication is linear over GF(2)), where T0/T1 are 8-entry byte
// tables held in two dwords (v_perm selects from {S0:S1}) and T2 a 4-entry
// table in one dword; the three partial products and the accumulator are
// combined with v_bitop3_b32 (3-input XOR).  The 256 possible tables live in
// LDS (8 KB) and are read with wave-uniform (broadcast) addresses.
//
// Work unit: one wavefront per (group, column tile) -- a tile spans
// 64 lanes x 4W bytes of every shard of the group -- so the coefficients are
// wave-uniform even when every group has its own decode matrix.  The hot
// uniform encode (RS(20,10)) additionally has a bit-sliced, build-time
// specialised kernel (bitslice.hip).
#include "rsmi_internal.hpp"

namespace rsmi {

namespace {

constexpr int kRB = 10;  // output rows accumulated per pass over the inputs

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ int wave_id_uniform() {
    return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

// Load the 256 x {T0lo,T0hi,T1lo,T1hi} and 256 x T2 tables into LDS.
__device__ __forceinline__ void load_ptab(const uint32_t *ptab, uint4 *s01, uint32_t *s2) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        const uint4 *src = reinterpret_cast<const uint4 *>(ptab + i * kPtabDwords);
        s01[i] = src[0];
        s2[i] = ptab[i * kPtabDwords + 4];
    }
    __syncthreads();
}

struct TileJob {
    uint8_t *gbase;           // shard 0 of the group
    int64_t sstride;
    int len, k, rows;
    const uint8_t *in_slots;  // nullptr: input j is slot j
    const uint8_t *out_slots; // nullptr: output r is slot k + r
    const uint8_t *coef;      // rows x k, row-major
};

// One wave: out[r] = sum_j coef[r][j] * in[j] over the lane's 4W bytes.
template <int W>
__device__ __forceinline__ void apply_tile(const TileJob &J, int tile_off, const uint4 *s01,
                                           const uint32_t *s2) {
    const int lane = threadIdx.x & 63;
    const int off = tile_off + lane * (4 * W);
    int nw = (J.len - off + 3) >> 2;  // words holding at least one payload byte
    nw = nw < 0 ? 0 : (nw > W ? W : nw);
    for (int rb = 0; rb < J.rows; rb += kRB) {
        const int nr = (J.rows - rb) < kRB ? (J.rows - rb) : kRB;
        uint32_t acc[kRB][W];
#pragma unroll
        for (int r = 0; r < kRB; ++r)
#pragma unroll
            for (int w = 0; w < W; ++w) acc[r][w] = 0;
        for (int j = 0; j < J.k; ++j) {
            const int slot = J.in_slots ? J.in_slots[j] : j;
            const uint32_t *src =
                reinterpret_cast<const uint32_t *>(J.gbase + slot * J.sstride + off);
            uint32_t x[W];
            if (nw == W) {
#pragma unroll
                for (int w = 0; w < W; ++w) x[w] = src[w];
            } else {
#pragma unroll
                for (int w = 0; w < W; ++w) x[w] = (w < nw) ? src[w] : 0u;
            }
            uint32_t q0[W], q1[W], q2[W];
#pragma unroll
            for (int w = 0; w < W; ++w) {
                q0[w] = x[w] & 0x07070707u;
                q1[w] = (x[w] >> 3) & 0x07070707u;
                q2[w] = (x[w] >> 6) & 0x03030303u;
            }
            const uint8_t *crow = J.coef + (size_t)rb * J.k + j;
#pragma unroll
            for (int r = 0; r < kRB; ++r) {
                if (r < nr) {
                    const uint32_t c = crow[(size_t)r * J.k];
                    if (c) {
                        const uint4 t = s01[c];
                        const uint32_t t2 = s2[c];
#pragma unroll
                        for (int w = 0; w < W; ++w) {
                            const uint32_t p0 = __builtin_amdgcn_perm(t.y, t.x, q0[w]);
                            const uint32_t p1 = __builtin_amdgcn_perm(t.w, t.z, q1[w]);
                            const uint32_t p2 = __builtin_amdgcn_perm(t2, t2, q2[w]);
                            acc[r][w] = acc[r][w] ^ xor3(p0, p1, p2);
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int r = 0; r < kRB; ++r) {
            if (r < nr) {
                const int slot = J.out_slots ? J.out_slots[rb + r] : J.k + rb + r;
                uint32_t *dst = reinterpret_cast<uint32_t *>(J.gbase + slot * J.sstride + off);
#pragma unroll
                for (int w = 0; w < W; ++w)
                    if (w < nw) dst[w] = acc[r][w];
            }
        }
    }
}

template <int W>
__global__ __launch_bounds__(256) void k_encode_generic(UniformArgs a, const uint8_t *parity_rows,
                                                        const uint32_t *ptab) {
    __shared__ uint4 s01[256];
    __shared__ uint32_t s2[256];
    load_ptab(ptab, s01, s2);
    const int64_t items = a.ngroups * a.tiles;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    for (int64_t it = (int64_t)blockIdx.x * 4 + wave_id_uniform(); it < items; it += nwaves) {
        const int64_t g = it / a.tiles;
        const int tile = (int)(it - g * a.tiles);
        TileJob J{a.base + g * a.group_stride, a.shard_stride, a.len, a.k, a.n - a.k,
                  nullptr, nullptr, parity_rows};
        apply_tile<W>(J, tile * 256 * W, s01, s2);
    }
}

template <int W>
__global__ __launch_bounds__(256) void k_decode_apply(UniformArgs a, const uint8_t *plans,
                                                      const uint32_t *ptab) {
    __shared__ uint4 s01[256];
    __shared__ uint32_t s2[256];
    load_ptab(ptab, s01, s2);
    const int m = a.n - a.k;
    const PlanLayout L(a.k, a.k < m ? a.k : m);
    const int64_t items = a.ngroups * a.tiles;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    for (int64_t it = (int64_t)blockIdx.x * 4 + wave_id_uniform(); it < items; it += nwaves) {
        const int64_t g = it / a.tiles;
        const int tile = (int)(it - g * a.tiles);
        const uint8_t *plan = plans + g * L.stride;
        const int status = *reinterpret_cast<const int32_t *>(plan);
        const int e = plan[4];
        if (status != RSMI_DEC_OK || e == 0) continue;
        TileJob J{a.base + g * a.group_stride, a.shard_stride, a.len, a.k, e,
                  plan + 8, plan + 8 + a.k, plan + L.coef_off};
        apply_tile<W>(J, tile * 256 * W, s01, s2);
    }
}

// ---- decode plans: one wavefront per group --------------------------------
// Selection = first k present shards in ascending order (lib/rs.cpp:24-39).
// With E = missing data rows (|E| = e) and R = the e parity rows selected,
// d_E = A^-1 (p_R + B d_P), A = enc[R][E], B = enc[R][P].  Gauss-Jordan on the
// augmented [A | M] (M's column per survivor: unit vector for a parity
// survivor, enc[R][s] for a data survivor) leaves [I | coef].  The inverse is
// unique, so coef equals the rows fec_decode derives (fec.cpp:795-825, 861-868).
__device__ __forceinline__ uint8_t gmul_lds(const uint8_t *lexp, const uint8_t *llog, uint32_t a,
                                            uint32_t b) {
    return (a && b) ? lexp[llog[a] + llog[b]] : 0;
}

__global__ __launch_bounds__(64) void k_decode_plan(UniformArgs a, const uint8_t *present,
                                                    const uint8_t *parity_rows, uint8_t *plans,
                                                    int32_t *status_out, const uint8_t *gftab) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *lexp = smem;          // 512
    uint8_t *llog = smem + 512;    // 256
    uint8_t *lsel = smem + 768;    // 256
    uint8_t *lmiss = smem + 1024;  // 256
    uint8_t *aug = smem + 1280;    // emax * (emax + k)
    const int lane = threadIdx.x;
    const int k = a.k, n = a.n, m = n - k;
    const PlanLayout L(k, k < m ? k : m);
    for (int i = lane; i < 768; i += 64) smem[i] = gftab[i];
    __syncthreads();
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int64_t g = blockIdx.x; g < a.ngroups; g += gridDim.x) {
        const uint8_t *pr = present + g * n;
        uint8_t *plan = plans + g * L.stride;
        int cnt = 0;
        for (int b = 0; b < n && cnt < k; b += 64) {
            const int idx = b + lane;
            const bool f = idx < n && pr[idx] != 0;
            const uint64_t mk = __ballot(f);
            const int rank = cnt + __popcll(mk & lt);
            if (f && rank < k) lsel[rank] = (uint8_t)idx;
            cnt += __popcll(mk);
        }
        int st = RSMI_DEC_OK;
        int e = 0;
        if (cnt < k) {
            st = RSMI_DEC_TOO_FEW;
        } else {
            for (int b = 0; b < k; b += 64) {
                const int idx = b + lane;
                const bool ms = idx < k && pr[idx] == 0;
                const uint64_t mk = __ballot(ms);
                if (ms) lmiss[e + __popcll(mk & lt)] = (uint8_t)idx;
                e += __popcll(mk);
            }
        }
        __syncthreads();
        if (st == RSMI_DEC_OK && e > 0) {
            const int W = e + k;
            for (int t = lane; t < e * W; t += 64) {
                const int r = t / W, c = t - r * W;
                const int R = lsel[k - e + r];
                const uint8_t *prow = parity_rows + (size_t)(R - k) * k;
                uint8_t v;
                if (c < e) {
                    v = prow[lmiss[c]];
                } else {
                    const int s = lsel[c - e];
                    v = (s >= k) ? (uint8_t)(s == R) : prow[s];
                }
                aug[t] = v;
            }
            __syncthreads();
            for (int p = 0; p < e; ++p) {
                const uint32_t piv = aug[p * W + p];
                if (piv == 0) { st = RSMI_DEC_SINGULAR; break; }
                const uint32_t ipiv = lexp[255 - llog[piv]];
                for (int c = p + 1 + lane; c < W; c += 64)
                    aug[p * W + c] = gmul_lds(lexp, llog, ipiv, aug[p * W + c]);
                __syncthreads();
                const int cols = W - p - 1;
                for (int t = lane; t < e * cols; t += 64) {
                    const int r = t / cols;
                    if (r == p) continue;
                    const int c = p + 1 + (t - r * cols);
                    const uint32_t f = aug[r * W + p];
                    if (f) aug[r * W + c] ^= gmul_lds(lexp, llog, f, aug[p * W + c]);
                }
                __syncthreads();
            }
            if (st == RSMI_DEC_OK) {
                for (int t = lane; t < e * k; t += 64) {
                    const int r = t / k, c = t - r * k;
                    plan[L.coef_off + t] = aug[r * W + e + c];
                }
                for (int t = lane; t < k; t += 64) plan[8 + t] = lsel[t];
                for (int t = lane; t < e; t += 64) plan[8 + k + t] = lmiss[t];
            }
        }
        if (lane == 0) {
            *reinterpret_cast<int32_t *>(plan) = st;
            plan[4] = (uint8_t)(st == RSMI_DEC_OK ? e : 0);
            if (status_out) status_out[g] = st;
        }
        __syncthreads();
    }
}

// ---- the reference's placement after a two-kernel decode --------------------
// k_decode_apply rebuilt each missing data row in its own slot; fec_decode
// leaves it in the buffer of the parity survivor its shuffle moves into data[i]
// (fec.cpp:755-788, 872-877; ref_slot_of).  One wave per group moves the rows
// there (16-byte pieces up to round_up(len, 16), inside the slot padding) and
// writes the group's slot map (0xFF: an erased row of a group with too few).
__global__ __launch_bounds__(64) void k_decode_ref_move(UniformArgs a, const uint8_t *plans,
                                                        const uint8_t *present, uint8_t *slot_map) {
    const int k = a.k, m = a.n - a.k, lane = threadIdx.x;
    const PlanLayout L(k, k < m ? k : m);
    const int pieces = (a.len + 15) >> 4;
    for (int64_t g = blockIdx.x; g < a.ngroups; g += gridDim.x) {
        const uint8_t *plan = plans + g * L.stride;
        const int st = *reinterpret_cast<const int32_t *>(plan);
        const int e = st == RSMI_DEC_OK ? plan[4] : 0;
        const uint8_t *sel = plan + 8, *miss = plan + 8 + k;
        uint8_t *gb = a.base + g * a.group_stride;
        for (int r = 0; r < e; ++r) {
            const uint4 *src = reinterpret_cast<const uint4 *>(gb + miss[r] * a.shard_stride);
            uint4 *dst = reinterpret_cast<uint4 *>(gb + ref_slot_of(k, e, sel, miss[r]) * a.shard_stride);
            for (int p = lane; p < pieces; p += 64) dst[p] = src[p];
        }
        if (slot_map) {
            for (int i = lane; i < k; i += 64) {
                uint8_t v = present[g * a.n + i] ? (uint8_t)i : (uint8_t)0xFF;
                if (v == 0xFF && e > 0) v = (uint8_t)ref_slot_of(k, e, sel, i);
                slot_map[g * k + i] = v;
            }
        }
    }
}

// ---- ragged encode: one wavefront per group, tile width chosen per group ----
__global__ __launch_bounds__(256) void k_encode_ragged(const rsmi_group *groups, int64_t ngroups,
                                                       uint8_t *base, const uint64_t *code_dir,
                                                       const uint32_t *ptab) {
    __shared__ uint4 s01[256];
    __shared__ uint32_t s2[256];
    load_ptab(ptab, s01, s2);
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    for (int64_t g = (int64_t)blockIdx.x * 4 + wave_id_uniform(); g < ngroups; g += nwaves) {
        const rsmi_group d = groups[g];
        const int k = d.k, n = d.n;
        if (k < 1 || n <= k || n > 256) continue;
        const uint8_t *rows = reinterpret_cast<const uint8_t *>(code_dir[k * 257 + n]);
        if (!rows) continue;
        TileJob J{base + d.offset, (int64_t)d.shard_stride, (int)d.len, k, n - k,
                  nullptr, nullptr, rows};
        const int len = (int)d.len;
        if (len <= 256) {
            apply_tile<1>(J, 0, s01, s2);
        } else if (len <= 512) {
            apply_tile<2>(J, 0, s01, s2);
        } else if (len <= 768) {
            apply_tile<3>(J, 0, s01, s2);
        } else if (len <= 1024) {
            apply_tile<4>(J, 0, s01, s2);
        } else {
            for (int off = 0; off < len; off += 1280) apply_tile<5>(J, off, s01, s2);
        }
    }
}

// ---- synthetic SplitMix64 data ---------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_fill_data(int k, int len, uint8_t *base, int64_t gs,
                                                   int64_t ss, int64_t g0, int64_t ngroups,
                                                   uint64_t seed) {
    const int wpr = (len + 3) >> 2;  // words per shard row
    const int64_t total = ngroups * k * (int64_t)wpr;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = t / ((int64_t)k * wpr);
        const int rem = (int)(t - g * k * wpr);
        const int j = rem / wpr, w = rem - j * wpr;
        const uint64_t s0 = seed ^ (uint64_t)(g0 + g);
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int off = 4 * w + b;
            if (off < len) {
                const uint64_t q = (uint64_t)j * len + off;
                const uint64_t word = mix64(s0 + (q / 8 + 1) * 0x9E3779B97F4A7C15ull);
                v |= (uint32_t)((word >> (8 * (q % 8))) & 0xFF) << (8 * b);
            }
        }
        *reinterpret_cast<uint32_t *>(base + g * gs + j * ss + 4 * w) = v;
    }
}

// ragged fill: one block per group (grid-stride), data rows of group g get
// stream (seed ^ (g0 + g)) laid out like k_fill_data.
__global__ __launch_bounds__(256) void k_fill_ragged(const rsmi_group *groups, int64_t ngroups,
                                                     uint8_t *base, int64_t g0, uint64_t seed) {
    for (int64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
        const rsmi_group d = groups[g];
        const int len = (int)d.len, k = d.k;
        const int wpr = (len + 3) >> 2;
        const uint64_t s0 = seed ^ (uint64_t)(g0 + g);
        for (int t = threadIdx.x; t < k * wpr; t += blockDim.x) {
            const int j = t / wpr, w = t - j * wpr;
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int off = 4 * w + b;
                if (off < len) {
                    const uint64_t q = (uint64_t)j * len + off;
                    const uint64_t word = mix64(s0 + (q / 8 + 1) * 0x9E3779B97F4A7C15ull);
                    v |= (uint32_t)((word >> (8 * (q % 8))) & 0xFF) << (8 * b);
                }
            }
            *reinterpret_cast<uint32_t *>(base + d.offset + (int64_t)j * d.shard_stride + 4 * w) = v;
        }
    }
}

// ---- measured copy peak and read:write mixes (bench.py's hbm_copy_peak) -------
// A wave moves U (or R) 16-byte words per lane from one contiguous range of
// its own, 1 KiB per instruction (a block-strided layout, words 4 KiB apart
// per thread, measured 27 % slower at 8 words per thread: each wave's loads
// then fall 4 KiB apart); every load is issued before the first store; NT:
// nontemporal loads and stores.  nbytes % 16 == 0; the tail checks each word.
typedef uint32_t cp_word __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy_peak(cp_word *__restrict__ dst, const cp_word *__restrict__ src,
                                                   int64_t nwords) {
    const int64_t w0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 * U) + (threadIdx.x & 63);
    cp_word v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t w = w0 + u * 64;
        if (w < nwords) v[u] = NT ? __builtin_nontemporal_load(src + w) : src[w];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t w = w0 + u * 64;
        if (w < nwords) {
            if (NT) __builtin_nontemporal_store(v[u], dst + w);
            else dst[w] = v[u];
        }
    }
}

// Read:write mixes: each lane reads R words (its wave's contiguous range, as
// above) and writes W, each the XOR of a share of what it read (W = 0: nothing
// is written unless the XOR of all R words is the sentinel, which synthetic
// input never holds).  Nontemporal, like the codec kernels' streams.  Whole
// blocks only (the host rounds the read size down).
template <int R, int W>
__global__ __launch_bounds__(256) void k_mix_peak(cp_word *__restrict__ dst, const cp_word *__restrict__ src) {
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t r0 = wave * (64 * R) + lane;
    cp_word v[R];
#pragma unroll
    for (int u = 0; u < R; ++u) v[u] = __builtin_nontemporal_load(src + r0 + u * 64);
    if (W == 0) {
        cp_word x = v[0];
#pragma unroll
        for (int u = 1; u < R; ++u) x ^= v[u];
        if (x.x == 0x9E3779B9u && x.y == 0x7F4A7C15u && x.z == 0xF39CC060u && x.w == 0x5CEDC834u)
            dst[lane] = x;
        return;
    }
    const int64_t w0 = wave * (64 * W) + lane;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        cp_word x = v[w];
#pragma unroll
        for (int u = w + W; u < R; u += W) x ^= v[u];
        __builtin_nontemporal_store(x, dst + w0 + w * 64);
    }
}

int grid_for(int64_t waves) {
    int64_t blocks = (waves + 3) / 4;
    const int64_t cap = 256 * 8;  // ~8 resident 256-thread blocks per CU
    if (blocks > cap) blocks = cap;
    return blocks < 1 ? 1 : (int)blocks;
}

}  // namespace

hipError_t launch_encode_generic(const UniformArgs &a, int W, const uint8_t *parity_rows,
                                 const uint32_t *ptab, hipStream_t s) {
    const int grid = grid_for(a.ngroups * a.tiles);
    switch (W) {
        case 1: k_encode_generic<1><<<grid, 256, 0, s>>>(a, parity_rows, ptab); break;
        case 2: k_encode_generic<2><<<grid, 256, 0, s>>>(a, parity_rows, ptab); break;
        case 3: k_encode_generic<3><<<grid, 256, 0, s>>>(a, parity_rows, ptab); break;
        case 4: k_encode_generic<4><<<grid, 256, 0, s>>>(a, parity_rows, ptab); break;
        default: k_encode_generic<5><<<grid, 256, 0, s>>>(a, parity_rows, ptab); break;
    }
    return hipGetLastError();
}

hipError_t launch_decode_plan(const UniformArgs &a, const uint8_t *present,
                              const uint8_t *parity_rows, uint8_t *plans, int32_t *status,
                              const uint8_t *gftab, hipStream_t s) {
    const int m = a.n - a.k;
    const int emax = a.k < m ? a.k : m;
    const size_t lds = 1280 + (size_t)emax * (emax + a.k);
    int64_t grid = a.ngroups < 256 * 16 ? a.ngroups : 256 * 16;
    if (grid < 1) grid = 1;
    k_decode_plan<<<(int)grid, 64, lds, s>>>(a, present, parity_rows, plans, status, gftab);
    return hipGetLastError();
}

hipError_t launch_decode_apply(const UniformArgs &a, int W, const uint8_t *plans,
                               const uint32_t *ptab, hipStream_t s) {
    const int grid = grid_for(a.ngroups * a.tiles);
    switch (W) {
        case 1: k_decode_apply<1><<<grid, 256, 0, s>>>(a, plans, ptab); break;
        case 2: k_decode_apply<2><<<grid, 256, 0, s>>>(a, plans, ptab); break;
        case 3: k_decode_apply<3><<<grid, 256, 0, s>>>(a, plans, ptab); break;
        case 4: k_decode_apply<4><<<grid, 256, 0, s>>>(a, plans, ptab); break;
        default: k_decode_apply<5><<<grid, 256, 0, s>>>(a, plans, ptab); break;
    }
    return hipGetLastError();
}

hipError_t launch_decode_ref_move(const UniformArgs &a, const uint8_t *plans, const uint8_t *present,
                                  uint8_t *slot_map, hipStream_t s) {
    int64_t grid = a.ngroups < 256 * 16 ? a.ngroups : 256 * 16;
    if (grid < 1) grid = 1;
    k_decode_ref_move<<<(int)grid, 64, 0, s>>>(a, plans, present, slot_map);
    return hipGetLastError();
}

hipError_t launch_copy_peak(uint8_t *dst, const uint8_t *src, int64_t nbytes, int variant, hipStream_t s) {
    const int64_t nw = nbytes / 16;
    if (variant >= 4) {  // read:write mixes, nbytes read
        auto d = reinterpret_cast<cp_word *>(dst);
        auto r = reinterpret_cast<const cp_word *>(src);
        switch (variant) {
            case 4: k_mix_peak<4, 0><<<(unsigned)(nw / (256 * 4)), 256, 0, s>>>(d, r); break;
            case 5: k_mix_peak<4, 2><<<(unsigned)(nw / (256 * 4)), 256, 0, s>>>(d, r); break;
            default: k_mix_peak<6, 1><<<(unsigned)(nw / (256 * 6)), 256, 0, s>>>(d, r); break;
        }
        return hipGetLastError();
    }
    const int U = (variant & 1) ? 8 : 4;
    const int64_t grid = (nw + 256 * U - 1) / (256 * U);
    auto d = reinterpret_cast<cp_word *>(dst);
    auto r = reinterpret_cast<const cp_word *>(src);
    switch (variant) {
        case 0: k_copy_peak<4, false><<<(unsigned)grid, 256, 0, s>>>(d, r, nw); break;
        case 1: k_copy_peak<8, false><<<(unsigned)grid, 256, 0, s>>>(d, r, nw); break;
        case 2: k_copy_peak<4, true><<<(unsigned)grid, 256, 0, s>>>(d, r, nw); break;
        default: k_copy_peak<8, true><<<(unsigned)grid, 256, 0, s>>>(d, r, nw); break;
    }
    return hipGetLastError();
}

hipError_t launch_encode_ragged(const rsmi_group *groups, int64_t ngroups, uint8_t *base,
                                const uint64_t *code_dir, const uint32_t *ptab, hipStream_t s) {
    const int grid = grid_for(ngroups);
    k_encode_ragged<<<grid, 256, 0, s>>>(groups, ngroups, base, code_dir, ptab);
    return hipGetLastError();
}

hipError_t launch_fill_data(int k, int len, uint8_t *base, int64_t group_stride,
                            int64_t shard_stride, int64_t g0, int64_t ngroups, uint64_t seed,
                            hipStream_t s) {
    const int64_t total = ngroups * k * (int64_t)((len + 3) / 4);
    int64_t grid = (total + 255) / 256;
    if (grid > 256 * 32) grid = 256 * 32;
    if (grid < 1) grid = 1;
    k_fill_data<<<(int)grid, 256, 0, s>>>(k, len, base, group_stride, shard_stride, g0, ngroups,
                                          seed);
    return hipGetLastError();
}

hipError_t launch_fill_ragged(const rsmi_group *groups, int64_t ngroups, uint8_t *base,
                              int64_t g0, uint64_t seed, hipStream_t s) {
    const int64_t grid = ngroups < 256 * 32 ? ngroups : 256 * 32;
    k_fill_ragged<<<(int)(grid < 1 ? 1 : grid), 256, 0, s>>>(groups, ngroups, base, g0, seed);
    return hipGetLastError();
}

}  // namespace rsmi
