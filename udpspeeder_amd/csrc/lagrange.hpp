// lagrange.hpp -- decode coefficients in Lagrange form and their wave-level
// helpers, shared by the batched decode (decode.hip) and the one-group
// drop-in kernels (oneshot.hip).  Included inside namespace rsmi's
// anonymous namespace of each translation unit.
#pragma once

// ---- Lagrange form of the decode coefficients ------------------------------------
// fec_new's code is systematic Vandermonde (lib/fec.cpp:665-720): shard i is
// the value at the point x_i = (i ? alpha^(i-1) : 0) of the polynomial P of
// degree < k whose values at x_0..x_{k-1} are the data shards.  Any k
// survivors S fix P, so a missing data row d is
//     d = sum_{s in S} L_s(x_d) * shard_s,
//     L_s(x_d) = prod_{t in S, t != s} (x_d ^ x_t) / (x_s ^ x_t),
// and the matrix [L_s(x_d)] is the inverse fec_decode's Gauss-Jordan builds
// (lib/fec.cpp:795-825, 425-549): both are the unique left inverse of the
// survivors' rows of the encoding matrix, so the bytes are the same for any
// input, codeword or not.  In logs (lz: log with lz[0] = 0, so t = s drops out
// of every sum by itself):
//     log L_s(x_d) = A_d - lz[x_d ^ x_s] - B_s   (mod 255),
//     A_d = sum_{t in S} lz[x_d ^ x_t],   B_s = sum_{t in S} lz[x_s ^ x_t].
// Lane s computes B_s (k independent LDS byte lookups) and lz[x_d ^ x_s] for
// every missing row d; A_d is a wave sum of the latter (DPP, two rows packed
// per 32-bit sum).  The coefficient's v_perm split table is read straight by
// its log (tl01 / tl2 below), so no exp step and no pivot chain: a handful of
// independent lookups in place of e dependent elimination steps.  Every
// coefficient is nonzero (distinct points), so every one has a log.
constexpr int kLTabBytes = 5632;  // tl01[255] (4096) | tl2[255] (1024) | px[256] | lz[256]

struct LTables {
    const uint4 *t01;      // split table of alpha^v, v = 0..254 (T0lo T0hi T1lo T1hi)
    const uint32_t *t2;    // ... its T2
    const uint8_t *px;     // px[i] = x_i, the evaluation point of shard i
    const uint8_t *lz;     // lz[v] = log v, lz[0] = 0
};

// The image sits in gftab at kGfLtabOff (api.cpp init_device builds it):
// one independent 16-byte load per piece, no gftab -> ptab chain.
static_assert(kGfLtabBytes == kLTabBytes, "LTables image size");
__device__ __forceinline__ LTables load_ltables(uint8_t *smem, const uint32_t *,
                                                const uint8_t *gftab) {
    const uint4 *src = reinterpret_cast<const uint4 *>(gftab + kGfLtabOff);
    uint4 *dst = reinterpret_cast<uint4 *>(smem);
    for (int i = threadIdx.x; i < kLTabBytes / 16; i += blockDim.x) dst[i] = src[i];
    return LTables{reinterpret_cast<const uint4 *>(smem), reinterpret_cast<const uint32_t *>(smem + 4096),
                   smem + 5120, smem + 5376};
}

// Sum of x over the wave, in every lane's result (Kogge-Stone within each row
// of 16 lanes, then the row sums through row_bcast:15 / row_bcast:31).
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false); // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false); // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// B_s = sum_{t < k} lz[x_s ^ x_t] for lane s (xs: lane s holds x_s), in two
// chains of independent lookups.
__device__ __forceinline__ uint32_t lagrange_b(int k, uint32_t xs, const LTables &T) {
    uint32_t b0 = 0, b1 = 0;
    int t = 0;
    for (; t + 1 < k; t += 2) {
        const uint32_t x0 = (uint32_t)__builtin_amdgcn_readlane((int)xs, t);
        const uint32_t x1 = (uint32_t)__builtin_amdgcn_readlane((int)xs, t + 1);
        b0 += T.lz[xs ^ x0];
        b1 += T.lz[xs ^ x1];
    }
    if (t < k) b0 += T.lz[xs ^ (uint32_t)__builtin_amdgcn_readlane((int)xs, t)];
    return b0 + b1;
}

// log L_s(x_d) for the e <= NR rows d whose points lane d of xm holds; lane s
// < k (survivor s: point xs, B_s in B) gets store(r, v) with v the log of
// coefficient (row r, survivor s), 0..254.
template <int NR, class Store>
__device__ __forceinline__ void lagrange_rows(int k, int e, uint32_t xs, uint32_t B, uint32_t xm,
                                              const LTables &T, int lane, Store store) {
    const bool act = lane < k;
    // lz[x_d ^ x_s] of rows 2i and 2i + 1 packed in q[i] (each half <= 254,
    // and a wave sum of halves <= 64 * 254 < 2^16): A_d for two rows per sum
    constexpr int NQ = (NR + 1) / 2;
    uint32_t q[NQ], A[NQ];
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        q[i] = 0;
        A[i] = 0;
        if (2 * i < e) {
            const uint32_t x0 = (uint32_t)__builtin_amdgcn_readlane((int)xm, 2 * i);
            uint32_t v = T.lz[x0 ^ xs];
            if (2 * i + 1 < e) {
                const uint32_t x1 = (uint32_t)__builtin_amdgcn_readlane((int)xm, 2 * i + 1);
                v |= (uint32_t)T.lz[x1 ^ xs] << 16;
            }
            q[i] = act ? v : 0u;
            A[i] = wave_sum(q[i]);
        }
    }
    if (act) {
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            if (r < e) {
                const uint32_t sh = (r & 1) * 16;
                const uint32_t a = (A[r >> 1] >> sh) & 0xFFFFu, l = (q[r >> 1] >> sh) & 0xFFFFu;
                // A + 255 * 64 - l - B > 0 (l + B <= 64 * 254), then mod 255
                uint32_t v = a + 255u * 64u - l - B;
                v = (v & 255u) + (v >> 8);       // <= 255 + 127
                v = (v & 255u) + (v >> 8);       // <= 255
                v = min(v, v - 255u);            // 255 -> 0
                store(r, v);
            }
        }
    }
}
