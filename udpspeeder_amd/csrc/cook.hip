// cook.hip -- batched packet cook / de_cook for gfx950.
//
// Semantics: packet.cpp do_cook (:303-308) and de_cook (:310-326), see
// include/rsmi_cook.h.  One half-wave (32 lanes) owns one packet; a lane owns a
// 48-byte chunk (three 16-byte pieces) of each 1536-byte round of it.
//
// The transform is byte-parallel: piece P of the output is the input piece
// XOR a key-stream window (KS[p] = key[p % strlen(key)], precomputed per
// context, read 16-B aligned from L1/L2) XOR an IV window (the packet's IV
// repeated in LDS, read as five dwords and funnel-shifted by P mod iv_len).
//
// CRC-32 (packet.cpp:236-257) is the only serial part.  Raw CRC (register init
// 0, no final xor) is linear, with Z_d = "feed d zero bytes" a linear map on
// the 32-bit register:
//   * each lane folds its chunk with slicing-by-8 (8 x 256-word LDS tables);
//   * lane l's value is shifted to the round end by Z_{48(31-l)} and the 32
//     lanes XOR-reduce with ds_swizzle (no lookups in the reduction);
//   * rounds chain through Z_1536;
//   * the message is zero-padded to whole rounds, so the result is finally
//     un-shifted by Z_{-z} (z = padded - len) -- three nibble-table maps for
//     the three hex digits of z.
// crc32h's init ~0 is folded in by complementing the first 4 bytes of the
// zero-padded message, its final ~ at the end.  Linear maps are applied as
// eight 16-entry nibble tables (512 B per map) so all of them fit in LDS.
//
// Cook writes pieces wholly below len as it goes; the (at most four) pieces
// that hold the appended crc/iv/iv_len tail are rebuilt after the CRC is known,
// from a 64-byte per-packet overlay in LDS.  De_cook reads the IV and the
// stored crc first, then writes every piece in its single pass.
#include "rsmi_internal.hpp"
#include "../../include/rsmi_cook.h"

namespace rsmi {
namespace {

constexpr int kThreads = 512;           // 8 waves = 16 packets in flight per block
constexpr int kChunk = 48;              // bytes per lane per round
constexpr int kRound = 32 * kChunk;     // 1536
constexpr int kScr = 368;               // per-packet LDS: iv2[288] | overlay[64] | misc[16]

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));  // packet pieces: 4-byte aligned

__device__ __forceinline__ u32x4 ld_piece(const uint8_t *p) {
    return *reinterpret_cast<const u32x4_a4 *>(p);
}
__device__ __forceinline__ void st_piece(uint8_t *p, u32x4 v) {
    *reinterpret_cast<u32x4_a4 *>(p) = v;
}

// CRC register after 8 bytes (dwords a, b little-endian) from register c.
__device__ __forceinline__ uint32_t slice8(const uint32_t *T, uint32_t c, uint32_t a, uint32_t b) {
    const uint32_t x = c ^ a;
    uint32_t r = xor3(T[7 * 256 + (x & 0xff)], T[6 * 256 + ((x >> 8) & 0xff)],
                      T[5 * 256 + ((x >> 16) & 0xff)]);
    r = xor3(r, T[4 * 256 + (x >> 24)], T[3 * 256 + (b & 0xff)]);
    r = xor3(r, T[2 * 256 + ((b >> 8) & 0xff)], T[256 + ((b >> 16) & 0xff)]);
    return r ^ T[b >> 24];
}

// A linear map of the CRC register held as 8 nibble tables of 16 words.
__device__ __forceinline__ uint32_t nib_map(const uint32_t *M, uint32_t c) {
    uint32_t r = xor3(M[c & 15], M[16 + ((c >> 4) & 15)], M[32 + ((c >> 8) & 15)]);
    r = xor3(r, M[48 + ((c >> 12) & 15)], M[64 + ((c >> 16) & 15)]);
    r = xor3(r, M[80 + ((c >> 20) & 15)], M[96 + ((c >> 24) & 15)]);
    return r ^ M[112 + (c >> 28)];
}

// XOR over the 32 lanes of this half-wave (ds_swizzle xor-mode stays in 32 lanes).
__device__ __forceinline__ uint32_t half_xor(uint32_t c) {
    c ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)c, 0x041F);
    c ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)c, 0x081F);
    c ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)c, 0x101F);
    c ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)c, 0x201F);
    c ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)c, 0x401F);
    return c;
}

// Byte masks of a 16-byte piece whose first v bytes are selected.
__device__ __forceinline__ u32x4 piece_mask(int v) {
    u32x4 m;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int nb = v - 4 * d;
        m[d] = nb >= 4 ? ~0u : (nb <= 0 ? 0u : ((1u << (8 * nb)) - 1u));
    }
    return m;
}

// IV bytes iv[(pos + t) % ivl], t = 0..15, from the repeated IV in LDS.
__device__ __forceinline__ u32x4 iv_window(const uint32_t *iv2w, uint32_t pos, uint32_t ivl,
                                           uint32_t magic) {
    uint32_t r = pos - __umulhi(pos, magic) * ivl;
    if (r >= ivl) r -= ivl;
    const uint32_t *w = iv2w + (r >> 2);
    const uint32_t sh = r & 3;
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
    return u32x4{__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                 __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
}

__device__ __forceinline__ uint32_t mod_ivl(uint32_t pos, uint32_t ivl, uint32_t magic) {
    uint32_t r = pos - __umulhi(pos, magic) * ivl;
    return r >= ivl ? r - ivl : r;
}

__device__ __forceinline__ uint64_t splitmix(uint64_t seed, uint64_t idx, uint64_t w) {
    uint64_t z = (seed ^ idx) + (w + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t unshift(const uint32_t *U, uint32_t c, uint32_t z) {
    c = nib_map(U + 128 * (z & 15), c);
    c = nib_map(U + 128 * (16 + ((z >> 4) & 15)), c);
    return nib_map(U + 128 * (32 + (z >> 8)), c);
}

__device__ __forceinline__ int round16(int x) { return (x + 15) & ~15; }

__device__ __forceinline__ void load_tables(uint32_t *lds, const uint32_t *tabs) {
    for (int i = threadIdx.x; i < kCookTabWords / 4; i += kThreads)
        reinterpret_cast<u32x4 *>(lds)[i] = reinterpret_cast<const u32x4 *>(tabs)[i];
    __syncthreads();
}

// Uniform loop bound for the two packets of a wave.
__device__ __forceinline__ int wave_max(int v) {
    const int a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 32);
    return a > b ? a : b;
}

__global__ __launch_bounds__(kThreads) void k_cook(CookArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const bool ck = !(a.flags & RSMI_COOK_NO_CHECKSUM);
    const bool obs = !(a.flags & RSMI_COOK_NO_OBSCURE);
    const bool kx = a.ks != nullptr;
    if (ck) load_tables(lds, a.tabs);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, half = lane >> 5, hl = lane & 31;
    uint8_t *scr = reinterpret_cast<uint8_t *>(lds + kCookTabWords) + (wid * 2 + half) * kScr;
    uint32_t *iv2w = reinterpret_cast<uint32_t *>(scr);
    uint8_t *ovl = scr + 288;
    const uint32_t *T = lds;
    const int64_t npairs = (a.count + 1) >> 1;

    for (int64_t pw = (int64_t)blockIdx.x * (kThreads / 64) + wid; pw < npairs;
         pw += (int64_t)gridDim.x * (kThreads / 64)) {
        const int64_t pk = 2 * pw + half;
        const bool have = pk < a.count;
        int L = -1, ivl = 0;
        uint8_t *pkt = nullptr;
        uint64_t iw0 = 0;
        if (have) {
            L = a.len[pk];
            pkt = a.base + (a.offset ? a.offset[pk] : (uint64_t)pk * (uint64_t)a.stride);
            if (obs) {
                if (a.iv) {
                    ivl = a.iv_len[pk];
                } else {
                    iw0 = splitmix(a.seed, (uint64_t)pk, 0);
                    ivl = 4 + (int)(iw0 % 29u);
                }
            }
        }
        const int out = L + (ck ? 4 : 0) + (obs ? ivl + 1 : 0);
        const bool ok = have && L >= 0 && L <= RSMI_COOK_MAX_LEN && ivl <= RSMI_COOK_IV_MAX &&
                        round16(out) <= a.cap && ((uintptr_t)pkt & 3) == 0;
        const int ext = ok ? round16(out) : 0;
        if (ok && ivl) {  // iv repeated: iv2[t] = iv[t % ivl], t < ivl + 20
            for (int t = hl; t < ivl + 20; t += 32) {
                const int j = t % ivl;
                uint8_t b;
                if (a.iv)
                    b = a.iv[pk * RSMI_COOK_IV_MAX + j];
                else
                    b = (uint8_t)(splitmix(a.seed, (uint64_t)pk, 1 + (j >> 3)) >> (8 * (j & 7)));
                scr[t] = b;
            }
        }
        wave_sync();
        const uint32_t magic = ivl ? 0xFFFFFFFFu / (uint32_t)ivl : 0u;
        const int nr = (ext + kRound - 1) / kRound;
        const int nrm = wave_max(nr);
        uint32_t acc = 0;
        for (int r = 0; r < nrm; ++r) {
            uint32_t c = 0;
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const int P = r * kRound + hl * kChunk + p * 16;
                u32x4 d = {0, 0, 0, 0};
                if (P < ext) d = ld_piece(pkt + P);
                if (ck) {
                    u32x4 ci = d & piece_mask(L - P);
                    if (P == 0) ci.x = ~ci.x;
                    c = slice8(T, c, ci.x, ci.y);
                    c = slice8(T, c, ci.z, ci.w);
                }
                if (P < ext && P + 16 <= L) {  // wholly payload: obscure + xor, store now
                    u32x4 m = kx ? *reinterpret_cast<const u32x4 *>(a.ks + P) : u32x4{0, 0, 0, 0};
                    if (ivl) m ^= iv_window(iv2w, (uint32_t)P, (uint32_t)ivl, magic);
                    st_piece(pkt + P, d ^ m);
                }
            }
            if (ck) {  // the partner packet may need more rounds: only own rounds count
                c = half_xor(nib_map(T + kCookLane + 128 * hl, c));
                const uint32_t nacc = nib_map(T + kCookRound, acc) ^ c;
                acc = r < nr ? nacc : acc;
            }
        }
        uint32_t crc = 0;
        if (ck) crc = ~unshift(T + kCookUns, acc, (uint32_t)(nr * kRound - L));
        // ---- tail: crc (BE), iv, iv_len appended after the payload -------------
        const int P0 = L & ~15;
        if (ok) {
            for (int t = hl; t < 64; t += 32) {
                const int pos = P0 + t;
                uint32_t v = 0;
                if (pos >= L && pos < out) {
                    const int u = pos - L;
                    if (ck && u < 4) {
                        v = (crc >> (24 - 8 * u)) & 0xffu;
                        if (ivl) v ^= scr[mod_ivl((uint32_t)pos, (uint32_t)ivl, magic)];
                    } else {
                        const int w = u - (ck ? 4 : 0);
                        v = w < ivl ? scr[w] : (uint32_t)ivl;
                    }
                    if (kx) v ^= a.ks[pos];
                }
                ovl[t] = (uint8_t)v;
            }
        }
        wave_sync();
        if (ok && hl < 4) {
            const int P = P0 + 16 * hl;
            if (P < ext) {
                const u32x4 d = ld_piece(pkt + P);
                u32x4 m = kx ? *reinterpret_cast<const u32x4 *>(a.ks + P) : u32x4{0, 0, 0, 0};
                if (ivl) m ^= iv_window(iv2w, (uint32_t)P, (uint32_t)ivl, magic);
                const u32x4 o = *reinterpret_cast<const u32x4 *>(ovl + 16 * hl);
                const u32x4 lo = piece_mask(L - P), hi = piece_mask(out - P);
                st_piece(pkt + P, ((d ^ m) & lo) | (o & hi & ~lo) | (d & ~hi));
            }
        }
        if (have && hl == 0) a.out_len[pk] = ok ? out : -1;
        wave_sync();  // the scratch slice is rewritten by the next packet
    }
}

__global__ __launch_bounds__(kThreads) void k_decook(CookArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const bool ck = !(a.flags & RSMI_COOK_NO_CHECKSUM);
    const bool obs = !(a.flags & RSMI_COOK_NO_OBSCURE);
    const bool kx = a.ks != nullptr;
    if (ck) load_tables(lds, a.tabs);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, half = lane >> 5, hl = lane & 31;
    uint8_t *scr = reinterpret_cast<uint8_t *>(lds + kCookTabWords) + (wid * 2 + half) * kScr;
    uint32_t *iv2w = reinterpret_cast<uint32_t *>(scr);
    uint8_t *misc = scr + 352;
    const uint32_t *T = lds;
    const int64_t npairs = (a.count + 1) >> 1;

    for (int64_t pw = (int64_t)blockIdx.x * (kThreads / 64) + wid; pw < npairs;
         pw += (int64_t)gridDim.x * (kThreads / 64)) {
        const int64_t pk = 2 * pw + half;
        const bool have = pk < a.count;
        int L = -1;
        uint8_t *pkt = nullptr;
        if (have) {
            L = a.len[pk];
            pkt = a.base + (a.offset ? a.offset[pk] : (uint64_t)pk * (uint64_t)a.stride);
        }
        const bool ok = have && L >= 0 && L <= RSMI_COOK_MAX_LEN && round16(L) <= a.cap &&
                        ((uintptr_t)pkt & 3) == 0;
        // ---- de_obscure bounds (packet.cpp:93-100), read before any store ------
        int status = 0, ivl = 0, L1 = L;
        if (ok && obs) {
            if (L < 1) {
                status = -1;
            } else {
                const int v = pkt[L - 1] ^ (kx ? a.ks[L - 1] : 0);
                if (L < 1 + v) status = -1;
                else { ivl = v; L1 = L - 1 - v; }
            }
        }
        const uint32_t magic = ivl ? 0xFFFFFFFFu / (uint32_t)ivl : 0u;
        if (ok && ivl) {
            for (int t = hl; t < ivl + 20; t += 32) {
                const int pos = L1 + t % ivl;
                scr[t] = pkt[pos] ^ (kx ? a.ks[pos] : 0);
            }
        }
        wave_sync();
        // ---- rm_crc32 input (packet.cpp:337-346): stored crc, big-endian --------
        const int Lc = L1 - 4;
        const bool crc_on = ok && ck && status == 0 && Lc >= 0;
        if (ok && ck && status == 0 && Lc < 0) status = -1;
        if (crc_on && hl < 4) {
            const int pos = Lc + hl;
            uint32_t b = pkt[pos] ^ (kx ? a.ks[pos] : 0);
            if (ivl) b ^= scr[mod_ivl((uint32_t)pos, (uint32_t)ivl, magic)];
            misc[hl] = (uint8_t)b;
        }
        wave_sync();
        const uint32_t crc_in = crc_on ? __builtin_bswap32(*reinterpret_cast<const uint32_t *>(misc)) : 0u;
        const int ext = ok ? round16(L) : 0;
        const int nr = (ext + kRound - 1) / kRound;
        const int nrm = wave_max(nr);
        uint32_t acc = 0;
        for (int r = 0; r < nrm; ++r) {
            uint32_t c = 0;
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const int P = r * kRound + hl * kChunk + p * 16;
                u32x4 o = {0, 0, 0, 0};
                if (P < ext) {
                    const u32x4 d = ld_piece(pkt + P);
                    const u32x4 mk = kx ? *reinterpret_cast<const u32x4 *>(a.ks + P) : u32x4{0, 0, 0, 0};
                    const u32x4 mi = ivl ? iv_window(iv2w, (uint32_t)P, (uint32_t)ivl, magic)
                                         : u32x4{0, 0, 0, 0};
                    if (P + 16 <= L1) o = d ^ mk ^ mi;
                    else o = d ^ (mk & piece_mask(L - P)) ^ (mi & piece_mask(L1 - P));
                    st_piece(pkt + P, o);
                }
                if (ck) {
                    u32x4 ci = o & piece_mask(Lc - P);
                    if (P == 0) ci.x = ~ci.x;
                    c = slice8(T, c, ci.x, ci.y);
                    c = slice8(T, c, ci.z, ci.w);
                }
            }
            if (ck) {  // the partner packet may need more rounds: only own rounds count
                c = half_xor(nib_map(T + kCookLane + 128 * hl, c));
                const uint32_t nacc = nib_map(T + kCookRound, acc) ^ c;
                acc = r < nr ? nacc : acc;
            }
        }
        if (crc_on && ~unshift(T + kCookUns, acc, (uint32_t)(nr * kRound - Lc)) != crc_in) status = -1;
        if (have && hl == 0) a.out_len[pk] = (!ok || status) ? -1 : (ck ? Lc : L1);
        wave_sync();
    }
}

}  // namespace

size_t cook_lds_bytes() { return (size_t)kCookTabWords * 4 + (size_t)(kThreads / 32) * kScr; }

hipError_t launch_cook(const CookArgs &a, bool decook, int max_blocks, hipStream_t s) {
    if (a.count <= 0) return hipSuccess;
    const int64_t pairs = (a.count + 1) / 2;
    int64_t blocks = (pairs + kThreads / 64 - 1) / (kThreads / 64);
    if (blocks > max_blocks) blocks = max_blocks;
    const size_t lds = cook_lds_bytes();
    if (decook)
        k_decook<<<(unsigned)blocks, kThreads, lds, s>>>(a);
    else
        k_cook<<<(unsigned)blocks, kThreads, lds, s>>>(a);
    return hipGetLastError();
}

}  // namespace rsmi
