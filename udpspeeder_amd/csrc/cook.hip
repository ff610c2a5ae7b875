// cook.hip -- batched packet cook / de_cook for gfx950.
//
// Semantics: packet.cpp do_cook (:303-308) and de_cook (:310-326), see
// include/rsmi_cook.h.  kLpp lanes (8 by default, an eighth of a wave) own one
// packet, so a wave works on 64/kLpp packets at once.  A packet is walked in
// rounds of 96 16-byte pieces (1536 B); in a round lane l owns pieces l,
// l+kLpp, l+2kLpp, ..., so every load and store instruction covers 16*kLpp
// contiguous bytes of each of the wave's packets.
//
// The transform is byte-parallel: an output piece is the input piece XOR a
// key-stream window (KS[p] = key[p % strlen(key)], precomputed per context,
// read 16-B aligned from L1/L2) XOR an IV window (the packet's IV repeated in
// LDS, read as five dwords and funnel-shifted by P mod iv_len).
//
// CRC-32 (packet.cpp:236-257) is the only serial part.  Raw CRC (register init
// 0, no final xor) is linear, with Z_d = "feed d zero bytes" a linear map on
// the 32-bit register.  The message is zero-padded to Q whole pieces; then
//   * each piece's raw CRC comes from slicing-by-8 (8 x 256-word LDS tables);
//   * a lane folds its pieces Horner-style, h = Z_{16 kLpp}(h) ^ crc(piece);
//   * h is shifted to the end of the round's data by Z_{16k}, k = pieces after
//     the lane's last piece (always 0..kLpp-1: kLpp nibble-table maps), and the
//     packet's kLpp lanes XOR-reduce with ds_swizzle;
//   * a lane's pieces in successive rounds continue the same arithmetic
//     sequence (step 16 kLpp), so its Horner chain runs across rounds and is
//     shifted and reduced once per packet (COOK_ONE_CHAIN / COOKF_ONE_CHAIN;
//     the older form chained rounds as acc = Z_{16 Q_r}(acc) ^ round);
//   * the < 16 bytes of zero padding are removed with Z_{-z} (two nibble maps).
// crc32h's init ~0 is folded in by complementing the first 4 bytes of the
// padded message, its final ~ at the end.
//
// Cook keeps the (at most one per lane) piece that holds part of the appended
// crc/iv/iv_len tail in registers and rebuilds it after the CRC is known from a
// 64-byte per-packet overlay in LDS.  De_cook issues its first round of loads,
// then reads iv_len, the IV and the stored crc, then writes every piece.
#include "rsmi_internal.hpp"
#include "../../include/rsmi_cook.h"

namespace rsmi {
#include "frame_piece.hpp"
namespace {

#ifndef COOK_TRACE
#define COOK_TRACE 0  // measurement only: per wave-step phase timestamps of k_cook
#endif
#if COOK_TRACE
__device__ uint64_t *g_cook_trace;  // [wave step][8]: t0..t4 (rsmi_debug_cook_trace)
__device__ __forceinline__ uint64_t ctrace_now() {
    asm volatile("" ::: "memory");
    const uint64_t t = __builtin_amdgcn_s_memtime();
    asm volatile("" ::: "memory");
    return t;
}
#define CT(i) const uint64_t ct##i = ctrace_now()
#else
#define CT(i)
#endif
constexpr int kLpp = kCookLpp;          // lanes per packet
constexpr int kPpw = 64 / kLpp;         // packets per wave
constexpr int kPpl = 96 / kLpp;         // pieces per lane per round
#ifndef COOK_OCC
#define COOK_OCC (kLpp == 8 ? 4 : kLpp == 16 ? 5 : 6)  // waves per SIMD the register budget is cut for
#endif
#ifndef COOK_ABS_LDS
#define COOK_ABS_LDS 1  // CRC tables addressed from LDS address 0 (see tab_byte)
#endif
#ifndef COOK_SKIP
#define COOK_SKIP 1  // skip the CRC of piece slots past every packet's last crc piece of the wave
#endif
#ifndef COOK_SB
#define COOK_SB 1  // scheduling fence every COOK_SB pieces (0: none), bounds registers
#endif
#ifndef COOK_ONE_CHAIN
#define COOK_ONE_CHAIN 1  // k_cook: one Horner chain (pair) per lane across rounds, finished once
#endif
#ifndef COOK_DEFER
#define COOK_DEFER 0  // k_cook, bit 0: a piece's key-stream load issued before its CRC;
                      // bit 1: the round's stores after the round (in vmcnt, a store made
                      // the next piece's key-stream load wait for it)
#endif
#ifndef COOK_LINE
#define COOK_LINE 0  // k_cook: lane pieces on the 128-byte line grid of the packet (one-chain fold).
                     // Round 6 (profiles/r06/cook_line_ab.txt): cook 1.309-1.316 ms vs 1.275-1.278
                     // without, the fused run 2.87-2.91 vs 2.88-3.00 ms -- off (k_cook_frame's
                     // COOKF_LINE, whose plain stream it fixed, stays on)
#endif
#ifndef COOK_THREADS
#define COOK_THREADS (kLpp == 32 ? 512 : 256)
#endif
constexpr int kThreads = COOK_THREADS;  // LDS (tables per block) bounds residency
constexpr int kRound = 1536;            // 96 pieces per packet per round
constexpr int kScrCook = 144;           // per-packet LDS: iv2[64] | overlay[64] | misc[16]
constexpr int kScrDecook = 304;         // iv2[288] (iv_len up to 255) | misc[16]

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

#ifndef COOK_NT
#define COOK_NT 0  // 1: packet loads and stores non-temporal (read and written once)
#endif
#ifndef COOK_LD_NT
#define COOK_LD_NT COOK_NT  // ... the loads alone
#endif
#ifndef COOK_ST_NT
#define COOK_ST_NT COOK_NT  // ... the stores alone
#endif
__device__ __forceinline__ u32x4 ld_piece(const uint8_t *p) {
#if COOK_LD_NT
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4_a4 *>(p));
#else
    return *reinterpret_cast<const u32x4_a4 *>(p);
#endif
}
__device__ __forceinline__ void st_piece(uint8_t *p, u32x4 v) {
#if COOK_ST_NT
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4_a4 *>(p));
#else
    *reinterpret_cast<u32x4_a4 *>(p) = v;
#endif
}

// Table word at word index w + byte b of x (b = 0..3): the tables sit at LDS
// address 0 (the kernels' only LDS is the dynamic array, tables first), so the
// address is ((x >> 8b) & 0xff) * 4 + 4w -- the table base goes into the
// ds_read offset and the byte scale into one SDWA shift.  Through the generic
// pointer LLVM added the array's base as a register: v_bfe + v_lshl_add per
// lookup.
#if COOK_ABS_LDS
typedef const __attribute__((address_space(3))) uint32_t *lds_u32p;
__device__ __forceinline__ uint32_t tab_byte(const uint32_t *, int w, uint32_t x, int b) {
    return *(lds_u32p)(size_t)(4 * w + (((x >> (8 * b)) & 0xffu) << 2));
}
#else
__device__ __forceinline__ uint32_t tab_byte(const uint32_t *T, int w, uint32_t x, int b) {
    return T[w + ((x >> (8 * b)) & 0xffu)];
}
#endif

#if !COOK_S16
// CRC register after 8 bytes (dwords a, b little-endian) from register c.
__device__ __forceinline__ uint32_t slice8(const uint32_t *T, uint32_t c, uint32_t a, uint32_t b) {
    const uint32_t x = c ^ a;
    uint32_t r = xor3(tab_byte(T, 7 * 256, x, 0), tab_byte(T, 6 * 256, x, 1), tab_byte(T, 5 * 256, x, 2));
    r = xor3(r, tab_byte(T, 4 * 256, x, 3), tab_byte(T, 3 * 256, b, 0));
    r = xor3(r, tab_byte(T, 2 * 256, b, 1), tab_byte(T, 256, b, 2));
    return r ^ tab_byte(T, 0, b, 3);
}
#endif

// A linear map of the CRC register held as 8 nibble tables of 16 words.
__device__ __forceinline__ uint32_t nib_map(const uint32_t *M, uint32_t c) {
    uint32_t r = xor3(M[c & 15], M[16 + ((c >> 4) & 15)], M[32 + ((c >> 8) & 15)]);
    r = xor3(r, M[48 + ((c >> 12) & 15)], M[64 + ((c >> 16) & 15)]);
    r = xor3(r, M[80 + ((c >> 20) & 15)], M[96 + ((c >> 24) & 15)]);
    return r ^ M[112 + (c >> 28)];
}

// XOR over the kLpp lanes of one packet (ds_swizzle xor-mode, xor masks < kLpp).
__device__ __forceinline__ uint32_t group_xor(uint32_t c) {
    c ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)c, 0x041F);
    c ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)c, 0x081F);
    c ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)c, 0x101F);
    if (kLpp >= 16) c ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)c, 0x201F);
    if (kLpp == 32) c ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)c, 0x401F);
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

// IV bytes iv[(r + t) % ivl], t = 0..15, from the repeated IV in LDS (r < ivl).
__device__ __forceinline__ u32x4 iv_window_at(const uint32_t *iv2w, uint32_t r) {
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

__device__ __forceinline__ u32x4 iv_window(const uint32_t *iv2w, uint32_t pos, uint32_t ivl,
                                           uint32_t magic) {
    return iv_window_at(iv2w, mod_ivl(pos, ivl, magic));
}

// Position of the IV cycle at the next piece a lane owns (16 kLpp bytes further).
__device__ __forceinline__ uint32_t iv_step(uint32_t r, uint32_t s512, uint32_t ivl) {
    r += s512;
    return r >= ivl ? r - ivl : r;
}

__device__ __forceinline__ uint64_t splitmix(uint64_t seed, uint64_t idx, uint64_t w) {
    uint64_t z = (seed ^ idx) + (w + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

#if COOK_NIB
// Word at byte offset o of table t (o a multiple of 4).
__device__ __forceinline__ uint32_t at(const uint32_t *t, uint32_t o) {
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(t) + o);
}

// Z_{16 kLpp} as eight nibble tables.
__device__ __forceinline__ uint32_t zh(const uint32_t *T, uint32_t c) {
    return nib_map(T + kCookZN, c);
}

// Raw CRC of one 16-byte piece: 32 nibble lookups, one level deep.
__device__ __forceinline__ uint32_t crc16(const uint32_t *T, u32x4 v) {
    const uint32_t *N = T + kCookNib;
    uint32_t r[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t lo = (v[d] << 2) & 0x3C3C3C3Cu, hi = (v[d] >> 2) & 0x3C3C3C3Cu;
        const uint32_t *Nd = N + 128 * d;
        uint32_t x = xor3(at(Nd, lo & 0xff), at(Nd + 16, hi & 0xff),
                          at(Nd + 32, (lo >> 8) & 0xff));
        x = xor3(x, at(Nd + 48, (hi >> 8) & 0xff), at(Nd + 64, (lo >> 16) & 0xff));
        x = xor3(x, at(Nd + 80, (hi >> 16) & 0xff), at(Nd + 96, lo >> 24));
        r[d] = x ^ at(Nd + 112, hi >> 24);
    }
    return xor3(r[0], r[1], r[2]) ^ r[3];
}
#else
// Z_{16 kLpp} as four byte tables.
__device__ __forceinline__ uint32_t zh(const uint32_t *T, uint32_t c) {
    return xor3(tab_byte(T, kCookZH, c, 0), tab_byte(T, kCookZH + 256, c, 1),
                tab_byte(T, kCookZH + 512, c, 2)) ^
           tab_byte(T, kCookZH + 768, c, 3);
}

#if COOK_S16
// Table word of T_k (byte followed by k zero bytes), k = 0..15.
__device__ __forceinline__ constexpr int tword(int k) { return k < 8 ? 256 * k : kCookS16 + 256 * (k - 8); }

// Raw CRC of one 16-byte piece: byte j through T_{15-j}, all 16 lookups independent.
__device__ __forceinline__ uint32_t crc16(const uint32_t *T, u32x4 v) {
    const uint32_t a = xor3(tab_byte(T, tword(15), v.x, 0), tab_byte(T, tword(14), v.x, 1),
                            tab_byte(T, tword(13), v.x, 2));
    const uint32_t b = xor3(tab_byte(T, tword(12), v.x, 3), tab_byte(T, tword(11), v.y, 0),
                            tab_byte(T, tword(10), v.y, 1));
    const uint32_t c = xor3(tab_byte(T, tword(9), v.y, 2), tab_byte(T, tword(8), v.y, 3),
                            tab_byte(T, tword(7), v.z, 0));
    const uint32_t d = xor3(tab_byte(T, tword(6), v.z, 1), tab_byte(T, tword(5), v.z, 2),
                            tab_byte(T, tword(4), v.z, 3));
    const uint32_t e = xor3(tab_byte(T, tword(3), v.w, 0), tab_byte(T, tword(2), v.w, 1),
                            tab_byte(T, tword(1), v.w, 2));
    return xor3(a, b, c) ^ xor3(d, e, tab_byte(T, tword(0), v.w, 3));
}
#else
// Raw CRC of one 16-byte piece.
__device__ __forceinline__ uint32_t crc16(const uint32_t *T, u32x4 v) {
    return slice8(T, slice8(T, 0u, v.x, v.y), v.z, v.w);
}
#endif
#endif

// Remove z < 16 trailing zero bytes: Z_{-z} = Z_{-(z&3)} o Z_{-4(z>>2)}.
__device__ __forceinline__ uint32_t unshift(const uint32_t *T, uint32_t c, uint32_t z) {
    const uint32_t *U = T + kCookUns;
    const uint32_t lo = z & 3, hi = z >> 2;
    const uint32_t c1 = nib_map(U + 128 * (lo ? lo - 1 : 0), c);
    c = lo ? c1 : c;
    const uint32_t c2 = nib_map(U + 128 * (hi ? hi + 2 : 0), c);
    return hi ? c2 : c;
}

// Z_{32 kLpp}: two piece slots of a lane (the two-chain fold's step).
__device__ __forceinline__ uint32_t zh2(const uint32_t *T, uint32_t c) {
    return xor3(tab_byte(T, kCookZH2, c, 0), tab_byte(T, kCookZH2 + 256, c, 1),
                tab_byte(T, kCookZH2 + 512, c, 2)) ^
           tab_byte(T, kCookZH2 + 768, c, 3);
}

// CRC of a round, folded one piece at a time: piece q (= kLpp p + lane, slot
// p) of the round, crc input v; qr = data pieces of the packet in this round
// (0..96).  TWO: even and odd slots fold as two Horner chains with step
// Z_{32 kLpp}; the data pieces are a prefix of the slots, so the other chain's
// last piece is one slot before the lane's last and joins it through Z_{16 kLpp}.
template <bool TWO>
struct RoundCrc {
    uint32_t h[2] = {0, 0};
    int last = -1, last_slot = -1;
    __device__ __forceinline__ void add(const uint32_t *T, u32x4 v, int p, int q, int qr) {
        const int c = TWO ? (p & 1) : 0;
        const uint32_t hn = (TWO ? zh2(T, h[c]) : zh(T, h[c])) ^ crc16(T, v);
        h[c] = q < qr ? hn : h[c];
        last = q < qr ? q : last;
        last_slot = q < qr ? p : last_slot;  // (a line-aligned grid shifts q against the slot)
    }
    // The round's raw CRC relative to the end of its data, in all kLpp lanes.
    __device__ __forceinline__ uint32_t finish(const uint32_t *T, int qr) const {
        uint32_t hh = h[0];
        if (TWO) {  // Z(0) = 0: an empty chain adds nothing
            const bool odd = last >= 0 && (last_slot & 1);
            hh = zh(T, odd ? h[0] : h[1]) ^ (odd ? h[1] : h[0]);
        }
        int k = qr - 1 - last;
        k = (last >= 0 && k >= 0 && k < kLpp) ? k : 0;
        const uint32_t c = nib_map(T + kCookLane + 128 * k, hh);
        return group_xor(last >= 0 ? c : 0u);
    }
};

// acc = Z_{16 qr}(acc): Z_{16 kLpp} (qr / kLpp) times, then the lane map
// Z_{16 (qr % kLpp)}.
__device__ __forceinline__ uint32_t shift_pieces(const uint32_t *T, uint32_t acc, int qr) {
#pragma unroll
    for (int i = 0; i < kPpl; ++i) {
        const uint32_t n = zh(T, acc);
        acc = i < qr / kLpp ? n : acc;
    }
    return nib_map(T + kCookLane + 128 * (qr % kLpp), acc);
}

__device__ __forceinline__ int round16(int x) { return (x + 15) & ~15; }

// acc = Z_{16 qr}(acc) for qr <= N kLpp pieces (shift_pieces for shorter rounds).
template <int N>
__device__ __forceinline__ uint32_t shift_pieces_n(const uint32_t *T, uint32_t acc, int qr) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const uint32_t n = zh(T, acc);
        acc = i < qr / kLpp ? n : acc;
    }
    return nib_map(T + kCookLane + 128 * (qr % kLpp), acc);
}


__device__ __forceinline__ void load_tables(uint32_t *lds, const uint32_t *tabs, int words) {
    for (int i = threadIdx.x; i < words / 4; i += kThreads)
        reinterpret_cast<u32x4 *>(lds)[i] = reinterpret_cast<const u32x4 *>(tabs)[i];
    __syncthreads();
}

// Uniform loop bound for the packets of a wave.
__device__ __forceinline__ int wave_max(int v) {
    int m = __builtin_amdgcn_readlane(v, 0);
#pragma unroll
    for (int s = 1; s < kPpw; ++s) m = max(m, __builtin_amdgcn_readlane(v, s * kLpp));
    return m;
}

__device__ __forceinline__ uint64_t packet_off(const CookArgs &a, int64_t pk) {
    if (a.pk) return (uint64_t)a.pk[pk].slot * (uint64_t)a.stride + (uint64_t)a.pk_off;
    return a.offset ? a.offset[pk] : (uint64_t)pk * (uint64_t)a.stride;
}

__device__ __forceinline__ int packet_len(const CookArgs &a, int64_t pk) {
    return a.pk ? a.pk[pk].len : a.len[pk];
}

// The N pieces of round r (N kLpp pieces a packet) owned by lane hl: zeros past ext.
template <int N>
__device__ __forceinline__ void load_round(u32x4 (&d)[N], const uint8_t *pkt, int r, int hl, int ext,
                                           int lead = 0) {
#pragma unroll
    for (int p = 0; p < N; ++p) {
        const int P = r * (16 * kLpp * N) + 16 * (kLpp * p + hl - lead);
        d[p] = (P >= 0 && P < ext) ? ld_piece(pkt + P) : u32x4{0, 0, 0, 0};
    }
}

// Key stream at packet offset P (>= -12: the stream has a 16-byte lead).
__device__ __forceinline__ u32x4 ks_piece(const CookArgs &a, int P) {
    return a.ks ? *reinterpret_cast<const u32x4_a4 *>(a.ks + P) : u32x4{0, 0, 0, 0};
}

// CRC input of piece P: bytes below n, the first 4 bytes complemented (init ~0).
// The byte mask is built only when some lane of the wave holds a piece that
// ends past n (a wave-uniform branch): most pieces are whole.
__device__ __forceinline__ u32x4 crc_in(u32x4 v, int P, int n) {
    if (__ballot(P + 16 > n)) v &= piece_mask(n - P);
    if (P == 0) v.x = ~v.x;
    return v;
}

// The same on the packet's 16-byte grid when the packet starts ph (0, 4, 8 or
// 12) bytes into a piece: piece P's bytes below ph are not the packet's (zero
// for the CRC: leading zeros leave a zero register as it is), the message's
// first 4 bytes are dword ph / 4 of piece 0.
__device__ __forceinline__ u32x4 crc_in_ph(u32x4 v, int P, int n, int ph) {
    if (__ballot(P + 16 > n)) v &= piece_mask(n - P);
    if (P == 0) {
        v &= ~piece_mask(ph);
#pragma unroll
        for (int d = 0; d < 4; ++d) v[d] = (4 * d == ph) ? ~v[d] : v[d];
    }
    return v;
}

// k_cook's round: COOK_PPL pieces per lane (kPpl: 1536 bytes per packet).
#ifndef COOK_PPL
#define COOK_PPL kPpl
#endif
constexpr int kPplC = COOK_PPL;
constexpr int kRoundC = 16 * kLpp * kPplC;

// PREX (a fused cooked run's list B with the parity cook in the encoder's
// epilogue, rsmi_internal.hpp EpiRec): an entry flagged kPrexFlag in len is
// read from the output, where the encoder stored its whole payload pieces
// already obscured and keyed and its other pieces plain (and k_expand_packets
// its header): those pieces' plain bytes are recovered for the CRC and not
// stored again; the header piece and the tail are cooked as usual.
template <bool PREX>
__global__ __launch_bounds__(kThreads, COOK_OCC) void k_cook(CookArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const bool ck = !(a.flags & RSMI_COOK_NO_CHECKSUM);
    const bool obs = !(a.flags & RSMI_COOK_NO_OBSCURE);
    if (ck) load_tables(lds, a.tabs, kCookTabWords);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, sub = lane / kLpp, hl = lane % kLpp;
    uint8_t *scr = reinterpret_cast<uint8_t *>(lds + kCookTabWords) + (wid * kPpw + sub) * kScrCook;
    uint32_t *iv2w = reinterpret_cast<uint32_t *>(scr);
    uint8_t *ovl = scr + 64;
    const uint32_t *T = lds;
    const int64_t nunits = (a.count + kPpw - 1) / kPpw;  // kPpw packets per wave step

    for (int64_t pw = (int64_t)blockIdx.x * (kThreads / 64) + wid; pw < nunits;
         pw += (int64_t)gridDim.x * (kThreads / 64)) {
        CT(0);
        const int64_t pk = kPpw * pw + sub;
        const bool have = pk < a.count;
        // the packet's index in its batch: IV draw, out_len and packed place
        const int64_t gi = have && a.pk_idx ? (int64_t)a.pk[pk].event : pk;
        int L = -1, ivl = 0;
        const uint64_t po = have ? packet_off(a, pk) : 0u;
        uint8_t *pkt = have ? a.base + po : nullptr;
        uint8_t *opkt = !have ? nullptr
                        : a.dst_off ? a.dst + a.dst_off[gi]
                                    : (a.dst ? a.dst : a.base) + po;  // where the output goes
        // a.phase: work on the 16-byte grid the packet sits in (an FEC packet
        // starts 8 bytes into one, RSMI_FEC_SLOT_PACKET): whole-piece loads and
        // stores line up with memory; the ph bytes before the packet are the
        // slot's scratch.  Grid coordinates below: packet byte x is grid byte x + ph.
        const int ph = (a.phase && have && ((uintptr_t)pkt & 3) == 0 &&
                        (((uintptr_t)pkt ^ (uintptr_t)opkt) & 15) == 0)
                           ? (int)((uintptr_t)pkt & 15) : 0;
        const uint8_t *pga = pkt - ph;
        uint8_t *oga = opkt - ph;
        const bool pre = PREX && have && (a.pk[pk].len & kPrexFlag);
        const uint8_t *sga = pre ? oga : pga;  // where the packet's bytes are read
        // COOK_LINE: the lanes count pieces from the 128-byte line the grid
        // starts in (`lead` pieces before it, untouched), so a load or store
        // instruction covers whole lines (an FEC packet's grid starts 112 B
        // into its slot's line: two instructions per line, as k_cook_frame's)
        const int lead = (COOK_LINE && have && (((uintptr_t)pga ^ (uintptr_t)oga) & 127) == 0)
                             ? (int)(((uintptr_t)pga & 127) >> 4) : 0;
        // round 0 is read up to the packet's cap (every packet owns cap bytes), so
        // these loads fly together with the length load instead of after it
        u32x4 cur[kPplC];
        load_round(cur, sga, 0, hl, have && ((uintptr_t)pkt & 3) == 0 ? min((a.cap + ph) & ~15, kRoundC) : 0,
                   lead);
        if (have) {
            L = PREX ? (packet_len(a, pk) & ~kPrexFlag) : packet_len(a, pk);
            if (obs) ivl = a.iv ? a.iv_len[pk] : 4 + (int)(splitmix(a.seed, (uint64_t)gi, 0) % 29u);
        }
        const int out = L + (ck ? 4 : 0) + (obs ? ivl + 1 : 0);
        // (a packed output has room for any iv_len <= RSMI_COOK_IV_MAX)
        const int Lg = L + ph, outg = out + ph;  // payload end and output end on the grid
        const bool ok = have && L >= 0 && L <= RSMI_COOK_MAX_LEN && ivl <= RSMI_COOK_IV_MAX &&
                        (a.dst_off || round16(outg) - ph <= a.cap) && round16(Lg) - ph <= a.cap &&
                        ((uintptr_t)pkt & 3) == 0;
        const int ext = ok ? round16(outg) : 0;
        const uint32_t magic = ivl ? 0xFFFFFFFFu / (uint32_t)ivl : 0u;
        if (ok && ivl && !a.iv && 8 * hl < ivl) {  // device-drawn IV: 8 bytes per draw, one per lane
            const uint64_t z = splitmix(a.seed, (uint64_t)gi, 1 + (uint64_t)hl);
            reinterpret_cast<uint32_t *>(ovl)[2 * hl] = (uint32_t)z;
            reinterpret_cast<uint32_t *>(ovl)[2 * hl + 1] = (uint32_t)(z >> 32);
        }
        wave_sync();
        if (ok && ivl) {  // iv repeated: iv2[t] = iv[t % ivl], t < ivl + 20 (<= 52)
            for (int t = hl; t < ivl + 20; t += kLpp) {
                const uint32_t j = mod_ivl((uint32_t)t, (uint32_t)ivl, magic);
                scr[t] = a.iv ? a.iv[pk * RSMI_COOK_IV_MAX + j] : ovl[j];
            }
        }
        wave_sync();
        CT(1);
        const uint32_t sstep = ivl ? mod_ivl(16u * kLpp, (uint32_t)ivl, magic) : 0u;
        const int Q = (Lg + 15) >> 4;           // pieces holding payload (crc input)
        const int P0 = Lg & ~15;                // first piece that holds tail bytes
        const int nrm = wave_max((ext + 16 * lead + kRoundC - 1) / kRoundC);
        uint32_t acc = 0;
        u32x4 dt = {0, 0, 0, 0};                // this lane's tail piece, if any
        int Pt = -1;
#if COOK_ONE_CHAIN
        RoundCrc<COOK_2CH != 0> rcx;  // slot s = r kPplC + p over all rounds (see k_cook_frame)
#endif
        for (int r = 0; r < nrm; ++r) {
            // rounds past the first (long packets); a packed output's tail may
            // end past the source slot, whose bytes there are never used
            if (r) load_round(cur, sga, r, hl, min(ext, (a.cap + ph) & ~15), lead);
            // (round r's slot p holds piece kLpp (r kPplC + p) + hl - lead)
            const int qr = min(max(Q + lead - kPplC * kLpp * r, 0), kPplC * kLpp);
            // pieces at or past every packet's last crc piece in this round:
            // skip their CRC (a wave-uniform branch per piece slot)
            const int qr_max = COOK_SKIP ? wave_max(qr) : kPplC * kLpp;
#if COOK_ONE_CHAIN
            RoundCrc<COOK_2CH != 0> &rc = rcx;
#else
            RoundCrc<COOK_2CH != 0> rc;
#endif
            uint32_t ivr = ivl ? mod_ivl((uint32_t)(r * kRoundC + 16 * (hl - lead) + 128 * ivl - ph),
                                         (uint32_t)ivl, magic)
                               : 0u;
#pragma unroll
            for (int p = 0; p < kPplC; ++p) {
                const int P = r * kRoundC + 16 * (kLpp * p + hl - lead);  // grid offset
                // wholly payload (the head piece's bytes before the packet are scratch)
                const bool whole = P >= 0 && P < ext && P + 16 <= Lg;
                // cooked by the encoder: a payload piece (past the header piece)
                const bool done = PREX && pre && whole && P >= 16;
                u32x4 m = {0, 0, 0, 0};
                if (done) {
                    m = ks_piece(a, P - ph);
                    if (ivl) m ^= iv_window_at(iv2w, ivr);
                    cur[p] ^= m;  // its plain bytes, for the CRC
                }
                if ((COOK_DEFER & 1) && whole) {  // the key stream's load flies during the CRC
                    m = ks_piece(a, P - ph);
                    if (ivl) m ^= iv_window_at(iv2w, ivr);
                }
#if COOK_ONE_CHAIN
                if (ck && kLpp * p < qr_max && P >= 0) {
                    const int sl = r * kPplC + p;
                    rc.add(T, crc_in_ph(cur[p], P, Lg, ph), sl, kLpp * sl + hl - lead, Q);
                }
#else
                if (ck && kLpp * p < qr_max) rc.add(T, crc_in_ph(cur[p], P, Lg, ph), p, kLpp * p + hl, qr);
#endif
                if (done) {
                } else if (whole) {  // obscure + xor
                    if (!(COOK_DEFER & 1)) {
                        m = ks_piece(a, P - ph);
                        if (ivl) m ^= iv_window_at(iv2w, ivr);
                    }
                    if (COOK_DEFER & 2) cur[p] ^= m;  // stored after the round
                    else st_piece(oga + P, cur[p] ^ m);
                } else if (P < ext && P >= P0) {
                    dt = cur[p];
                    Pt = P;
                }
                if (ivl) ivr = iv_step(ivr, sstep, (uint32_t)ivl);
                if (COOK_SB && p % COOK_SB == COOK_SB - 1)
                    __builtin_amdgcn_sched_barrier(0);  // COOK_SB pieces' lookups at a time
            }
            if (COOK_DEFER & 2) {
#pragma unroll
                for (int p = 0; p < kPplC; ++p) {
                    const int P = r * kRoundC + 16 * (kLpp * p + hl - lead);
                    if (P >= 0 && P < ext && P + 16 <= Lg && !(PREX && pre && P >= 16)) st_piece(oga + P, cur[p]);
                }
            }
#if !COOK_ONE_CHAIN
            if (ck) {
                const uint32_t c = rc.finish(T, qr);
                const uint32_t nacc = (r ? shift_pieces_n<kPplC>(T, acc, qr) : 0u) ^ c;
                acc = qr > 0 ? nacc : acc;
            }
#endif
        }
#if COOK_ONE_CHAIN
        if (ck) acc = rcx.finish(T, Q);
#endif
        CT(2);
        uint32_t crc = 0;
        if (ck && L > 0) crc = ~unshift(T, acc, (uint32_t)(16 * Q - Lg));
        // ---- tail: crc (BE), iv, iv_len appended after the payload -------------
        if (ok) {
            for (int t = hl; t < 64; t += kLpp) {
                const int pos = P0 + t - ph;  // packet offset of overlay byte t
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
                }
                ovl[t] = (uint8_t)v;  // the key stream goes on with the tail piece below
            }
        }
        wave_sync();
        CT(3);
        if (Pt >= 0) {
            // the overlay holds the tail bytes before encrypt_0: the piece's key
            // stream covers payload and tail alike (one 16-B load, where a byte
            // load per tail byte stood in the overlay loop's dependent chain)
            const u32x4 k = ks_piece(a, Pt - ph);
            u32x4 m = k;
            if (ivl) m ^= iv_window(iv2w, (uint32_t)(Pt + 16 * ivl - ph), (uint32_t)ivl, magic);
            const u32x4 o = *reinterpret_cast<const u32x4 *>(ovl + (Pt - P0));
            const u32x4 lo = piece_mask(Lg - Pt), hi = piece_mask(outg - Pt);
            st_piece(oga + Pt, ((dt ^ m) & lo) | ((o ^ k) & hi & ~lo) | (dt & ~hi));
        }
        if (have && hl == 0) a.out_len[gi] = ok ? out : -1;
        wave_sync();  // the scratch slice is rewritten by the next packet
#if COOK_TRACE
        CT(4);
        if (lane == 0 && g_cook_trace) {
            uint64_t *t = g_cook_trace + pw * 8;
            t[0] = ct0; t[1] = ct1; t[2] = ct2; t[3] = ct3; t[4] = ct4; t[5] = (uint64_t)nrm;
        }
#endif
    }
}

__global__ __launch_bounds__(kThreads, COOK_OCC) void k_decook(CookArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const bool ck = !(a.flags & RSMI_COOK_NO_CHECKSUM);
    const bool obs = !(a.flags & RSMI_COOK_NO_OBSCURE);
    if (ck) load_tables(lds, a.tabs, kCookTabDecook);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, sub = lane / kLpp, hl = lane % kLpp;
    uint8_t *scr = reinterpret_cast<uint8_t *>(lds + kCookTabDecook) + (wid * kPpw + sub) * kScrDecook;
    uint32_t *iv2w = reinterpret_cast<uint32_t *>(scr);
    uint8_t *misc = scr + 288;
    const uint32_t *T = lds;
    const int64_t nunits = (a.count + kPpw - 1) / kPpw;  // kPpw packets per wave step

    for (int64_t pw = (int64_t)blockIdx.x * (kThreads / 64) + wid; pw < nunits;
         pw += (int64_t)gridDim.x * (kThreads / 64)) {
        const int64_t pk = kPpw * pw + sub;
        const bool have = pk < a.count;
        // (de_cook keeps its round-0 loads behind the length: loading up to the
        // cap here spills registers and measured slower)
        int L = -1;
        uint8_t *pkt = nullptr, *opkt = nullptr, *mpkt = nullptr;
        if (have) {
            L = packet_len(a, pk);
            const uint64_t po = packet_off(a, pk);
            pkt = a.base + po;
            opkt = (a.dst ? a.dst : a.base) + po;  // where the output goes
            if (a.mirror) mpkt = a.mirror + po;    // and its copy (the host's)
        }
        const bool ok = have && L >= 0 && L <= RSMI_COOK_MAX_LEN && round16(L) <= a.cap &&
                        ((uintptr_t)pkt & 3) == 0;
        const int ext = ok ? round16(L) : 0;
        u32x4 cur[kPpl];
        load_round(cur, pkt, 0, hl, ext);       // in flight while the tail is parsed
        // ---- de_obscure bounds (packet.cpp:93-100), read before any store ------
        int status = 0, ivl = 0, L1 = L;
        if (ok && obs) {
            if (L < 1) {
                status = -1;
            } else {
                const int v = pkt[L - 1] ^ (a.ks ? a.ks[L - 1] : 0);
                if (L < 1 + v) status = -1;
                else { ivl = v; L1 = L - 1 - v; }
            }
        }
        const uint32_t magic = ivl ? 0xFFFFFFFFu / (uint32_t)ivl : 0u;
        const uint32_t sstep = ivl ? mod_ivl(16u * kLpp, (uint32_t)ivl, magic) : 0u;
        if (ok && ivl) {
            // the IV repeated (iv2[t] = iv[t % ivl], t < ivl + 20): the first
            // kIvPre steps' byte loads are issued together before any store
            // (iv_len <= 32 + ... as the reference sends it needs no more),
            // then the rest (iv_len up to 255 is accepted on the wire)
            constexpr int kIvPre = (52 + kLpp - 1) / kLpp;
            uint32_t bv[kIvPre];
#pragma unroll
            for (int i = 0; i < kIvPre; ++i) {
                const int t = hl + kLpp * i;
                bv[i] = 0;
                if (t < ivl + 20) {
                    const int pos = L1 + (int)mod_ivl((uint32_t)t, (uint32_t)ivl, magic);
                    bv[i] = pkt[pos] ^ (a.ks ? a.ks[pos] : 0);
                }
            }
#pragma unroll
            for (int i = 0; i < kIvPre; ++i)
                if (hl + kLpp * i < ivl + 20) scr[hl + kLpp * i] = (uint8_t)bv[i];
            for (int t = hl + kLpp * kIvPre; t < ivl + 20; t += kLpp) {
                const int pos = L1 + (int)mod_ivl((uint32_t)t, (uint32_t)ivl, magic);
                scr[t] = pkt[pos] ^ (a.ks ? a.ks[pos] : 0);
            }
        }
        wave_sync();
        // ---- rm_crc32 input (packet.cpp:337-346): stored crc, big-endian --------
        const int Lc = L1 - 4;
        const bool crc_on = ok && ck && status == 0 && Lc >= 0;
        if (ok && ck && status == 0 && Lc < 0) status = -1;
        if (crc_on && hl < 4) {
            const int pos = Lc + hl;
            uint32_t b = pkt[pos] ^ (a.ks ? a.ks[pos] : 0);
            if (ivl) b ^= scr[mod_ivl((uint32_t)pos, (uint32_t)ivl, magic)];
            misc[hl] = (uint8_t)b;
        }
        wave_sync();
        const uint32_t want = crc_on ? __builtin_bswap32(*reinterpret_cast<const uint32_t *>(misc)) : 0u;
        const int Q = (Lc + 15) >> 4;
        const int nrm = wave_max((ext + kRound - 1) / kRound);
        uint32_t acc = 0;
        for (int r = 0; r < nrm; ++r) {
            if (r) load_round(cur, pkt, r, hl, ext);   // rounds past the first (long packets)
            const int qr = crc_on ? min(max(Q - 96 * r, 0), 96) : 0;
            const int qr_max = COOK_SKIP ? wave_max(qr) : 96;
            RoundCrc<false> rc;
            uint32_t ivr = ivl ? mod_ivl((uint32_t)(r * kRound + 16 * hl), (uint32_t)ivl, magic) : 0u;
#pragma unroll
            for (int p = 0; p < kPpl; ++p) {
                const int P = r * kRound + 16 * (kLpp * p + hl);
                u32x4 o = {0, 0, 0, 0};
                if (P < ext) {
                    const u32x4 mk = ks_piece(a, P);
                    const u32x4 mi = ivl ? iv_window_at(iv2w, ivr) : u32x4{0, 0, 0, 0};
                    if (P + 16 <= L1) o = cur[p] ^ mk ^ mi;
                    else o = cur[p] ^ (mk & piece_mask(L - P)) ^ (mi & piece_mask(L1 - P));
                    st_piece(opkt + P, o);
                    if (mpkt) st_piece(mpkt + P, o);
                }
                if (ck && kLpp * p < qr_max) rc.add(T, crc_in(o, P, Lc), p, kLpp * p + hl, qr);
                if (ivl) ivr = iv_step(ivr, sstep, (uint32_t)ivl);
                if (COOK_SB && p % COOK_SB == COOK_SB - 1) __builtin_amdgcn_sched_barrier(0);
            }
            if (ck) {
                const uint32_t c = rc.finish(T, qr);
                const uint32_t nacc = (r ? shift_pieces(T, acc, qr) : 0u) ^ c;
                acc = qr > 0 ? nacc : acc;
            }
        }
        if (crc_on) {
            const uint32_t got = Lc > 0 ? ~unshift(T, acc, (uint32_t)(16 * Q - Lc)) : 0u;
            if (got != want) status = -1;
        }
        if (have && hl == 0) a.out_len[pk] = (!ok || status) ? -1 : (ck ? Lc : L1);
        wave_sync();
    }
}

// ---- the fused framing cook -------------------------------------------------
// k_cook with k_frame in front: each list-A packet is a data packet of a clean
// shard (FrameGroup.nclean), so its bytes are the 8-byte header followed by
// the shard's stream -- blob positions i * fec_len.. in mode 0, the shard's
// own [u16 len][payload] zero-padded in mode 1 (fec_manager.cpp:318-344, the
// stream layout of k_frame, frame_piece.hpp).  A packet sits 8 bytes into its
// 16-byte grid (RSMI_FEC_SLOT_PACKET), so grid piece 0 holds the header and
// grid piece 1 + q is exactly shard piece q: each is assembled from the source
// records, stored plain into the slot (the encoder reads it) and cooked into
// the output in the same pass -- the framing's writes and the cook's reads of
// the data packets are one kernel.  The <= kFuseRecs records a
// shard overlaps are staged per packet in LDS.
constexpr int kScrFuse = kScrCook + 8 * kFuseRecs + 4 * (kFuseRecs + 1) + 12;  // + record addr / off
// k_cook_frame stages a shard's records one lane per record (hl < nrec)
static_assert(kFuseRecs <= kLpp, "k_cook_frame needs a lane per source record (COOK_LPP >= kFuseRecs)");
// Third rounds (32 pieces, 512 bytes per packet): a round's assembly keeps
// its pieces' source windows in flight, twice the registers of a plain load.
// 4 pieces per lane fit 125 VGPRs with no spill; 6 spilled 8 and measured
// 1 % slower, 8 and 12 (fewer waves) 13 and 21 % (profiles/r04/fused_knobs).
#ifndef COOKF_PPL
#define COOKF_PPL (kPpl / 3)
#endif
#ifndef COOKF_OCC
#define COOKF_OCC COOK_OCC
#endif
#ifndef COOKF_PROBE
#define COOKF_PROBE 0  // measurement only (wrong output): 1 no plain slot stores, 2 no cooked
                       // stores, 4 no source loads (zeros), 8 no plain header piece
#endif
#ifndef COOKF_ONE_CHAIN
#define COOKF_ONE_CHAIN 1  // k_cook_frame: one Horner chain per lane across its rounds
#endif
#ifndef COOKF_LINE
#define COOKF_LINE 1  // k_cook_frame: lane pieces on the 128-byte line grid of the slot
#endif
static_assert(!COOKF_LINE || COOKF_ONE_CHAIN, "COOKF_LINE shifts the pieces of the one-chain fold only");
static_assert(!COOK_LINE || COOK_ONE_CHAIN, "COOK_LINE shifts the pieces of the one-chain fold only");
constexpr int kPplF = COOKF_PPL;
constexpr int kRoundF = 16 * kLpp * kPplF;

// A packet's staged records: blob offsets off[0..n] (off[n] = the end of the
// last), payload addresses addr[0..n).
struct LdsRecs {
    const uint64_t *a;
    const uint32_t *o;
    __device__ __forceinline__ uint32_t off(uint32_t j) const { return o[j]; }
    __device__ __forceinline__ uint32_t len(uint32_t j) const { return o[j + 1] - o[j] - 2; }
    __device__ __forceinline__ const uint8_t *addr(uint32_t j) const {
        return reinterpret_cast<const uint8_t *>(a[j]);
    }
};

__global__ __launch_bounds__(kThreads, COOKF_OCC) void k_cook_frame(CookArgs a, FuseArgs f) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const bool ck = !(a.flags & RSMI_COOK_NO_CHECKSUM);
    const bool obs = !(a.flags & RSMI_COOK_NO_OBSCURE);
    if (ck) load_tables(lds, a.tabs, kCookTabDecook);
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, sub = lane / kLpp, hl = lane % kLpp;
    uint8_t *scr = reinterpret_cast<uint8_t *>(lds + kCookTabDecook) + (wid * kPpw + sub) * kScrFuse;
    uint32_t *iv2w = reinterpret_cast<uint32_t *>(scr);
    uint8_t *ovl = scr + 64;
    uint64_t *raddr = reinterpret_cast<uint64_t *>(scr + kScrCook);
    uint32_t *roff = reinterpret_cast<uint32_t *>(scr + kScrCook + 8 * kFuseRecs);
    const uint32_t *T = lds;
    const int64_t nunits = (a.count + kPpw - 1) / kPpw;

    for (int64_t pw = (int64_t)blockIdx.x * (kThreads / 64) + wid; pw < nunits;
         pw += (int64_t)gridDim.x * (kThreads / 64)) {
        const int64_t pk = kPpw * pw + sub;
        const bool have = pk < a.count;
        const int64_t gi = have ? (int64_t)a.pk[pk].event : pk;
        int L = -1, ivl = 0;
        FrameGroup G{};
        int64_t slot = 0;
        if (have) {
            slot = a.pk[pk].slot;
            L = a.pk[pk].len;
            G = f.groups[f.job[pk]];
        }
        const uint64_t po = have ? (uint64_t)slot * (uint64_t)a.stride + (uint64_t)a.pk_off : 0u;
        uint8_t *pkt = have ? a.base + po : nullptr;
        uint8_t *opkt = !have ? nullptr : a.dst_off ? a.dst + a.dst_off[gi] : a.dst + po;
        const int ph = (int)((uintptr_t)pkt & 15);
        uint8_t *pga = pkt - ph;
        uint8_t *oga = opkt - ph;
        // COOKF_LINE: the lanes' piece grid starts on the 128-byte line that
        // holds the packet's first grid piece (the slot start: that piece is
        // 112 B in), `lead` pieces before it, which no lane touches -- so one
        // store instruction writes whole lines of the plain slot (and of a
        // slot-layout output), where the packet's own grid made every line
        // two stores of different rounds (1.24x the plain stream's bytes,
        // profiles/r05/cook_frame_probes)
        const int lead = COOKF_LINE ? (int)(((uintptr_t)pga & 127) >> 4) : 0;
        const uint32_t i = (uint32_t)(slot - (int64_t)G.slot0);  // shard index in its group
        const bool m0 = G.mode == 0;
        const uint32_t fl = G.fec_len;
        // the records the shard overlaps: j0 = the one holding its first byte
        // (mode 1: the shard's own), j1 = the first past its end
        const uint32_t rj = have ? f.rec[pk] : 1u;
        const uint32_t j0 = m0 ? rj >> 8 : i, nrec = rj & 255u;  // (found by the planner)
        if (have && hl < (int)nrec && nrec <= (uint32_t)kFuseRecs) {
            const FrameSrc r = f.srcs[G.src0 + j0 + hl];
            raddr[hl] = (uint64_t)(uintptr_t)f.carry.resolve(r.addr);
            const uint32_t o = m0 ? r.off : 0u;
            roff[hl] = o;
            if (hl == (int)nrec - 1) roff[nrec] = o + 2 + r.len;
        }
        // shards cfirst..nclean-1 are cooked here, nclean..nfr-1 only framed
        // (their stale blob bytes come later; list B cooks them)
        const bool ckit = have && i < G.nclean;
        if (ckit && obs) ivl = 4 + (int)(splitmix(a.seed, (uint64_t)gi, 0) % 29u);
        const int out = L + (ck ? 4 : 0) + (obs ? ivl + 1 : 0);
        const int Lg = L + ph, outg = out + ph;
        // whole grid pieces of the plain packet: header, then the shard to fec_len
        const int pext = 16 + (int)((fl + 15) & ~15u);
        const bool ok = have && ph == 8 && (((uintptr_t)opkt & 15) == 8) && L >= 0 &&
                        L <= RSMI_COOK_MAX_LEN && nrec <= (uint32_t)kFuseRecs && i >= G.cfirst &&
                        i < G.nfr &&
                        (a.dst_off || round16(outg) - ph <= a.cap) && pext - ph <= a.cap;
        const bool cookit = ok && ckit;
        const int ext = cookit ? round16(outg) : 0;
        const int xall = ok ? max(ext, pext) : 0;  // pieces to assemble
        const uint32_t magic = ivl ? 0xFFFFFFFFu / (uint32_t)ivl : 0u;
        if (ok && ivl && 8 * hl < ivl) {
            const uint64_t z = splitmix(a.seed, (uint64_t)gi, 1 + (uint64_t)hl);
            reinterpret_cast<uint32_t *>(ovl)[2 * hl] = (uint32_t)z;
            reinterpret_cast<uint32_t *>(ovl)[2 * hl + 1] = (uint32_t)(z >> 32);
        }
        wave_sync();
        if (ok && ivl) {
            for (int t = hl; t < ivl + 20; t += kLpp) {
                const uint32_t j = mod_ivl((uint32_t)t, (uint32_t)ivl, magic);
                scr[t] = ovl[j];
            }
        }
        wave_sync();
        const LdsRecs rv{raddr, roff};
        const uint32_t sbase = m0 ? i * fl : 0u;                   // stream position of shard byte 0
        const uint32_t slen = m0 ? G.blob_len : roff[1];           // stream end
        const uint32_t w1 = (uint32_t)G.mode |
                            (m0 ? ((uint32_t)G.k << 8 | (uint32_t)G.m << 16) : 0u) |
                            ((G.idx0 + i) & 0xffu) << 24;         // header (fec_manager.cpp:318-333)
        const uint32_t sstep = ivl ? mod_ivl(16u * kLpp, (uint32_t)ivl, magic) : 0u;
        const int Q = cookit ? (Lg + 15) >> 4 : 0;
        const int P0 = Lg & ~15;
        const int nrm = wave_max((xall + 16 * lead + kRoundF - 1) / kRoundF);
        uint32_t acc = 0;
        u32x4 dt = {0, 0, 0, 0};
        int Pt = -1;
#if COOKF_ONE_CHAIN
        // a lane's pieces in every round continue one arithmetic sequence (slot
        // s = r kPplF + p, step 16 kLpp), so its Horner chain runs across the
        // rounds and is finished once: no per-round lane maps, swizzles and
        // Z_{16 qr} shifts (for a 1.2 KB packet, 72 of a lane's ~270 lookups)
        RoundCrc<false> rcx;
#endif
        for (int r = 0; r < nrm; ++r) {
            // ---- frame: the round's pieces from the staged records
            u32x4 cur[kPplF];
            int slow = 0;  // bit p: piece p crosses a record or stream boundary
            const uint8_t *A[kPplF];
#pragma unroll
            for (int p = 0; p < kPplF; ++p) {
                const int P = r * kRoundF + 16 * (kLpp * p + hl - lead);
                A[p] = reinterpret_cast<const uint8_t *>(raddr);  // readable dummy
                if (P > 0 && P < xall) {
                    const uint32_t b = sbase + (uint32_t)(P - 16);
                    const uint32_t bb = m0 ? max(b, 4u) : b;
                    uint32_t t = 0;
                    for (uint32_t u = 1; u < nrec; ++u) t = roff[u] <= bb ? u : t;
                    const uint32_t q0 = roff[t] + 2, q1 = roff[t + 1];
                    if (nrec && b >= q0 && b + 16 <= q1) A[p] = rv.addr(t) + (b - q0);
                    else slow |= 1 << p;
                }
            }
#pragma unroll
            for (int p = 0; p < kPplF; ++p)
                cur[p] = (COOKF_PROBE & 4) ? u32x4{0, 0, 0, 0} : fpiece::window(A[p], 0, 16);
#pragma unroll
            for (int p = 0; p < kPplF; ++p) {
                const int P = r * kRoundF + 16 * (kLpp * p + hl - lead);
                if (P == 0) {
                    cur[p] = u32x4{0u, 0u, __builtin_bswap32(G.seq), w1};
                } else if (P >= xall || P < 0) {
                    cur[p] = u32x4{0u, 0u, 0u, 0u};
                } else if (slow & (1 << p)) {
                    const uint32_t b = sbase + (uint32_t)(P - 16);
                    const uint32_t bb = m0 ? max(b, 4u) : b;
                    uint32_t t = 0;
                    for (uint32_t u = 1; u < nrec; ++u) t = roff[u] <= bb ? u : t;
                    cur[p] = fpiece::stream_piece(rv, t, nrec, (int64_t)b, (int64_t)slen, m0, G.nsrc);
                }
                if (P >= 0 && P < pext && ok && !(COOKF_PROBE & 1) && !((COOKF_PROBE & 8) && P == 0))
                    st_piece(pga + P, cur[p]);  // the plain packet, for the encoder
            }
            // ---- cook (k_cook's round, one Horner chain)
            // (lead: round r's slot p holds pieces kLpp (r kPplF + p) + hl - lead)
            const int qr = min(max(Q + lead - kPplF * kLpp * r, 0), kPplF * kLpp);
            const int qr_max = COOK_SKIP ? wave_max(qr) : kPplF * kLpp;
#if COOKF_ONE_CHAIN
            RoundCrc<false> &rc = rcx;
#else
            RoundCrc<false> rc;
#endif
            uint32_t ivr = ivl ? mod_ivl((uint32_t)(r * kRoundF + 16 * (hl - lead) + 128 * ivl - ph), (uint32_t)ivl,
                                         magic)
                               : 0u;
#pragma unroll
            for (int p = 0; p < kPplF; ++p) {
                const int P = r * kRoundF + 16 * (kLpp * p + hl - lead);
#if COOKF_ONE_CHAIN
                if (ck && kLpp * p < qr_max && P >= 0) {
                    const int sl = r * kPplF + p;  // the lane's slot over all rounds
                    rc.add(T, crc_in_ph(cur[p], P, Lg, ph), sl, kLpp * sl + hl - lead, Q);
                }
#else
                if (ck && kLpp * p < qr_max) rc.add(T, crc_in_ph(cur[p], P, Lg, ph), p, kLpp * p + hl, qr);
#endif
                if (P >= 0 && P < ext && P + 16 <= Lg) {
                    u32x4 m = ks_piece(a, P - ph);
                    if (ivl) m ^= iv_window_at(iv2w, ivr);
                    if (!(COOKF_PROBE & 2)) st_piece(oga + P, cur[p] ^ m);
                } else if (P < ext && P >= P0) {
                    dt = cur[p];
                    Pt = P;
                }
                if (ivl) ivr = iv_step(ivr, sstep, (uint32_t)ivl);
                if (COOK_SB && p % COOK_SB == COOK_SB - 1) __builtin_amdgcn_sched_barrier(0);
            }
#if !COOKF_ONE_CHAIN
            if (ck) {
                const uint32_t c = rc.finish(T, qr);
                const uint32_t nacc = (r ? shift_pieces_n<kPplF>(T, acc, qr) : 0u) ^ c;
                acc = qr > 0 ? nacc : acc;
            }
#endif
        }
#if COOKF_ONE_CHAIN
        if (ck) acc = rcx.finish(T, Q);
#endif
        uint32_t crc = 0;
        if (ck && L > 0 && cookit) crc = ~unshift(T, acc, (uint32_t)(16 * Q - Lg));
        if (cookit) {
            for (int t = hl; t < 64; t += kLpp) {
                const int pos = P0 + t - ph;
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
                }
                ovl[t] = (uint8_t)v;
            }
        }
        wave_sync();
        if (Pt >= 0) {
            const u32x4 k = ks_piece(a, Pt - ph);
            u32x4 m = k;
            if (ivl) m ^= iv_window(iv2w, (uint32_t)(Pt + 16 * ivl - ph), (uint32_t)ivl, magic);
            const u32x4 o = *reinterpret_cast<const u32x4 *>(ovl + (Pt - P0));
            const u32x4 lo = piece_mask(Lg - Pt), hi = piece_mask(outg - Pt);
            st_piece(oga + Pt, ((dt ^ m) & lo) | ((o ^ k) & hi & ~lo) | (dt & ~hi));
        }
        // (a packet only framed here gets its out_len from list B's cook)
        if (have && hl == 0 && (cookit || !ok)) a.out_len[gi] = ok ? out : -1;
        wave_sync();
    }
}

}  // namespace

size_t cook_lds_bytes(bool decook) {
    return (size_t)(decook ? kCookTabDecook : kCookTabWords) * 4 +
           (size_t)(kThreads / kLpp) * (decook ? kScrDecook : kScrCook);
}

hipError_t launch_cook_frame(const CookArgs &a, const FuseArgs &f, int max_blocks, hipStream_t s) {
    if (a.count <= 0) return hipSuccess;
    const int64_t units = (a.count + kPpw - 1) / kPpw;
    int64_t blocks = (units + kThreads / 64 - 1) / (kThreads / 64);
    if (blocks > max_blocks) blocks = max_blocks;
    const size_t lds = (size_t)kCookTabDecook * 4 + (size_t)(kThreads / kLpp) * kScrFuse;
    k_cook_frame<<<(unsigned)blocks, kThreads, lds, s>>>(a, f);
    return hipGetLastError();
}

hipError_t launch_cook(const CookArgs &a, bool decook, int max_blocks, hipStream_t s) {
    if (a.count <= 0) return hipSuccess;
    const int64_t units = (a.count + kPpw - 1) / kPpw;
    int64_t blocks = (units + kThreads / 64 - 1) / (kThreads / 64);
    if (blocks > max_blocks) blocks = max_blocks;
    const size_t lds = cook_lds_bytes(decook);
    if (decook)
        k_decook<<<(unsigned)blocks, kThreads, lds, s>>>(a);
    else if (a.prex)
        k_cook<true><<<(unsigned)blocks, kThreads, lds, s>>>(a);
    else
        k_cook<false><<<(unsigned)blocks, kThreads, lds, s>>>(a);
    return hipGetLastError();
}

}  // namespace rsmi

#if COOK_TRACE
extern "C" int rsmi_debug_cook_trace(void *dev_ptr) {  // measurement builds only
    return hipMemcpyToSymbol(HIP_SYMBOL(rsmi::g_cook_trace), &dev_ptr, sizeof(dev_ptr)) == hipSuccess ? 0 : -1;
}
#endif
