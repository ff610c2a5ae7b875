// decode.hip -- batched RS decode for gfx950: one wavefront per group builds
// that group's decode matrix and streams the reconstruction.
//
// Semantics are rs_decode2's (lib/rs.cpp:21-40 -> lib/fec.cpp:838-882): the k
// survivors used are the first k present shards in ascending index order; a
// missing data row d_j is a fixed GF(2^8) combination of them.  With E the
// missing data rows (|E| = e) and R the e parity rows among the survivors,
//     d_E = A^-1 (p_R + B d_P),   A = enc[R][E],  B = enc[R][P]
// Gauss-Jordan on [A | M] (M's column per survivor: a unit vector for a parity
// survivor, enc[R][s] for a data survivor) leaves [I | coef]; the inverse is
// unique, so coef equals the rows fec_decode derives.  No pivot search is
// needed: every leading minor of A is a square submatrix of the code's parity
// rows, invertible because the code is MDS.  Rebuilt rows are written into
// their own (data) slots.
//
// Per wave and group:
//   1. ballot the group's present flags -> sel[k], miss[e], status;
//   2. issue the first RING survivor loads (they fly during step 3);
//   3. Gauss-Jordan with column c of [A | M] in lane c (e bytes in registers,
//      W = e + k <= 64; wider systems use the wave's LDS slice); multiplies by
//      a wave-uniform factor go through that factor's v_perm split table;
//      expand every coefficient into its split table (5 dwords, see
//      kernels.hip) in LDS;
//   4. stream: per survivor, 5 dwords per lane (one 1-KiB dwordx4 wave-load +
//      one 256-B dword wave-load cover a 1280-B tile), GF multiply-accumulate
//      into the row accumulators, prefetch survivor j+RING; store the rows.
// Buffer descriptors with out-of-range offsets handle ragged tails: those
// loads read 0 and those stores are dropped.
//
// Kernels: k_decode_fused (uniform batch: one code, the code's parity rows in
// LDS), k_decode_ragged (every group its own k, n, len, stride; parity rows
// read through the device code directory) and k_decode_ragged_big (one
// workgroup per group for the groups the one-wave form defers: e > 10, k > 32
// or a slot extent >= 2 GiB).
#include "rsmi_internal.hpp"

namespace rsmi {
namespace {

constexpr int kWaves = 4;      // waves per block (one group each)
#ifndef DEC_RING
#define DEC_RING 2             // fused kernel: survivors in flight (2 at 5 waves/SIMD: decode -1 %,
                               // C2 worst -1.5 % against 4 at 4 waves/SIMD, profiles/r03/dec_occ5_ab.txt)
#endif
#ifndef DEC_LD_AUX
#define DEC_LD_AUX 2           // cache policy of the survivor loads: nt (bench step: decode
                               // 0.466 vs 0.475 ms with default-policy loads, encode unchanged)
#endif
#ifndef DEC_RAG_LD_AUX
#define DEC_RAG_LD_AUX DEC_LD_AUX  // ... of the ragged kernels' survivor loads (TileIO)
#endif
#ifndef DEC_ST_AUX
#define DEC_ST_AUX 16          // cache policy of the uniform kernel's rebuilt-row stores: sc1
                               // (round 5, scripts/gpu_ab.sh c2: C2 random 0.389-0.395 vs 0.397-0.403 ms
                               // with default stores; profiles/r05/c2_store_policy_ab)
#endif
#ifndef DEC_ST_AUX_BIG
#define DEC_ST_AUX_BIG 2       // ... for a group rebuilding >= DEC_ST_BIG_E rows: nt (C2 worst case,
                               // 5 rows per group: 0.431-0.435 vs 0.449 ms with sc1, 0.465 default)
#endif
#ifndef DEC_ST_BIG_E
#define DEC_ST_BIG_E 5            // (4: C2 random 0.385-0.387 vs 0.381-0.383 ms at 5)
#endif
#ifndef DEC_REF_ST_AUX
#define DEC_REF_ST_AUX 16      // store policy of the reference-placement rows (over the parity survivors
                               // just read): sc1 as for own slots (round 6, profiles/r06/c2_place_ab.txt:
                               // C2 random 0.3768-0.3789 ms vs own slots 0.3775-0.3783; default policy
                               // 0.380-0.383, nt 0.398; the pattern probe's "last survivors' slots" gain
                               // does not carry over to the kernel)
#endif
#ifndef DEC_REF_ST_AUX_BIG
#define DEC_REF_ST_AUX_BIG 2
#endif
#ifndef DEC_RAG_ST_AUX
#define DEC_RAG_ST_AUX 16      // cache policy of the ragged kernels' rebuilt-row stores: sc1 (C3 decode
                               // 0.135-0.136 vs 0.137-0.138 ms default, 0.145-0.148 nt)
#endif
constexpr int kRing = DEC_RING;  // survivors in flight per wave
constexpr int kRows = 10;      // max e handled by the one-wave kernels
constexpr int kPass = 5;       // rows accumulated per pass over the survivors
#ifndef DEC_FPASS
#define DEC_FPASS 5            // ... in the fused uniform kernel (<= kTabRows)
#endif
constexpr int kFPass = DEC_FPASS;
constexpr int kTile = 1280;    // bytes per lane-tile pass (64 x 16 + 64 x 4)
#ifndef DEC_ST_SGPR
#define DEC_ST_SGPR 0          // 1: row offset of the rebuilt-row stores in soffset (see bitslice.hip
                               // DevIO::store: no hazard wait state is inserted for that form)
#endif
#ifndef DEC_OCC
#define DEC_OCC 5              // waves per SIMD the fused kernel's register budget is cut for
#endif
#ifndef DEC_FAKE
#define DEC_FAKE 0             // measurement only: rows computed per survivor (0 = e, the real decode)
#endif
#ifndef DEC_NOMEM
#define DEC_NOMEM 0            // measurement only: survivor loads all hit one cached slot
#endif
#ifndef DEC_RAG_RING4
#define DEC_RAG_RING4 2  // ragged kernels: survivors in flight for 16-byte lane pieces
#endif
#ifndef DEC_RAG_RING5
#define DEC_RAG_RING5 2  // ... and for 20-byte pieces (round 4: 2 at 7 waves/SIMD in the merged class launch, 0.139-0.142 vs 0.1425 ms for 3 at 6)
#endif
#ifndef DEC_RAG_UNCOND_W
#define DEC_RAG_UNCOND_W 4  // ragged kernels: unconditional ring refills for tile widths >= this
#endif
#ifndef DEC_RAG_ALLROWS
#define DEC_RAG_ALLROWS 0  // ragged kernels: tile widths <= this multiply every row of a pass
                           // (no per-row scalar compare and branch per survivor).  Round 6
                           // (profiles/r06/c3_allrows_ab.txt): C3 decode 0.153 ms for W <= 2,
                           // 0.477 ms for every width, against 0.138-0.142 ms guarded
#endif
#ifndef DEC_RAG_DEEP
#define DEC_RAG_DEEP 1  // ragged kernel: 16 / W survivors in flight for 4- and 8-byte lane pieces
#endif
#ifndef DEC_XCD
#define DEC_XCD 1              // XCD-contiguous group ranges (see k_decode_fused; ~0.5 %)
#endif
#ifndef DEC_ROWGUARD
#define DEC_ROWGUARD 1         // fused kernel: row guards on an opaque SGPR (see the MAC loop)
#endif
#ifndef DEC_GRID_PER_CU
#define DEC_GRID_PER_CU 8      // fused kernel: blocks per CU in the (persistent) grid
#endif
#ifndef DEC_PAIR
#define DEC_PAIR 0             // uniform kernel: fold survivors in pairs (fewer XORs, more VGPRs)
#endif
#ifndef DEC_ORDER
#define DEC_ORDER 1            // ring loads issued in slot order (precise vmcnt in the survivor loop)
#endif
constexpr int kDefer = 0x100;  // internal status: left for k_decode_ragged_big
#ifndef DEC_TRACE
#define DEC_TRACE 0            // measurement only: per-group phase timestamps of the class kernels
#endif
#if DEC_TRACE
__device__ uint64_t *g_dec_trace;  // [group][8]: t0 t1 t2 t3 info wave tk0 tk1 (rsmi_debug_dec_trace)
__device__ __forceinline__ uint64_t trace_now() {
    asm volatile("" ::: "memory");
    const uint64_t t = __builtin_amdgcn_s_memtime();
    asm volatile("" ::: "memory");
    return t;
}
#endif

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kTabBytes = 6144;  // smem: s01 | s2 | exp | log | inv, then per-kernel regions

// The block-shared tables: v_perm split tables of all 256 coefficients, GF
// exp/log and inverses.
struct Tables {
    const uint4 *s01;
    const uint32_t *s2;
    const uint8_t *lexp, *llog, *linv;
};

__device__ __forceinline__ Tables load_tables(uint8_t *smem, const uint32_t *ptab,
                                              const uint8_t *gftab) {
    uint4 *s01 = reinterpret_cast<uint4 *>(smem);              // 256 x 16 B
    uint32_t *s2 = reinterpret_cast<uint32_t *>(smem + 4096);  // 256 x 4 B
    uint8_t *lexp = smem + 5120;                               // 512
    uint8_t *llog = smem + 5632;                               // 256
    uint8_t *linv = smem + 5888;                               // 256: x^-1
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        s01[i] = reinterpret_cast<const uint4 *>(ptab + i * kPtabDwords)[0];
        s2[i] = ptab[i * kPtabDwords + 4];
    }
    for (int i = threadIdx.x; i < 768; i += blockDim.x) smem[5120 + i] = gftab[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x)
        linv[i] = i ? gftab[255 - gftab[512 + i]] : 0;  // exp[255 - log x]
    return Tables{s01, s2, lexp, llog, linv};
}

__device__ __forceinline__ uint32_t gmul(const uint8_t *lexp, const uint8_t *llog, uint32_t a,
                                         uint32_t b) {
    return (a && b) ? lexp[llog[a] + llog[b]] : 0u;
}

#include "lagrange.hpp"

struct WaveLds {  // per-wave LDS slice
    uint8_t *sel, *miss, *aug;
    uint32_t *tab;  // k_decode_fused: [k][kRows] entries of 8 dwords (T0lo T0hi T1lo T1hi T2 - - -)
    // ragged kernels: coefficient (j, r)'s split table is t01[j * rows + r]
    // (T0lo T0hi T1lo T1hi) and t2[j * rows + r] (T2): 20 bytes, not 32
    uint4 *t01;
    uint32_t *t2;
    int rows;
};


// fused kernel: split-table rows per survivor in the wave's slice, one block
// of kPass rows at a time (each block's Lagrange coefficients are computed
// when its pass starts)
constexpr int kTabRows = 5;

__host__ __device__ inline int wave_lds_bytes(int k) {
    return 512 + k * kTabRows * 32;  // sel[256] miss[256] tab[k * kTabRows * 32]
}

// Ragged kernels' slice: sel[64] miss[64] t01[k*rows] t2[k*rows] (k <= 32;
// the split tables of one block of `rows` missing rows at a time).
__host__ __device__ inline int rag_lds_bytes(int k, int rows) { return 128 + k * rows * 20; }

__device__ __forceinline__ WaveLds rag_slice(uint8_t *wl, int k, int rows) {
    uint4 *t01 = reinterpret_cast<uint4 *>(wl + 128);
    return WaveLds{wl, wl + 64, nullptr, nullptr, t01,
                   reinterpret_cast<uint32_t *>(t01 + k * rows), rows};
}

// ---- 1. survivor selection (rs.cpp:24-39) ------------------------------------
// flag(b, idx) is the present flag of shard idx (b = idx rounded down to 64);
// writes sel[0..k) (the first k present, ascending) and miss[0..e) (missing
// data rows, ascending).  Returns the present count, e in e_out.
template <class Flag>
__device__ __forceinline__ int select_survivors(int k, int n, Flag flag, const WaveLds &L, int lane,
                                                int &e_out) {
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    int cnt = 0, e = 0;
    for (int b = 0; b < n && cnt < k; b += 64) {
        const int idx = b + lane;
        const bool f = idx < n && flag(b, idx);
        const uint64_t mk = __ballot(f);
        const int rank = cnt + __popcll(mk & lt);
        if (f && rank < k) L.sel[rank] = (uint8_t)idx;
        cnt += __popcll(mk);
    }
    if (cnt >= k) {
        for (int b = 0; b < k; b += 64) {
            const int idx = b + lane;
            const bool ms = idx < k && !flag(b, idx);
            const uint64_t mk = __ballot(ms);
            if (ms) L.miss[e + __popcll(mk & lt)] = (uint8_t)idx;
            e += __popcll(mk);
        }
    }
    // values that steer control flow are wave-uniform: say so, or the
    // compiler wraps every buffer op below in a waterfall loop
    e_out = __builtin_amdgcn_readfirstlane(e);
    return __builtin_amdgcn_readfirstlane(cnt);
}

// Lagrange coefficients (see LTables above) for k <= 64 survivors, e <= NR
// missing data rows: lane s < k holds survivor s's shard index in sel_lane,
// lane d < e missing row d's in miss_lane.  Leaves coef[r][j]'s split table at
// (t01, t2)[j * rows + r], where Rebuild reads them.
template <int NR>
__device__ __forceinline__ void lagrange_coefs(int k, int e, uint32_t sel_lane, uint32_t miss_lane,
                                               const WaveLds &L, const LTables &T, int lane) {
    const uint32_t xs = T.px[sel_lane & 255u];
    const uint32_t xm = T.px[miss_lane & 255u];
    const uint32_t B = lagrange_b(k, xs, T);
    const int base = lane * L.rows;
    lagrange_rows<NR>(k, e, xs, B, xm, T, lane, [&](int r, uint32_t v) {
        L.t01[base + r] = T.t01[v];
        L.t2[base + r] = T.t2[v];
    });
    wave_sync();
}

// Tile geometry for W dwords per lane: W = 1, 2, 4 is one 4W-byte load per
// lane (a 256W-byte tile); W = 5 is a 16-byte load plus a dword load (1280 B).
template <int W>
struct TileIO {
    static_assert(W == 1 || W == 2 || W == 4 || W == 5, "lane pieces must divide 16");
    static constexpr int kBytes = 256 * W;
    uint32_t v16, v4;  // per-lane offsets of the two loads (v4 unused for W <= 4)
    __device__ __forceinline__ void set(int toff, int tlen, int lane) {
        const int a = (W == 5 ? 16 : 4 * W) * lane;
        v16 = a < tlen ? (uint32_t)(toff + a) : 0x80000000u;
        v4 = (W == 5 && 1024 + 4 * lane < tlen) ? (uint32_t)(toff + 1024 + 4 * lane) : 0x80000000u;
    }
    __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, uint32_t so, uint32_t (&x)[W]) const {
        if constexpr (W == 1) {
            x[0] = __builtin_amdgcn_raw_buffer_load_b32(r, v16, so, DEC_RAG_LD_AUX);
        } else if constexpr (W == 2) {
            typedef uint32_t u2 __attribute__((ext_vector_type(2)));
            const u2 v = __builtin_amdgcn_raw_buffer_load_b64(r, v16, so, DEC_RAG_LD_AUX);
            x[0] = v.x; x[1] = v.y;
        } else {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, v16, so, DEC_RAG_LD_AUX);
            x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
            if constexpr (W == 5) x[4] = __builtin_amdgcn_raw_buffer_load_b32(r, v4, so, DEC_RAG_LD_AUX);
        }
    }
    // offsets in the VGPR, soffset 0 (see bitslice_kern.hpp DevIO::store)
    __device__ __forceinline__ void store(__amdgpu_buffer_rsrc_t r, uint32_t so, const uint32_t (&y)[W]) const {
        if constexpr (W == 1) {
            __builtin_amdgcn_raw_buffer_store_b32(y[0], r, v16 + so, 0, DEC_RAG_ST_AUX);
        } else if constexpr (W == 2) {
            typedef uint32_t u2 __attribute__((ext_vector_type(2)));
            const u2 v = {y[0], y[1]};
            __builtin_amdgcn_raw_buffer_store_b64(v, r, v16 + so, 0, DEC_RAG_ST_AUX);
        } else {
            const u32x4 v = {y[0], y[1], y[2], y[3]};
            __builtin_amdgcn_raw_buffer_store_b128(v, r, v16 + so, 0, DEC_RAG_ST_AUX);
            if constexpr (W == 5) __builtin_amdgcn_raw_buffer_store_b32(y[4], r, v4 + so, 0, DEC_RAG_ST_AUX);
        }
    }
};

// ---- 2 + 4. survivor streaming ---------------------------------------------------
// One group's reconstruction: the wave-uniform descriptor covers the group's
// n slots; survivor j's slot offset sits in lane j of so_lane, missing row
// r's in lane r of mo_lane.  W dwords per lane: the ragged kernel picks the
// narrowest tile that covers a short group, so its MACs do not run over empty
// lanes.
template <int W>
struct Rebuild {
    // narrow tiles keep more survivors in flight in the same registers (16
    // dwords of ring): short groups are latency-bound, not VGPR-bound
    static constexpr int R = DEC_RAG_DEEP && W <= 2 ? 16 / W : (W == 4 ? DEC_RAG_RING4 : DEC_RAG_RING5);
    __amdgpu_buffer_rsrc_t rsrc, rnull;  // rnull: num_records 0, every load reads 0
    uint32_t so_lane, mo_lane;
    int k, e, len, lpad;
    TileIO<W> io;
    uint32_t rq[R][W];

    // Ring slot q <- survivor j.  For the wide tiles (W >= 4, rings of 2-3)
    // the refills are unconditional: past the last survivor they go through
    // rnull (no memory access, zeros).  A refill under "if (j < k)" makes
    // rq[q] a loop-carried phi of old and new values, and the compiler then
    // loads into spare registers and copies them back at the bottom of the
    // loop behind an s_waitcnt vmcnt(0): every iteration waited for the loads
    // it had just issued.  The narrow tiles keep the guard: their deep rings
    // (8-16 slots) would issue that many dead loads per group, and the depth
    // hides the wait anyway.
    static constexpr bool kUncond = W >= DEC_RAG_UNCOND_W;
    static constexpr bool kAllRows = W <= DEC_RAG_ALLROWS;
    __device__ __forceinline__ void load(int q, int j) {
        if (kUncond) {
            const bool ok = j < k;
            io.load(ok ? rsrc : rnull, (uint32_t)__builtin_amdgcn_readlane(so_lane, ok ? j : 0), rq[q]);
        } else if (j < k) {
            io.load(rsrc, (uint32_t)__builtin_amdgcn_readlane(so_lane, j), rq[q]);
        }
    }
    // whole cache lines where the slot has room (rsmi.h padding rule)
    __device__ __forceinline__ void start_tile(int toff, int lane) {
        io.set(toff, lpad - toff, lane);
#pragma unroll
        for (int q = 0; q < R; ++q) load(q, q);
    }
    // Rows [rb0, rb0 + nrows) (their coefficients at table rows 0..nrows-1),
    // in passes over (tile, block of kPass rows); the first pass's loads were
    // issued by start_tile(0) before the coefficients.
    __device__ __forceinline__ void run(const WaveLds &L, int lane, int rb0, int nrows) {
        const int rend = rb0 + nrows;
        for (int toff = 0; toff < len; toff += TileIO<W>::kBytes) {
            for (int rb = rb0; rb < rend; rb += kPass) {
                if (toff || rb != rb0) start_tile(toff, lane);
                uint32_t acc[kPass][W];
#pragma unroll
                for (int r = 0; r < kPass; ++r)
#pragma unroll
                    for (int w = 0; w < W; ++w) acc[r][w] = 0;
                // a VGPR zero the compiler cannot see through: the per-survivor
                // table addresses become one VALU add each (rows at immediate
                // offsets) instead of a v_mov of an SGPR address per row
                int z = 0;
                asm volatile("" : "+v"(z));
                for (int jb = 0; jb < k; jb += R) {
#pragma unroll
                    for (int q = 0; q < R; ++q) {
                        const int j = jb + q;
                        // the 3-bit split selectors of the survivor's W dwords
                        uint32_t a0[W], a1[W], a2[W];
                        if (j < k) {
#pragma unroll
                            for (int w = 0; w < W; ++w) {
                                a0[w] = rq[q][w] & 0x07070707u;
                                a1[w] = (rq[q][w] >> 3) & 0x07070707u;
                                a2[w] = (rq[q][w] >> 6) & 0x03030303u;
                            }
                        }
                        // ring slot q took survivor j: load survivor j + R into it
                        load(q, j + R);
                        if (j < k) {
                            const uint4 *ta = L.t01 + (z + j * L.rows + (rb - rb0));
                            const uint32_t *ta2 = L.t2 + (z + j * L.rows + (rb - rb0));
                            int nr = rend - rb;  // opaque SGPR: see k_decode_fused's row guards
                            asm volatile("" : "+s"(nr));
#pragma unroll
                            for (int r = 0; r < kPass; ++r) {
                                // kAllRows: every row of the pass, no per-row branch (rows
                                // past nr read stale table entries and are never stored)
                                if (kAllRows || r < nr) {
                                    const uint4 t = ta[r];
                                    const uint32_t t2 = ta2[r];
#pragma unroll
                                    for (int w = 0; w < W; ++w)
                                        acc[r][w] ^= xor3(__builtin_amdgcn_perm(t.y, t.x, a0[w]),
                                                          __builtin_amdgcn_perm(t.w, t.z, a1[w]),
                                                          __builtin_amdgcn_perm(t2, t2, a2[w]));
                                }
                            }
                        }
                    }
                }
#pragma unroll
                for (int r = 0; r < kPass; ++r)
                    if (rb + r < rend) io.store(rsrc, __builtin_amdgcn_readlane(mo_lane, rb + r), acc[r]);
            }
        }
    }
};

// descriptor base through readfirstlane (cdna_hip_programming.md T20)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t group_rsrc(const uint8_t *gbase, uint32_t bytes) {
    const uint64_t gb = (uint64_t)(uintptr_t)gbase;
    const uint64_t gbu = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(gb >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)gb);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<uint8_t *>(gbu), 0, (int)bytes,
                                             0x00020000);
}

// The uniform kernel keeps its own straight-line form (not Rebuild / the
// helper functions): written that way it fits 4 waves/SIMD without spills.
// LDAUX / STAUX: cache policy of the survivor loads and rebuilt-row stores --
// DEC_LD_AUX / DEC_ST_AUX for HBM; sc0|sc1 (system scope, coherent with the
// host) when the shards are pinned host memory read over PCIe
// (rsmi_decode_pinned's zero-copy path).
// REF: the reference's placement (rsmi_decode_dev_ref): rebuilt data row i
// goes over the parity survivor fec_decode's shuffle leaves in data[i]
// (fec.cpp:755-788, 872-877), and slot_map (may be null) receives, per group,
// the slot now holding each data row.
template <int LDAUX, int STAUX, int STBIG, int REF>
__global__ __launch_bounds__(256, DEC_OCC) void k_decode_fused(UniformArgs a, const uint8_t *present,
                                                      const uint8_t *prows, int32_t *status_out,
                                                      const uint32_t *ptab, const uint8_t *gftab,
                                                      uint8_t *slot_map) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int k = a.k, n = a.n;
    (void)prows;
    const int wbytes = wave_lds_bytes(k);
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    // LTables | per wave: sel[256] miss[256] tab[k][kTabRows] (8 dwords per entry)
    uint8_t *wl = smem + kLTabBytes + wid * wbytes;
    WaveLds L{wl, wl + 256, nullptr, reinterpret_cast<uint32_t *>(wl + 512)};

    // the LTables image (Lagrange coefficients need no parity rows)
    const LTables LT = load_ltables(smem, ptab, gftab);
    __syncthreads();

    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    // DEC_NOMEM (measurement only): every survivor load reads group 0's slot 0
    const __amdgpu_buffer_rsrc_t rsrc0 = __builtin_amdgcn_make_buffer_rsrc(a.base, 0, 4096, 0x00020000);
    const int64_t nwaves = (int64_t)gridDim.x * kWaves;
    // DEC_XCD: blocks b, b+8, ... (dispatched to one XCD) take adjacent groups
    const int64_t bid = (DEC_XCD && (gridDim.x & 7) == 0)
                            ? (int64_t)(blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3)
                            : (int64_t)blockIdx.x;
    const int64_t g0 = bid * kWaves + wid;
    // present flags of the first 64 shards, prefetched one group ahead
    uint32_t pf = (g0 < a.ngroups && lane < n) ? present[g0 * n + lane] : 0u;
    uint32_t pf_next = 0;
    for (int64_t g = g0; g < a.ngroups; g += nwaves, pf = pf_next) {
#if DEC_TRACE
        const uint64_t tr0 = trace_now();
#endif
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
            // nothing moves: data row i stays in slot i (0xFF: erased, too few)
            if (REF && slot_map && lane < k) slot_map[g * k + lane] = pf ? (uint8_t)lane : (uint8_t)0xFF;
            continue;
        }
        // REF: the slot rebuilt row r (lane r) goes to.  fec_decode packs the
        // k survivors sel[] (ascending: s = k - e data shards, then parity)
        // and its shuffle moves each data survivor home, swapping the
        // displaced packet into the vacated position; position x < s
        // therefore passes its final occupant along the chain
        // x -> sel[x] -> ... (strictly increasing) to the first position >= s,
        // which still holds its parity packet: row miss[r] ends in that
        // packet's buffer (pinned against decode_small.npz's ptr_out).
        uint32_t ref_slot = 0;
        if (REF) {
            if (lane < e) {
                int x = L.miss[lane];
                const int s = k - e;
                while (x < s) x = L.sel[x];
                ref_slot = L.sel[x];
            }
            if (slot_map) {
                uint8_t *tmp = L.miss + 128;  // scratch: the slice's miss[] holds e <= 10 entries
                if (lane < e) tmp[L.miss[lane]] = (uint8_t)ref_slot;
                wave_sync();
                if (lane < k) slot_map[g * k + lane] = pf ? (uint8_t)lane : tmp[lane];
            }
        }

#if DEC_TRACE
        const uint64_t tr1 = trace_now();
#endif
        // ---- 2. descriptor + first loads ---------------------------------------
        // descriptor inputs through readfirstlane (cdna_hip_programming.md T20)
        const uint64_t gb = (uint64_t)(uintptr_t)(a.base + g * a.group_stride);
        const uint64_t gbu = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(gb >> 32)) << 32) |
                             (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)gb);
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<uint8_t *>(gbu), 0, (int)(a.n * a.shard_stride), 0x00020000);
        // num_records 0: the ring's loads past the last survivor read zeros
        // without touching memory (see Rebuild::load for why they are not
        // skipped instead)
        const __amdgpu_buffer_rsrc_t rnull = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<uint8_t *>(gbu), 0, 0, 0x00020000);
        const uint32_t ss = (uint32_t)a.shard_stride;
        // survivor j's shard offset lives in lane j (k <= 64 on this path):
        // v_readlane gives the scalar soffset without an LDS round trip
        const uint32_t sel_lane = lane < k ? (uint32_t)L.sel[lane] : 0u;
        const uint32_t so_lane = sel_lane * ss;
        const uint32_t mo_lane = (lane < e ? (uint32_t)L.miss[lane] : 0u) * ss;
        const uint32_t ref_lane = ref_slot * ss;
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
                const bool ok = q < k;
                const uint32_t so = __builtin_amdgcn_readlane(so_lane, ok ? q : 0);
                const __amdgpu_buffer_rsrc_t r = DEC_NOMEM ? rsrc0 : (ok ? rsrc : rnull);
                rq[q] = __builtin_amdgcn_raw_buffer_load_b128(r, v16, DEC_NOMEM ? 0u : so, LDAUX);
                rd[q] = __builtin_amdgcn_raw_buffer_load_b32(r, v4, DEC_NOMEM ? 0u : so, LDAUX);
#if DEC_ORDER
                // issue the ring in slot order: the survivor loop refills
                // slot 0 first, and the waitcnt pass merges this entry state
                // with the loop's own; slots issued here in another order make
                // that merge pessimistic (vmcnt(0) at the top of every ring
                // cycle, so only one survivor's compute hides each load)
                __builtin_amdgcn_sched_barrier(0);
#endif
            }
        };
        start_tile(0);  // the first survivors fly while the matrix is inverted

        // ---- 3. Gauss-Jordan on [A | M], e x (e+k) ------------------------------
        // ---- 3. coefficients: Lagrange form (see LTables), computed per block
        // of kFPass rows when the block's pass starts, below

#if DEC_TRACE
        const uint64_t tr2 = trace_now();
#endif
        // ---- 4. stream the survivors: passes over (tile, block of kFPass rows) --
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
        // (unconditional: past the last survivor through rnull)
        auto refill = [&](int q, int j) {
            const bool ok = j + kRing < k;
            const uint32_t so = __builtin_amdgcn_readlane(so_lane, ok ? j + kRing : 0);
            const __amdgpu_buffer_rsrc_t r = DEC_NOMEM ? rsrc0 : (ok ? rsrc : rnull);
            rq[q] = __builtin_amdgcn_raw_buffer_load_b128(r, v16, DEC_NOMEM ? 0u : so, LDAUX);
            rd[q] = __builtin_amdgcn_raw_buffer_load_b32(r, v4, DEC_NOMEM ? 0u : so, LDAUX);
        };
        for (int rb = 0; rb < e; rb += kFPass) {
            if (rb) start_tile(0);  // block 0's first loads are already in flight
            {   // coefficients of rows rb .. rb + kFPass - 1 into the slice's table rows
                const uint32_t xs = LT.px[sel_lane & 255u];
                const uint32_t B = lagrange_b(k, xs, LT);
                const uint32_t xm = lane + rb < e ? (uint32_t)LT.px[L.miss[lane + rb]] : 0u;
                lagrange_rows<kFPass>(k, e - rb < kFPass ? e - rb : kFPass, xs, B, xm, LT, lane,
                                     [&](int r, uint32_t v) {
                                         uint32_t *dst = L.tab + (lane * kTabRows + r) * 8;
                                         reinterpret_cast<uint4 *>(dst)[0] = LT.t01[v];
                                         dst[4] = LT.t2[v];
                                     });
                wave_sync();
            }
            const int rt = rb;  // table row of row rb + r: r
            for (int toff = 0; toff < a.len; toff += kTile) {
                if (toff) start_tile(toff);  // the pass's first loads
                uint32_t acc[kFPass][5];
#pragma unroll
                for (int r = 0; r < kFPass; ++r)
#pragma unroll
                    for (int w = 0; w < 5; ++w) acc[r][w] = 0;
                int z = 0;  // VGPR zero: one address add per survivor (see Rebuild::run)
                asm volatile("" : "+v"(z));
                for (int jb = 0; jb < k; jb += kRing) {
#pragma unroll
                    for (int q = 0; q < kRing; q += DEC_PAIR ? 2 : 1) {
                        const int j = jb + q;
                        if (DEC_PAIR && j + 1 < k) {
                            // two survivors per step: their six split products
                            // fold into a row with three 3-input XORs
                            uint32_t a0[5], a1[5], a2[5], b0[5], b1[5], b2[5];
                            split(rq[q], rd[q], a0, a1, a2);
                            split(rq[q + 1], rd[q + 1], b0, b1, b2);
                            refill(q, j);
                            refill(q + 1, j + 1);
                            const uint32_t *ta = L.tab + (j * kTabRows + rb - rt) * 8;
                            const uint32_t *tb = ta + kTabRows * 8;
#pragma unroll
                            for (int r = 0; r < kFPass; ++r) {
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
                        } else {
                            uint32_t a0[5], a1[5], a2[5];
                            if (j < k) split(rq[q], rd[q], a0, a1, a2);
                            refill(q, j);  // every iteration: see Rebuild::run
                            if (j >= k) continue;
                            const uint32_t *ta = L.tab + (z + (j * kTabRows + rb - rt) * 8);
                            // rows in this pass, as an opaque SGPR per survivor: a
                            // loop-invariant "rb + r < e" is hoisted as a lane-mask
                            // boolean and re-materialised with v_cndmask + v_cmp at
                            // every use (2 VALU per row and survivor)
                            int nr = e - rb;
                            if (DEC_ROWGUARD) asm volatile("" : "+s"(nr));
#pragma unroll
                            for (int r = 0; r < kFPass; ++r) {
                                if (DEC_FAKE ? r < DEC_FAKE : r < nr) {  // DEC_FAKE: measurement only
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
                // the store policy by the group's write share: a group that
                // rebuilds many rows streams them past the caches (STBIG)
                // REF: the last pass writes over the parity survivors (every
                // read of this tile is behind it); earlier passes park their
                // rows in their own (erased) slots, moved after the last pass
                const uint32_t dst_lane = (REF && rb + kFPass >= e) ? ref_lane : mo_lane;
                auto store_rows = [&](auto aux) {
                    constexpr int AUX = decltype(aux)::value;
#pragma unroll
                    for (int r = 0; r < kFPass; ++r) {
                        if (rb + r < e) {
                            const uint32_t so = __builtin_amdgcn_readlane(dst_lane, rb + r);
                            const u32x4 v = {acc[r][0], acc[r][1], acc[r][2], acc[r][3]};
#if DEC_ST_SGPR
                            __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, v16, so, AUX);
                            __builtin_amdgcn_raw_buffer_store_b32(acc[r][4], rsrc, v4, so, AUX);
#else
                            __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, v16 + so, 0, AUX);
                            __builtin_amdgcn_raw_buffer_store_b32(acc[r][4], rsrc, v4 + so, 0, AUX);
#endif
                        }
                    }
                };
                if (STAUX != STBIG && e >= DEC_ST_BIG_E)
                    store_rows(std::integral_constant<int, STBIG>{});
                else
                    store_rows(std::integral_constant<int, STAUX>{});
            }
        }
        if (REF && e > kFPass) {
            // rows of the earlier passes: own slot -> their parity survivor
            // (each lane moves the bytes it stored; the fences order the
            // stores before the loads, which bypass the CU cache)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            const int moved = (e - 1) / kFPass * kFPass;
            for (int toff = 0; toff < a.len; toff += kTile) {
                const int tlen = lpad - toff;
                const uint32_t c16 = (16 * lane < tlen) ? (uint32_t)(toff + 16 * lane) : 0x80000000u;
                const uint32_t c4 = (1024 + 4 * lane < tlen) ? (uint32_t)(toff + 1024 + 4 * lane) : 0x80000000u;
                for (int r = 0; r < moved; ++r) {
                    const uint32_t src = __builtin_amdgcn_readlane(mo_lane, r);
                    const uint32_t dst = __builtin_amdgcn_readlane(ref_lane, r);
                    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, c16, src, 1);
                    const uint32_t d = __builtin_amdgcn_raw_buffer_load_b32(rsrc, c4, src, 1);
                    __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, c16 + dst, 0, STAUX);
                    __builtin_amdgcn_raw_buffer_store_b32(d, rsrc, c4 + dst, 0, STAUX);
                }
            }
        }
        if (lane == 0 && status_out) status_out[g] = RSMI_DEC_OK;
#if DEC_TRACE
        if (lane == 0 && g_dec_trace) {  // phases of the group (scripts/c2_trace.py)
            uint64_t *t = g_dec_trace + g * 8;
            t[0] = tr0; t[1] = tr1; t[2] = tr2; t[3] = trace_now();
            t[4] = (uint64_t)5 | ((uint64_t)k << 8) | ((uint64_t)e << 16) | ((uint64_t)a.len << 32);
            t[5] = (uint64_t)(bid * kWaves + wid);
        }
#endif
        wave_sync();  // the LDS slice is rewritten by the next group
    }
}

// ---- ragged batches ---------------------------------------------------------------
// One wave per group; each group its own (k, n, len, shard_stride, offset) from
// its rsmi_group descriptor, present flags as a 256-bit mask per group (8
// words: bit j of word j/32 = shard j received), parity rows through the
// device code directory.  Groups this form cannot take (e > NR, k > kmax, or
// n slots spanning >= 2 GiB) get kDefer for k_decode_ragged_big.
#ifndef DEC_RAG_W
#define DEC_RAG_W 1  // ragged kernel: tile width per group (0: always 1280-byte tiles)
#endif
#ifndef DEC_RAG_OCC
#define DEC_RAG_OCC 4  // waves per SIMD the ragged (single-kernel) form's registers are cut for
#endif
// class kernels (plans): waves per SIMD per tile width
#ifndef DEC_CLS_OCC1
#define DEC_CLS_OCC1 8
#endif
#ifndef DEC_CLS_OCC2
#define DEC_CLS_OCC2 8
#endif
#ifndef DEC_CLS_OCC4
#define DEC_CLS_OCC4 8
#endif
#ifndef DEC_CLS_OCC5
#define DEC_CLS_OCC5 7
#endif
constexpr int kClsRows = 5;  // class kernels: e <= 5 in registers, more is deferred
#ifndef DEC_MIX
#define DEC_MIX 2  // class launches: 0 one per class, 1 W = 5 alone + the others in one, 2 all in one
#endif
using RagTables = LTables;
constexpr int kRagTabBytes = kLTabBytes;
__device__ __forceinline__ RagTables load_rag_tables(uint8_t *smem, const uint32_t *ptab, const uint8_t *gftab) {
    return load_ltables(smem, ptab, gftab);
}

// One group's wave-uniform description.
struct GroupDesc {
    int64_t g;          // status index
    int k, n, len;
    uint32_t ss;
    uint64_t off;
    const uint8_t *rows;  // the code's parity rows, (n-k) x k (nullptr when n == k)
};

// One group.  WC = tile width (1, 2, 4, 5), or 0: chosen per group.
// flag(b, idx) is shard idx's present flag (b = idx rounded down to 64).
// A deferral mark: the class kernels raise *word to `epoch` (atomic max) when
// they leave a group for k_decode_ragged_big, which does nothing unless
// *word >= its epoch.  Calls number their epochs upwards, so concurrent calls
// on one plan can only make the big kernel scan needlessly, never skip.
struct DeferMark {
    uint32_t *word;  // nullptr: no mark (the big kernel always scans)
    uint32_t epoch;
};

struct NoHook {
    __device__ void operator()() const {}
};

// The reference's placement (RefOut.on; rsmi_decode_dev_ref's rule, ref_slot_of
// over the slice's sel[]): the slot of the parity survivor fec_decode's
// shuffle leaves in data[row].
__device__ __forceinline__ int ref_slot_lds(const uint8_t *sel, int k, int e, int row) {
    int x = row;
    while (x < k - e) x = sel[x];
    return sel[x];
}

// A group's slot map: i for a present data row, its reference slot for a
// rebuilt one (decoded groups: k <= 64 on these kernels), 0xFF for an erased
// row of a group that was not decoded (any k).
template <class Flag>
__device__ __forceinline__ void write_slot_map(const RefOut &ro, int64_t g, int k, int e, bool decoded,
                                               Flag flag, const WaveLds &L, int lane) {
    if (!ro.map) return;
    const int lim = k < ro.stride ? k : ro.stride;
    for (int b = 0; b < lim; b += 64) {
        const int i = b + lane;
        const bool p = flag(b, i);  // (wave-wide: flag reads lanes of the present words)
        if (i < lim)
            ro.map[g * ro.stride + i] =
                p ? (uint8_t)i : decoded ? (uint8_t)ref_slot_lds(L.sel, k, e, i) : (uint8_t)0xFF;
    }
}

// Move rows [0, nrows) of the group from their own (erased) slots to their
// reference slots: 16-byte pieces over the padded length, the stores ordered
// before the loads, which read past the CU cache (other lanes wrote them).
__device__ __forceinline__ void ref_move_rows(__amdgpu_buffer_rsrc_t rsrc, const WaveLds &L, int k, int e,
                                              int nrows, uint32_t ss, int lpad, int lane) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    for (int r = 0; r < nrows; ++r) {
        const int row = L.miss[r];
        const uint32_t src = (uint32_t)row * ss;
        const uint32_t dst = (uint32_t)__builtin_amdgcn_readfirstlane(ref_slot_lds(L.sel, k, e, row)) * ss;
        for (int p = 16 * lane; p < lpad; p += 1024) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (uint32_t)p, src, 1);
            __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, (uint32_t)p + dst, 0, DEC_RAG_ST_AUX);
        }
    }
}

// after_select() runs once, right after the survivor selection (the class
// kernels fetch the next group's present words there).
// Rows rb0 .. rb0 + NR - 1 of the group's missing data rows (the slice holds
// split tables for NR rows; Lagrange coefficients need no elimination, so a
// group with e > NR is never deferred: the caller runs it again with rb0 + NR
// while this returns true, and the status is written by the last call).
template <int WC, int NR, class Flag, class Hook = NoHook>
__device__ __forceinline__ bool ragged_group_run(const GroupDesc &D, Flag flag, uint8_t *base,
                                                 int32_t *status_out, const RagTables &T,
                                                 const WaveLds &L, int kmax, int lane,
                                                 DeferMark dm = DeferMark{nullptr, 0},
                                                 Hook after_select = Hook{}, int rb0 = 0,
                                                 RefOut ro = RefOut{nullptr, 0, 0}) {
    const int64_t g = D.g;
    const int k = D.k, n = D.n, len = D.len;
    const uint32_t ss = D.ss;
    const uint64_t off = D.off;
    const uint8_t *rows = D.rows;
    if (k < 1 || n < k || n > 256 || (n > k && !rows)) {
        after_select();
        if (lane == 0) status_out[g] = RSMI_DEC_UNSUPPORTED;
        return false;
    }
#if DEC_TRACE
    const uint64_t tr0 = trace_now();
#endif
    int e;
    const int cnt = select_survivors(k, n, flag, L, lane, e);
    wave_sync();
    after_select();
#if DEC_TRACE
    const uint64_t tr1 = trace_now();
#endif
    if (cnt < k || e == 0) {
        if (lane == 0) status_out[g] = cnt < k ? RSMI_DEC_TOO_FEW : RSMI_DEC_OK;
        if (ro.on) write_slot_map(ro, g, k, e, false, flag, L, lane);
        return false;
    }
    if (k > kmax || (uint64_t)n * ss >= 0x80000000ull) {
        if (lane == 0) {
            status_out[g] = kDefer;
            if (dm.word) atomicMax(dm.word, dm.epoch);
        }
        return false;
    }
    const int lpad = rag_lpad((uint32_t)len, ss);
    const uint32_t sel_lane = lane < k ? (uint32_t)L.sel[lane] : 0u;
    auto rebuild = [&](auto wc) {
        constexpr int W = decltype(wc)::value;
        Rebuild<W> B;
        B.rsrc = group_rsrc(base + off, (uint32_t)(n * ss));
        B.rnull = group_rsrc(base + off, 0u);
        B.k = k;
        B.e = e;
        B.len = len;
        B.lpad = lpad;
        // rows rb0 .. rb0 + nb0 - 1 of the e missing ones (lane d: row rb0 + d)
        const uint32_t miss_lane = lane + rb0 < e ? (uint32_t)L.miss[lane + rb0] : 0u;
        B.so_lane = sel_lane * ss;
        const int nb0 = e - rb0 < NR ? e - rb0 : NR;
        // the reference's placement: the group's last pass of kPass rows (the
        // last block's, B.run makes kPass-row passes per tile) writes over
        // the parity survivors -- every read of the tile is behind its stores
        // -- and the rows before it park in their own slots, moved after it
        const bool last = rb0 + NR >= e;
        const int lastpass = (nb0 - 1) / kPass * kPass;  // its first row, relative to rb0
        B.mo_lane = (ro.on && last && lane >= lastpass && lane + rb0 < e
                         ? (uint32_t)ref_slot_lds(L.sel, k, e, (int)miss_lane) : miss_lane) * ss;
        if (len > 0) B.start_tile(0, lane);  // the first survivors fly while the coefficients form
        lagrange_coefs<NR>(k, nb0, sel_lane, miss_lane, L, T, lane);  // distinct points: never singular
#if DEC_TRACE
        const uint64_t tr2 = trace_now();
#endif
        if (len > 0) B.run(L, lane, 0, nb0);
        if (ro.on && last && rb0 + lastpass > 0 && len > 0)
            ref_move_rows(B.rsrc, L, k, e, rb0 + lastpass, ss, lpad, lane);
        const int st = RSMI_DEC_OK;
#if DEC_TRACE
        const uint64_t tr3 = trace_now();
        if (lane == 0 && g_dec_trace) {
            uint64_t *t = g_dec_trace + g * 8;
            t[0] = tr0; t[1] = tr1; t[2] = tr2; t[3] = tr3;
            t[4] = (uint64_t)W | ((uint64_t)k << 8) | ((uint64_t)e << 16) | ((uint64_t)len << 32);
        }
#endif
        return st;
    };
    int st;
    if constexpr (WC != 0) {
        st = rebuild(std::integral_constant<int, WC>{});
    } else {
        const int w = DEC_RAG_W ? rag_width(lpad) : 5;
        if (w == 1) st = rebuild(std::integral_constant<int, 1>{});
        else if (w == 2) st = rebuild(std::integral_constant<int, 2>{});
        else if (w == 4) st = rebuild(std::integral_constant<int, 4>{});
        else st = rebuild(std::integral_constant<int, 5>{});
    }
    if (rb0 + NR < e) return true;  // more rows: the status waits for the last block
    if (lane == 0) status_out[g] = st;
    if (ro.on) write_slot_map(ro, g, k, e, true, flag, L, lane);
    return false;
}

// One group from its rsmi_group descriptor (scalar loads) and the code
// directory; w8 is present word (lane & 7) of the group.
template <int WC, int NR>
__device__ __forceinline__ void ragged_group(int64_t g, const rsmi_group &d, uint32_t w8,
                                             uint8_t *base, int32_t *status_out,
                                             const uint64_t *code_dir, const RagTables &T,
                                             const WaveLds &L, int kmax, int lane, RefOut ro) {
    GroupDesc D;
    D.g = g;
    D.k = __builtin_amdgcn_readfirstlane(d.k);
    D.n = __builtin_amdgcn_readfirstlane(d.n);
    D.len = __builtin_amdgcn_readfirstlane(d.len);
    D.ss = __builtin_amdgcn_readfirstlane(d.shard_stride);
    D.off = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(d.offset >> 32)) << 32) |
            (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)d.offset);
    D.rows = (D.k >= 1 && D.n > D.k && D.n <= 256)
                 ? reinterpret_cast<const uint8_t *>(code_dir[D.k * 257 + D.n])
                 : nullptr;
    for (int rb0 = 0;; rb0 += NR) {
        const bool more = ragged_group_run<WC, NR>(
            D,
            [&](int b, int idx) {
                // words b/32 and b/32 + 1 cover shards b..b+63 (readlane ignores exec)
                const uint32_t lo = __builtin_amdgcn_readlane(w8, (b >> 5) & 7);
                const uint32_t hi = __builtin_amdgcn_readlane(w8, ((b >> 5) + 1) & 7);
                return ((((idx & 32) ? hi : lo) >> (idx & 31)) & 1u) != 0;
            },
            base, status_out, T, L, kmax, lane, DeferMark{nullptr, 0}, NoHook{}, rb0, ro);
        wave_sync();  // the LDS slice is rewritten by the next block or group
        if (!more) break;
    }
}

// Every group of the batch, tile width chosen per group (rsmi_decode_ragged_dev:
// descriptors on the device, no plan).
__global__ __launch_bounds__(256, DEC_RAG_OCC) void k_decode_ragged(
    const rsmi_group *__restrict__ groups, int64_t ngroups, uint8_t *base,
    const uint32_t *__restrict__ present, int32_t *status_out, const uint64_t *__restrict__ code_dir,
    const uint32_t *ptab, const uint8_t *gftab, int kmax, RefOut ro) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const RagTables T = load_rag_tables(smem, ptab, gftab);
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane0 = threadIdx.x & 63;
    const WaveLds L = rag_slice(smem + kRagTabBytes + wid * rag_lds_bytes(kmax, kRows), kmax, kRows);
    __syncthreads();
    const int64_t nwaves = (int64_t)gridDim.x * kWaves;
    for (int64_t g = (int64_t)blockIdx.x * kWaves + wid; g < ngroups; g += nwaves) {
        // lane-derived values are recomputed per group: hoisted out of the
        // loop they stay live across the four tile-width bodies and spill
        int lane = lane0;
        asm volatile("" : "+v"(lane));
        const rsmi_group d = groups[g];
        ragged_group<0, kRows>(g, d, present[g * 8 + (lane & 7)], base, status_out, code_dir, T, L,
                               kmax, lane, ro);
        wave_sync();  // the LDS slice is rewritten by the next group
    }
}

// Plans: the groups of one tile-width class, registers cut for that width so
// short groups run at up to 8 waves per SIMD: C3's groups are latency-bound
// (a chain of dependent round trips per group).  Workgroup b takes the groups
// the plan dealt it (ragged.cpp: longest first onto the least-loaded
// workgroup) as 8-dword records {offset lo, hi, stride, len, k | n << 16,
// status index, parity-rows pointer lo, hi} at rec[wst[b] .. wst[b+1]): the
// records and their 8 present words come into LDS with two block-wide loads,
// and the block's waves take groups from an LDS counter, so a wave whose
// groups lost many data shards (long eliminations and multiplies: costs the
// plan cannot see) does not hold the round up while its neighbours idle.
// One class workgroup: its cnt records at rec[i0 ..) (and their present
// words) staged in LDS, its waves taking groups from an LDS counter.
template <int W>
__device__ __forceinline__ void cls_block(const uint32_t *__restrict__ rec, uint32_t i0, uint32_t cnt,
                                          int maxb, uint8_t *base, const uint32_t *__restrict__ present,
                                          int32_t *status_out, const uint32_t *ptab, const uint8_t *gftab,
                                          int kmax, DeferMark dm, int b, RefOut ro) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
#if DEC_TRACE
    const uint64_t tk0 = trace_now();
#endif
    uint32_t *srec = reinterpret_cast<uint32_t *>(smem + kRagTabBytes + kClsWaves * rag_lds_bytes(kmax, kClsRows));
    uint32_t *spw = srec + (size_t)maxb * 8;
    uint32_t *next = spw + (size_t)maxb * 8;
    for (uint32_t t = threadIdx.x; t < cnt * 8; t += blockDim.x) srec[t] = rec[(size_t)i0 * 8 + t];
    if (threadIdx.x == 0) *next = 0;
    const RagTables T = load_rag_tables(smem, ptab, gftab);
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const WaveLds L = rag_slice(smem + kRagTabBytes + wid * rag_lds_bytes(kmax, kClsRows), kmax, kClsRows);
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < cnt * 8; t += blockDim.x)
        spw[t] = present[(size_t)srec[(t & ~7u) + 5] * 8 + (t & 7u)];
    __syncthreads();
#if DEC_TRACE
    const uint64_t tk1 = trace_now();
    const int w = b * kClsWaves + wid;
#else
    (void)b;
#endif
    for (;;) {
        uint32_t i = 0;
        if (lane == 0) i = __hip_atomic_fetch_add(next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        i = (uint32_t)__builtin_amdgcn_readfirstlane(i);
        if (i >= cnt) break;
        const uint32_t r = srec[i * 8 + (lane & 7)];
        const uint32_t pw = spw[i * 8 + (lane & 7)];
        GroupDesc D;
        // (readlane returns int: every dword goes through uint32_t before it
        // is widened, or a low half with bit 31 set sign-extends into the
        // high half of a 64-bit offset or pointer)
        auto dw = [&](int f) { return (uint32_t)__builtin_amdgcn_readlane(r, f); };
        const uint32_t kn = dw(4);
        D.g = (int64_t)dw(5);
        D.k = (int)(kn & 0xFFFFu);
        D.n = (int)(kn >> 16);
        D.len = (int)dw(3);
        D.ss = dw(2);
        D.off = ((uint64_t)dw(1) << 32) | (uint64_t)dw(0);
        D.rows = reinterpret_cast<const uint8_t *>((uintptr_t)(((uint64_t)dw(7) << 32) | (uint64_t)dw(6)));
#if DEC_TRACE
        if (lane == 0 && g_dec_trace) {
            uint64_t *tt = g_dec_trace + D.g * 8;
            tt[5] = (uint64_t)w; tt[6] = tk0; tt[7] = tk1;
        }
#endif
        // lane-derived values (LDS row addresses) are recomputed per group:
        // hoisted out of the loop they stay live across it and spill
        for (int rb0 = 0;; rb0 += kClsRows) {  // blocks of kClsRows missing rows
            int lane_g = lane;
            asm volatile("" : "+v"(lane_g));
            const bool more = ragged_group_run<W, kClsRows>(
                D,
                [&](int bb, int idx) {
                    const uint32_t lo = __builtin_amdgcn_readlane(pw, (bb >> 5) & 7);
                    const uint32_t hi = __builtin_amdgcn_readlane(pw, ((bb >> 5) + 1) & 7);
                    return ((((idx & 32) ? hi : lo) >> (idx & 31)) & 1u) != 0;
                },
                base, status_out, T, L, kmax, lane_g, dm, NoHook{}, rb0, ro);
            wave_sync();  // the LDS slice is rewritten by the next block or group
            if (!more) break;
        }
    }
}

template <int W, int OCC>
__global__ __launch_bounds__(64 * kClsWaves, OCC) void k_decode_ragged_cls(
    const uint32_t *__restrict__ rec, const uint32_t *__restrict__ wst, int nb, int maxb, uint8_t *base,
    const uint32_t *__restrict__ present, int32_t *status_out, const uint32_t *ptab,
    const uint8_t *gftab, int kmax, DeferMark dm, RefOut ro) {
    const int b = blockIdx.x;
    if (b >= nb) return;  // (whole block: before any barrier)
    cls_block<W>(rec, wst[b], wst[b + 1] - wst[b], maxb, base, present, status_out, ptab, gftab, kmax, dm, b,
                 ro);
}

// Several classes in one launch (DEC_MIX): the grid is the classes' workgroups
// back to back, widest class first, so the short narrow-tile groups fill the
// tail the long wide-tile groups leave instead of each class paying its own
// ramp and drain.  CMASK: bit c = class c included (0: W = 1 ... 3: W = 5).
struct MixGrid {
    const uint32_t *wst[4];
    int nb[4];
};
template <int OCC, int CMASK>
__global__ __launch_bounds__(64 * kClsWaves, OCC) void k_decode_ragged_mix(
    const uint32_t *__restrict__ rec, MixGrid M, int maxb, uint8_t *base,
    const uint32_t *__restrict__ present, int32_t *status_out, const uint32_t *ptab,
    const uint8_t *gftab, int kmax, DeferMark dm, RefOut ro) {
    int b = blockIdx.x;
#define RSMI_MIX_CLASS(c, W)                                                                        \
    if (CMASK & (1 << c)) {                                                                         \
        if (b < M.nb[c]) {                                                                          \
            cls_block<W>(rec, M.wst[c][b], M.wst[c][b + 1] - M.wst[c][b], maxb, base, present,      \
                         status_out, ptab, gftab, kmax, dm, b, ro);                                 \
            return;                                                                                 \
        }                                                                                           \
        b -= M.nb[c];                                                                               \
    }
    RSMI_MIX_CLASS(3, 5)
    RSMI_MIX_CLASS(2, 4)
    RSMI_MIX_CLASS(1, 2)
    RSMI_MIX_CLASS(0, 1)
#undef RSMI_MIX_CLASS
}

// The deferred groups: one 256-thread workgroup per group.  Gauss-Jordan on
// [A | M] in LDS (e x (e + k) <= 128 x 256 bytes for n <= 256), coefficients
// left in place, then each thread rebuilds dwords of up to 8 rows at a time
// with the v_perm split tables.  Not a hot path: big codes only.
constexpr int kBigAug = 128 * 256;
constexpr int kBigRows = 8;

__global__ __launch_bounds__(256) void k_decode_ragged_big(
    const rsmi_group *groups, int64_t ngroups, uint8_t *base, const uint32_t *present,
    int32_t *status_out, const uint64_t *code_dir, const uint32_t *ptab, const uint8_t *gftab,
    const uint32_t *defer_word, uint32_t epoch, RefOut ro) {
    // plans: nothing to do unless a class kernel marked a deferral this call
    if (defer_word && (uint32_t)__builtin_amdgcn_readfirstlane(*defer_word) < epoch) return;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const Tables T = load_tables(smem, ptab, gftab);
    uint8_t *sel = smem + kTabBytes, *miss = sel + 256, *aug = miss + 256;
    __shared__ int s_e, s_n;
    __shared__ int64_t s_list[256];
    const int tid = threadIdx.x, lane = tid & 63;
    // Each block takes 256 consecutive statuses at a time (one coalesced load)
    // and works through the deferred ones among them: usually none, and a
    // group-at-a-time scan cost a dependent load per group.
    for (int64_t g0 = (int64_t)blockIdx.x * 256; g0 < ngroups; g0 += (int64_t)gridDim.x * 256) {
        if (tid == 0) s_n = 0;
        __syncthreads();
        if (g0 + tid < ngroups && status_out[g0 + tid] == kDefer)
            s_list[atomicAdd(&s_n, 1)] = g0 + tid;
        __syncthreads();
        const int nlist = s_n;
        for (int li = 0; li < nlist; ++li) {
            const int64_t g = s_list[li];
            const rsmi_group d = groups[g];
            const int k = d.k, n = d.n, len = (int)d.len;
            const uint64_t ss = d.shard_stride;
            uint8_t *gb = base + d.offset;
            const uint8_t *rows = reinterpret_cast<const uint8_t *>(code_dir[k * 257 + n]);
            const uint32_t *pw = present + g * 8;
            if (tid < 64) {  // wave 0 selects (the one-wave kernel found >= k present)
                const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
                int cnt = 0, e = 0;
                for (int b = 0; b < n && cnt < k; b += 64) {
                    const int idx = b + lane;
                    const bool f = idx < n && ((pw[idx >> 5] >> (idx & 31)) & 1u);
                    const uint64_t mk = __ballot(f);
                    const int rank = cnt + __popcll(mk & lt);
                    if (f && rank < k) sel[rank] = (uint8_t)idx;
                    cnt += __popcll(mk);
                }
                for (int b = 0; b < k; b += 64) {
                    const int idx = b + lane;
                    const bool ms = idx < k && !((pw[idx >> 5] >> (idx & 31)) & 1u);
                    const uint64_t mk = __ballot(ms);
                    if (ms) miss[e + __popcll(mk & lt)] = (uint8_t)idx;
                    e += __popcll(mk);
                }
                if (lane == 0) s_e = e;
            }
            __syncthreads();
            const int e = s_e, W = e + k;
            for (int t = tid; t < e * W; t += 256) {
                const int r = t / W, c = t - r * W;
                const int R = sel[k - e + r];
                const uint8_t *pr = rows + (R - k) * k;
                uint8_t v;
                if (c < e) {
                    v = pr[miss[c]];
                } else {
                    const int s = sel[c - e];
                    v = (s >= k) ? (uint8_t)(s == R) : pr[s];
                }
                aug[t] = v;
            }
            __syncthreads();
            int st = RSMI_DEC_OK;
            for (int p = 0; p < e; ++p) {
                const uint32_t piv = aug[p * W + p];
                if (piv == 0) {
                    st = RSMI_DEC_SINGULAR;
                    break;
                }
                const uint32_t ipiv = T.lexp[255 - T.llog[piv]];
                for (int c = p + 1 + tid; c < W; c += 256)
                    aug[p * W + c] = (uint8_t)gmul(T.lexp, T.llog, ipiv, aug[p * W + c]);
                __syncthreads();
                const int cols = W - p - 1;
                for (int t = tid; t < e * cols; t += 256) {
                    const int r = t / cols;
                    if (r == p) continue;
                    const int c = p + 1 + (t - r * cols);
                    const uint32_t f = aug[r * W + p];
                    if (f) aug[r * W + c] ^= (uint8_t)gmul(T.lexp, T.llog, f, aug[p * W + c]);
                }
                __syncthreads();
            }
            if (st == RSMI_DEC_OK) {
                // coef[r][j] = aug[r][e + j]; rows in blocks of kBigRows, dwords per thread
                const int words = (len + 3) >> 2;
                for (int rb = 0; rb < e; rb += kBigRows) {
                    for (int w = tid; w < words; w += 256) {
                        uint32_t acc[kBigRows];
    #pragma unroll
                        for (int r = 0; r < kBigRows; ++r) acc[r] = 0;
                        for (int j = 0; j < k; ++j) {
                            const uint32_t x =
                                *reinterpret_cast<const uint32_t *>(gb + sel[j] * ss + 4 * w);
                            const uint32_t a0 = x & 0x07070707u, a1 = (x >> 3) & 0x07070707u,
                                           a2 = (x >> 6) & 0x03030303u;
    #pragma unroll
                            for (int r = 0; r < kBigRows; ++r) {
                                if (rb + r < e) {
                                    const uint32_t c = aug[(rb + r) * W + e + j];
                                    const uint4 t = T.s01[c];
                                    const uint32_t t2 = T.s2[c];
                                    acc[r] ^= xor3(__builtin_amdgcn_perm(t.y, t.x, a0),
                                                   __builtin_amdgcn_perm(t.w, t.z, a1),
                                                   __builtin_amdgcn_perm(t2, t2, a2));
                                }
                            }
                        }
    #pragma unroll
                        for (int r = 0; r < kBigRows; ++r)
                            if (rb + r < e)
                                *reinterpret_cast<uint32_t *>(gb + miss[rb + r] * ss + 4 * w) = acc[r];
                    }
                }
                if (ro.on) {
                    // the reference's placement: every row from its own slot
                    // to the parity survivor fec_decode's shuffle picks (all
                    // reads of the survivors are behind the barrier)
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    __syncthreads();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    const int pieces = (len + 15) >> 4;
                    for (int t = tid; t < e * pieces; t += 256) {
                        const int r = t / pieces, p = t - r * pieces;
                        const int dst = ref_slot_lds(sel, k, e, miss[r]);
                        *reinterpret_cast<u32x4 *>(gb + dst * ss + 16 * p) =
                            __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(gb + miss[r] * ss + 16 * p));
                    }
                }
            }
            if (ro.on && ro.map) {
                const uint32_t *pw8 = present + g * 8;
                for (int i = tid; i < k && i < ro.stride; i += 256) {
                    const bool p = (pw8[i >> 5] >> (i & 31)) & 1u;
                    ro.map[g * ro.stride + i] = p ? (uint8_t)i
                                              : st == RSMI_DEC_OK ? (uint8_t)ref_slot_lds(sel, k, e, i)
                                                                  : (uint8_t)0xFF;
                }
            }
            if (tid == 0) status_out[g] = st;
            __syncthreads();  // sel / miss / aug are rewritten by the next group
        }
    }
}

}  // namespace

bool decode_fused_ok(int k, int n, int64_t group_stride, int64_t shard_stride, int len) {
    const int m = n - k;
    const int emax = k < m ? k : m;
    return emax <= kRows && k <= 64 && n * shard_stride < (int64_t(1) << 31) && len > 0 &&
           kLTabBytes + kWaves * wave_lds_bytes(k) <= 64 * 1024 && group_stride >= n * shard_stride;
}

hipError_t launch_decode_fused(const UniformArgs &a, const uint8_t *present,
                               const uint8_t *parity_rows, int32_t *status,
                               const uint32_t *ptab, const uint8_t *gftab, hipStream_t s,
                               bool host_shards, bool ref, uint8_t *slot_map) {
    const size_t lds = kLTabBytes + (size_t)kWaves * wave_lds_bytes(a.k);
    int64_t blocks = (a.ngroups + kWaves - 1) / kWaves;
    const int64_t cap = 256 * DEC_GRID_PER_CU;
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    if (host_shards)
        k_decode_fused<3, 3, 3, 0><<<(unsigned)blocks, 64 * kWaves, lds, s>>>(a, present, parity_rows,
                                                                         status, ptab, gftab, nullptr);
    else if (ref)
        k_decode_fused<DEC_LD_AUX, DEC_REF_ST_AUX, DEC_REF_ST_AUX_BIG, 1>
            <<<(unsigned)blocks, 64 * kWaves, lds, s>>>(a, present, parity_rows, status, ptab, gftab, slot_map);
    else
        k_decode_fused<DEC_LD_AUX, DEC_ST_AUX, DEC_ST_AUX_BIG, 0><<<(unsigned)blocks, 64 * kWaves, lds, s>>>(
            a, present, parity_rows, status, ptab, gftab, nullptr);
    return hipGetLastError();
}


hipError_t launch_decode_ragged(const rsmi_group *groups, int64_t ngroups, uint8_t *base,
                                const uint32_t *present_bits, int32_t *status, int kmax,
                                const uint64_t *code_dir, const uint32_t *ptab,
                                const uint8_t *gftab, hipStream_t s, RefOut ro) {
    if (ngroups <= 0) return hipSuccess;
    kmax = kmax < 1 ? 1 : (kmax > 32 ? 32 : kmax);  // larger k: the workgroup kernel
    const size_t lds = kRagTabBytes + (size_t)kWaves * rag_lds_bytes(kmax, kRows);
    int64_t blocks = (ngroups + kWaves - 1) / kWaves;
    if (blocks > 256 * 8) blocks = 256 * 8;
    k_decode_ragged<<<(unsigned)blocks, 64 * kWaves, lds, s>>>(groups, ngroups, base, present_bits,
                                                              status, code_dir, ptab, gftab, kmax, ro);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_decode_ragged_big(groups, ngroups, base, present_bits, status, code_dir, ptab,
                                    gftab, s, nullptr, 0, ro);
}

// tables | wave slices | records | present words | counter
size_t cls_lds_bytes(int kmax, int maxb) {
    kmax = kmax < 1 ? 1 : (kmax > 32 ? 32 : kmax);
    return kRagTabBytes + (size_t)kClsWaves * rag_lds_bytes(kmax, kClsRows) + (size_t)maxb * 64 + 16;
}

int decode_cls_occupancy(int c) {
    static const int occ[4] = {DEC_CLS_OCC1, DEC_CLS_OCC2, DEC_CLS_OCC4, DEC_CLS_OCC5};
    return occ[c & 3];
}

hipError_t launch_decode_ragged_cls(const rsmi_group *groups, const ClsLaunch &C, uint8_t *base,
                                    const uint32_t *present_bits, int32_t *status, int kmax,
                                    const uint64_t *code_dir, const uint32_t *ptab,
                                    const uint8_t *gftab, hipStream_t s, const hipStream_t cs[4]) {
    kmax = kmax < 1 ? 1 : (kmax > 32 ? 32 : kmax);  // larger k: the workgroup kernel
    auto launch = [&](auto kern, int c) {
        const int nb = C.nw[c];
        if (nb <= 0) return hipSuccess;
        // tables | wave slices | records | present words | counter
        const size_t lds = cls_lds_bytes(kmax, C.maxb[c]);
        kern<<<(unsigned)nb, 64 * kClsWaves, lds, cs[c]>>>(C.rec, C.wst[c], nb, C.maxb[c], base,
                                                        present_bits, status, ptab, gftab, kmax,
                                                        DeferMark{C.defer, C.epoch}, C.ref);
        return hipGetLastError();
    };
    // classes in one launch: CMASK's classes, OCC waves per SIMD
    auto mix = [&](auto kern, int cmask) {
        MixGrid M{};
        int nb = 0, maxb = 0;
        for (int c = 0; c < 4; ++c) {
            M.wst[c] = C.wst[c];
            M.nb[c] = (cmask >> c) & 1 ? C.nw[c] : 0;
            nb += M.nb[c];
            if (M.nb[c] > 0) maxb = maxb > C.maxb[c] ? maxb : C.maxb[c];
        }
        if (nb <= 0) return hipSuccess;
        kern<<<(unsigned)nb, 64 * kClsWaves, cls_lds_bytes(kmax, maxb), cs[3]>>>(
            C.rec, M, maxb, base, present_bits, status, ptab, gftab, kmax, DeferMark{C.defer, C.epoch}, C.ref);
        return hipGetLastError();
    };
    hipError_t e = hipSuccess;
    if (DEC_MIX == 2) return mix(k_decode_ragged_mix<DEC_CLS_OCC5, 15>, 15);
    e = launch(k_decode_ragged_cls<5, DEC_CLS_OCC5>, 3);
    if (DEC_MIX == 1) return e == hipSuccess ? mix(k_decode_ragged_mix<DEC_CLS_OCC4, 7>, 7) : e;
    if (e == hipSuccess) e = launch(k_decode_ragged_cls<4, DEC_CLS_OCC4>, 2);
    if (e == hipSuccess) e = launch(k_decode_ragged_cls<2, DEC_CLS_OCC2>, 1);
    if (e == hipSuccess) e = launch(k_decode_ragged_cls<1, DEC_CLS_OCC1>, 0);
    return e;
}

hipError_t launch_decode_ragged_big(const rsmi_group *groups, int64_t ngroups, uint8_t *base,
                                    const uint32_t *present_bits, int32_t *status,
                                    const uint64_t *code_dir, const uint32_t *ptab,
                                    const uint8_t *gftab, hipStream_t s, const uint32_t *defer_word,
                                    uint32_t epoch, RefOut ro) {
    // one block per CU at most: when nothing was deferred (the usual case
    // for plans) every block only reads the mark and leaves, and 1,024 of
    // them cost 5 us of launch and drain per decode call (C3, rocprofv3)
    int64_t bb = (ngroups + 255) / 256;
    if (bb > 256) bb = 256;
    k_decode_ragged_big<<<(unsigned)bb, 256, kTabBytes + 512 + kBigAug, s>>>(
        groups, ngroups, base, present_bits, status, code_dir, ptab, gftab, defer_word, epoch, ro);
    return hipGetLastError();
}

}  // namespace rsmi

#if DEC_TRACE
extern "C" int rsmi_debug_dec_trace(void *dev_ptr) {  // measurement builds only
    return hipMemcpyToSymbol(HIP_SYMBOL(rsmi::g_dec_trace), &dev_ptr, sizeof(dev_ptr)) == hipSuccess ? 0 : -1;
}
#endif
