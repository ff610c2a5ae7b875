// gf256.hpp -- host-side GF(2^8) arithmetic and code construction for rsmi.
//
// Field: polynomial 1+x^2+x^3+x^4+x^8 (0x11D), generator alpha = 2, exactly the
// field of lib/fec.cpp (allPp[8], fec.cpp:140; generate_gf fec.cpp:260-321).
// The systematic encoding matrix follows fec_new (fec.cpp:665-720): Vandermonde
// rows at the points {0, alpha^0, alpha^1, ...}, top k x k inverted, bottom
// rows multiplied by that inverse, top replaced by I.
//
// Everything here is tiny and runs once per (k,n) (the role of get_code,
// rs.cpp:42-55) or once per decode pattern; the byte streams go through the
// HIP kernels in kernels.hip.
#pragma once
#include <cstdint>
#include <vector>

namespace rsmi {

struct GF {
    uint8_t exp[512];   // alpha^i, doubled (fec.cpp:308-310)
    int log[256];       // log[0] = 255 sentinel (fec.cpp:307)
    uint8_t inv[256];   // inv[0] = 0 (fec.cpp:317)
    uint8_t mul[256][256];
    GF();
    uint8_t m(uint8_t a, uint8_t b) const { return mul[a][b]; }
};

const GF &gf();  // process-wide immutable tables, built once (thread-safe static init)

// n x k row-major systematic encoding matrix; false if (k,n) invalid
// (fec_new's k > 256 || n > 256 || k > n check, fec.cpp:676-680).
bool build_enc_matrix(int k, int n, std::vector<uint8_t> &out);

// In-place k x k inverse; false if singular.
bool invert(uint8_t *a, int k);

// Decode coefficients for one group, following the survivor-selection rule of
// rs_decode (rs.cpp:24-39: the first k present indices in ascending order).
//   present[n] (nonzero = present); enc = n x k matrix.
// On success returns e = number of missing data rows, fills
//   sel[k]      survivor slots used (ascending),
//   miss[e]     missing data rows (ascending),
//   coef[e*k]   row r: d[miss[r]] = sum_c coef[r*k+c] * shard[sel[c]].
// Returns -1 if fewer than k present (rs.cpp:31-32), -2 if singular.
int decode_coeffs(int k, int n, const uint8_t *enc, const uint8_t *present,
                  uint8_t *sel, uint8_t *miss, uint8_t *coef);

// 3-bit split tables used by the v_perm GF multiply (kernels.hip): for a
// constant c, T0[v] = c*v (v<8), T1[v] = c*(v<<3) (v<8), T2[v] = c*(v<<6) (v<4),
// packed little-endian as 5 dwords {T0[0..3], T0[4..7], T1[0..3], T1[4..7], T2}.
void perm_tables(uint8_t c, uint32_t out[5]);

}  // namespace rsmi
