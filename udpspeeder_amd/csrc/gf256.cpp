// gf256.cpp -- see gf256.hpp.
#include "gf256.hpp"

#include <cstring>

namespace rsmi {

GF::GF() {
    unsigned v = 1;
    for (int i = 0; i < 255; ++i) {
        exp[i] = (uint8_t)v;
        log[v] = i;
        v <<= 1;
        if (v & 0x100) v ^= 0x11D;
    }
    for (int i = 255; i < 512; ++i) exp[i] = exp[i - 255];
    log[0] = 255;
    inv[0] = 0;
    for (int i = 1; i < 256; ++i) inv[i] = exp[(255 - log[i]) % 255];
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b)
            mul[a][b] = (a && b) ? exp[log[a] + log[b]] : 0;
}

const GF &gf() {
    static const GF tables;  // C++11 magic static: built once, thread-safe
    return tables;
}

bool invert(uint8_t *a, int k) {
    const GF &F = gf();
    std::vector<uint8_t> aug((size_t)k * 2 * k, 0);
    for (int r = 0; r < k; ++r) {
        std::memcpy(&aug[(size_t)r * 2 * k], a + (size_t)r * k, k);
        aug[(size_t)r * 2 * k + k + r] = 1;
    }
    const int w = 2 * k;
    for (int c = 0; c < k; ++c) {
        int p = -1;
        for (int r = c; r < k; ++r)
            if (aug[(size_t)r * w + c]) { p = r; break; }
        if (p < 0) return false;
        if (p != c)
            for (int x = 0; x < w; ++x) std::swap(aug[(size_t)p * w + x], aug[(size_t)c * w + x]);
        uint8_t *pr = &aug[(size_t)c * w];
        const uint8_t *s = F.mul[F.inv[pr[c]]];
        for (int x = 0; x < w; ++x) pr[x] = s[pr[x]];
        for (int r = 0; r < k; ++r) {
            if (r == c) continue;
            uint8_t *rr = &aug[(size_t)r * w];
            const uint8_t f = rr[c];
            if (!f) continue;
            const uint8_t *fm = F.mul[f];
            for (int x = 0; x < w; ++x) rr[x] ^= fm[pr[x]];
        }
    }
    for (int r = 0; r < k; ++r) std::memcpy(a + (size_t)r * k, &aug[(size_t)r * w + k], k);
    return true;
}

bool build_enc_matrix(int k, int n, std::vector<uint8_t> &out) {
    if (k < 1 || n < k || k > 256 || n > 256) return false;
    const GF &F = gf();
    std::vector<uint8_t> v((size_t)n * k, 0);
    v[0] = 1;  // evaluation point 0: row e0
    for (int r = 1; r < n; ++r)
        for (int c = 0; c < k; ++c) v[(size_t)r * k + c] = F.exp[((r - 1) * c) % 255];
    if (!invert(v.data(), k)) return false;  // top is V(0, a^0..a^(k-2)): never singular
    out.assign((size_t)n * k, 0);
    for (int c = 0; c < k; ++c) out[(size_t)c * k + c] = 1;
    for (int r = k; r < n; ++r)
        for (int c = 0; c < k; ++c) {
            uint8_t acc = 0;
            for (int i = 0; i < k; ++i) acc ^= F.mul[v[(size_t)r * k + i]][v[(size_t)i * k + c]];
            out[(size_t)r * k + c] = acc;
        }
    return true;
}

int decode_coeffs(int k, int n, const uint8_t *enc, const uint8_t *present, uint8_t *sel,
                  uint8_t *miss, uint8_t *coef) {
    const GF &F = gf();
    int cnt = 0;
    for (int i = 0; i < n && cnt < k; ++i)
        if (present[i]) sel[cnt++] = (uint8_t)i;
    if (cnt < k) return -1;
    // Data rows present in the selection are exactly the present data rows
    // (they have the smallest indices); the parity rows used are sel[k-e..k-1].
    int e = 0;
    for (int j = 0; j < k; ++j)
        if (!present[j]) miss[e++] = (uint8_t)j;
    if (e == 0) return 0;
    // A = enc[R][E] (e x e), B = enc[R][P]; d_E = A^-1 p_R + A^-1 B d_P.
    std::vector<uint8_t> A((size_t)e * e);
    const uint8_t *R = sel + (k - e);
    for (int r = 0; r < e; ++r)
        for (int c = 0; c < e; ++c) A[(size_t)r * e + c] = enc[(size_t)R[r] * k + miss[c]];
    if (!invert(A.data(), e)) return -2;
    // Column c of coef corresponds to survivor sel[c].
    for (int r = 0; r < e; ++r) {
        for (int c = 0; c < k; ++c) {
            const int s = sel[c];
            uint8_t acc = 0;
            if (s >= k) {  // parity survivor: A^-1[r][position in R]
                acc = A[(size_t)r * e + (c - (k - e))];
            } else {       // data survivor: (A^-1 B)[r][s]
                for (int t = 0; t < e; ++t)
                    acc ^= F.mul[A[(size_t)r * e + t]][enc[(size_t)R[t] * k + s]];
            }
            coef[(size_t)r * k + c] = acc;
        }
    }
    return e;
}

void perm_tables(uint8_t c, uint32_t out[5]) {
    const GF &F = gf();
    uint8_t t0[8], t1[8], t2[4];
    for (int v = 0; v < 8; ++v) { t0[v] = F.mul[c][v]; t1[v] = F.mul[c][v << 3]; }
    for (int v = 0; v < 4; ++v) t2[v] = F.mul[c][v << 6];
    std::memcpy(&out[0], t0, 4);
    std::memcpy(&out[1], t0 + 4, 4);
    std::memcpy(&out[2], t1, 4);
    std::memcpy(&out[3], t1 + 4, 4);
    std::memcpy(&out[4], t2, 4);
}

}  // namespace rsmi
