/*
 * rs_oracle.c -- TEST INFRASTRUCTURE ONLY (the CPU checker, never the product).
 *
 * A clean-room, plain-C restatement of the Reed-Solomon erasure code that
 * UDPspeeder vendors as lib/fec.cpp (Rizzo 1997) and wraps in lib/rs.cpp.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker.  The product path
 * (udpspeeder_amd/, librsmi.so) never links or calls it.
 *
 * Parity pinning: this restatement is checked byte-for-byte against golden
 * vectors produced by the reference itself (oracle/_ref, built from
 * /root/reference/lib/{fec,rs}.cpp by oracle/Makefile; fixtures written by
 * oracle/gen_golden.py into tests/golden/), including the reference's only
 * in-tree known-answer test (misc.cpp:335-361).
 *
 * Every function cites the reference lines whose behaviour it restates.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

typedef uint8_t gf;

/* ---- GF(2^8) with primitive polynomial 1+x^2+x^3+x^4+x^8 (0x11D) ------
 * lib/fec.cpp:131-149 (allPp[8] = "101110001"), generate_gf 260-321.
 * exp table is doubled so exp[a+b] needs no reduction (fec.cpp:308-310);
 * log[0] holds the sentinel 255 (fec.cpp:307); inverse[0] = 0 (fec.cpp:317). */
static gf g_exp[510];
static int g_log[256];
static gf g_inv[256];
static gf g_mul[256][256];
static int g_ready = 0;

static void orc_gf_init(void) {
    if (g_ready) return;
    unsigned v = 1;
    for (int i = 0; i < 255; i++) {          /* alpha^i, alpha = x = 2 */
        g_exp[i] = (gf)v;
        g_log[v] = i;
        v <<= 1;
        if (v & 0x100) v ^= 0x11D;
    }
    g_log[0] = 255;
    for (int i = 0; i < 255; i++) g_exp[i + 255] = g_exp[i];
    g_inv[0] = 0;
    g_inv[1] = 1;
    for (int i = 2; i < 256; i++) g_inv[i] = g_exp[255 - g_log[i]];
    /* fec.cpp:202-212: mul table from logs, row/column 0 forced to 0 */
    for (int a = 0; a < 256; a++)
        for (int b = 0; b < 256; b++)
            g_mul[a][b] = (a && b) ? g_exp[g_log[a] + g_log[b]] : 0;
    g_ready = 1;
}

/* Exported accessors so tests can pin the tables themselves. */
void orc_gf_tables(uint8_t *exp510, int32_t *log256, uint8_t *inv256) {
    orc_gf_init();
    memcpy(exp510, g_exp, 510);
    for (int i = 0; i < 256; i++) log256[i] = g_log[i];
    memcpy(inv256, g_inv, 256);
}
uint8_t orc_gf_mul(uint8_t a, uint8_t b) { orc_gf_init(); return g_mul[a][b]; }

/* ---- k x k Gauss-Jordan inverse over GF(2^8) --------------------------
 * Role of invert_mat (fec.cpp:425-549) / invert_vdm (fec.cpp:563-617).  The
 * inverse of a non-singular matrix is unique, so any exact elimination gives
 * the reference's bytes; this one uses partial pivoting on an augmented copy.
 * Returns 0 on success, 1 if singular (fec.cpp:469-497 error paths). */
static int gf_invert(gf *a, int k) {
    gf *aug = (gf *)malloc((size_t)k * 2 * k);
    if (!aug) return 1;
    for (int r = 0; r < k; r++) {
        memcpy(aug + (size_t)r * 2 * k, a + (size_t)r * k, k);
        memset(aug + (size_t)r * 2 * k + k, 0, k);
        aug[(size_t)r * 2 * k + k + r] = 1;
    }
    for (int c = 0; c < k; c++) {
        int p = -1;
        for (int r = c; r < k; r++)
            if (aug[(size_t)r * 2 * k + c]) { p = r; break; }
        if (p < 0) { free(aug); return 1; }
        if (p != c)
            for (int x = 0; x < 2 * k; x++) {
                gf t = aug[(size_t)p * 2 * k + x];
                aug[(size_t)p * 2 * k + x] = aug[(size_t)c * 2 * k + x];
                aug[(size_t)c * 2 * k + x] = t;
            }
        gf *pr = aug + (size_t)c * 2 * k;
        gf s = g_inv[pr[c]];
        for (int x = 0; x < 2 * k; x++) pr[x] = g_mul[s][pr[x]];
        for (int r = 0; r < k; r++) {
            if (r == c) continue;
            gf *rr = aug + (size_t)r * 2 * k;
            gf f = rr[c];
            if (!f) continue;
            for (int x = 0; x < 2 * k; x++) rr[x] ^= g_mul[f][pr[x]];
        }
    }
    for (int r = 0; r < k; r++)
        memcpy(a + (size_t)r * k, aug + (size_t)r * 2 * k + k, k);
    free(aug);
    return 0;
}

/* ---- systematic encoding matrix, n x k row-major ----------------------
 * fec_new (fec.cpp:665-720): Vandermonde rows at evaluation points
 * {0, alpha^0, alpha^1, ...}: row 0 = e0 (fec.cpp:691-693), row r >= 1 has
 * column c = alpha^((r-1)*c mod 255) (fec.cpp:694-697).  Invert the top k x k
 * (fec.cpp:705), bottom = V_bot * V_top^-1 (fec.cpp:706), top = I
 * (fec.cpp:710-712).  Invalid (k,n) -> -1 (fec.cpp:676-680). */
int orc_enc_matrix(int k, int n, uint8_t *out /* n*k */) {
    orc_gf_init();
    if (k < 1 || n < k || k > 256 || n > 256) return -1;
    gf *v = (gf *)calloc((size_t)n * k, 1);
    if (!v) return -1;
    v[0] = 1;
    for (int r = 1; r < n; r++)
        for (int c = 0; c < k; c++)
            v[(size_t)r * k + c] = g_exp[((r - 1) * c) % 255];
    if (gf_invert(v, k)) { free(v); return -1; }  /* never singular: distinct points */
    memset(out, 0, (size_t)n * k);
    for (int c = 0; c < k; c++) out[(size_t)c * k + c] = 1;
    for (int r = k; r < n; r++)
        for (int c = 0; c < k; c++) {
            gf acc = 0;
            for (int i = 0; i < k; i++)
                acc ^= g_mul[v[(size_t)r * k + i]][v[(size_t)i * k + c]];
            out[(size_t)r * k + c] = acc;
        }
    free(v);
    return 0;
}

/* Lazy (k,n) -> matrix cache: role of get_code (rs.cpp:42-55).  Single
 * threaded like the reference; tests use it from one thread. */
static uint8_t *g_codes[257][257];
static const uint8_t *code_for(int k, int n) {
    if (k < 1 || n < k || k > 256 || n > 256) return NULL;
    if (!g_codes[k][n]) {
        uint8_t *m = (uint8_t *)malloc((size_t)n * k);
        if (!m || orc_enc_matrix(k, n, m)) { free(m); return NULL; }
        g_codes[k][n] = m;
    }
    return g_codes[k][n];
}

/* dst ^= c * src over sz bytes: addmul1 (fec.cpp:336-376), skipped for c=0. */
static void addmul(gf *dst, const gf *src, gf c, int sz) {
    if (!c) return;
    const gf *row = g_mul[c];
    for (int i = 0; i < sz; i++) dst[i] ^= row[src[i]];
}

/* ---- rs_encode2 (rs.cpp:56-59 -> rs_encode rs.cpp:11-19 -> fec_encode
 * fec.cpp:727-750): for each parity index i in [k,n): zero data[i], then
 * accumulate enc[i][j] * data[j] for j < k.  Returns -1 for invalid (k,n)
 * where the reference would dereference a NULL code. */
int orc_encode(int k, int n, uint8_t **data, int size) {
    const uint8_t *m = code_for(k, n);
    if (!m) return -1;
    for (int i = k; i < n; i++) {
        memset(data[i], 0, size);
        for (int j = 0; j < k; j++) addmul(data[i], data[j], m[(size_t)i * k + j], size);
    }
    return 0;
}

/* ---- rs_decode2 (rs.cpp:61-64 -> rs_decode rs.cpp:21-40 -> fec_decode
 * fec.cpp:838-882), including the in-place pointer permutation:
 *  1. pack non-null pointers to the front, remember their indices, null the
 *     rest (rs.cpp:24-38); fewer than k -> -1 (rs.cpp:31-32);
 *  2. shuffle: move each received data shard (index < k) to its own slot
 *     (fec.cpp:755-788); a conflict -> 1;
 *  3. for every slot row < k still holding a parity shard, rebuild data row
 *     `row` = sum_col Dinv[row][col] * pkt[col] where D's row i is e_i for a
 *     data shard and enc[index[i]] for a parity shard (fec.cpp:795-825,
 *     861-868), then copy it over that parity buffer (fec.cpp:872-877). */
int orc_decode(int k, int n, uint8_t **data, int size) {
    const uint8_t *m = code_for(k, n);
    if (!m) return 1;
    int *index = (int *)malloc(sizeof(int) * (size_t)n);
    int count = 0;
    for (int i = 0; i < n; i++)
        if (data[i]) index[count++] = i;
    if (count < k) { free(index); return -1; }
    for (int i = 0; i < n; i++) data[i] = (i < count) ? data[index[i]] : NULL;

    /* shuffle (fec.cpp:755-788) */
    for (int i = 0; i < k;) {
        if (index[i] >= k || index[i] == i) { i++; continue; }
        int c = index[i];
        if (index[c] == c) { free(index); return 1; }
        int ti = index[i]; index[i] = index[c]; index[c] = ti;
        uint8_t *tp = data[i]; data[i] = data[c]; data[c] = tp;
    }
    gf *dm = (gf *)malloc((size_t)k * k);
    for (int i = 0; i < k; i++) {
        if (index[i] < k) {
            memset(dm + (size_t)i * k, 0, k);
            dm[(size_t)i * k + i] = 1;
        } else if (index[i] < n) {
            memcpy(dm + (size_t)i * k, m + (size_t)index[i] * k, k);
        } else { free(dm); free(index); return 1; }
    }
    if (gf_invert(dm, k)) { free(dm); free(index); return 1; }
    gf **fresh = (gf **)calloc((size_t)(unsigned)k, sizeof(gf *));
    for (int row = 0; row < k; row++) {
        if (index[row] < k) continue;
        fresh[row] = (gf *)calloc((size_t)(size > 0 ? size : 1), 1);
        for (int col = 0; col < k; col++)
            addmul(fresh[row], data[col], dm[(size_t)row * k + col], size);
    }
    for (int row = 0; row < k; row++)
        if (fresh[row]) { memcpy(data[row], fresh[row], size); free(fresh[row]); }
    free(fresh);
    free(dm);
    free(index);
    return 0;
}

/* ---- strided batch helpers (device-layout twins, used by tests/bench) --
 * Group g's shard j lives at buf + g*group_stride + j*shard_stride. */
int orc_encode_batch(int k, int n, uint8_t *buf, int64_t group_stride,
                     int64_t shard_stride, int len, int64_t ngroups) {
    uint8_t *ptrs[256];
    for (int64_t g = 0; g < ngroups; g++) {
        for (int j = 0; j < n; j++) ptrs[j] = buf + g * group_stride + j * shard_stride;
        if (orc_encode(k, n, ptrs, len)) return -1;
    }
    return 0;
}

/* Decode each group whose present flags are given as bytes [ngroups][n]
 * (nonzero = present).  Recovered data rows are written into their OWN
 * slot (j < k), the batched device contract; the pointer dance of
 * orc_decode happens on a private pointer array.  status[g] = 0/-1/1. */
int orc_decode_batch(int k, int n, uint8_t *buf, int64_t group_stride,
                     int64_t shard_stride, int len, int64_t ngroups,
                     const uint8_t *present, int32_t *status) {
    uint8_t *ptrs[256];
    uint8_t *tmp = (uint8_t *)malloc((size_t)k * (len > 0 ? len : 1));
    int bad = 0;
    for (int64_t g = 0; g < ngroups; g++) {
        uint8_t *base = buf + g * group_stride;
        for (int j = 0; j < n; j++)
            ptrs[j] = present[g * n + j] ? base + j * shard_stride : NULL;
        int rc = orc_decode(k, n, ptrs, len);
        status[g] = rc;
        if (rc) { bad++; continue; }
        /* ptrs[0..k-1] now point at recovered rows; stage then scatter so a
         * recovered row living in another missing row's slot is not clobbered */
        for (int j = 0; j < k; j++) memcpy(tmp + (size_t)j * len, ptrs[j], len);
        for (int j = 0; j < k; j++)
            if (!present[g * n + j]) memcpy(base + j * shard_stride, tmp + (size_t)j * len, len);
    }
    free(tmp);
    return bad;
}

/* ---- rs_from_str (fec_manager.h:40-136): "x1:y1,x2:y2,..." -> dense table
 * rs_par[x-1] = (x, y) for x = 1..x_last.  Returns x_last (rs_cnt) or -1.
 * Interpolation (fec_manager.h:122): y = pre_y + (now_y-pre_y)*(x-pre_x)/dist
 * + 0.9999 in double, truncated; clamp so x+y <= 255 (fec_manager.h:124-127). */
int orc_rs_from_str(const char *s, uint8_t *xs, uint8_t *ys /* >= 255 each */) {
    /* string_to_vec(s, ",") (common.cpp:919-934) is strtok: tokens between
     * commas, empty ones skipped; each is sscanf'd with "%d:%d" (trailing
     * characters ignored) */
    int px[256], py[256], cnt = 0;
    char tok[4096];
    const char *p = s;
    while (*p) {
        const char *c = strchr(p, ',');
        size_t n = c ? (size_t)(c - p) : strlen(p);
        if (n > 0) {
            int x, y;
            if (n >= sizeof(tok)) return -1;
            memcpy(tok, p, n);
            tok[n] = 0;
            if (sscanf(tok, "%d:%d", &x, &y) != 2) return -1;
            if (x < 1 || y < 0 || x + y > 255) return -1;
            if (cnt >= 256) return -1;
            px[cnt] = x; py[cnt] = y; cnt++;
        }
        p += n;
        if (*p == ',') p++;
    }
    if (cnt < 1) return -1;
    for (int i = 1; i < cnt; i++)
        if (px[i] <= px[i - 1]) return -1;
    for (int i = 1; i <= px[0]; i++) { xs[i - 1] = (uint8_t)i; ys[i - 1] = (uint8_t)py[0]; }
    for (int i = 1; i < cnt; i++) {
        int nx = px[i], ny = py[i], ox = px[i - 1], oy = py[i - 1];
        xs[nx - 1] = (uint8_t)nx; ys[nx - 1] = (uint8_t)ny;
        for (int j = ox + 1; j <= nx - 1; j++) {
            double dist = nx - ox;
            int y = (int)(oy + (ny - oy) * (j - ox) / dist + 0.9999);
            if (j + y > 255) y = 255 - j;
            xs[j - 1] = (uint8_t)j; ys[j - 1] = (uint8_t)y;
        }
    }
    return px[cnt - 1];
}
