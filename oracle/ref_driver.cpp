// ref_driver.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Our own thin batch driver around the UNMODIFIED reference codec
// (/root/reference/lib/fec.cpp + lib/rs.cpp, compiled from where they lie by
// oracle/Makefile into oracle/_ref/libref_rs.so, which is git-ignored).  It
// adds nothing to the reference's arithmetic: it only builds the char*
// pointer arrays that fec_manager.cpp builds (fec_manager.cpp:364, 632, 710)
// and loops over many groups, optionally on several threads, so that
// tests/golden generation and bench.py's cpu_baseline leg can drive the
// real rs_encode2 / rs_decode2 (lib/rs.h:41,43) over a batch.
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <thread>
#include <vector>
#include "rs.h"  // from /root/reference/lib (include path set by the Makefile)

void *get_code(int k, int n);  // lib/rs.cpp:43 (not declared in rs.h)

extern "C" {

// Warm the reference's lazy, unsynchronised (k,n) cache (rs.cpp:42-55) from a
// single thread before any multi-threaded use.
int ref_prewarm(int k, int n) { return get_code(k, n) != 0 ? 0 : -1; }

static void enc_range(int k, int n, uint8_t *buf, int64_t gs, int64_t ss, int len,
                      int64_t g0, int64_t g1) {
    char *ptrs[256];
    for (int64_t g = g0; g < g1; g++) {
        for (int j = 0; j < n; j++) ptrs[j] = (char *)(buf + g * gs + j * ss);
        rs_encode2(k, n, ptrs, len);
    }
}

int ref_encode_batch(int k, int n, uint8_t *buf, int64_t gs, int64_t ss, int len,
                     int64_t ngroups, int nthreads) {
    if (ref_prewarm(k, n)) return -1;
    if (nthreads <= 1) { enc_range(k, n, buf, gs, ss, len, 0, ngroups); return 0; }
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; t++) {
        int64_t g0 = ngroups * t / nthreads, g1 = ngroups * (t + 1) / nthreads;
        th.emplace_back(enc_range, k, n, buf, gs, ss, len, g0, g1);
    }
    for (auto &x : th) x.join();
    return 0;
}

// Decode groups in place the way fec_manager does: pointer array with nulls
// for erased shards, rs_decode2, then (if write_back) copy recovered rows
// data[0..k-1] into their own slots so callers can compare buffers.
static void dec_range(int k, int n, uint8_t *buf, int64_t gs, int64_t ss, int len,
                      const uint8_t *present, int32_t *status, int write_back,
                      int64_t g0, int64_t g1) {
    char *ptrs[256];
    for (int64_t g = g0; g < g1; g++) {
        uint8_t *base = buf + g * gs;
        for (int j = 0; j < n; j++)
            ptrs[j] = present[g * n + j] ? (char *)(base + j * ss) : 0;
        int rc = rs_decode2(k, n, ptrs, len);
        status[g] = rc;
        if (rc || !write_back) continue;
        for (int j = 0; j < k; j++)
            if (!present[g * n + j]) memmove(base + j * ss, ptrs[j], len);
    }
}

int ref_decode_batch(int k, int n, uint8_t *buf, int64_t gs, int64_t ss, int len,
                     int64_t ngroups, const uint8_t *present, int32_t *status,
                     int write_back, int nthreads) {
    if (ref_prewarm(k, n)) return -1;
    if (nthreads <= 1) {
        dec_range(k, n, buf, gs, ss, len, present, status, write_back, 0, ngroups);
        return 0;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; t++) {
        int64_t g0 = ngroups * t / nthreads, g1 = ngroups * (t + 1) / nthreads;
        th.emplace_back(dec_range, k, n, buf, gs, ss, len, present, status, write_back, g0, g1);
    }
    for (auto &x : th) x.join();
    return 0;
}

// One rs_decode2 call on n shards of one group, reporting the pointer
// permutation it leaves behind as slot indices (-1 = null) so the drop-in
// shim's in-place semantics (lib/rs.h:25-38) can be pinned.
int ref_decode_ptrs(int k, int n, uint8_t *buf, int64_t ss, int len,
                    const int32_t *in_slot, int32_t *out_slot) {
    char *ptrs[256];
    for (int j = 0; j < n; j++) ptrs[j] = in_slot[j] >= 0 ? (char *)(buf + in_slot[j] * ss) : 0;
    int rc = rs_decode2(k, n, ptrs, len);
    for (int j = 0; j < n; j++)
        out_slot[j] = ptrs[j] ? (int32_t)(((uint8_t *)ptrs[j] - buf) / ss) : -1;
    return rc;
}

}  // extern "C"
