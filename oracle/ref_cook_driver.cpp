// TEST INFRASTRUCTURE ONLY -- never shipped, never on the product path.
//
// Thin extern "C" driver around the REAL reference packet transforms
// (/root/reference/packet.cpp, compiled unmodified from where it lies by
// oracle/Makefile together with the reference sources it links against).
// Used to pin oracle/cook_oracle.c and to generate tests/golden/cook_*.npz.
//
//   do_cook   packet.cpp:303-308  (put_crc32 :327-336, do_obscure :77-91, encrypt_0 :32-39)
//   de_cook   packet.cpp:310-326  (decrypt_0 :41-48, de_obscure :93-106, rm_crc32 :337-346)
//   crc32h    packet.cpp:236-257
//
// The reference draws the obscure IV from its own mt19937 (common.cpp:147-186,
// seeded from std::random_device), so do_cook output is not reproducible run to
// run; callers recover (iv_len, iv) from the cooked bytes, which is exact.
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "common.h"
#include "misc.h"
#include "packet.h"

// Defined in packet.cpp with these signatures (packet.h declares older ones).
int do_obscure(char *data, int &len);
int de_obscure(char *data, int &len);
unsigned int crc32h(unsigned char *message, int len);

extern "C" {

void ref_cook_config(int no_checksum, int no_obscure, int no_xor, const char *key, int ivmin,
                     int ivmax) {
    disable_checksum = no_checksum;
    disable_obscure = no_obscure;
    disable_xor = no_xor;
    std::memset(key_string, 0, sizeof(key_string));
    if (key) std::strncpy(key_string, key, sizeof(key_string) - 1);
    iv_min = ivmin;
    iv_max = ivmax;
}

uint32_t ref_crc32h(const uint8_t *p, int len) { return crc32h((unsigned char *)p, len); }

// In place; returns the cooked length.
int ref_do_cook(uint8_t *buf, int len) {
    do_cook((char *)buf, len);
    return len;
}

// In place; returns de_cook's status and the resulting length via *len.
int ref_de_cook(uint8_t *buf, int *len) { return de_cook((char *)buf, *len); }

// Batch de_cook over a strided array of packets (CPU baseline).  de_cook is
// deterministic and touches no shared state, so it threads safely.
void ref_de_cook_batch(uint8_t *base, int64_t npk, int64_t stride, const int32_t *len,
                       int32_t *out_len, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
        th.emplace_back([=] {
            for (int64_t i = t; i < npk; i += nthreads) {
                int l = len[i];
                int rc = de_cook((char *)(base + i * stride), l);
                out_len[i] = rc == 0 ? l : -1;
            }
        });
    for (auto &x : th) x.join();
}

// Batch do_cook (single thread: the reference's PRNG is a shared global).
void ref_do_cook_batch(uint8_t *base, int64_t npk, int64_t stride, const int32_t *len,
                       int32_t *out_len) {
    for (int64_t i = 0; i < npk; ++i) {
        int l = len[i];
        do_cook((char *)(base + i * stride), l);
        out_len[i] = l;
    }
}

}  // extern "C"
