// cook_host.cpp -- host side of the batched packet cook / de_cook (include/rsmi_cook.h).
//
// Builds the CRC-32 table blob the kernels keep in LDS (slicing-by-8 tables and
// the nibble-table forms of the zero-feed maps Z_d, see cook.hip) and the
// per-context key stream KS[p] = key[p % strlen(key)] (encrypt_0,
// packet.cpp:32-39), then validates and launches.
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "rsmi_internal.hpp"
#include "../../include/rsmi_cook.h"

namespace rsmi {
void set_error(const std::string &m);
}

struct rsmi_cook_ctx {
    int device = -1;
    int flags = 0;
    int max_blocks = 0;
    uint32_t *tabs = nullptr;
    uint8_t *ks = nullptr;  // NULL when there is no XOR stage; position p at ks[p], p >= -kCookKsLead
    uint8_t *ks_mem = nullptr;  // the allocation (ks - kCookKsLead)
    uint8_t *zks = nullptr;     // no XOR stage: a zero stream of the same extent (the encoder epilogue's)
    // synchronous host path
    std::mutex mu;
    uint8_t *hbuf = nullptr;
    size_t hcap = 0;
};

namespace {

int fail(int code, const std::string &m) {
    rsmi::set_error(m);
    return code;
}

// Reflected CRC-32, poly 0xEDB88320 (crc32h, packet.cpp:236-257).
struct CrcTables {
    uint32_t t0[256];
    uint8_t inv_top[256];  // T0[v] >> 24 is a permutation of v: inverts one zero-byte feed
    std::vector<uint32_t> blob;

    uint32_t feed0(uint32_t c) const { return (c >> 8) ^ t0[c & 0xff]; }
    uint32_t unfeed0(uint32_t c) const {
        const uint32_t v = inv_top[c >> 24];
        return ((c ^ t0[v]) << 8) | v;
    }
    // Nibble tables of the map c -> Z_d(c) (d < 0: the inverse map).
    void put_map(uint32_t *dst, int d) const {
        uint32_t basis[32];
        for (int b = 0; b < 32; ++b) {
            uint32_t c = 1u << b;
            for (int i = 0; i < (d < 0 ? -d : d); ++i) c = d < 0 ? unfeed0(c) : feed0(c);
            basis[b] = c;
        }
        for (int i = 0; i < 8; ++i)
            for (int v = 0; v < 16; ++v) {
                uint32_t r = 0;
                for (int b = 0; b < 4; ++b)
                    if (v >> b & 1) r ^= basis[4 * i + b];
                dst[16 * i + v] = r;
            }
    }

    // Z_d (d > 0) as four byte tables: Z(c) = B0[c & 255] ^ B1[c >> 8 & 255] ^ ...
    void put_bytemap(uint32_t *dst, int d) const {
        uint32_t basis[32];
        for (int b = 0; b < 32; ++b) {
            uint32_t c = 1u << b;
            for (int i = 0; i < d; ++i) c = feed0(c);
            basis[b] = c;
        }
        for (int t = 0; t < 4; ++t)
            for (int v = 0; v < 256; ++v) {
                uint32_t r = 0;
                for (int b = 0; b < 8; ++b)
                    if (v >> b & 1) r ^= basis[8 * t + b];
                dst[256 * t + v] = r;
            }
    }

    CrcTables() {
        for (uint32_t v = 0; v < 256; ++v) {
            uint32_t c = v;
            for (int b = 0; b < 8; ++b) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
            t0[v] = c;
            inv_top[c >> 24] = (uint8_t)v;
        }
        blob.assign(rsmi::kCookTabWords, 0);
        for (int v = 0; v < 256; ++v) blob[v] = t0[v];
        for (int k = 1; k < 8; ++k)
            for (int v = 0; v < 256; ++v) blob[256 * k + v] = feed0(blob[256 * (k - 1) + v]);
        for (int k = 0; k < rsmi::kCookLpp; ++k) put_map(&blob[rsmi::kCookLane + 128 * k], 16 * k);
        // Z_{16 kCookLpp} (a lane's step to its next piece) as four byte tables:
        // Z(c) = B0[c & 255] ^ B1[c >> 8 & 255] ^ ...
        put_bytemap(&blob[rsmi::kCookZH], 16 * rsmi::kCookLpp);
        if (COOK_2CH) put_bytemap(&blob[rsmi::kCookZH2], 32 * rsmi::kCookLpp);
        for (int c = 1; c < 4; ++c) put_map(&blob[rsmi::kCookUns + 128 * (c - 1)], -c);
        for (int c = 1; c < 4; ++c) put_map(&blob[rsmi::kCookUns + 128 * (2 + c)], -4 * c);
        if (COOK_S16)  // T_8..T_15, each one zero byte past the one before (T_7 first)
            for (int k = 8; k < 16; ++k) {
                const uint32_t *src = k == 8 ? &blob[256 * 7] : &blob[rsmi::kCookS16 + 256 * (k - 9)];
                for (int v = 0; v < 256; ++v) blob[rsmi::kCookS16 + 256 * (k - 8) + v] = feed0(src[v]);
            }
        if (!COOK_NIB) return;
        // nibble i of a piece is the low (i even) or high nibble of byte i / 2
        for (int i = 0; i < 32; ++i)
            for (uint32_t v = 0; v < 16; ++v) {
                uint32_t c = 0;
                for (int j = 0; j < 16; ++j)
                    c = feed0(c ^ (j == i / 2 ? (i & 1 ? v << 4 : v) : 0u));
                blob[rsmi::kCookNib + 16 * i + v] = c;
            }
        put_map(&blob[rsmi::kCookZN], 16 * rsmi::kCookLpp);
    }
};

const CrcTables &crc_tables() {
    static const CrcTables t;
    return t;
}

int check_batch(const rsmi_packet_batch *b) {
    if (!b || b->count < 0 || b->cap < 0 || b->reserved != 0 || b->stride < 0)
        return fail(RSMI_ERR_INVALID, "invalid packet batch");
    if (b->count > 0 && (!b->base || !b->len || !b->out_len))
        return fail(RSMI_ERR_INVALID, "packet batch needs base, len and out_len");
    return RSMI_OK;
}

rsmi::CookArgs make_args(const rsmi_cook_ctx *c, const rsmi_packet_batch *b) {
    rsmi::CookArgs a{};
    a.base = b->base;
    a.offset = b->offset;
    a.stride = b->stride;
    a.count = b->count;
    a.cap = b->cap;
    a.flags = c->flags;
    a.len = b->len;
    a.out_len = b->out_len;
    a.tabs = c->tabs;
    a.ks = c->ks;
    return a;
}

int launch(const rsmi::CookArgs &a, const rsmi_cook_ctx *c, bool decook, hipStream_t s) {
    const hipError_t e = rsmi::launch_cook(a, decook, c->max_blocks, s);
    if (e != hipSuccess)
        return fail(RSMI_ERR_HIP, std::string(decook ? "decook" : "cook") + " launch: " +
                                      hipGetErrorString(e));
    return RSMI_OK;
}

}  // namespace

extern "C" int rsmi_cook_ctx_create(const char *key, int flags, rsmi_cook_ctx **out) {
    if (!out || (flags & ~7)) return fail(RSMI_ERR_INVALID, "invalid cook context arguments");
    *out = nullptr;
    const size_t klen = key ? std::strlen(key) : 0;
    rsmi_cook_ctx *c = new rsmi_cook_ctx();
    c->flags = flags;
    int cus = 0;
    if (hipGetDevice(&c->device) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess) {
        delete c;
        return fail(RSMI_ERR_HIP, "hipGetDevice (no usable GPU?)");
    }
    // LDS per block bounds residency: as many blocks per CU as 160 KiB holds
    const int per_cu = (int)((160 * 1024) / rsmi::cook_lds_bytes(true));
    c->max_blocks = cus * (per_cu > 0 ? per_cu : 1) * 2;
    const CrcTables &t = crc_tables();
    hipError_t e = hipMalloc(&c->tabs, sizeof(uint32_t) * t.blob.size());
    if (e == hipSuccess)
        e = hipMemcpy(c->tabs, t.blob.data(), sizeof(uint32_t) * t.blob.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess && klen && !(flags & RSMI_COOK_NO_XOR)) {
        // key[p % klen] for p in [-kCookKsLead, kCookKsBytes): the lead serves the
        // phase pieces' bytes before a packet (never used, kept periodic)
        const int lead = rsmi::kCookKsLead;
        std::vector<uint8_t> ks(rsmi::kCookKsBytes + lead);
        for (size_t i = 0; i < ks.size(); ++i)
            ks[i] = (uint8_t)key[(size_t)(((int64_t)i - lead) % (int64_t)klen + klen) % klen];
        e = hipMalloc(&c->ks_mem, ks.size());
        if (e == hipSuccess) e = hipMemcpy(c->ks_mem, ks.data(), ks.size(), hipMemcpyHostToDevice);
        if (e == hipSuccess) c->ks = c->ks_mem + lead;
    } else if (e == hipSuccess) {
        // the cooking encoder XORs a key stream unconditionally (a branch there
        // costs it its registers): zeros
        const size_t bytes = rsmi::kCookKsBytes + rsmi::kCookKsLead;
        e = hipMalloc(&c->ks_mem, bytes);
        if (e == hipSuccess) e = hipMemset(c->ks_mem, 0, bytes);
        if (e == hipSuccess) c->zks = c->ks_mem + rsmi::kCookKsLead;
    }
    if (e != hipSuccess) {
        rsmi_cook_ctx_destroy(c);
        return fail(RSMI_ERR_NOMEM, std::string("cook context: ") + hipGetErrorString(e));
    }
    *out = c;
    return RSMI_OK;
}

extern "C" void rsmi_cook_ctx_destroy(rsmi_cook_ctx *c) {
    if (!c) return;
    if (c->tabs) (void)hipFree(c->tabs);
    if (c->ks_mem) (void)hipFree(c->ks_mem);
    if (c->hbuf) (void)hipFree(c->hbuf);
    delete c;
}

extern "C" int rsmi_cook_dev(const rsmi_cook_ctx *c, const rsmi_packet_batch *b,
                             const uint8_t *iv, const uint8_t *iv_len, uint64_t seed,
                             void *stream) {
    if (!c) return fail(RSMI_ERR_INVALID, "null cook context");
    if (int rc = check_batch(b)) return rc;
    if ((iv == nullptr) != (iv_len == nullptr))
        return fail(RSMI_ERR_INVALID, "iv and iv_len must both be given or both be NULL");
    rsmi::CookArgs a = make_args(c, b);
    a.iv = iv;
    a.iv_len = iv_len;
    a.seed = seed;
    return launch(a, c, false, (hipStream_t)stream);
}

extern "C" int rsmi_decook_dev(const rsmi_cook_ctx *c, const rsmi_packet_batch *b, void *stream) {
    if (!c) return fail(RSMI_ERR_INVALID, "null cook context");
    if (int rc = check_batch(b)) return rc;
    return launch(make_args(c, b), c, true, (hipStream_t)stream);
}

extern "C" int rsmi_cook_to(const rsmi_cook_ctx *c, const rsmi_packet_batch *b, uint8_t *out,
                            const uint8_t *iv, const uint8_t *iv_len, uint64_t seed, void *stream) {
    if (!c) return fail(RSMI_ERR_INVALID, "null cook context");
    if (int rc = check_batch(b)) return rc;
    if ((iv == nullptr) != (iv_len == nullptr))
        return fail(RSMI_ERR_INVALID, "iv and iv_len must both be given or both be NULL");
    if (!out || ((uintptr_t)out & 15)) return fail(RSMI_ERR_INVALID, "out must be a 16-aligned pointer");
    rsmi::CookArgs a = make_args(c, b);
    a.dst = out;
    a.iv = iv;
    a.iv_len = iv_len;
    a.seed = seed;
    return launch(a, c, false, (hipStream_t)stream);
}

extern "C" int rsmi_decook_mirror(const rsmi_cook_ctx *c, const rsmi_packet_batch *b, uint8_t *mirror,
                                  void *stream) {
    if (!c) return fail(RSMI_ERR_INVALID, "null cook context");
    if (int rc = check_batch(b)) return rc;
    if (!mirror || ((uintptr_t)mirror & 15)) return fail(RSMI_ERR_INVALID, "mirror must be a 16-aligned pointer");
    rsmi::CookArgs a = make_args(c, b);
    a.mirror = mirror;
    return launch(a, c, true, (hipStream_t)stream);
}

extern "C" int rsmi_decook_to(const rsmi_cook_ctx *c, const rsmi_packet_batch *b, uint8_t *out,
                              void *stream) {
    if (!c) return fail(RSMI_ERR_INVALID, "null cook context");
    if (int rc = check_batch(b)) return rc;
    if (!out || ((uintptr_t)out & 15)) return fail(RSMI_ERR_INVALID, "out must be a 16-aligned pointer");
    rsmi::CookArgs a = make_args(c, b);
    a.dst = out;
    return launch(a, c, true, (hipStream_t)stream);
}

namespace rsmi {
int cook_ctx_flags(const rsmi_cook_ctx *c) { return c->flags; }
const uint8_t *cook_ctx_ks(const rsmi_cook_ctx *c) { return c->ks ? c->ks : c->zks; }

int cook_packets(const rsmi_cook_ctx *c, uint8_t *slots, int64_t S, const rsmi_fenc_packet *pk,
                 int64_t npk, int32_t *out_len, uint8_t *dst, const int64_t *dst_off, uint64_t seed,
                 hipStream_t s, bool prex) {
    CookArgs a{};
    a.prex = prex ? 1 : 0;
    a.base = slots;
    a.dst = dst;
    a.dst_off = dst_off;
    a.pk = pk;
    a.pk_off = kSlotHeader;
    a.pk_idx = 1;
    a.phase = 1;  // slot bytes before a packet are the slot's own scratch (RSMI_FEC_SLOT_PACKET)
    a.stride = S;
    a.count = npk;
    a.cap = (int32_t)(S - kSlotHeader);
    a.flags = c->flags;
    a.out_len = out_len;
    a.seed = seed;
    a.tabs = c->tabs;
    a.ks = c->ks;
    return launch(a, c, false, s);
}
int cook_frame_packets(const rsmi_cook_ctx *c, uint8_t *slots, int64_t S, const rsmi_fenc_packet *pk,
                       int64_t npk, int32_t *out_len, uint8_t *dst, const int64_t *dst_off, uint64_t seed,
                       const FuseArgs &f, hipStream_t s) {
    if (npk <= 0) return RSMI_OK;
    CookArgs a{};
    a.base = slots;
    a.dst = dst;
    a.dst_off = dst_off;
    a.pk = pk;
    a.pk_off = kSlotHeader;
    a.pk_idx = 1;
    a.phase = 1;
    a.stride = S;
    a.count = npk;
    a.cap = (int32_t)(S - kSlotHeader);
    a.flags = c->flags;
    a.out_len = out_len;
    a.seed = seed;
    a.tabs = c->tabs;
    a.ks = c->ks;
    const hipError_t e = launch_cook_frame(a, f, c->max_blocks, s);
    if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("cook_frame launch: ") + hipGetErrorString(e));
    return RSMI_OK;
}
}  // namespace rsmi

namespace {

// Host batch: packets [count][stride] then len, out_len, iv, iv_len in one
// device allocation; copy in, launch, copy back.
int host_run(rsmi_cook_ctx *c, bool decook, uint8_t *host, int64_t stride, int64_t count,
             int32_t cap, const int32_t *len, int32_t *out_len, const uint8_t *iv,
             const uint8_t *iv_len, uint64_t seed) {
    if (!c || count < 0 || stride < 0 || cap < 0 || cap > stride || (count && (!host || !len || !out_len)))
        return fail(RSMI_ERR_INVALID, "invalid host cook arguments");
    if (stride % 4) return fail(RSMI_ERR_INVALID, "stride must be a multiple of 4");
    if (count == 0) return RSMI_OK;
    const size_t dbytes = (size_t)(stride * count);
    const size_t o_len = (dbytes + 255) & ~size_t(255);
    const size_t o_out = o_len + (((size_t)count * 4 + 255) & ~size_t(255));
    const size_t o_iv = o_out + (((size_t)count * 4 + 255) & ~size_t(255));
    const size_t o_ivl = o_iv + (((size_t)count * RSMI_COOK_IV_MAX + 255) & ~size_t(255));
    const size_t need = o_ivl + (size_t)count + 16;
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->hcap < need) {
        if (c->hbuf) (void)hipFree(c->hbuf);
        c->hbuf = nullptr;
        c->hcap = 0;
        if (hipMalloc(&c->hbuf, need) != hipSuccess) return fail(RSMI_ERR_NOMEM, "hipMalloc(host cook)");
        c->hcap = need;
    }
    uint8_t *d = c->hbuf;
    hipError_t e = hipMemcpy(d, host, dbytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d + o_len, len, (size_t)count * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess && iv) e = hipMemcpy(d + o_iv, iv, (size_t)count * RSMI_COOK_IV_MAX, hipMemcpyHostToDevice);
    if (e == hipSuccess && iv_len) e = hipMemcpy(d + o_ivl, iv_len, (size_t)count, hipMemcpyHostToDevice);
    if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("host cook H2D: ") + hipGetErrorString(e));
    rsmi_packet_batch b{d, nullptr, stride, count, cap, 0,
                        reinterpret_cast<const int32_t *>(d + o_len),
                        reinterpret_cast<int32_t *>(d + o_out)};
    rsmi::CookArgs a = make_args(c, &b);
    a.iv = iv ? d + o_iv : nullptr;
    a.iv_len = iv ? d + o_ivl : nullptr;
    a.seed = seed;
    if (int rc = launch(a, c, decook, nullptr)) return rc;
    e = hipMemcpy(host, d, dbytes, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out_len, d + o_out, (size_t)count * 4, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("host cook D2H: ") + hipGetErrorString(e));
    return RSMI_OK;
}

}  // namespace

extern "C" int rsmi_cook_host(const rsmi_cook_ctx *c, uint8_t *host, int64_t stride, int64_t count,
                              int32_t cap, const int32_t *len, int32_t *out_len, const uint8_t *iv,
                              const uint8_t *iv_len, uint64_t seed) {
    if ((iv == nullptr) != (iv_len == nullptr))
        return fail(RSMI_ERR_INVALID, "iv and iv_len must both be given or both be NULL");
    return host_run(const_cast<rsmi_cook_ctx *>(c), false, host, stride, count, cap, len, out_len,
                    iv, iv_len, seed);
}

extern "C" int rsmi_decook_host(const rsmi_cook_ctx *c, uint8_t *host, int64_t stride,
                                int64_t count, int32_t cap, const int32_t *len, int32_t *out_len) {
    return host_run(const_cast<rsmi_cook_ctx *>(c), true, host, stride, count, cap, len, out_len,
                    nullptr, nullptr, 0);
}
