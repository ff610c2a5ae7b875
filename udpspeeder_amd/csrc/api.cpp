// api.cpp -- host runtime of librsmi.so: per-device state (GF tables, resident
// codes, decode workspaces), argument validation, the extern "C" batched API
// of include/rsmi.h, and the synchronous host-memory variants used by the
// drop-in shim (compat.cpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gf256.hpp"
#include "rsmi_internal.hpp"

namespace rsmi {
std::atomic<int> g_opt_cls_cap{0};  // RSMI_OPT_CLS_REC_CAP (read by ragged.cpp)
namespace {

thread_local std::string g_err;
thread_local int g_last_enc = RSMI_ENC_NONE;  // rsmi_last_encoder
std::atomic<int> g_opt_oneshot{1};              // RSMI_OPT_ONE_GROUP
std::atomic<int> g_opt_server{-1};              // RSMI_OPT_ONE_SERVER: idle us (-1: not read yet)
std::atomic<int> g_opt_server_life{-1};         // RSMI_OPT_ONE_SERVER_LIFE: ms (-1: not read yet)
std::atomic<int> g_opt_bitslice{1};
std::atomic<int> g_opt_fused{1};
std::atomic<int> g_opt_parity_cook{-1};        // RSMI_OPT_PARITY_COOK (-1: not read yet)

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char *what) {
    return fail(RSMI_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define RSMI_HIP(call, what)                          \
    do {                                              \
        hipError_t e_ = (call);                       \
        if (e_ != hipSuccess) return hip_fail(e_, what); \
    } while (0)

struct Code {
    int k = 0, n = 0;
    std::vector<uint8_t> host;    // n x k
    uint8_t *dev_rows = nullptr;  // (n-k) x k parity rows on the device
};

struct Workspace {
    uint8_t *ptr = nullptr;
    size_t bytes = 0;
};

// Streams and buffers of the pinned host<->device pipelines (rsmi_encode_pinned,
// rsmi_decode_pinned): one of each per device, one call at a time.
struct Pipeline {
    static constexpr int kDepth = 3;
    std::mutex mu;
    hipStream_t st[kDepth] = {};
    uint8_t *dev[kDepth] = {};
    size_t bytes = 0;
    int32_t *dstat[kDepth] = {};  // decode: status and present flags per stage
    uint8_t *dpres[kDepth] = {};
    int64_t cap = 0;
    uint8_t *hpin = nullptr;      // decode: pinned copies of present / status (pageable
    size_t hpin_bytes = 0;        // small copies would block the issuing thread)
};

struct Device {
    int id = -1;
    std::mutex mu;
    uint32_t *ptab = nullptr;     // 256 x kPtabDwords
    uint8_t *gftab = nullptr;     // exp[512] | log[256]
    uint64_t *code_dir = nullptr; // 257*257 device pointers to parity rows
    std::map<int, Code> codes;    // key k*257+n
    std::map<hipStream_t, Workspace> ws;
    // host-path resources (guarded by hmu, held for a whole host call)
    std::mutex hmu;
    hipStream_t hstream = nullptr;
    uint8_t *pinned = nullptr;
    size_t pinned_bytes = 0;
    uint8_t *hdev = nullptr;
    size_t hdev_bytes = 0;
    int32_t *hstatus_dev = nullptr;
    size_t hstatus_cap = 0;
    Pipeline penc, pdec, pzc;  // pzc: rsmi_decode_pinned's zero-copy path
    Pipeline prag;             // rsmi_encode_ragged_pinned / rsmi_decode_ragged_pinned
    // one group per call (oneshot.hip): pinned staging the kernel reads and
    // writes over PCIe, a completion flag, guarded by one_mu
    std::mutex one_mu;
    hipStream_t one_stream = nullptr;
    uint8_t *one_pin = nullptr, *one_dev = nullptr;  // host / device address of the staging
    size_t one_bytes = 0;
    uint32_t one_seq = 0;
    // the resident one-group server (oneshot.hip k_one_server), guarded by one_mu
    OneSrvCtl *srv_pin = nullptr, *srv_dev = nullptr;
    OneSrvDev *srv_dv = nullptr;  // device memory of the server's stop / exit words
    uint32_t srv_gen = 0;
    bool srv_running = false;
};

std::mutex g_devs_mu;
std::map<int, std::unique_ptr<Device>> g_devs;

int init_device(Device &D) {
    // caller holds D.mu
    if (D.ptab) return RSMI_OK;
    std::vector<uint32_t> pt(256 * kPtabDwords, 0);
    for (int c = 0; c < 256; ++c) perm_tables((uint8_t)c, &pt[(size_t)c * kPtabDwords]);
    const GF &F = gf();
    // exp[512] | log[256] | pad | the ragged decode's Lagrange tables at
    // kGfLtabOff (decode.hip LTables: the split table of alpha^v by v, the
    // evaluation point of each shard index, log with log 0 = 0), copied into
    // LDS by each workgroup with one 16-byte load per piece
    std::vector<uint8_t> gt(kGfLtabOff + kGfLtabBytes, 0);
    std::memcpy(gt.data(), F.exp, 512);
    for (int i = 0; i < 256; ++i) gt[512 + i] = (uint8_t)F.log[i];
    {
        uint8_t *lt = gt.data() + kGfLtabOff;
        for (int v = 0; v < 256; ++v) {
            const uint32_t c = F.exp[v < 255 ? v : 0];
            std::memcpy(lt + 16 * v, &pt[(size_t)c * kPtabDwords], 16);
            std::memcpy(lt + 4096 + 4 * v, &pt[(size_t)c * kPtabDwords + 4], 4);
            lt[5120 + v] = v ? F.exp[v - 1] : 0;
            lt[5376 + v] = v ? (uint8_t)F.log[v] : 0;
        }
    }
    RSMI_HIP(hipMalloc(&D.ptab, pt.size() * 4), "hipMalloc(ptab)");
    RSMI_HIP(hipMalloc(&D.gftab, gt.size()), "hipMalloc(gftab)");
    RSMI_HIP(hipMalloc(&D.code_dir, sizeof(uint64_t) * 257 * 257), "hipMalloc(code_dir)");
    RSMI_HIP(hipMemcpy(D.ptab, pt.data(), pt.size() * 4, hipMemcpyHostToDevice), "upload ptab");
    RSMI_HIP(hipMemcpy(D.gftab, gt.data(), gt.size(), hipMemcpyHostToDevice), "upload gftab");
    RSMI_HIP(hipMemset(D.code_dir, 0, sizeof(uint64_t) * 257 * 257), "clear code_dir");
    return RSMI_OK;
}

// Returns the state of the current device, initialised; nullptr on error.
Device *current(int *rc) {
    int id = -1;
    hipError_t e = hipGetDevice(&id);
    if (e != hipSuccess) {
        *rc = hip_fail(e, "hipGetDevice (no usable GPU?)");
        return nullptr;
    }
    Device *D;
    {
        std::lock_guard<std::mutex> lk(g_devs_mu);
        auto &slot = g_devs[id];
        if (!slot) {
            slot.reset(new Device());
            slot->id = id;
        }
        D = slot.get();
    }
    std::lock_guard<std::mutex> lk(D->mu);
    *rc = init_device(*D);
    return *rc == RSMI_OK ? D : nullptr;
}

// caller holds D.mu
int ensure_code(Device &D, int k, int n, const Code **out) {
    if (k < 1 || n < k || k > 256 || n > 256)
        return fail(RSMI_ERR_INVALID, "invalid (k,n): need 1 <= k <= n <= 256");
    const int key = k * 257 + n;
    auto it = D.codes.find(key);
    if (it == D.codes.end()) {
        Code c;
        c.k = k;
        c.n = n;
        if (!build_enc_matrix(k, n, c.host)) return fail(RSMI_ERR_INVALID, "matrix build failed");
        const size_t rows = (size_t)(n - k) * k;
        if (rows) {
            RSMI_HIP(hipMalloc(&c.dev_rows, rows), "hipMalloc(code)");
            RSMI_HIP(hipMemcpy(c.dev_rows, c.host.data() + (size_t)k * k, rows,
                               hipMemcpyHostToDevice), "upload code");
            const uint64_t p = (uint64_t)(uintptr_t)c.dev_rows;
            RSMI_HIP(hipMemcpy(D.code_dir + key, &p, sizeof(p), hipMemcpyHostToDevice),
                     "code_dir entry");
        }
        it = D.codes.emplace(key, std::move(c)).first;
        // no build-time network: compile one in the background (bitslice_rtc.cpp)
        if (n > k && !has_bitslice(k, n)) bitslice_rtc_request({{k, n}});
    }
    *out = &it->second;
    return RSMI_OK;
}

// caller holds D.mu
int ensure_ws(Device &D, hipStream_t s, size_t bytes, uint8_t **out) {
    Workspace &w = D.ws[s];
    if (w.bytes < bytes) {
        if (w.ptr) {
            // the old buffer may still be in use by work queued on s
            RSMI_HIP(hipStreamSynchronize(s), "hipStreamSynchronize(ws grow)");
            RSMI_HIP(hipFree(w.ptr), "hipFree(ws)");
            w.ptr = nullptr;
            w.bytes = 0;
        }
        RSMI_HIP(hipMalloc(&w.ptr, bytes), "hipMalloc(decode workspace)");
        w.bytes = bytes;
    }
    *out = w.ptr;
    return RSMI_OK;
}

int check_uniform(int k, int n, const void *base, int64_t gs, int64_t ss, int len,
                  int64_t ngroups) {
    if (k < 1 || n < k || k > 256 || n > 256)
        return fail(RSMI_ERR_INVALID, "invalid (k,n): need 1 <= k <= n <= 256");
    if (len < 0 || ngroups < 0) return fail(RSMI_ERR_INVALID, "negative len/ngroups");
    if (ngroups > 0 && len > 0 && !base) return fail(RSMI_ERR_INVALID, "null base");
    if (ss % 16 || gs % 16 || ((uintptr_t)base) % 16)
        return fail(RSMI_ERR_INVALID, "base, shard_stride and group_stride must be 16-aligned");
    if (ss < len) return fail(RSMI_ERR_INVALID, "shard_stride < len");
    return RSMI_OK;
}

int tile_words(int len) {
    int w = (len + 255) / 256;
    return w < 1 ? 1 : (w > 5 ? 5 : w);
}

UniformArgs make_args(int k, int n, uint8_t *base, int64_t gs, int64_t ss, int len,
                      int64_t ngroups, int *W) {
    *W = tile_words(len);
    UniformArgs a;
    a.base = base;
    a.group_stride = gs;
    a.shard_stride = ss;
    a.len = len;
    a.k = k;
    a.n = n;
    a.tiles = (len + 256 * *W - 1) / (256 * *W);
    if (a.tiles < 1) a.tiles = 1;
    a.ngroups = ngroups;
    return a;
}

size_t plan_bytes(int k, int n, int64_t ngroups) {
    const int m = n - k;
    const PlanLayout L(k, k < m ? k : m);
    return (size_t)L.stride * (size_t)(ngroups > 0 ? ngroups : 1);
}

}  // namespace

// ---- internal entry points shared with compat.cpp -------------------------
int encode_dev(int k, int n, uint8_t *base, int64_t gs, int64_t ss, int len, int64_t ngroups,
               hipStream_t s) {
    int rc = check_uniform(k, n, base, gs, ss, len, ngroups);
    if (rc) return rc;
    Device *D = current(&rc);
    if (!D) return rc;
    const Code *C;
    {
        std::lock_guard<std::mutex> lk(D->mu);
        rc = ensure_code(*D, k, n, &C);
        if (rc) return rc;
    }
    if (n == k || len == 0 || ngroups == 0) return RSMI_OK;
    int W;
    UniformArgs a = make_args(k, n, base, gs, ss, len, ngroups, &W);
    hipError_t e = hipErrorNotSupported;
    // build-time network, else the run-time one once compiled (NotSupported
    // until then), else the generic table kernel
    if (g_opt_bitslice.load()) e = launch_encode_bitslice(a, s);
    g_last_enc = e == hipErrorNotSupported ? RSMI_ENC_GENERIC
                 : has_bitslice(k, n)      ? RSMI_ENC_BITSLICE
                                           : RSMI_ENC_BITSLICE_RTC;
    if (e == hipErrorNotSupported) e = launch_encode_generic(a, W, C->dev_rows, D->ptab, s);
    if (e != hipSuccess) return hip_fail(e, "encode launch");
    return RSMI_OK;
}

bool parity_cook_enabled() {
    int v = g_opt_parity_cook.load();
    if (v < 0) {  // RSMI_PARITY_COOK=1 turns it on for a process (A/B runs)
        const char *e = std::getenv("RSMI_PARITY_COOK");
        v = (e && *e && *e != '0') ? 1 : 0;
        int expect = -1;
        g_opt_parity_cook.compare_exchange_strong(expect, v);
        v = g_opt_parity_cook.load();
    }
    return v > 0;
}

bool encode_cooked_ok(int k, int n, int64_t gs, int64_t ss, int len, int64_t ngroups) {
    if (!g_opt_bitslice.load() || n <= k || len <= 0 || ngroups <= 0 || k > 256 || n > 256 || ss % 16 ||
        gs % 16 || ss < len)
        return false;
    int W;
    return bitslice_cooked_ok(make_args(k, n, nullptr, gs, ss, len, ngroups, &W));
}

// encode_dev with the parity cook in the epilogue (the caller checked
// encode_cooked_ok; the kernels and records are described at EpiRec).
int encode_dev_cooked(int k, int n, uint8_t *base, int64_t gs, int64_t ss, int len, int64_t ngroups,
                      const CookEpi &ep, hipStream_t s) {
    int rc = check_uniform(k, n, base, gs, ss, len, ngroups);
    if (rc) return rc;
    Device *D = current(&rc);
    if (!D) return rc;
    const Code *C;
    {
        std::lock_guard<std::mutex> lk(D->mu);
        rc = ensure_code(*D, k, n, &C);
        if (rc) return rc;
    }
    int W;
    UniformArgs a = make_args(k, n, base, gs, ss, len, ngroups, &W);
    const hipError_t e = launch_encode_bitslice_cooked(a, ep, s);
    if (e != hipSuccess) return hip_fail(e, "cooking encode launch");
    g_last_enc = RSMI_ENC_BITSLICE;
    return RSMI_OK;
}

int decode_dev(int k, int n, uint8_t *base, int64_t gs, int64_t ss, int len, int64_t ngroups,
               const uint8_t *present, int32_t *status, hipStream_t s, bool ref = false,
               uint8_t *slot_map = nullptr) {
    int rc = check_uniform(k, n, base, gs, ss, len, ngroups);
    if (rc) return rc;
    if (ngroups > 0 && !present) return fail(RSMI_ERR_INVALID, "null present");
    Device *D = current(&rc);
    if (!D) return rc;
    const Code *C;
    uint8_t *plans = nullptr;
    const bool fused = g_opt_fused.load() && n > k && decode_fused_ok(k, n, gs, ss, len);
    {
        std::lock_guard<std::mutex> lk(D->mu);
        rc = ensure_code(*D, k, n, &C);
        if (rc) return rc;
        if (!fused) {
            rc = ensure_ws(*D, s, plan_bytes(k, n, ngroups), &plans);
            if (rc) return rc;
        }
    }
    if (ngroups == 0) return RSMI_OK;
    int W;
    UniformArgs a = make_args(k, n, base, gs, ss, len, ngroups, &W);
    if (fused) {
        hipError_t e = launch_decode_fused(a, present, C->dev_rows, status, D->ptab, D->gftab, s,
                                           false, ref, slot_map);
        if (e != hipSuccess) return hip_fail(e, "fused decode launch");
        return RSMI_OK;
    }
    hipError_t e = launch_decode_plan(a, present, C->dev_rows, plans, status, D->gftab, s);
    if (e != hipSuccess) return hip_fail(e, "decode plan launch");
    if (n > k && len > 0) {
        e = launch_decode_apply(a, W, plans, D->ptab, s);
        if (e != hipSuccess) return hip_fail(e, "decode apply launch");
    }
    if (ref) {
        e = launch_decode_ref_move(a, plans, present, slot_map, s);
        if (e != hipSuccess) return hip_fail(e, "decode placement launch");
    }
    return RSMI_OK;
}

int prepare_code(int k, int n) {
    int rc;
    Device *D = current(&rc);
    if (!D) return rc;
    std::lock_guard<std::mutex> lk(D->mu);
    const Code *C;
    return ensure_code(*D, k, n, &C);
}

int reserve(int k, int n, int64_t ngroups, hipStream_t s) {
    if (k < 1 || n < k || k > 256 || n > 256 || ngroups < 0)
        return fail(RSMI_ERR_INVALID, "invalid reserve arguments");
    int rc;
    Device *D = current(&rc);
    if (!D) return rc;
    std::lock_guard<std::mutex> lk(D->mu);
    const Code *C;
    rc = ensure_code(*D, k, n, &C);
    if (rc) return rc;
    uint8_t *ws;
    return ensure_ws(*D, s, plan_bytes(k, n, ngroups), &ws);
}

int encode_ragged_dev(const rsmi_group *dg, int64_t ngroups, uint8_t *base, hipStream_t s) {
    if (ngroups < 0) return fail(RSMI_ERR_INVALID, "negative ngroups");
    if (ngroups == 0) return RSMI_OK;
    if (!dg || !base) return fail(RSMI_ERR_INVALID, "null descriptors/base");
    int rc;
    Device *D = current(&rc);
    if (!D) return rc;
    hipError_t e = launch_encode_ragged(dg, ngroups, base, D->code_dir, D->ptab, s);
    if (e != hipSuccess) return hip_fail(e, "ragged encode launch");
    return RSMI_OK;
}

int decode_ragged_dev(const rsmi_group *dg, int64_t ngroups, uint8_t *base,
                      const uint32_t *present_bits, int32_t *status, int kmax, hipStream_t s,
                      RefOut ro = RefOut{nullptr, 0, 0}) {
    if (ngroups < 0) return fail(RSMI_ERR_INVALID, "negative ngroups");
    if (ngroups == 0) return RSMI_OK;
    if (!dg || !base || !present_bits || !status)
        return fail(RSMI_ERR_INVALID, "null descriptors/base/present_bits/status");
    if (((uintptr_t)base) % 16) return fail(RSMI_ERR_INVALID, "base must be 16-aligned");
    int rc;
    Device *D = current(&rc);
    if (!D) return rc;
    hipError_t e = launch_decode_ragged(dg, ngroups, base, present_bits, status, kmax,
                                        D->code_dir, D->ptab, D->gftab, s, ro);
    if (e != hipSuccess) return hip_fail(e, "ragged decode launch");
    return RSMI_OK;
}

int decode_ragged_cls_dev(const rsmi_group *dg, int64_t ngroups, const ClsLaunch &C, uint8_t *base,
                          const uint32_t *present_bits, int32_t *status, int kmax, hipStream_t s) {
    if (ngroups <= 0) return RSMI_OK;
    if (!base || !present_bits || !status)
        return fail(RSMI_ERR_INVALID, "null base/present_bits/status");
    if (((uintptr_t)base) % 16) return fail(RSMI_ERR_INVALID, "base must be 16-aligned");
    int rc;
    Device *D = current(&rc);
    if (!D) return rc;
    // Classes run one after another on s: forking them over four streams
    // (event fork/join) measured slower, 0.240 vs 0.217 ms for C3.
    const hipStream_t cs[4] = {s, s, s, s};
    hipError_t e = launch_decode_ragged_cls(dg, C, base, present_bits, status, kmax, D->code_dir,
                                            D->ptab, D->gftab, s, cs);
    // the plan knows whether any group can be deferred (e never defers: the
    // class kernels take any e in row blocks); without one, no big launch
    if (e == hipSuccess && C.need_big)
        e = launch_decode_ragged_big(dg, ngroups, base, present_bits, status, D->code_dir, D->ptab,
                                     D->gftab, s, C.defer, C.epoch, C.ref);
    if (e != hipSuccess) return hip_fail(e, "ragged decode launch");
    return RSMI_OK;
}

const uint8_t *device_code_rows(int k, int n) {
    int rc;
    Device *D = current(&rc);
    if (!D) return nullptr;
    std::lock_guard<std::mutex> lk(D->mu);
    auto it = D->codes.find(k * 257 + n);
    return it == D->codes.end() ? nullptr : it->second.dev_rows;
}

uint64_t *device_code_dir(int *rc) {
    Device *D = current(rc);
    return D ? D->code_dir : nullptr;
}

const uint32_t *device_ptab(int *rc) {
    Device *D = current(rc);
    return D ? D->ptab : nullptr;
}

// ---- synchronous host-memory path (pinned staging, internal stream) --------
namespace {
int host_buffers(Device &D, size_t bytes, int64_t ngroups) {
    // caller holds D.hmu
    if (!D.hstream) RSMI_HIP(hipStreamCreateWithFlags(&D.hstream, hipStreamNonBlocking),
                             "hipStreamCreate");
    if (D.pinned_bytes < bytes) {
        if (D.pinned) (void)hipHostFree(D.pinned);
        D.pinned = nullptr;
        D.pinned_bytes = 0;
        RSMI_HIP(hipHostMalloc(&D.pinned, bytes, hipHostMallocDefault), "hipHostMalloc");
        D.pinned_bytes = bytes;
    }
    if (D.hdev_bytes < bytes) {
        if (D.hdev) (void)hipFree(D.hdev);
        D.hdev = nullptr;
        D.hdev_bytes = 0;
        RSMI_HIP(hipMalloc(&D.hdev, bytes), "hipMalloc(host path)");
        D.hdev_bytes = bytes;
    }
    if ((int64_t)D.hstatus_cap < ngroups) {
        if (D.hstatus_dev) (void)hipFree(D.hstatus_dev);
        D.hstatus_dev = nullptr;
        RSMI_HIP(hipMalloc(&D.hstatus_dev, sizeof(int32_t) * (size_t)ngroups), "hipMalloc(st)");
        D.hstatus_cap = (size_t)ngroups;
    }
    return RSMI_OK;
}
}  // namespace

// ---- the resident one-group server --------------------------------------------
int server_idle_us() {
    int v = g_opt_server.load();
    if (v < 0) {  // first use: RSMI_ONE_SERVER_IDLE_US overrides the default (0 = off)
        const char *env = getenv("RSMI_ONE_SERVER_IDLE_US");
        v = env ? std::max(0, atoi(env)) : 20000;
        int expect = -1;
        if (!g_opt_server.compare_exchange_strong(expect, v)) v = g_opt_server.load();
    }
    return v;
}

// The server's lifetime cap (relaunched by the next call after it): the
// reference's own latency budget, fec_manager.h:30 (timeout = 8 ms), so a
// device-wide synchronisation waits at most about that long for it even under
// steady traffic.
int server_life_ms() {
    int v = g_opt_server_life.load();
    if (v < 0) {
        const char *env = getenv("RSMI_ONE_SERVER_LIFE_MS");
        v = env ? std::max(1, atoi(env)) : 8;
        int expect = -1;
        if (!g_opt_server_life.compare_exchange_strong(expect, v)) v = g_opt_server_life.load();
    }
    return v;
}

std::mutex g_srv_list_mu;
std::vector<Device *> g_srv_devs;  // devices whose server may be running

void stop_servers_at_exit() {
    std::lock_guard<std::mutex> lk(g_srv_list_mu);
    for (Device *D : g_srv_devs)
        if (D->srv_pin) reinterpret_cast<volatile uint32_t *>(&D->srv_pin->quit)[0] = 1u;
}

// Pinned memory of the one-group path (staging, server control block):
// RSMI_ONE_HOSTMEM = 0 hipHostMallocDefault, 1 coherent, 2 uncached (A/B knob).
unsigned one_hostmem_flags() {
    static const unsigned f = [] {
        const char *e = getenv("RSMI_ONE_HOSTMEM");
        const int v = e ? atoi(e) : 0;
        return v == 1 ? (unsigned)hipHostMallocCoherent : v == 2 ? (unsigned)hipHostMallocUncached
                                                                 : (unsigned)hipHostMallocDefault;
    }();
    return f;
}

// caller holds D.one_mu
int launch_server(Device &D, uint32_t done0, uint32_t idle_us) {
    if (!D.srv_pin) {
        void *hp = nullptr, *dp = nullptr;
        RSMI_HIP(hipHostMalloc(&hp, sizeof(OneSrvCtl), one_hostmem_flags()), "hipHostMalloc(server)");
        RSMI_HIP(hipHostGetDevicePointer(&dp, hp, 0), "hipHostGetDevicePointer(server)");
        std::memset(hp, 0, sizeof(OneSrvCtl));
        RSMI_HIP(hipMalloc(&D.srv_dv, sizeof(OneSrvDev)), "hipMalloc(server)");
        D.srv_pin = static_cast<OneSrvCtl *>(hp);
        D.srv_dev = static_cast<OneSrvCtl *>(dp);
        std::lock_guard<std::mutex> lk(g_srv_list_mu);
        if (g_srv_devs.empty()) std::atexit(stop_servers_at_exit);
        g_srv_devs.push_back(&D);
    }
    reinterpret_cast<volatile uint32_t *>(&D.srv_pin->quit)[0] = 0u;
    const uint32_t gen = ++D.srv_gen;
    hipError_t e = launch_one_server(D.srv_dev, D.srv_dv, D.ptab, D.gftab, gen, done0, idle_us,
                                     (uint32_t)server_life_ms(), D.one_stream);
    if (e != hipSuccess) return hip_fail(e, "one-group server launch");
    D.srv_running = true;
    return RSMI_OK;
}

// caller holds D.one_mu; the job's inputs are in staging.  Every word of the
// job block carries the seq beside its dword of OneArgs (OneSrvCtl).
int post_to_server(Device &D, const OneArgs &a, uint32_t idle_us) {
    if (!D.srv_pin || !D.srv_running) {
        int rc = launch_server(D, a.seq - 1, idle_us);
        if (rc) return rc;
    }
    uint32_t w[kOneJobWords] = {};
    static_assert(sizeof(OneArgs) <= sizeof(w), "OneArgs fits the job block");
    std::memcpy(w, &a, sizeof(OneArgs));
    std::atomic_thread_fence(std::memory_order_release);  // the inputs before any job word
    volatile uint64_t *job = D.srv_pin->job;
    for (int i = 0; i < kOneJobWords; ++i) job[i] = ((uint64_t)a.seq << 32) | w[i];
    return RSMI_OK;
}

// caller holds D.one_mu: stop a running server and wait for it to end
int stop_server_locked(Device &D) {
    if (!D.srv_pin || !D.srv_running) return RSMI_OK;
    reinterpret_cast<volatile uint32_t *>(&D.srv_pin->quit)[0] = 1u;
    RSMI_HIP(hipStreamSynchronize(D.one_stream), "stop one-group server");
    D.srv_running = false;
    return RSMI_OK;
}

// Stop a running server and wait for it (RSMI_OPT_ONE_SERVER 0, rsmi_quiesce).
int stop_server(Device &D) {
    std::lock_guard<std::mutex> lk(D.one_mu);
    return stop_server_locked(D);
}

// Every device's server stopped (the next drop-in call relaunches its own).
int stop_all_servers() {
    std::vector<Device *> ds;
    {
        std::lock_guard<std::mutex> lk(g_srv_list_mu);
        ds = g_srv_devs;
    }
    int cur = -1;
    (void)hipGetDevice(&cur);
    int rc = RSMI_OK;
    for (Device *D : ds) {
        (void)hipSetDevice(D->id);
        rc = stop_server(*D);
        if (rc) break;
    }
    if (cur >= 0) (void)hipSetDevice(cur);
    return rc;
}

// One group, host buffers, one kernel (oneshot.hip): the shards the kernel
// needs are copied into pinned staging, the kernel reads them over PCIe,
// writes the output rows back into staging and raises a flag this thread
// spins on.  Returns 1 when the code/shape is outside the kernel's range (the
// caller takes the staged path), else RSMI_OK or an error.
int one_group_op(Device &D, bool decode, int k, int n, uint8_t *const *ptrs, uint8_t *const *out,
                 int len, const uint8_t *present, int32_t *status) {
    const int ss = (len + 15) & ~15;
    if (!one_group_ok(k, n, len, ss > 0 ? ss : 16, !decode)) return 1;
    const Code *C;
    int rc;
    {
        std::lock_guard<std::mutex> lk(D.mu);
        rc = ensure_code(D, k, n, &C);
        if (rc) return rc;
    }
    std::lock_guard<std::mutex> lk(D.one_mu);
    const int m = n - k;
    const size_t in_bytes = (size_t)n * ss, out_bytes = (size_t)(decode ? k : m) * ss;
    const size_t need = in_bytes + out_bytes + 128;
    if (!D.one_stream)
        RSMI_HIP(hipStreamCreateWithFlags(&D.one_stream, hipStreamNonBlocking), "hipStreamCreate(one)");
    if (D.one_bytes < need) {
        // a resident server still polls this staging, and CLR's hipHostFree
        // waits for every stream: stop it first (relaunched by the post below)
        rc = stop_server_locked(D);
        if (rc) return rc;
        if (D.one_pin) (void)hipHostFree(D.one_pin);
        D.one_pin = D.one_dev = nullptr;
        D.one_bytes = 0;
        const size_t cap = std::max<size_t>(need, 64 * 1024);
        RSMI_HIP(hipHostMalloc(&D.one_pin, cap, one_hostmem_flags()), "hipHostMalloc(one)");
        void *dp = nullptr;
        RSMI_HIP(hipHostGetDevicePointer(&dp, D.one_pin, 0), "hipHostGetDevicePointer(one)");
        D.one_dev = static_cast<uint8_t *>(dp);
        D.one_bytes = cap;
        std::memset(D.one_pin, 0, cap);
    }
    uint8_t *in = D.one_pin, *rows = D.one_pin + in_bytes;
    uint8_t *tail = D.one_pin + D.one_bytes - 128;  // status | pad | flags[kOneSrvWgs]
    int rows_out = m;  // encode: the parity rows; decode: the missing data rows
    if (decode) {
        rows_out = 0;
        for (int j = 0; j < k; ++j) rows_out += present[j] ? 0 : 1;
    }
    const bool multi = one_multi_ok(k, n, len, ss > 0 ? ss : 16, rows_out);
    const int idle_us = multi ? server_idle_us() : 0;
    if (!multi && D.srv_running) {  // the single-workgroup kernel queues on the server's stream
        rc = stop_server_locked(D);
        if (rc) return rc;
    }
    volatile uint32_t *flags = idle_us > 0 ? D.srv_pin ? D.srv_pin->flags : nullptr
                                           : reinterpret_cast<volatile uint32_t *>(tail + 64);
    const int nflags = multi ? kOneSrvWgs : 1;
    OneArgs a{};
    a.in = D.one_dev;
    a.out = D.one_dev + in_bytes;
    a.rows = C->dev_rows;
    a.ptab = D.ptab;
    a.gftab = D.gftab;
    a.status = reinterpret_cast<int32_t *>(D.one_dev + (tail - D.one_pin));
    a.flag = reinterpret_cast<uint32_t *>(D.one_dev + (tail + 64 - D.one_pin));
    a.seq = ++D.one_seq;
    a.k = k;
    a.n = n;
    a.len = len;
    a.ss = ss > 0 ? ss : 16;
    a.encode = decode ? 0 : 1;
    if (decode) {
        // only the survivors the kernel will read: the first k present (rs.cpp:24-39)
        int cnt = 0;
        for (int j = 0; j < n; ++j) {
            if (!present[j]) continue;
            a.present[j >> 5] |= 1u << (j & 31);
            if (cnt++ < k && len) std::memcpy(in + (size_t)j * ss, ptrs[j], (size_t)len);
        }
    } else if (len) {
        for (int j = 0; j < k; ++j) std::memcpy(in + (size_t)j * ss, ptrs[j], (size_t)len);
    }
    std::atomic_thread_fence(std::memory_order_release);
    if (idle_us > 0) {
        rc = post_to_server(D, a, (uint32_t)idle_us);
        if (rc) return rc;
        flags = D.srv_pin->flags;
    } else {
        hipError_t e = multi ? launch_one_multi(a, D.one_stream) : launch_one_group(a, D.one_stream);
        if (e != hipSuccess) return hip_fail(e, "one-group kernel launch");
    }
    // spin on the completion words (one per workgroup of the multi-workgroup
    // kernels); a kernel that never raises them surfaces its error through the
    // stream after a bound.  With the server: a server that ended (idle or
    // lifetime) before it ran this job is relaunched, and the new one takes
    // the pending job.
    auto all_done = [&] {
        for (int i = 0; i < nflags; ++i)
            if (flags[i] != a.seq) return false;
        return true;
    };
    const auto t0 = std::chrono::steady_clock::now();
    while (!all_done()) {
        __builtin_ia32_pause();
        if (idle_us > 0 && reinterpret_cast<volatile uint32_t *>(&D.srv_pin->exit_gen)[0] == D.srv_gen) {
            if (all_done()) break;  // it finished this job, then went idle
            rc = launch_server(D, a.seq - 1, (uint32_t)idle_us);
            if (rc) return rc;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
            if (idle_us > 0) reinterpret_cast<volatile uint32_t *>(&D.srv_pin->quit)[0] = 1u;
            RSMI_HIP(hipStreamSynchronize(D.one_stream), "one-group kernel");
            D.srv_running = false;
            if (!all_done()) return fail(RSMI_ERR_HIP, "one-group kernel did not complete");
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    const int32_t st = *reinterpret_cast<volatile int32_t *>(tail);
    if (status) *status = st;
    if (decode) {
        if (st != RSMI_DEC_OK || !len) return RSMI_OK;
        int r = 0;  // rebuilt rows come out in ascending missing-index order
        for (int j = 0; j < k; ++j)
            if (!present[j]) std::memcpy(out[j], rows + (size_t)(r++) * ss, (size_t)len);
    } else if (len) {
        for (int j = k; j < n; ++j) std::memcpy(ptrs[j], rows + (size_t)(j - k) * ss, (size_t)len);
    }
    return RSMI_OK;
}

// Gather host shards into a packed device layout [g][n][ss] (ss =
// round_up(len,16)), run the device op on the internal stream, scatter back.
// ptrs[g*n + j] is shard j of group g (may be null for an erased shard when
// decoding).  Encode writes parity rows j >= k; decode writes recovered data
// rows j < k whose pointer was null into out[g*k + j] (non-null required).
int host_op_ptrs(bool decode, int k, int n, uint8_t *const *ptrs, uint8_t *const *out, int len,
                 int64_t ngroups, const uint8_t *present, int32_t *status) {
    if (k < 1 || n < k || k > 256 || n > 256)
        return fail(RSMI_ERR_INVALID, "invalid (k,n): need 1 <= k <= n <= 256");
    if (len < 0 || ngroups < 0) return fail(RSMI_ERR_INVALID, "negative len/ngroups");
    if (ngroups == 0) return RSMI_OK;
    int rc;
    Device *D = current(&rc);
    if (!D) return rc;
    if (ngroups == 1 && n > k && g_opt_oneshot.load()) {
        rc = one_group_op(*D, decode, k, n, ptrs, out, len, present, status);
        if (rc != 1) return rc;
    }
    std::lock_guard<std::mutex> hl(D->hmu);
    const int64_t ss = len > 0 ? (len + 15) / 16 * 16 : 16;
    const int64_t dgs = ss * n;
    const size_t data_bytes = (size_t)(dgs * ngroups);
    const size_t pres_bytes = decode ? (size_t)(n * ngroups + 15) / 16 * 16 : 0;
    rc = host_buffers(*D, data_bytes + pres_bytes, ngroups);
    if (rc) return rc;
    uint8_t *P = D->pinned;
    for (int64_t g = 0; g < ngroups; ++g)
        for (int j = 0; j < n; ++j) {
            const bool have = decode ? present[g * n + j] != 0 : (j < k);
            if (have && len) std::memcpy(P + g * dgs + j * ss, ptrs[g * n + j], len);
        }
    if (decode) std::memcpy(P + data_bytes, present, (size_t)n * ngroups);
    hipStream_t s = D->hstream;
    RSMI_HIP(hipMemcpyAsync(D->hdev, P, data_bytes + pres_bytes, hipMemcpyHostToDevice, s),
             "H2D");
    if (decode)
        rc = decode_dev(k, n, D->hdev, dgs, ss, len, ngroups, D->hdev + data_bytes,
                        D->hstatus_dev, s);
    else
        rc = encode_dev(k, n, D->hdev, dgs, ss, len, ngroups, s);
    if (rc) {
        (void)hipStreamSynchronize(s);
        return rc;
    }
    RSMI_HIP(hipMemcpyAsync(P, D->hdev, data_bytes, hipMemcpyDeviceToHost, s), "D2H");
    std::vector<int32_t> st;
    if (decode) {
        st.resize((size_t)ngroups);
        RSMI_HIP(hipMemcpyAsync(st.data(), D->hstatus_dev, sizeof(int32_t) * ngroups,
                                hipMemcpyDeviceToHost, s), "D2H status");
    }
    RSMI_HIP(hipStreamSynchronize(s), "hipStreamSynchronize(host path)");
    for (int64_t g = 0; g < ngroups; ++g) {
        if (decode) {
            if (status) status[g] = st[(size_t)g];
            if (st[(size_t)g] != RSMI_DEC_OK) continue;
            for (int j = 0; j < k; ++j)
                if (!present[g * n + j] && len)
                    std::memcpy(out[g * k + j], P + g * dgs + j * ss, len);
        } else {
            for (int j = k; j < n; ++j)
                if (len) std::memcpy(ptrs[g * n + j], P + g * dgs + j * ss, len);
        }
    }
    return RSMI_OK;
}

int host_op(bool decode, int k, int n, uint8_t *base, int64_t gs, int64_t ss, int len,
            int64_t ngroups, const uint8_t *present, int32_t *status) {
    if (k < 1 || n < k || k > 256 || n > 256)
        return fail(RSMI_ERR_INVALID, "invalid (k,n): need 1 <= k <= n <= 256");
    if (ngroups < 0) return fail(RSMI_ERR_INVALID, "negative ngroups");
    std::vector<uint8_t *> p((size_t)(ngroups * n)), o(decode ? (size_t)(ngroups * k) : 0);
    for (int64_t g = 0; g < ngroups; ++g) {
        for (int j = 0; j < n; ++j) p[(size_t)(g * n + j)] = base + g * gs + j * ss;
        if (decode)
            for (int j = 0; j < k; ++j) o[(size_t)(g * k + j)] = base + g * gs + j * ss;
    }
    return host_op_ptrs(decode, k, n, p.data(), o.data(), len, ngroups, present, status);
}

// ---- pipelined host <-> device encode / decode (rsmi_*_pinned) ------------
int check_encode_pinned(int k, int n, const uint8_t *hd, int64_t dgs, uint8_t *hp, int64_t pgs,
                        int64_t ss, int len, int64_t ngroups, int64_t chunk) {
    int rc = check_uniform(k, n, nullptr, 16, ss, len, 0);
    if (rc) return rc;
    if (ngroups < 0 || chunk < 1 || (ngroups && (!hd || (!hp && n > k))) || dgs < k * ss ||
        (n > k && pgs < (n - k) * ss))
        return fail(RSMI_ERR_INVALID, "invalid encode_pinned arguments");
    return RSMI_OK;
}

// The pipeline on the calling thread's current device (D), with pipeline P:
// the device's own, or a multi-device worker's (rsmi_use_devices).
int encode_pinned_on(Device &D, Pipeline &P, int k, int n, const uint8_t *hd, int64_t dgs, uint8_t *hp,
                     int64_t pgs, int64_t ss, int len, int64_t ngroups, int64_t chunk) {
    int rc;
    (void)D;
    std::lock_guard<std::mutex> lk(P.mu);  // one call at a time per pipeline
    const int64_t dgs_dev = (int64_t)n * ss;
    const size_t need = (size_t)(dgs_dev * chunk);
    if (P.bytes < need) {
        for (int i = 0; i < Pipeline::kDepth; ++i) {
            if (P.dev[i]) (void)hipFree(P.dev[i]);
            P.dev[i] = nullptr;
        }
        P.bytes = 0;
        for (int i = 0; i < Pipeline::kDepth; ++i)
            RSMI_HIP(hipMalloc(&P.dev[i], need), "hipMalloc(pipeline)");
        P.bytes = need;
    }
    for (int i = 0; i < Pipeline::kDepth; ++i)
        if (!P.st[i]) RSMI_HIP(hipStreamCreateWithFlags(&P.st[i], hipStreamNonBlocking),
                               "hipStreamCreate(pipeline)");
    const int m = n - k;
    int64_t c = 0;
    for (int64_t g0 = 0; g0 < ngroups; g0 += chunk, ++c) {
        const int64_t cnt = std::min(chunk, ngroups - g0);
        const int b = (int)(c % Pipeline::kDepth);
        hipStream_t s = P.st[b];
        RSMI_HIP(hipMemcpy2DAsync(P.dev[b], dgs_dev, hd + g0 * dgs, dgs, (size_t)k * ss, cnt,
                                  hipMemcpyHostToDevice, s), "H2D data");
        rc = encode_dev(k, n, P.dev[b], dgs_dev, ss, len, cnt, s);
        if (rc) return rc;
        RSMI_HIP(hipMemcpy2DAsync(hp + g0 * pgs, pgs, P.dev[b] + (size_t)k * ss, dgs_dev,
                                  (size_t)m * ss, cnt, hipMemcpyDeviceToHost, s), "D2H parity");
    }
    for (int i = 0; i < Pipeline::kDepth; ++i)
        RSMI_HIP(hipStreamSynchronize(P.st[i]), "hipStreamSynchronize(pipeline)");
    return RSMI_OK;
}

int decode_zero_copy(Device &D, Pipeline &P, int k, int n, uint8_t *hs_dev, int64_t hgs, int64_t ss, int len,
                     int64_t ngroups, const uint8_t *present, int32_t *status) {
    std::lock_guard<std::mutex> lk(P.mu);  // one call at a time per pipeline
    const Code *C;
    int rc;
    {
        std::lock_guard<std::mutex> dl(D.mu);
        rc = ensure_code(D, k, n, &C);
        if (rc) return rc;
    }
    // present flags and statuses go through pinned staging in chunks of up
    // to kChunk groups (a few MB of device buffers, whatever the batch)
    constexpr int64_t kChunk = 1 << 18;
    const int64_t cap = std::min<int64_t>(ngroups, kChunk);
    if (P.cap < cap) {
        for (int i = 0; i < 2; ++i) {
            if (P.dstat[i]) (void)hipFree(P.dstat[i]);
            if (P.dpres[i]) (void)hipFree(P.dpres[i]);
            P.dstat[i] = nullptr;
            P.dpres[i] = nullptr;
        }
        if (P.hpin) (void)hipHostFree(P.hpin);
        P.hpin = nullptr;
        P.cap = 0;
        for (int i = 0; i < 2; ++i) {
            RSMI_HIP(hipMalloc(&P.dstat[i], sizeof(int32_t) * (size_t)cap), "hipMalloc(status)");
            RSMI_HIP(hipMalloc(&P.dpres[i], (size_t)(256 * cap)), "hipMalloc(present)");
        }
        RSMI_HIP(hipHostMalloc(&P.hpin, 2 * (size_t)(256 + 4) * (size_t)cap, hipHostMallocDefault),
                 "hipHostMalloc(pin)");
        P.cap = cap;
    }
    for (int i = 0; i < 2; ++i)
        if (!P.st[i]) RSMI_HIP(hipStreamCreateWithFlags(&P.st[i], hipStreamNonBlocking),
                               "hipStreamCreate(zero-copy)");
    // two chunks in flight: staging of chunk c+1's flags overlaps chunk c's kernel
    uint8_t *hp[2] = {P.hpin, P.hpin + (size_t)(256 + 4) * (size_t)cap};
    int64_t prev_g0[2] = {-1, -1}, prev_cnt[2] = {0, 0};
    auto finish = [&](int b) -> int {
        if (prev_g0[b] < 0) return RSMI_OK;
        RSMI_HIP(hipStreamSynchronize(P.st[b]), "hipStreamSynchronize(zero-copy)");
        if (status)
            std::memcpy(status + prev_g0[b], hp[b] + (size_t)n * cap, sizeof(int32_t) * (size_t)prev_cnt[b]);
        prev_g0[b] = -1;
        return RSMI_OK;
    };
    int64_t c = 0;
    for (int64_t g0 = 0; g0 < ngroups; g0 += cap, ++c) {
        const int64_t cnt = std::min(cap, ngroups - g0);
        const int b = (int)(c & 1);
        rc = finish(b);
        if (rc) return rc;
        hipStream_t s = P.st[b];
        std::memcpy(hp[b], present + g0 * n, (size_t)(n * cnt));
        RSMI_HIP(hipMemcpyAsync(P.dpres[b], hp[b], (size_t)(n * cnt), hipMemcpyHostToDevice, s),
                 "H2D present");
        int W;
        UniformArgs a = make_args(k, n, hs_dev + g0 * hgs, hgs, ss, len, cnt, &W);
        hipError_t e = launch_decode_fused(a, P.dpres[b], C->dev_rows, P.dstat[b], D.ptab, D.gftab, s,
                                           /*host_shards=*/true);
        if (e != hipSuccess) return hip_fail(e, "zero-copy decode launch");
        RSMI_HIP(hipMemcpyAsync(hp[b] + (size_t)n * cap, P.dstat[b], sizeof(int32_t) * (size_t)cnt,
                                hipMemcpyDeviceToHost, s), "D2H status");
        prev_g0[b] = g0;
        prev_cnt[b] = cnt;
    }
    for (int b = 0; b < 2; ++b) {
        rc = finish(b);
        if (rc) return rc;
    }
    return RSMI_OK;
}

// The device address of host range [p, p + bytes) when all of it lies in one
// pinned, device-mapped allocation (hipHostMalloc, torch pin_memory,
// hipHostRegister'ed), else nullptr: a kernel may then read and write it over
// PCIe.  Anything else (pageable memory, a range running past the allocation)
// never reaches a kernel.
uint8_t *mapped_host_range(uint8_t *p, size_t bytes) {
    const bool dbg = getenv("RSMI_DEBUG_PINNED") != nullptr;
    hipPointerAttribute_t at;
    hipError_t e = hipPointerGetAttributes(&at, p);
    if (e != hipSuccess) {
        if (dbg) fprintf(stderr, "rsmi: pinned? %p: hipPointerGetAttributes %d\n", (void *)p, (int)e);
        (void)hipGetLastError();
        return nullptr;
    }
    if (dbg)
        fprintf(stderr, "rsmi: pinned? %p: type %d dev %p host %p flags %u\n", (void *)p, (int)at.type,
                at.devicePointer, at.hostPointer, at.allocationFlags);
    if (at.type != hipMemoryTypeHost || !at.devicePointer || !at.hostPointer) return nullptr;
    // [p, p + bytes) lies in ONE allocation when its first and last bytes
    // report the same range start (RANGE_SIZE reads 0 for a 4 GiB pinned
    // block on ROCm 7.2, so the size is not trusted)
    void *start = nullptr, *start_last = nullptr;
    hipError_t e1 = hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p);
    hipError_t e2 = hipPointerGetAttribute(&start_last, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR,
                                           (hipDeviceptr_t)(p + bytes - 1));
    if (dbg)
        fprintf(stderr, "rsmi: pinned? range %d %d start %p start(last byte) %p need %zu\n", (int)e1, (int)e2,
                start, start_last, bytes);
    if (e1 != hipSuccess || e2 != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (!start || start != start_last || p < static_cast<const uint8_t *>(start)) return nullptr;
    hipPointerAttribute_t at_last;
    if (hipPointerGetAttributes(&at_last, p + bytes - 1) != hipSuccess || at_last.type != hipMemoryTypeHost) {
        (void)hipGetLastError();
        return nullptr;
    }
    return static_cast<uint8_t *>(at.devicePointer) + (p - static_cast<uint8_t *>(at.hostPointer));
}

thread_local int g_last_pinned = 0;  // rsmi_last_decode_pinned_path

int check_decode_pinned(int k, int n, uint8_t *hs, int64_t hgs, int64_t ss, int len, int64_t ngroups,
                        const uint8_t *present, int64_t chunk) {
    int rc = check_uniform(k, n, nullptr, 16, ss, len, 0);
    if (rc) return rc;
    if (ngroups < 0 || chunk < 1 || (ngroups && (!hs || !present)) || hgs < n * ss)
        return fail(RSMI_ERR_INVALID, "invalid decode_pinned arguments");
    return RSMI_OK;
}

int decode_pinned_on(Device &Dref, Pipeline &pdec, Pipeline &pzc, int k, int n, uint8_t *hs, int64_t hgs,
                     int64_t ss, int len, int64_t ngroups, const uint8_t *present, int32_t *status,
                     int64_t chunk) {
    int rc;
    Device *D = &Dref;
    // Zero-copy: shards in pinned host memory are read by the fused decode
    // kernel itself over PCIe -- only the k survivors it selects (lib/rs.cpp:
    // 24-39) -- and it writes only the rebuilt rows back; nothing is staged.
    uint8_t *hs_dev = nullptr;
    if (g_opt_fused.load() && n > k && decode_fused_ok(k, n, hgs, ss, len) && hgs % 16 == 0 &&
        (uintptr_t)hs % 16 == 0)
        hs_dev = mapped_host_range(hs, (size_t)((ngroups - 1) * hgs + (int64_t)n * ss));
    g_last_pinned = hs_dev ? RSMI_PINNED_ZERO_COPY : RSMI_PINNED_STAGED;
    if (hs_dev) return decode_zero_copy(*D, pzc, k, n, hs_dev, hgs, ss, len, ngroups, present, status);
    Pipeline &P = pdec;
    std::lock_guard<std::mutex> lk(P.mu);  // one call at a time per pipeline
    int32_t **dstat = P.dstat;
    uint8_t **dpres = P.dpres;
    int64_t &cap = P.cap;
    uint8_t *&hpin = P.hpin;
    size_t &hpin_bytes = P.hpin_bytes;
    const size_t pin_need = (size_t)(n * ngroups + 64) + sizeof(int32_t) * (size_t)ngroups;
    if (hpin_bytes < pin_need) {
        if (hpin) (void)hipHostFree(hpin);
        hpin = nullptr;
        hpin_bytes = 0;
        RSMI_HIP(hipHostMalloc(&hpin, pin_need, hipHostMallocDefault), "hipHostMalloc(pin)");
        hpin_bytes = pin_need;
    }
    uint8_t *pres_pin = hpin;
    int32_t *stat_pin = reinterpret_cast<int32_t *>(hpin + ((n * ngroups + 63) & ~int64_t(63)));
    std::memcpy(pres_pin, present, (size_t)(n * ngroups));
    const int64_t dgs = (int64_t)n * ss;
    const size_t need = (size_t)(dgs * chunk);
    if (P.bytes < need || cap < chunk) {
        for (int i = 0; i < Pipeline::kDepth; ++i) {
            if (P.dev[i]) (void)hipFree(P.dev[i]);
            if (dstat[i]) (void)hipFree(dstat[i]);
            if (dpres[i]) (void)hipFree(dpres[i]);
            P.dev[i] = nullptr;
            dstat[i] = nullptr;
            dpres[i] = nullptr;
        }
        P.bytes = 0;
        cap = 0;
        for (int i = 0; i < Pipeline::kDepth; ++i) {
            RSMI_HIP(hipMalloc(&P.dev[i], need), "hipMalloc(pipeline)");
            RSMI_HIP(hipMalloc(&dstat[i], sizeof(int32_t) * chunk), "hipMalloc(status)");
            RSMI_HIP(hipMalloc(&dpres[i], (size_t)(n * chunk)), "hipMalloc(present)");
        }
        P.bytes = need;
        cap = chunk;
    }
    for (int i = 0; i < Pipeline::kDepth; ++i)
        if (!P.st[i]) RSMI_HIP(hipStreamCreateWithFlags(&P.st[i], hipStreamNonBlocking),
                               "hipStreamCreate(pipeline)");
    for (int i = 0; i < Pipeline::kDepth; ++i) {
        rc = reserve(k, n, chunk, P.st[i]);
        if (rc) return rc;
    }
    int64_t c = 0;
    for (int64_t g0 = 0; g0 < ngroups; g0 += chunk, ++c) {
        const int64_t cnt = std::min(chunk, ngroups - g0);
        const int b = (int)(c % Pipeline::kDepth);
        hipStream_t s = P.st[b];
        RSMI_HIP(hipMemcpy2DAsync(P.dev[b], dgs, hs + g0 * hgs, hgs, (size_t)dgs, cnt,
                                  hipMemcpyHostToDevice, s), "H2D shards");
        RSMI_HIP(hipMemcpyAsync(dpres[b], pres_pin + g0 * n, (size_t)(n * cnt),
                                hipMemcpyHostToDevice, s), "H2D present");
        rc = decode_dev(k, n, P.dev[b], dgs, ss, len, cnt, dpres[b], dstat[b], s);
        if (rc) return rc;
        RSMI_HIP(hipMemcpy2DAsync(hs + g0 * hgs, hgs, P.dev[b], dgs, (size_t)k * ss, cnt,
                                  hipMemcpyDeviceToHost, s), "D2H data rows");
        RSMI_HIP(hipMemcpyAsync(stat_pin + g0, dstat[b], sizeof(int32_t) * cnt,
                                hipMemcpyDeviceToHost, s), "D2H status");
    }
    for (int i = 0; i < Pipeline::kDepth; ++i)
        RSMI_HIP(hipStreamSynchronize(P.st[i]), "hipStreamSynchronize(pipeline)");
    if (status) std::memcpy(status, stat_pin, sizeof(int32_t) * (size_t)ngroups);
    return RSMI_OK;
}

// ---- several devices behind the host-memory entry points ------
//
// FEC groups are independent, so a host batch splits into contiguous group
// ranges, one per listed device, with no exchange between them: each range
// runs the single-device pipeline above on its own host thread, HIP streams
// and (for the staged paths) device buffers, and its results land in its own
// part of the caller's host arrays.  Every device has its own PCIe link, so
// the end-to-end rate of the pinned paths -- PCIe-bound on one device -- adds
// up across devices.  A device may be listed more than once (two workers,
// two pipelines on one device: the 1-GPU test of the partition).
struct Worker {
    int dev = -1;
    Pipeline penc, pdec, pzc, prag;  // this worker's own pipelines
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::function<void()> task;
    bool quit = false, busy = false;
};

struct MultiDev {
    std::mutex call_mu;  // one multi-device call at a time (the workers have one task slot)
    std::mutex cfg_mu;
    std::vector<std::unique_ptr<Worker>> workers;
};

MultiDev &multi() {
    static MultiDev *m = new MultiDev();  // never destroyed: workers may outlive static teardown
    return *m;
}

void free_pipeline(Pipeline &P) {
    for (int i = 0; i < Pipeline::kDepth; ++i) {
        if (P.st[i]) (void)hipStreamDestroy(P.st[i]);
        if (P.dev[i]) (void)hipFree(P.dev[i]);
        if (P.dstat[i]) (void)hipFree(P.dstat[i]);
        if (P.dpres[i]) (void)hipFree(P.dpres[i]);
        P.st[i] = nullptr;
        P.dev[i] = nullptr;
        P.dstat[i] = nullptr;
        P.dpres[i] = nullptr;
    }
    if (P.hpin) (void)hipHostFree(P.hpin);
    P.hpin = nullptr;
    P.bytes = P.hpin_bytes = 0;
    P.cap = 0;
}

void worker_loop(Worker *W) {
    (void)hipSetDevice(W->dev);  // the thread's current device for everything it runs
    for (;;) {
        std::function<void()> t;
        {
            std::unique_lock<std::mutex> lk(W->mu);
            W->cv.wait(lk, [&] { return W->quit || (W->busy && W->task); });
            if (W->quit && !W->task) break;
            t = std::move(W->task);
            W->task = nullptr;
        }
        t();
        {
            std::lock_guard<std::mutex> lk(W->mu);
            W->busy = false;
        }
        W->cv.notify_all();
    }
    free_pipeline(W->penc);
    free_pipeline(W->pdec);
    free_pipeline(W->pzc);
    free_pipeline(W->prag);
}

void stop_workers(std::vector<std::unique_ptr<Worker>> &ws) {
    for (auto &W : ws) {
        {
            std::lock_guard<std::mutex> lk(W->mu);
            W->quit = true;
        }
        W->cv.notify_all();
    }
    for (auto &W : ws)
        if (W->th.joinable()) W->th.join();
    ws.clear();
}

// Contiguous ranges [bounds[i], bounds[i+1]) of n items over `parts` parts:
// near-equal counts (cost null), or near-equal summed cost -- the cut before
// part i is the first item whose prefix sum reaches i/parts of the total
// (shard.balanced_ranges; C3's ragged groups weigh (k+m)*len).
void split_ranges(int64_t n, const int64_t *cost, int parts, int64_t *bounds) {
    if (parts < 1) return;  // (callers reject parts < 1)
    bounds[0] = 0;
    bounds[parts] = n;
    if (!cost) {
        for (int i = 1; i < parts; ++i) bounds[i] = (int64_t)((__int128)n * i / parts);
        return;
    }
    std::vector<long double> pre((size_t)n + 1, 0.0L);
    for (int64_t g = 0; g < n; ++g) pre[(size_t)g + 1] = pre[(size_t)g] + (long double)cost[g];
    const long double total = pre[(size_t)n];
    for (int i = 1; i < parts; ++i) {
        const long double target = total * i / parts;
        bounds[i] = (int64_t)(std::lower_bound(pre.begin(), pre.end(), target) - pre.begin());
        if (bounds[i] > n) bounds[i] = n;
        if (bounds[i] < bounds[i - 1]) bounds[i] = bounds[i - 1];
    }
}

// run_split's answer when no device list is set: the caller runs the call on
// its own current device.  Decided under call_mu, so a concurrent
// rsmi_use_devices(.., 0) cannot turn a split call into a silent no-op.
constexpr int kNoWorkers = 0x52534d31;  // never a status: fn returns RSMI_OK or a negative RSMI_ERR_*

// Runs fn(worker, g0, count) for every listed device's range, in parallel, and
// returns the first failure (its message moved to the calling thread), or
// kNoWorkers.  cost (may be null): per-group weights the ranges balance.
int run_split(int64_t ngroups, const std::function<int(Worker &, int64_t, int64_t)> &fn,
              const int64_t *cost = nullptr) {
    MultiDev &M = multi();
    std::lock_guard<std::mutex> call(M.call_mu);
    std::vector<Worker *> ws;
    {
        std::lock_guard<std::mutex> lk(M.cfg_mu);
        for (auto &W : M.workers) ws.push_back(W.get());
    }
    const int parts = (int)ws.size();
    if (parts < 1) return kNoWorkers;
    std::vector<int64_t> b((size_t)parts + 1);
    split_ranges(ngroups, cost, parts, b.data());
    std::vector<int> rcs((size_t)parts, RSMI_OK);
    std::vector<std::string> errs((size_t)parts);
    for (int i = 0; i < parts; ++i) {
        Worker *W = ws[(size_t)i];
        const int64_t g0 = b[(size_t)i], cnt = b[(size_t)i + 1] - b[(size_t)i];
        std::lock_guard<std::mutex> lk(W->mu);
        W->task = [&, W, i, g0, cnt] {
            rcs[(size_t)i] = cnt > 0 ? fn(*W, g0, cnt) : RSMI_OK;
            if (rcs[(size_t)i]) errs[(size_t)i] = g_err;  // the worker thread's message
        };
        W->busy = true;
        W->cv.notify_all();
    }
    for (Worker *W : ws) {
        std::unique_lock<std::mutex> lk(W->mu);
        W->cv.wait(lk, [&] { return !W->busy; });
    }
    for (int i = 0; i < parts; ++i)
        if (rcs[(size_t)i]) {
            g_err = "device " + std::to_string(ws[(size_t)i]->dev) + ": " + errs[(size_t)i];
            return rcs[(size_t)i];
        }
    return RSMI_OK;
}

int set_devices(const int32_t *devs, int32_t n) {
    if (n < 0 || n > 64 || (n > 0 && !devs)) return fail(RSMI_ERR_INVALID, "rsmi_use_devices: bad arguments");
    if (n > 0) {
        int count = 0;
        hipError_t e = hipGetDeviceCount(&count);
        if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount (no usable GPU?)");
        for (int i = 0; i < n; ++i)
            if (devs[i] < 0 || devs[i] >= count)
                return fail(RSMI_ERR_INVALID, "rsmi_use_devices: device " + std::to_string(devs[i]) +
                                                  " out of range (" + std::to_string(count) + " devices)");
    }
    MultiDev &M = multi();
    std::lock_guard<std::mutex> call(M.call_mu);  // no call in flight while the pool changes
    std::vector<std::unique_ptr<Worker>> old;
    {
        std::lock_guard<std::mutex> lk(M.cfg_mu);
        old.swap(M.workers);
    }
    stop_workers(old);
    std::vector<std::unique_ptr<Worker>> fresh;
    for (int i = 0; i < n; ++i) {
        fresh.emplace_back(new Worker());
        fresh.back()->dev = devs[i];
        fresh.back()->th = std::thread(worker_loop, fresh.back().get());
    }
    std::lock_guard<std::mutex> lk(M.cfg_mu);
    M.workers.swap(fresh);
    return RSMI_OK;
}

int get_devices(int32_t *out, int32_t cap) {
    MultiDev &M = multi();
    std::lock_guard<std::mutex> lk(M.cfg_mu);
    const int n = (int)M.workers.size();
    for (int i = 0; i < n && i < cap && out; ++i) out[i] = M.workers[(size_t)i]->dev;
    return n;
}

int encode_pinned(int k, int n, const uint8_t *hd, int64_t dgs, uint8_t *hp, int64_t pgs,
                  int64_t ss, int len, int64_t ngroups, int64_t chunk) {
    int rc = check_encode_pinned(k, n, hd, dgs, hp, pgs, ss, len, ngroups, chunk);
    if (rc) return rc;
    if (ngroups == 0 || n == k || len == 0) return RSMI_OK;
    rc = run_split(ngroups, [&](Worker &W, int64_t g0, int64_t cnt) {
        int r;
        Device *D = current(&r);
        if (!D) return r;
        return encode_pinned_on(*D, W.penc, k, n, hd + g0 * dgs, dgs, hp + g0 * pgs, pgs, ss, len, cnt,
                                chunk);
    });
    if (rc != kNoWorkers) return rc;
    Device *D = current(&rc);
    if (!D) return rc;
    return encode_pinned_on(*D, D->penc, k, n, hd, dgs, hp, pgs, ss, len, ngroups, chunk);
}

int decode_pinned(int k, int n, uint8_t *hs, int64_t hgs, int64_t ss, int len, int64_t ngroups,
                  const uint8_t *present, int32_t *status, int64_t chunk) {
    int rc = check_decode_pinned(k, n, hs, hgs, ss, len, ngroups, present, chunk);
    if (rc) return rc;
    if (ngroups == 0) return RSMI_OK;
    {
        std::atomic<int> paths{0};
        rc = run_split(ngroups, [&](Worker &W, int64_t g0, int64_t cnt) {
            int r;
            Device *D = current(&r);
            if (!D) return r;
            r = decode_pinned_on(*D, W.pdec, W.pzc, k, n, hs + g0 * hgs, hgs, ss, len, cnt, present + g0 * n,
                                 status ? status + g0 : nullptr, chunk);
            paths.fetch_or(g_last_pinned);  // (the worker thread's own record)
            return r;
        });
        if (rc != kNoWorkers) {
            g_last_pinned = paths.load();  // both bits when the ranges took different paths
            return rc;
        }
    }
    Device *D = current(&rc);
    if (!D) return rc;
    return decode_pinned_on(*D, D->pdec, D->pzc, k, n, hs, hgs, ss, len, ngroups, present, status, chunk);
}

// ---- ragged host batches (mode-0 mixes in pinned host memory) -------------------
// rsmi_encode_ragged_pinned / rsmi_decode_ragged_pinned: a range of groups
// [g0, g0 + cnt) in chunks of at most `chunk` groups, each chunk's byte span
// H2D -> the ragged kernel on rebased descriptors -> span D2H, on the
// pipeline's three streams.  The groups are in ascending, non-overlapping
// offset order (check_ragged_host), so a chunk is one contiguous span.
int ragged_pinned_on(Pipeline &P, bool decode, const rsmi_group *groups, int64_t g0, int64_t cnt,
                     uint8_t *hb, const uint32_t *pbits, int32_t *status, int64_t chunk, int kmax) {
    std::lock_guard<std::mutex> lk(P.mu);
    // the range's codes resident on this thread's device (get_code's role)
    {
        std::vector<int> seen;
        for (int64_t g = g0; g < g0 + cnt; ++g) {
            const int key = groups[g].k * 257 + groups[g].n;
            if (std::find(seen.begin(), seen.end(), key) != seen.end()) continue;
            seen.push_back(key);
            const int rc = prepare_code(groups[g].k, groups[g].n);
            if (rc) return rc;
        }
    }
    auto span = [&](int64_t a, int64_t b) {  // bytes of groups [a, b)
        const rsmi_group &l = groups[b - 1];
        return (size_t)(l.offset + (uint64_t)l.n * l.shard_stride - groups[a].offset);
    };
    size_t need = 16;
    for (int64_t c0 = g0; c0 < g0 + cnt; c0 += chunk) need = std::max(need, span(c0, std::min(g0 + cnt, c0 + chunk)));
    const size_t meta = (size_t)chunk * (sizeof(rsmi_group) + 32 + 4) + 64;  // descriptors | bits | status
    if (P.bytes < need || P.cap < chunk) {
        for (int i = 0; i < Pipeline::kDepth; ++i) {
            if (P.dev[i]) (void)hipFree(P.dev[i]);
            if (P.dpres[i]) (void)hipFree(P.dpres[i]);
            P.dev[i] = P.dpres[i] = nullptr;
        }
        if (P.hpin) (void)hipHostFree(P.hpin);
        P.hpin = nullptr;
        P.bytes = P.hpin_bytes = 0;
        P.cap = 0;
        for (int i = 0; i < Pipeline::kDepth; ++i) {
            RSMI_HIP(hipMalloc(&P.dev[i], need), "hipMalloc(ragged pipeline)");
            RSMI_HIP(hipMalloc(&P.dpres[i], meta), "hipMalloc(ragged pipeline meta)");
        }
        RSMI_HIP(hipHostMalloc(&P.hpin, meta * Pipeline::kDepth, hipHostMallocDefault), "hipHostMalloc(ragged)");
        P.bytes = need;
        P.hpin_bytes = meta * Pipeline::kDepth;
        P.cap = chunk;
    }
    for (int i = 0; i < Pipeline::kDepth; ++i)
        if (!P.st[i]) RSMI_HIP(hipStreamCreateWithFlags(&P.st[i], hipStreamNonBlocking), "hipStreamCreate(pipeline)");
    const size_t o_bits = ((size_t)chunk * sizeof(rsmi_group) + 15) & ~(size_t)15;
    const size_t o_stat = o_bits + (size_t)chunk * 32;
    int64_t pend_g[Pipeline::kDepth], pend_n[Pipeline::kDepth];
    for (int i = 0; i < Pipeline::kDepth; ++i) pend_n[i] = 0;
    // a stage's status comes back through its pinned meta area: copied out
    // once the stage's stream has drained, before the stage is reused
    auto drain = [&](int b) -> int {
        RSMI_HIP(hipStreamSynchronize(P.st[b]), "hipStreamSynchronize(ragged pipeline)");
        if (decode && pend_n[b] > 0 && status)
            std::memcpy(status + pend_g[b], P.hpin + (size_t)b * meta + o_stat, (size_t)pend_n[b] * 4);
        pend_n[b] = 0;
        return RSMI_OK;
    };
    int64_t c = 0;
    for (int64_t c0 = g0; c0 < g0 + cnt; c0 += chunk, ++c) {
        const int64_t c1 = std::min(g0 + cnt, c0 + chunk), nc = c1 - c0;
        const int b = (int)(c % Pipeline::kDepth);
        int rc = drain(b);
        if (rc) return rc;
        hipStream_t s = P.st[b];
        uint8_t *hm = P.hpin + (size_t)b * meta;
        rsmi_group *rd = reinterpret_cast<rsmi_group *>(hm);
        const uint64_t base_off = groups[c0].offset;
        int km = 1;
        for (int64_t g = c0; g < c1; ++g) {
            rd[g - c0] = groups[g];
            rd[g - c0].offset -= base_off;
            km = std::max<int>(km, groups[g].k);
        }
        const size_t bytes = span(c0, c1);
        if (decode) std::memcpy(hm + o_bits, pbits + (size_t)c0 * 8, (size_t)nc * 32);
        RSMI_HIP(hipMemcpyAsync(P.dpres[b], hm, decode ? o_stat : (size_t)nc * sizeof(rsmi_group),
                                hipMemcpyHostToDevice, s), "H2D ragged meta");
        RSMI_HIP(hipMemcpyAsync(P.dev[b], hb + base_off, bytes, hipMemcpyHostToDevice, s), "H2D ragged span");
        const rsmi_group *dg = reinterpret_cast<const rsmi_group *>(P.dpres[b]);
        if (decode) {
            int32_t *dst = reinterpret_cast<int32_t *>(P.dpres[b] + o_stat);
            rc = decode_ragged_dev(dg, nc, P.dev[b], reinterpret_cast<const uint32_t *>(P.dpres[b] + o_bits), dst,
                                   std::min(km, kmax), s);
            if (rc) return rc;
            RSMI_HIP(hipMemcpyAsync(hm + o_stat, dst, (size_t)nc * 4, hipMemcpyDeviceToHost, s), "D2H status");
            pend_g[b] = c0;
            pend_n[b] = nc;
        } else {
            rc = encode_ragged_dev(dg, nc, P.dev[b], s);
            if (rc) return rc;
        }
        RSMI_HIP(hipMemcpyAsync(hb + base_off, P.dev[b], bytes, hipMemcpyDeviceToHost, s), "D2H ragged span");
    }
    for (int i = 0; i < Pipeline::kDepth; ++i) {
        const int rc = drain(i);
        if (rc) return rc;
    }
    return RSMI_OK;
}

int check_ragged_host(const rsmi_group *groups, int64_t ngroups, const uint8_t *hb, int64_t chunk) {
    if (ngroups < 0 || chunk < 1) return fail(RSMI_ERR_INVALID, "negative ngroups or chunk_groups < 1");
    if (ngroups > 0 && (!groups || !hb)) return fail(RSMI_ERR_INVALID, "null groups/host_base");
    uint64_t end = 0;
    for (int64_t g = 0; g < ngroups; ++g) {
        const rsmi_group &d = groups[g];
        if (d.k < 1 || d.n < d.k || d.n > 256 || d.shard_stride % 16 || d.shard_stride < d.len ||
            d.offset % 16 || d.reserved)
            return fail(RSMI_ERR_INVALID, "invalid descriptor at group " + std::to_string(g));
        if (d.offset < end)
            return fail(RSMI_ERR_INVALID, "groups must be in ascending, non-overlapping offset order (group " +
                                              std::to_string(g) + ")");
        end = d.offset + (uint64_t)d.n * d.shard_stride;
    }
    if (((uintptr_t)hb) % 16) return fail(RSMI_ERR_INVALID, "host_base must be 16-aligned");
    return RSMI_OK;
}

// Split over the device list by each group's bytes n * len (the PCIe and HBM
// work both scale with them: SURVEY 8(e)'s balanced ranges for C3).
int ragged_pinned(bool decode, const rsmi_group *groups, int64_t ngroups, uint8_t *hb, const uint32_t *pbits,
                  int32_t *status, int64_t chunk) {
    int rc = check_ragged_host(groups, ngroups, hb, chunk);
    if (rc) return rc;
    if (decode && ngroups > 0 && !pbits) return fail(RSMI_ERR_INVALID, "null present_bits");
    if (ngroups == 0) return RSMI_OK;
    int kmax = 1;
    std::vector<int64_t> cost((size_t)ngroups);
    for (int64_t g = 0; g < ngroups; ++g) {
        cost[(size_t)g] = (int64_t)groups[g].n * groups[g].len;
        kmax = std::max<int>(kmax, groups[g].k);
    }
    rc = run_split(
        ngroups,
        [&](Worker &W, int64_t g0, int64_t cnt) {
            return ragged_pinned_on(W.prag, decode, groups, g0, cnt, hb, pbits, status, chunk, kmax);
        },
        cost.data());
    if (rc != kNoWorkers) return rc;
    Device *D = current(&rc);
    if (!D) return rc;
    return ragged_pinned_on(D->prag, decode, groups, 0, ngroups, hb, pbits, status, chunk, kmax);
}

const char *last_error() { return g_err.c_str(); }
std::atomic<int> &opt_bitslice() { return g_opt_bitslice; }

void set_error(const std::string &m) { g_err = m; }

}  // namespace rsmi

// ===== extern "C" surface (include/rsmi.h) ===================================
extern "C" {

int rsmi_version(void) { return 0x000100; }

int rsmi_option(int option, int value) {
    if (option == RSMI_OPT_BITSLICE) return rsmi::g_opt_bitslice.exchange(value ? 1 : 0);
    if (option == RSMI_OPT_FUSED_DECODE) return rsmi::g_opt_fused.exchange(value ? 1 : 0);
    if (option == RSMI_OPT_ONE_GROUP) return rsmi::g_opt_oneshot.exchange(value ? 1 : 0);
    if (option == RSMI_OPT_CLS_REC_CAP) return rsmi::g_opt_cls_cap.exchange(value > 0 ? value : 0);
    if (option == RSMI_OPT_ONE_SERVER) {
        const int prev = rsmi::server_idle_us();
        rsmi::g_opt_server.store(value > 0 ? value : 0);
        if (value <= 0) {  // stop every running server (the next calls launch per call)
            const int rc = rsmi::stop_all_servers();
            if (rc) return rc;
        }
        return prev;
    }
    if (option == RSMI_OPT_PARITY_COOK) {
        const int prev = rsmi::parity_cook_enabled() ? 1 : 0;
        rsmi::g_opt_parity_cook.store(value ? 1 : 0);
        return prev;
    }
    if (option == RSMI_OPT_ONE_SERVER_LIFE) {
        const int prev = rsmi::server_life_ms();
        if (value < 1) {
            rsmi::set_error("RSMI_OPT_ONE_SERVER_LIFE: lifetime must be >= 1 ms");
            return RSMI_ERR_INVALID;
        }
        rsmi::g_opt_server_life.store(value);
        return prev;
    }
    rsmi::set_error("unknown option");
    return RSMI_ERR_INVALID;
}

int rsmi_quiesce(void) { return rsmi::stop_all_servers(); }

int rsmi_encode_ragged_pinned(const rsmi_group *groups, int64_t ngroups, uint8_t *host_base,
                              int64_t chunk_groups) {
    return rsmi::ragged_pinned(false, groups, ngroups, host_base, nullptr, nullptr, chunk_groups);
}

int rsmi_decode_ragged_pinned(const rsmi_group *groups, int64_t ngroups, uint8_t *host_base,
                              const uint32_t *present_bits, int32_t *status, int64_t chunk_groups) {
    return rsmi::ragged_pinned(true, groups, ngroups, host_base, present_bits, status, chunk_groups);
}

int rsmi_init(void) {
    int rc;
    return rsmi::current(&rc) ? RSMI_OK : rc;
}

const char *rsmi_last_error(void) { return rsmi::last_error(); }

int rsmi_get_matrix(int k, int n, uint8_t *out) {
    std::vector<uint8_t> m;
    if (!out || !rsmi::build_enc_matrix(k, n, m)) {
        rsmi::set_error("invalid (k,n) or null out");
        return RSMI_ERR_INVALID;
    }
    std::memcpy(out, m.data(), m.size());
    return RSMI_OK;
}

int rsmi_decode_matrix(int k, int n, const uint8_t *present, uint8_t *sel, uint8_t *miss,
                       uint8_t *coef) {
    if (k < 1 || n < k || k > 256 || n > 256 || !present || !sel || !miss || !coef) {
        rsmi::set_error("invalid decode_matrix arguments");
        return RSMI_ERR_INVALID;
    }
    std::vector<uint8_t> m;
    if (!rsmi::build_enc_matrix(k, n, m)) {
        rsmi::set_error("matrix build failed");
        return RSMI_ERR_INVALID;
    }
    const int e = rsmi::decode_coeffs(k, n, m.data(), present, sel, miss, coef);
    if (e == -2) {
        rsmi::set_error("singular decode matrix");
        return RSMI_ERR_INVALID;
    }
    return e;
}

int rsmi_prepare_code(int k, int n) { return rsmi::prepare_code(k, n); }

int rsmi_last_encoder(void) { return rsmi::g_last_enc; }

int rsmi_last_decode_pinned_path(void) { return rsmi::g_last_pinned; }


int rsmi_use_devices(const int32_t *devices, int32_t n) { return rsmi::set_devices(devices, n); }

int rsmi_get_devices(int32_t *out, int32_t cap) { return rsmi::get_devices(out, cap); }

int rsmi_split_ranges(int64_t n, const int64_t *cost, int32_t parts, int64_t *bounds) {
    if (n < 0 || parts < 1 || !bounds) return rsmi::fail(RSMI_ERR_INVALID, "rsmi_split_ranges: bad arguments");
    if (cost)
        for (int64_t g = 0; g < n; ++g)
            if (cost[g] < 0) return rsmi::fail(RSMI_ERR_INVALID, "rsmi_split_ranges: negative cost");
    rsmi::split_ranges(n, cost, parts, bounds);
    return RSMI_OK;
}

int rsmi_reserve(int k, int n, int64_t ngroups, void *stream) {
    return rsmi::reserve(k, n, ngroups, (hipStream_t)stream);
}

int rsmi_encode_dev(int k, int n, uint8_t *base, int64_t gs, int64_t ss, int len,
                    int64_t ngroups, void *stream) {
    return rsmi::encode_dev(k, n, base, gs, ss, len, ngroups, (hipStream_t)stream);
}

int rsmi_decode_dev(int k, int n, uint8_t *base, int64_t gs, int64_t ss, int len,
                    int64_t ngroups, const uint8_t *present, int32_t *status, void *stream) {
    return rsmi::decode_dev(k, n, base, gs, ss, len, ngroups, present, status,
                            (hipStream_t)stream);
}

int rsmi_decode_dev_ref(int k, int n, uint8_t *base, int64_t gs, int64_t ss, int len,
                        int64_t ngroups, const uint8_t *present, int32_t *status,
                        uint8_t *slot_map, void *stream) {
    return rsmi::decode_dev(k, n, base, gs, ss, len, ngroups, present, status,
                            (hipStream_t)stream, true, slot_map);
}

int rsmi_ref_slot_map(int k, int n, const uint8_t *present, uint8_t *slot_map) {
    if (k < 1 || n < k || n > 256 || !present || !slot_map)
        return rsmi::fail(RSMI_ERR_INVALID, "invalid rsmi_ref_slot_map arguments");
    uint8_t sel[256];
    int cnt = 0, e = 0;
    for (int j = 0; j < n && cnt < k; ++j)
        if (present[j]) sel[cnt++] = (uint8_t)j;
    if (cnt < k) {
        for (int i = 0; i < k; ++i) slot_map[i] = present[i] ? (uint8_t)i : (uint8_t)0xFF;
        return -1;
    }
    for (int i = 0; i < k; ++i) e += !present[i];
    for (int i = 0; i < k; ++i)
        slot_map[i] = present[i] ? (uint8_t)i : (uint8_t)rsmi::ref_slot_of(k, e, sel, i);
    return e;
}

int rsmi_encode_ragged(const rsmi_group *groups, int64_t ngroups, uint8_t *base, void *stream) {
    if (ngroups == 0) return RSMI_OK;
    rsmi_ragged_plan *plan = nullptr;
    int rc = rsmi_ragged_plan_create(groups, ngroups, &plan);
    if (rc) return rc;
    rc = rsmi_encode_ragged_plan(plan, base, stream);
    const hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    rsmi_ragged_plan_destroy(plan);
    if (rc) return rc;
    if (e != hipSuccess) {
        rsmi::set_error(std::string("ragged encode: ") + hipGetErrorString(e));
        return RSMI_ERR_HIP;
    }
    return RSMI_OK;
}

int rsmi_decode_ragged_dev_ref(const rsmi_group *groups, int64_t ngroups, uint8_t *base,
                               const uint32_t *present_bits, int32_t *status, int kmax,
                               uint8_t *slot_map, int32_t map_stride, void *stream) {
    if (slot_map && map_stride < 1) return rsmi::fail(RSMI_ERR_INVALID, "map_stride < 1");
    return rsmi::decode_ragged_dev(groups, ngroups, base, present_bits, status, kmax, (hipStream_t)stream,
                                   rsmi::RefOut{slot_map, map_stride, 1});
}

int rsmi_decode_ragged_dev(const rsmi_group *groups, int64_t ngroups, uint8_t *base,
                           const uint32_t *present_bits, int32_t *status, int kmax, void *stream) {
    return rsmi::decode_ragged_dev(groups, ngroups, base, present_bits, status, kmax,
                                   (hipStream_t)stream);
}

int rsmi_decode_ragged(const rsmi_group *groups, int64_t ngroups, uint8_t *base,
                       const uint32_t *present_bits, int32_t *status, void *stream) {
    if (ngroups == 0) return RSMI_OK;
    rsmi_ragged_plan *plan = nullptr;
    int rc = rsmi_ragged_plan_create(groups, ngroups, &plan);
    if (rc) return rc;
    rc = rsmi_decode_ragged_plan(plan, base, present_bits, status, stream);
    const hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    rsmi_ragged_plan_destroy(plan);
    if (rc) return rc;
    if (e != hipSuccess) {
        rsmi::set_error(std::string("ragged decode: ") + hipGetErrorString(e));
        return RSMI_ERR_HIP;
    }
    return RSMI_OK;
}

int rsmi_encode_ragged_dev(const rsmi_group *groups, int64_t ngroups, uint8_t *base,
                           void *stream) {
    return rsmi::encode_ragged_dev(groups, ngroups, base, (hipStream_t)stream);
}

int rsmi_encode_host(int k, int n, uint8_t *base, int64_t gs, int64_t ss, int len,
                     int64_t ngroups) {
    return rsmi::host_op(false, k, n, base, gs, ss, len, ngroups, nullptr, nullptr);
}

int rsmi_decode_host(int k, int n, uint8_t *base, int64_t gs, int64_t ss, int len,
                     int64_t ngroups, const uint8_t *present, int32_t *status) {
    if (ngroups > 0 && !present) {
        rsmi::set_error("null present");
        return RSMI_ERR_INVALID;
    }
    return rsmi::host_op(true, k, n, base, gs, ss, len, ngroups, present, status);
}

int rsmi_encode_pinned(int k, int n, const uint8_t *hd, int64_t dgs, uint8_t *hp, int64_t pgs,
                       int64_t ss, int len, int64_t ngroups, int64_t chunk) {
    return rsmi::encode_pinned(k, n, hd, dgs, hp, pgs, ss, len, ngroups, chunk);
}

int rsmi_decode_pinned(int k, int n, uint8_t *hs, int64_t hgs, int64_t ss, int len,
                       int64_t ngroups, const uint8_t *present, int32_t *status, int64_t chunk) {
    return rsmi::decode_pinned(k, n, hs, hgs, ss, len, ngroups, present, status, chunk);
}

int rsmi_fill_data(int k, int len, uint8_t *base, int64_t gs, int64_t ss, int64_t g0,
                   int64_t ngroups, uint64_t seed, void *stream) {
    if (k < 1 || len < 0 || ngroups < 0 || ss % 4 || gs % 4 || ss < len || ((uintptr_t)base) % 4) {
        rsmi::set_error("invalid fill arguments");
        return RSMI_ERR_INVALID;
    }
    if (ngroups == 0 || len == 0) return RSMI_OK;
    hipError_t e = rsmi::launch_fill_data(k, len, base, gs, ss, g0, ngroups, seed,
                                          (hipStream_t)stream);
    if (e != hipSuccess) {
        rsmi::set_error(std::string("fill launch: ") + hipGetErrorString(e));
        return RSMI_ERR_HIP;
    }
    return RSMI_OK;
}

int rsmi_fill_ragged(const rsmi_group *groups, int64_t ngroups, uint8_t *base, int64_t g0,
                     uint64_t seed, void *stream) {
    if (ngroups < 0 || (ngroups > 0 && (!groups || !base))) {
        rsmi::set_error("invalid fill_ragged arguments");
        return RSMI_ERR_INVALID;
    }
    if (ngroups == 0) return RSMI_OK;
    hipError_t e = rsmi::launch_fill_ragged(groups, ngroups, base, g0, seed, (hipStream_t)stream);
    if (e != hipSuccess) {
        rsmi::set_error(std::string("fill_ragged launch: ") + hipGetErrorString(e));
        return RSMI_ERR_HIP;
    }
    return RSMI_OK;
}

int rsmi_copy_peak(uint8_t *dst, const uint8_t *src, int64_t nbytes, int variant, void *stream) {
    if (nbytes < 0 || nbytes % 16 || variant < 0 || variant > 6 || ((uintptr_t)dst | (uintptr_t)src) % 16 ||
        (variant >= 4 && nbytes % (16 * 256 * 24)) ||
        (nbytes > 0 && (!dst || !src)) || nbytes / 16 / (256 * 4) >= 0x7FFFFFFF) {
        rsmi::set_error("invalid copy_peak arguments");
        return RSMI_ERR_INVALID;
    }
    if (nbytes == 0) return RSMI_OK;
    hipError_t e = rsmi::launch_copy_peak(dst, src, nbytes, variant, (hipStream_t)stream);
    if (e != hipSuccess) {
        rsmi::set_error(std::string("copy_peak launch: ") + hipGetErrorString(e));
        return RSMI_ERR_HIP;
    }
    return RSMI_OK;
}

}  // extern "C"
