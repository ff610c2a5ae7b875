// ragged.cpp -- ragged-batch plans (mode-0 mix: every group its own k, n, len).
//
// A plan is built once on the host from the rsmi_group descriptors and kept on
// the device, like an FFT plan: launches over the same batch layout reuse it
// (and are graph-capturable).  When every group's (k,n) has a bit-sliced
// network the plan buckets groups by code and maps every 16-byte column to
// (group, piece): one launch of k_bs_ragged covers the buckets of build-time
// codes, and each run-time compiled code (bitslice_rtc.cpp) gets one launch
// over its own bucket -- if all of those are compiled when the plan is made
// (plan creation does not wait: rsmi_wait_code).  Otherwise the plan falls
// back to the generic one-wave-per-group kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <utility>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "rsmi_internal.hpp"

#ifndef RSMI_DEC_CLASSES
#define RSMI_DEC_CLASSES 1  // plan decodes: one register-cut kernel per tile-width class
#endif
#ifndef RAG_CLS_SLOTS_DIV
#define RAG_CLS_SLOTS_DIV 1  // decode classes: resident wave slots per class / this = its waves.
                             // Round 6 (profiles/r06/c3_clsdiv_ab.txt): 2 -> C3 decode 0.138-0.140 ms,
                             // 4 -> 0.142-0.143, against 0.138-0.139 at 1: the workgroups' prologues
                             // overlap the older ones' streams, fewer and longer-lived ones buy nothing
#endif
#ifndef RAG_LPT
#define RAG_LPT 1  // bit-sliced ragged waves: costliest code first (0: code-list order)
#endif
static constexpr bool kRagLptOrder = RAG_LPT != 0;

namespace rsmi {
int prepare_code(int k, int n);
const uint8_t *device_code_rows(int k, int n);
void set_error(const std::string &m);
uint64_t *device_code_dir(int *rc);
int decode_ragged_dev(const rsmi_group *dg, int64_t ngroups, uint8_t *base,
                      const uint32_t *present_bits, int32_t *status, int kmax, hipStream_t s, RefOut ro);
int decode_ragged_cls_dev(const rsmi_group *dg, int64_t ngroups, const ClsLaunch &C, uint8_t *base,
                          const uint32_t *present_bits, int32_t *status, int kmax, hipStream_t s);
const uint32_t *device_ptab(int *rc);
extern std::atomic<int> g_opt_cls_cap;  // RSMI_OPT_CLS_REC_CAP (api.cpp)
}  // namespace rsmi

struct rsmi_ragged_plan {
    int device = -1;
    int64_t ngroups = 0;
    int kmax = 1;             // largest k in the batch (sizes the decode kernel's LDS)
    bool bitslice = false;
    uint32_t bytes = 0;       // extent of the batch from base (bitslice path)
    uint32_t nwaves = 0;
    uint32_t nwaves_builtin = 0;  // waves [0, nwaves_builtin) belong to build-time codes
    struct RtcBucket {
        int k, n;
        uint32_t first, count;  // slice of the wave list
    };
    std::vector<RtcBucket> rtc;
    uint8_t *mem = nullptr;   // one device allocation: groups | colmap | waves
    rsmi_group *d_groups = nullptr;
    uint32_t *d_colmap = nullptr;
    uint32_t *d_waves = nullptr;
    // decode: group records by tile-width class (rag_width), dealt to waves
    // (d_cls, wave-major; class c's wave offsets at d_wst + wst_first[c])
    rsmi::ClsLaunch cls{};
    uint32_t *d_cls = nullptr;
    std::atomic<uint32_t> epoch{0};  // decode calls so far (the deferral mark, ClsLaunch)
};

namespace {

int fail(int code, const std::string &m) {
    rsmi::set_error(m);
    return code;
}

}  // namespace

extern "C" int rsmi_ragged_plan_create(const rsmi_group *g, int64_t ngroups,
                                       rsmi_ragged_plan **out) {
    if (!out || ngroups < 0 || (ngroups > 0 && !g))
        return fail(RSMI_ERR_INVALID, "invalid ragged plan arguments");
    *out = nullptr;
    uint64_t extent = 0;
    int kmax = 1;
    bool need_big = false;
    bool bs = ngroups < (int64_t(1) << 20);
    std::vector<int> code_of((size_t)ngroups, -1);
    std::vector<uint8_t> seen(257 * 257, 0);
    std::map<int, int> rtc_index;  // k*257+n -> position in rtc_codes
    std::vector<std::pair<int, int>> rtc_codes;
    for (int64_t i = 0; i < ngroups; ++i) {
        const rsmi_group &d = g[i];
        if (d.k < 1 || d.n < d.k || d.n > 256 || d.reserved != 0 || d.offset % 16 ||
            d.shard_stride % 16 || d.shard_stride < d.len)
            return fail(RSMI_ERR_INVALID, "bad rsmi_group at index " + std::to_string(i));
        kmax = std::max(kmax, (int)d.k);
        const int key = d.k * 257 + d.n;
        if (!seen[key]) {
            seen[key] = 1;
            int rc = rsmi::prepare_code(d.k, d.n);
            if (rc) return rc;
        }
        if (d.n == d.k || d.len == 0) continue;  // nothing to compute
        // the class decode kernels defer these to the workgroup kernel
        if (d.k > 32 || (uint64_t)d.n * d.shard_stride >= 0x80000000ull) need_big = true;
        const uint64_t end = d.offset + (uint64_t)(d.n - 1) * d.shard_stride +
                             ((d.len + 15u) & ~15u);
        extent = std::max(extent, end);
        int ci = rsmi::bitslice_code_index(d.k, d.n);
        if (ci < 0) {
            if (rsmi::bitslice_rtc_eligible(d.k, d.n)) {
                auto it = rtc_index.find(key);
                if (it == rtc_index.end()) {
                    it = rtc_index.emplace(key, (int)rtc_codes.size()).first;
                    rtc_codes.push_back({(int)d.k, (int)d.n});
                }
                ci = rsmi::bitslice_builtin_count() + it->second;
            } else {
                bs = false;
            }
        }
        if (d.len > 65536) bs = false;
        code_of[(size_t)i] = ci;
    }
    if (extent >= 0x80000000ull) bs = false;
    // codes without a build-time network: prepare_code above queued their
    // compiles; the plan takes the bit-sliced path only if every one is ready
    // now (rsmi_wait_code first to be sure) and never waits for them itself
    for (auto &c : rtc_codes)
        if (bs && !rsmi::bitslice_rtc_function(c.first, c.second, rsmi::kRtcRagged)) bs = false;

    rsmi_ragged_plan *P = new rsmi_ragged_plan();
    if (hipGetDevice(&P->device) != hipSuccess) {
        delete P;
        return fail(RSMI_ERR_HIP, "hipGetDevice (no usable GPU?)");
    }
    P->ngroups = ngroups;
    P->kmax = kmax;
    P->bitslice = bs;
    P->cls.need_big = need_big ? 1 : 0;
    P->bytes = (uint32_t)std::min<uint64_t>(extent, 0x7FFFFFFFull);
    std::vector<uint32_t> colmap, waves;
    if (bs) {
        // bucket -> column count (each bucket padded to whole 128-column waves)
        int nb = 0;
        for (int v : code_of) nb = std::max(nb, v + 1);
        std::vector<uint64_t> cols((size_t)nb, 0), base((size_t)nb, 0), fill((size_t)nb, 0);
        for (int64_t i = 0; i < ngroups; ++i)
            if (code_of[(size_t)i] >= 0) cols[(size_t)code_of[(size_t)i]] += (g[i].len + 15) / 16;
        uint64_t total = 0;
        for (int b = 0; b < nb; ++b) {
            base[(size_t)b] = total;
            total += (cols[(size_t)b] + 127) / 128 * 128;
        }
        if (total >= 0xFFFFFF80ull) {
            delete P;
            return fail(RSMI_ERR_INVALID, "ragged batch too large for one plan");
        }
        colmap.assign((size_t)total + 64, 0xFFFFFFFFu);  // +64: lane c0+64 of the last wave
        for (int64_t i = 0; i < ngroups; ++i) {
            const int b = code_of[(size_t)i];
            if (b < 0) continue;
            const uint32_t pcs = (g[i].len + 15) / 16;
            uint64_t c = base[(size_t)b] + fill[(size_t)b];
            for (uint32_t p = 0; p < pcs; ++p) colmap[(size_t)(c + p)] = ((uint32_t)i << 12) | p;
            fill[(size_t)b] += pcs;
        }
        const int nbuiltin = rsmi::bitslice_builtin_count();
        // wave order of the built-in buckets: costliest code first (most rows,
        // then most data shards) so the grid's last dispatched waves are the
        // cheap ones and no big-code wave starts at the tail
        std::vector<int> order((size_t)nb);
        for (int b = 0; b < nb; ++b) order[(size_t)b] = b;
        if (kRagLptOrder)
            std::stable_sort(order.begin(), order.begin() + std::min(nb, nbuiltin), [](int a, int b) {
                const int ka = rsmi::bitslice_code_k(a), kb = rsmi::bitslice_code_k(b);
                const int na = rsmi::bitslice_code_n(a), nb2 = rsmi::bitslice_code_n(b);
                return na != nb2 ? na > nb2 : ka > kb;
            });
        for (int b : order) {
            if (b == nbuiltin) P->nwaves_builtin = (uint32_t)(waves.size() / 2);
            const uint32_t first = (uint32_t)(waves.size() / 2);
            for (uint64_t w = 0; w < (cols[(size_t)b] + 127) / 128; ++w) {
                waves.push_back((uint32_t)b);
                waves.push_back((uint32_t)(base[(size_t)b] + 128 * w));
            }
            if (b >= nbuiltin && cols[(size_t)b] > 0) {
                const auto &c = rtc_codes[(size_t)(b - nbuiltin)];
                P->rtc.push_back({c.first, c.second, first, (uint32_t)(waves.size() / 2) - first});
            }
        }
        P->nwaves = (uint32_t)(waves.size() / 2);
        if (nb <= nbuiltin) P->nwaves_builtin = P->nwaves;
    }
    // decode classes: the width each group's tiles take (decode.hip).  Each
    // class kernel runs one resident round of workgroups; the class's groups
    // are dealt to the workgroups longest-first onto the least-loaded one, on
    // an estimated cost, and a workgroup's waves take its groups one at a time
    // (decode.hip k_decode_ragged_cls).  A deal straight to waves could not see
    // the erasures, which set a group's elimination and multiply cost: the
    // slowest wave of a round ran 44 % past the median (profiles/r03 c3_trace).
    std::vector<uint32_t> cls, wst;
    int64_t wst_first[4] = {0, 0, 0, 0};
    {
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, P->device) != hipSuccess ||
            ncu < 1)
            ncu = 256;
        std::vector<std::vector<uint32_t>> by((size_t)4);
        for (int64_t i = 0; i < ngroups; ++i)
            by[(size_t)rsmi::rag_width_class(
                   rsmi::rag_width(rsmi::rag_lpad(g[i].len, g[i].shard_stride)))]
                .push_back((uint32_t)i);
        cls.reserve((size_t)ngroups * 8);
        for (int c = 0; c < 4; ++c) {
            auto &v = by[(size_t)c];
            const int W = c == 0 ? 1 : (c == 1 ? 2 : (c == 2 ? 4 : 5));
            const int occ = rsmi::decode_cls_occupancy(c);
            // RAG_CLS_SLOTS_DIV: the classes share one launch (DEC_MIX), so a
            // class sized to fill the device alone makes the launch several
            // rounds of short-lived workgroups, each paying its prologue
            // (tables, records, present words: 3-14 K cycles per wave,
            // profiles/r06/c3_trace.txt) for 1.3-3.4 groups a wave
            const int64_t slots = (int64_t)ncu * 4 * occ / RAG_CLS_SLOTS_DIV;
            // one wave per group at least: blocks of kClsWaves waves
            int64_t nb64 = (std::min<int64_t>((int64_t)v.size(), slots) + rsmi::kClsWaves - 1) /
                           rsmi::kClsWaves;
            // A workgroup stages its records in LDS (64 B each): cap them so
            // the class's occupancy holds (160 KiB of LDS per CU over occ
            // workgroups of kClsWaves waves, never past the 64 KiB a workgroup
            // may take).  Past the cap, more workgroups: the extra ones run
            // in later rounds as earlier ones retire.
            const size_t fixed = rsmi::cls_lds_bytes(kmax, 0);
            const size_t budget = std::min<size_t>(163840 / (size_t)occ, 65536);
            int64_t cap = budget > fixed + 64 * 16 ? (int64_t)((budget - fixed) / 64) : 16;
            if (rsmi::g_opt_cls_cap.load() > 0) cap = rsmi::g_opt_cls_cap.load();
            nb64 = std::max<int64_t>(nb64, ((int64_t)v.size() + cap - 1) / cap);
            if (nb64 > 0x7FFFFFFF) {
                delete P;
                return fail(RSMI_ERR_INVALID, "ragged plan: too many decode workgroups");
            }
            const int nb = (int)nb64;
            P->cls.nw[c] = nb;  // workgroups
            P->cls.maxb[c] = 0;
            wst_first[c] = (int64_t)wst.size();
            if (nb == 0) {
                wst.push_back((uint32_t)(cls.size() / 8));
                continue;
            }
            // cost: a fixed chain (descriptor, flags, code rows, elimination)
            // plus per survivor a load and a W-dword multiply
            auto cost = [&](uint32_t i) { return 24.0 + g[i].k * (2.0 + W); };
            std::stable_sort(v.begin(), v.end(), [&](uint32_t a, uint32_t b) { return cost(a) > cost(b); });
            std::vector<std::vector<uint32_t>> lists((size_t)nb);
            std::vector<std::pair<double, int>> heap;  // (load, block), min-heap
            heap.reserve((size_t)nb);
            for (int b = 0; b < nb; ++b) heap.push_back({0.0, b});
            auto gt = [](const std::pair<double, int> &a, const std::pair<double, int> &b) {
                return a.first > b.first || (a.first == b.first && a.second > b.second);
            };
            for (uint32_t i : v) {  // nb * cap >= |v|: the heap never runs dry
                std::pop_heap(heap.begin(), heap.end(), gt);
                heap.back().first += cost(i);
                auto &lst = lists[(size_t)heap.back().second];
                lst.push_back(i);
                if ((int64_t)lst.size() < cap)
                    std::push_heap(heap.begin(), heap.end(), gt);
                else
                    heap.pop_back();  // full: no more records for this workgroup
            }
            for (int b = 0; b < nb; ++b) {
                wst.push_back((uint32_t)(cls.size() / 8));
                P->cls.maxb[c] = std::max<int>(P->cls.maxb[c], (int)lists[(size_t)b].size());
                for (uint32_t i : lists[(size_t)b]) {  // the group's 8-dword record (decode.hip)
                    const rsmi_group &d = g[i];
                    const uint64_t rows = (uint64_t)(uintptr_t)rsmi::device_code_rows(d.k, d.n);
                    const uint32_t r8[8] = {(uint32_t)d.offset, (uint32_t)(d.offset >> 32), d.shard_stride,
                                            d.len, (uint32_t)d.k | ((uint32_t)d.n << 16), i,
                                            (uint32_t)rows, (uint32_t)(rows >> 32)};
                    cls.insert(cls.end(), r8, r8 + 8);
                }
            }
            wst.push_back((uint32_t)(cls.size() / 8));
        }
    }
    const size_t gbytes = sizeof(rsmi_group) * (size_t)ngroups;
    const size_t cbytes = sizeof(uint32_t) * colmap.size();
    const size_t wbytes = sizeof(uint32_t) * waves.size();
    const size_t dbytes = sizeof(uint32_t) * cls.size();
    const size_t sbytes = sizeof(uint32_t) * wst.size();
    const size_t goff = 0, coff = (gbytes + 255) & ~size_t(255),
                 woff = (coff + cbytes + 255) & ~size_t(255),
                 doff = (woff + wbytes + 255) & ~size_t(255),
                 soff = (doff + dbytes + 255) & ~size_t(255);
    const size_t all = soff + sbytes + 256;  // + the deferral word
    if (hipMalloc(&P->mem, all) != hipSuccess) {
        delete P;
        return fail(RSMI_ERR_NOMEM, "hipMalloc(ragged plan)");
    }
    P->d_groups = reinterpret_cast<rsmi_group *>(P->mem + goff);
    P->d_colmap = reinterpret_cast<uint32_t *>(P->mem + coff);
    P->d_waves = reinterpret_cast<uint32_t *>(P->mem + woff);
    P->d_cls = reinterpret_cast<uint32_t *>(P->mem + doff);
    uint32_t *d_wst = reinterpret_cast<uint32_t *>(P->mem + soff);
    P->cls.rec = P->d_cls;
    P->cls.defer = reinterpret_cast<uint32_t *>(P->mem + ((soff + sbytes + 127) & ~size_t(127)));
    for (int c = 0; c < 4; ++c) P->cls.wst[c] = d_wst + wst_first[c];
    hipError_t e = hipSuccess;
    if (gbytes) e = hipMemcpy(P->d_groups, g, gbytes, hipMemcpyHostToDevice);
    if (e == hipSuccess && cbytes) e = hipMemcpy(P->d_colmap, colmap.data(), cbytes,
                                                 hipMemcpyHostToDevice);
    if (e == hipSuccess && wbytes) e = hipMemcpy(P->d_waves, waves.data(), wbytes,
                                                 hipMemcpyHostToDevice);
    if (e == hipSuccess && dbytes) e = hipMemcpy(P->d_cls, cls.data(), dbytes,
                                                 hipMemcpyHostToDevice);
    if (e == hipSuccess && sbytes) e = hipMemcpy(d_wst, wst.data(), sbytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(P->cls.defer, 0, sizeof(uint32_t));
    if (e != hipSuccess) {
        (void)hipFree(P->mem);
        delete P;
        return fail(RSMI_ERR_HIP, std::string("ragged plan upload: ") + hipGetErrorString(e));
    }
    *out = P;
    return RSMI_OK;
}

extern "C" int rsmi_encode_ragged_plan(const rsmi_ragged_plan *P, uint8_t *base, void *stream) {
    if (!P) return fail(RSMI_ERR_INVALID, "null plan");
    if (P->ngroups == 0) return RSMI_OK;
    if (!base || ((uintptr_t)base) % 16) return fail(RSMI_ERR_INVALID, "base must be 16-aligned");
    hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    if (P->bitslice) {
        e = rsmi::launch_encode_bitslice_ragged(P->d_groups, P->d_colmap, P->d_waves,
                                                P->nwaves_builtin, base, P->bytes, s);
        for (size_t i = 0; e == hipSuccess && i < P->rtc.size(); ++i) {
            const auto &b = P->rtc[i];
            e = rsmi::launch_encode_bitslice_ragged_rtc(b.k, b.n, P->d_groups, P->d_colmap,
                                                        P->d_waves + 2 * (size_t)b.first, b.count,
                                                        base, P->bytes, s);
        }
    } else {
        int rc;
        const uint64_t *dir = rsmi::device_code_dir(&rc);
        if (!dir) return rc;
        const uint32_t *ptab = rsmi::device_ptab(&rc);
        if (!ptab) return rc;
        e = rsmi::launch_encode_ragged(P->d_groups, P->ngroups, base, dir, ptab, s);
    }
    if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("ragged launch: ") + hipGetErrorString(e));
    return RSMI_OK;
}

namespace {
int decode_plan_call(const rsmi_ragged_plan *P, uint8_t *base, const uint32_t *present_bits, int32_t *status,
                     rsmi::RefOut ro, void *stream) {
    if (!P) return fail(RSMI_ERR_INVALID, "null plan");
    if (RSMI_DEC_CLASSES) {
        rsmi::ClsLaunch C = P->cls;
        // a rising mark per call: the big kernel runs only if a call at or
        // after this one deferred (graph replays keep their captured mark and
        // may scan needlessly; never the reverse)
        C.epoch = const_cast<rsmi_ragged_plan *>(P)->epoch.fetch_add(1) + 1;
        C.ref = ro;
        return rsmi::decode_ragged_cls_dev(P->d_groups, P->ngroups, C, base, present_bits, status,
                                           P->kmax, (hipStream_t)stream);
    }
    return rsmi::decode_ragged_dev(P->d_groups, P->ngroups, base, present_bits, status, P->kmax,
                                   (hipStream_t)stream, ro);
}
}  // namespace

extern "C" int rsmi_decode_ragged_plan(const rsmi_ragged_plan *P, uint8_t *base,
                                       const uint32_t *present_bits, int32_t *status,
                                       void *stream) {
    return decode_plan_call(P, base, present_bits, status, rsmi::RefOut{nullptr, 0, 0}, stream);
}

extern "C" int rsmi_decode_ragged_plan_ref(const rsmi_ragged_plan *P, uint8_t *base,
                                           const uint32_t *present_bits, int32_t *status,
                                           uint8_t *slot_map, int32_t map_stride, void *stream) {
    if (slot_map && map_stride < 1) return fail(RSMI_ERR_INVALID, "map_stride < 1");
    return decode_plan_call(P, base, present_bits, status, rsmi::RefOut{slot_map, map_stride, 1}, stream);
}

extern "C" int rsmi_ragged_plan_uses_bitslice(const rsmi_ragged_plan *P) {
    return P && P->bitslice ? 1 : 0;
}

extern "C" void rsmi_ragged_plan_destroy(rsmi_ragged_plan *P) {
    if (!P) return;
    if (P->mem) (void)hipFree(P->mem);
    delete P;
}
