// fec_enc.cpp -- host side of the batched FEC framing (include/rsmi_fec.h).
//
// The planner replays fec_encode_manager_t::input() and ::output()
// (fec_manager.cpp:174-460) event by event.  Every decision there depends only
// on packet lengths, so it runs here without touching payload bytes.  It emits
// framing jobs for the GPU (frame.hip), the list of packets the reference's
// output() would have returned, and the encode launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <new>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "rsmi_internal.hpp"
#include "../../include/rsmi_fec.h"

namespace rsmi {
void set_error(const std::string &m);
const char *last_error();
}

using rsmi::CarryCopy;
using rsmi::FrameGroup;
using rsmi::FrameSrc;

namespace {

int fail(int code, const std::string &m) {
    rsmi::set_error(m);
    return code;
}

int round_up_div(int a, int b) { return (a + b - 1) / b; }  // common.cpp:747-749

// Payload addresses in a plan: a device address in the batch input, or a
// carry-tagged offset (rsmi::kCarryTag), resolved by the kernels, so planning
// needs no device.
using rsmi::kCarryBuf1;
using rsmi::kCarryTag;

struct Pending {
    uint64_t addr;  // batch-input device address or tagged carry offset
    uint32_t len;
    int64_t emitted;  // mode 1: index in this batch's packet list of its early send, -1 if none
    int64_t run;      // mode 1: the PacketRun of that send (its slot is set when the group closes)
};

// A growable array in pinned host memory (plain memory when no device is
// usable, e.g. planning-only on a CPU host), so a plan is uploaded straight
// from where the planner wrote it.
template <class T>
struct HostArr {
    T *p = nullptr;
    size_t n = 0, cap = 0;
    bool pinned = false;
    HostArr() = default;
    HostArr(const HostArr &) = delete;
    HostArr &operator=(const HostArr &) = delete;
    ~HostArr() { release(p, pinned); }
    static void release(T *q, bool pin) {
        if (!q) return;
        if (pin) (void)hipHostFree(q);
        else std::free(q);
    }
    void push_back(const T &v) {
        if (n == cap) reserve(cap ? 2 * cap : 1024);
        p[n++] = v;
    }
    void reserve(size_t c) {
        if (c <= cap) return;
        T *q = nullptr;
        bool pin = hipHostMalloc((void **)&q, c * sizeof(T), hipHostMallocDefault) == hipSuccess;
        if (!pin) {
            q = static_cast<T *>(std::malloc(c * sizeof(T)));
            if (!q) throw std::bad_alloc();
        }
        if (n) std::memcpy(q, p, n * sizeof(T));
        release(p, pinned);
        p = q;
        pinned = pin;
        cap = c;
    }
    void clear() { n = 0; }
    size_t size() const { return n; }
    bool empty() const { return n == 0; }
    T *data() const { return p; }
    T *begin() { return p; }
    T *end() { return p + n; }
    T &operator[](size_t i) { return p[i]; }
};

// A mode-0 group of this batch that still holds bytes of the blob buffer:
// positions [0, cl) were written by it; later, shorter blobs overwrite a prefix.
struct BlobHolder {
    int64_t slot0;
    int fec_len, cl;
};

// One encode launch over a run of consecutive groups with the same code and
// shard length.
struct Run {
    int64_t slot0, count;
    int k, n, len;
};

// The pinned arrays one batch's plan is uploaded from, and the event of its
// device run.  Two sets alternate, so batch i+1 is planned on the host while
// the GPU still uploads and runs batch i.
struct PlanSet {
    HostArr<FrameGroup> jobs;
    HostArr<FrameSrc> srcs;
    HostArr<CarryCopy> carry;
    HostArr<rsmi::ByteRun> stale;       // stale bytes of this batch's groups
    HostArr<rsmi::ByteRun> shadow_upd;  // the buffer at the batch end -> dshadow
    HostArr<rsmi_fenc_packet> packets;  // what output() returns, in order (rsmi_fenc_packets)
    HostArr<rsmi::PacketRun> pruns;     // the same as runs of slots (cooked runs upload these)
    HostArr<uint32_t> recs;             // per list-A packet: (first record << 8) | records its shard
                                        // overlaps (mode 0; the fused framing cook stages them)
    int64_t n_data_pk = 0, n_par_pk = 0;  // entries of the fused run's cook lists A (data shards the
                                          // fused framing cook frames) and B (the packets it does not cook)
    int32_t max_fl = 0;                   // largest fec_len of a group with list-A shards
    int64_t n_left = 0;                   // groups with data shards outside [cfirst, nfr) (k_frame's)
    uint32_t max_src = 0;  // most records of one job (> kFrameLdsSrc: k_frame reads them repeatedly)
    hipEvent_t done = nullptr;
    bool in_flight = false;
    // run by a collector: its event stands for this set's (one record per
    // flush instead of one per manager), and the stream it ran on (a run on
    // the same stream needs no cross-stream wait)
    std::shared_ptr<rsmi::SharedEv> ext;
    hipStream_t stream = nullptr;
    hipEvent_t ev() const { return ext ? ext->ev : done; }
};

}  // namespace

struct rsmi_fenc {
    rsmi_fec_config cfg;
    rsmi_fec_config next_cfg;
    bool has_next = false;
    uint32_t seq;
    int blob_len = 4;  // blob_encode_t::current_len (starts at sizeof(u32), :38-42)
    std::vector<Pending> pend;  // the open group's inputs, in order

    // ---- last plan
    PlanSet ps[2];
    int pcur = 1;              // ps[pcur] holds the last plan
    PlanSet *P = &ps[1];
    std::vector<int64_t> g_slot0;
    std::vector<int32_t> g_k, g_m, g_len;
    std::vector<uint32_t> g_seq;
    std::vector<Run> runs;
    // ---- mode 0's blob buffer (blob_encode_t::input_buf, fec_manager.h:257),
    // never cleared by the reference: the last data shard carries its bytes
    // past the blob's end (blob_encode_t::output, fec_manager.cpp:67-75).
    // Position p holds the byte of the latest blob longer than p.  `stack`
    // keeps this batch's groups that are such a latest writer for some
    // position (cl decreasing from the bottom, latest on top); the device copy
    // dshadow holds the buffer as of the batch start (zero beyond shadow_len).
    std::vector<BlobHolder> stack;
    int shadow_len = 0;
    int64_t n_slots = 0;
    int32_t stride_min = rsmi::kSlotShard;
    bool planned = false;
    bool plan_only = false;

    // ---- device side
    int device = -1;
    uint8_t *dplan = nullptr;
    size_t plan_cap = 0;
    uint8_t *dshadow = nullptr;  // kBlobBufBytes, zeroed at the first run
    uint8_t *dcarry[2] = {nullptr, nullptr};
    rsmi::EpiRec *depi = nullptr;  // parity cook in the encoder's epilogue: one record per slot
    size_t epi_cap = 0;            // records
    uint32_t epi_tag = 0;          // this encoder's runs' tags (records of older runs never match)
    int64_t last_epi_runs = 0;     // encoder runs of the last run_dev that cooked their parity
    size_t carry_cap[2] = {0, 0};
    int carry_cur = 0;  // pending packets live in dcarry[carry_cur] (or the batch input)
    size_t carry_need = 0;  // bytes of dcarry[carry_cur] the last plan fills

    int tail_x() const { return cfg.rs_cnt; }
    int y_of(int x) const { return cfg.rs_y[x - 1]; }
    // blob_encode_t::get_shard_len(n, next_packet_len), fec_manager.cpp:51-53
    int shard_len(int n, int next) const { return round_up_div(blob_len + 2 + next, n); }
};

namespace {

// The framing records (16 B per input packet, the plan's largest array) are
// read by k_frame straight from the pinned plan array over PCIe, once per
// group as its block starts, instead of being copied up first: the reads
// spread over the kernel's run and hide behind its work.  RSMI_FENC_SRC_COPY=1
// copies them up instead (A/B), as does a plan array that is not pinned.
const FrameSrc *mapped_srcs(const HostArr<FrameSrc> &a) {
    static const bool copy = [] {
        const char *v = std::getenv("RSMI_FENC_SRC_COPY");
        return v && *v && *v != '0';
    }();
    if (copy || !a.pinned || !a.p) return nullptr;
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, a.p, 0) != hipSuccess) return nullptr;
    return static_cast<const FrameSrc *>(d);
}

// RSMI_FENC_FUSE=0: cooked runs cook every packet after the encoder instead
// of framing and cooking the clean data packets in one pass (A/B).
bool fuse_enabled() {
    static const bool on = [] {
        const char *v = std::getenv("RSMI_FENC_FUSE");
        return !(v && *v == '0');
    }();
    return on;
}

// Device address of a pinned plan array (the kernels read it over PCIe), or
// NULL when it is not pinned.
template <class T>
const T *mapped(const HostArr<T> &a) {
    if (!a.pinned || !a.p) return nullptr;
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, a.p, 0) != hipSuccess) return nullptr;
    return static_cast<const T *>(d);
}

int wait_set(PlanSet &B) {
    if (B.in_flight) {
        hipError_t e = hipEventSynchronize(B.ev());
        if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("fenc wait: ") + hipGetErrorString(e));
        B.in_flight = false;
        B.ext.reset();
    }
    return RSMI_OK;
}

int grow(uint8_t **p, size_t *cap, size_t need, bool pinned) {
    if (need <= *cap) return RSMI_OK;
    size_t c = std::max(need + need / 4, *cap * 2);  // headroom: batch sizes wander
    c = (c + 4095) & ~size_t(4095);
    if (*p) (void)(pinned ? hipHostFree(*p) : hipFree(*p));
    *p = nullptr;
    *cap = 0;
    hipError_t e = pinned ? hipHostMalloc((void **)p, c, hipHostMallocDefault) : hipMalloc((void **)p, c);
    if (e != hipSuccess) return fail(RSMI_ERR_NOMEM, "fenc allocation failed");
    *cap = c;
    return RSMI_OK;
}

// Blob positions [a, b) of holder H -> runs into rows of the group at slot0
// (fec_len-byte rows), split at both groups' row boundaries.
void copy_from_holder(rsmi_fenc *E, int64_t slot0, int fec_len, const BlobHolder &H, int a, int b) {
    while (a < b) {
        const int doff = a % fec_len, soff = a % H.fec_len;
        const int n = std::min({b - a, fec_len - doff, H.fec_len - soff});
        E->P->stale.push_back(rsmi::ByteRun{(uint64_t)(slot0 + a / fec_len),
                                         (uint64_t)(H.slot0 + a / H.fec_len), (uint32_t)doff,
                                         (uint32_t)soff, (uint32_t)n, 0});
        a += n;
    }
}

// Mode 0: the bytes [cl, k*fec_len) of the group's data rows are whatever
// the blob buffer held there (k_frame wrote zeros; these runs overwrite them
// before the encode).  Then the group becomes the latest writer of [0, cl).
void stale_runs(rsmi_fenc *E, int64_t slot0, int k, int fec_len, int cl) {
    const int end = k * fec_len;
    std::vector<BlobHolder> &st = E->stack;
    for (int p = cl; p < end;) {
        // the latest holder with cl > p: the topmost such (cl decreases upward)
        int lo = 0, hi = (int)st.size();  // st[0, lo) have cl > p
        while (lo < hi) {
            const int mid = (lo + hi) / 2;
            if (st[mid].cl > p) lo = mid + 1;
            else hi = mid;
        }
        if (lo > 0) {
            const BlobHolder &H = st[lo - 1];
            const int q = std::min(end, H.cl);
            copy_from_holder(E, slot0, fec_len, H, p, q);
            p = q;
        } else {  // no writer in this batch: the buffer as of the batch start
            const int q = std::min(end, E->shadow_len);
            for (int a = p; a < q;) {
                const int doff = a % fec_len, n = std::min(q - a, fec_len - doff);
                E->P->stale.push_back(rsmi::ByteRun{(uint64_t)(slot0 + a / fec_len), rsmi::kShadowLoc,
                                                 (uint32_t)doff, (uint32_t)a, (uint32_t)n, 0});
                a += n;
            }
            break;  // beyond shadow_len the buffer is still zero, as k_frame wrote
        }
    }
    while (!st.empty() && st.back().cl <= cl) st.pop_back();
    st.push_back(BlobHolder{slot0, fec_len, cl});
}

// The blob buffer at the batch end, written back to the device copy: the top
// holder owns [0, cl_top), the one below it [cl_top, cl_below), ...
void shadow_update(rsmi_fenc *E) {
    int lo = 0;
    for (size_t i = E->stack.size(); i-- > 0;) {
        const BlobHolder &H = E->stack[i];
        for (int a = lo; a < H.cl;) {
            const int soff = a % H.fec_len, n = std::min(H.cl - a, H.fec_len - soff);
            E->P->shadow_upd.push_back(rsmi::ByteRun{rsmi::kShadowLoc, (uint64_t)(H.slot0 + a / H.fec_len),
                                                  (uint32_t)a, (uint32_t)soff, (uint32_t)n, 0});
            a += n;
        }
        lo = std::max(lo, H.cl);
    }
    E->shadow_len = std::max(E->shadow_len, lo);
}

// Data shards of the group being closed that the fused framing cook
// (k_cook_frame) frames, 0..nfr-1, and of those the ones it also cooks,
// 0..nclean-1.  Mode 1's are all clean ([u16 len][payload], zero padding).
// Mode 0's are framed while they overlap at most kFuseRecs records each (the
// kernel stages them per packet; their (first << 8) | count go to recs) and
// are clean when they end before the blob does (no stale blob-buffer bytes).
std::pair<int, int> fused_shards(rsmi_fenc *E, int k, int fec_len) {
    if (E->cfg.mode == 1) return {k, k};
    const int kc = std::min(k, E->blob_len / fec_len);
    // records' blob offsets: 4, then each after the last's 2 + len bytes
    size_t j0 = 0;  // the record holding the shard's first byte (or the last record)
    uint32_t o0 = 4;
    for (int i = 0; i < k; ++i) {
        const uint32_t s = (uint32_t)i * (uint32_t)fec_len, e = s + (uint32_t)fec_len;
        while (j0 + 1 < E->pend.size() && o0 + 2 + E->pend[j0].len <= s) {
            o0 += 2 + E->pend[j0].len;
            ++j0;
        }
        size_t j1 = j0;
        uint32_t o = o0;
        int n = 0;
        while (j1 < E->pend.size() && o < e) {
            if (o + 2 + E->pend[j1].len > s) ++n;  // (past the blob's end: none)
            o += 2 + E->pend[j1].len;
            ++j1;
        }
        if (n > rsmi::kFuseRecs) return {std::min(i, kc), i};
        E->P->recs.push_back(n ? (uint32_t)j0 << 8 | (uint32_t)n : 0u);
    }
    return {kc, k};
}

// Close the open group (the about_to_fec branch, fec_manager.cpp:248-367).
// Early-sent mode-1 packets of the group are pointed at their group slots.
void close_group(rsmi_fenc *E, int k, int m, int fec_len) {
    const int64_t slot0 = E->n_slots;
    const int n = k + m;
    E->n_slots += n;
    FrameGroup G{};
    G.slot0 = (uint64_t)slot0;
    G.seq = E->seq;
    G.fec_len = (uint32_t)fec_len;
    G.src0 = (uint32_t)E->P->srcs.size();
    G.nsrc = (uint32_t)E->pend.size();
    G.blob_len = (uint32_t)E->blob_len;
    G.nslots = (uint16_t)n;
    G.nframe = (uint16_t)k;
    G.mode = (uint8_t)E->cfg.mode;
    G.k = (uint8_t)k;
    G.m = (uint8_t)m;
    G.idx0 = 0;
    uint32_t off = 4;
    for (size_t j = 0; j < E->pend.size(); ++j) {
        const Pending &p = E->pend[j];
        E->P->srcs.push_back(FrameSrc{p.addr, p.len, E->cfg.mode == 0 ? off : 0u});
        off += 2 + p.len;
        if (p.emitted >= 0) {
            E->P->packets[(size_t)p.emitted].slot = slot0 + (int64_t)j;
            E->P->pruns[(size_t)p.run].slot = slot0 + (int64_t)j;
            E->P->pruns[(size_t)p.run].job = (int32_t)E->P->jobs.size();  // G, pushed below
        }
    }
    // mode 1: the shards whose packets went out in an earlier batch (carried,
    // at the front) are framed by k_frame; the rest were emitted in this one
    uint32_t cf = 0;
    if (E->cfg.mode == 1)
        while (cf < E->pend.size() && E->pend[cf].emitted < 0) ++cf;
    const std::pair<int, int> fs = fused_shards(E, k, fec_len);
    G.cfirst = (uint16_t)cf;
    G.nclean = (uint16_t)std::max((int)cf, fs.first);
    G.nfr = (uint16_t)std::max((int)cf, fs.second);
    if (G.nfr > G.cfirst) E->P->max_fl = std::max(E->P->max_fl, (int32_t)fec_len);
    if (G.cfirst > 0 || G.nfr < G.nframe) E->P->n_left += 1;
    E->P->jobs.push_back(G);
    E->P->max_src = std::max(E->P->max_src, E->cfg.mode == 0 ? G.nsrc : (uint32_t)G.nframe);
    if (E->cfg.mode == 0) stale_runs(E, slot0, k, fec_len, E->blob_len);
    E->g_slot0.push_back(slot0);
    E->g_k.push_back(k);
    E->g_m.push_back(m);
    E->g_len.push_back(fec_len);
    E->g_seq.push_back(E->seq);
    // pad_end of the encode kernels must stay inside the slot (rsmi.h padding rule)
    E->stride_min = std::max(E->stride_min, rsmi::kSlotShard + ((fec_len + 127) & ~127));
    if (m > 0) {
        const bool extend = !E->runs.empty() && E->runs.back().k == k && E->runs.back().n == n &&
                            E->runs.back().len == fec_len &&
                            E->runs.back().slot0 + E->runs.back().count * n == slot0;
        if (!extend) E->runs.push_back(Run{slot0, 0, k, n, fec_len});
        E->runs.back().count += 1;
    }
    // the group's encoder run (pad[0..1]; the cooked run sets pad[2] when that
    // run cooks its parity in the epilogue)
    const uint32_t ri = m > 0 ? (uint32_t)(E->runs.size() - 1) : 0xFFFFFFFFu;
    FrameGroup &J = E->P->jobs[E->P->jobs.size() - 1];
    J.pad[0] = (uint16_t)ri;
    J.pad[1] = (uint16_t)(ri >> 16);
    J.pad[2] = 0;
}

// Mode 1: the open group's last input goes out as a data packet now; its slot
// is known once the group closes (close_group) or the batch ends.
void emit_data(rsmi_fenc *E, int32_t event) {
    Pending &p = E->pend.back();
    p.emitted = (int64_t)E->P->packets.size();
    p.run = (int64_t)E->P->pruns.size();
    E->P->packets.push_back(rsmi_fenc_packet{-1, 8 + (int)p.len + 2, event});
    // (a mode-1 data shard is [u16 len][payload] zero-padded: always clean)
    E->P->pruns.push_back(rsmi::PacketRun{-1, 0, (int32_t)p.emitted, (int32_t)E->P->n_data_pk,
                                          (int32_t)E->P->n_par_pk, 8 + (int)p.len + 2, -1, 1, 1, 1, 0});
    E->P->max_fl = std::max(E->P->max_fl, (int32_t)p.len + 2);
    E->P->recs.push_back(1u);  // its own record (the kernel takes it from the slot)
    E->P->n_data_pk += 1;
}

// fec_encode_manager_t::input (fec_manager.cpp:206-447) for one event,
// followed by output() (:448-460): appends the packets output() would return.
int input_event(rsmi_fenc *E, int32_t event, bool has, int len, uint64_t addr) {
    if (E->pend.empty() && E->has_next) {  // fec_par.clone(g_fec_par) at counter 0 (:207-209)
        E->cfg = E->next_cfg;
        E->has_next = false;
    }
    const rsmi_fec_config &P = E->cfg;
    const int mode = P.mode;
    if (has && (len < 0 || len > 65535)) return -1;  // the reference asserts (:187, :57)
    if (mode == 0 && has && E->pend.empty()) {
        if (E->shard_len(E->tail_x(), len) > P.mtu) return -1;  // :217-223, "message too long"
    }
    const int cnt = (int)E->pend.size();
    if (!has && cnt == 0) return -1;  // :228-231
    bool about = !has;
    bool delayed = false;
    // :235-238 (input(0,0) passes len 0)
    if (mode == 0 && E->shard_len(E->tail_x(), has ? len : 0) > P.mtu) {
        about = true;
        delayed = true;
    }
    auto append = [&]() {  // fec_encode_manager_t::append (:174-204)
        E->pend.push_back(Pending{addr, (uint32_t)len, -1, -1});
        if (mode == 0) E->blob_len += 2 + len;
    };
    if (has && !delayed) append();
    const int counter = (int)E->pend.size();
    if (mode == 0 && counter == P.queue_len) about = true;
    if (mode == 1 && counter == E->tail_x()) about = true;

    if (about) {
        if (counter == 0) return -1;  // :252-255
        int k, m, fec_len;
        if (mode == 0) {
            const int tx = E->tail_x(), ty = E->y_of(tx);
            k = tx;
            m = ty;
            if (P.short_packet_optimize) {  // :264-288
                uint32_t best_len = (uint32_t)(E->shard_len(tx, 0) + P.header_overhead) * (uint32_t)(tx + ty);
                int best = tx;
                for (int i = 1; i < tx; ++i) {
                    const uint32_t sl = (uint32_t)E->shard_len(i, 0);
                    if (sl > (uint32_t)P.mtu) continue;
                    const uint32_t nl = (sl + (uint32_t)P.header_overhead) * (uint32_t)(i + E->y_of(i));
                    if (nl < best_len) {
                        best_len = nl;
                        best = i;
                    }
                }
                k = best;
                m = E->y_of(best);
            }
            fec_len = round_up_div(E->blob_len, k);  // blob_encode_t::output (:67-75)
        } else {
            k = counter;
            m = E->y_of(counter);
            fec_len = -1;
            for (const Pending &p : E->pend) fec_len = std::max(fec_len, (int)p.len + 2);
        }
        const int64_t first_pk = (int64_t)E->P->packets.size();
        // the packets output() returns (:318-346, fast send :376-393)
        if (mode == 0) {
            for (int i = 0; i < k + m; ++i)
                E->P->packets.push_back(rsmi_fenc_packet{-1, 8 + fec_len, event});
        } else {
            if (has) {  // the packet that completed the group goes with the parity (:376-381)
                emit_data(E, event);
            }
            for (int i = k; i < k + m; ++i)
                E->P->packets.push_back(rsmi_fenc_packet{-1, 8 + fec_len, event});
        }
        const int64_t slot0 = E->n_slots;
        close_group(E, k, m, fec_len);
        if (mode == 0) {
            for (int i = 0; i < k + m; ++i) E->P->packets[(size_t)(first_pk + i)].slot = slot0 + i;
            const FrameGroup &G = E->P->jobs[E->P->jobs.size() - 1];
            E->P->pruns.push_back(rsmi::PacketRun{slot0, 0, (int32_t)first_pk, (int32_t)E->P->n_data_pk,
                                                  (int32_t)E->P->n_par_pk, 8 + fec_len,
                                                  (int32_t)E->P->jobs.size() - 1, (uint16_t)(k + m),
                                                  G.nclean, G.nfr, 0});
            E->P->n_data_pk += G.nfr;
            E->P->n_par_pk += k + m - G.nclean;
        } else {
            int64_t q = first_pk + (has ? 1 : 0);
            if (m > 0) {
                E->P->pruns.push_back(rsmi::PacketRun{slot0 + k, 0, (int32_t)q, (int32_t)E->P->n_data_pk,
                                                      (int32_t)E->P->n_par_pk, 8 + fec_len,
                                                      (int32_t)E->P->jobs.size() - 1, (uint16_t)m, 0, 0, 0});
                E->P->n_par_pk += m;
            }
            for (int i = k; i < k + m; ++i) E->P->packets[(size_t)q++].slot = slot0 + i;
        }
        E->seq++;
        E->pend.clear();
        E->blob_len = 4;
    } else if (has && mode == 1) {  // encode_fast_send (:394-429): the data packet goes now
        emit_data(E, event);
    }
    if (has && delayed) append();  // :436-439
    return 0;
}

}  // namespace

namespace {
struct CookSpec {  // rsmi_fenc_run_cooked_dev: do_cook on the batch's packets after the encode
    const rsmi_cook_ctx *ctx;
    uint64_t seed;
    uint8_t *out;
    int32_t *out_len;
    int64_t out_cap;  // >= 0: packed output (rsmi_fenc_run_cooked_packed_dev)
};
int run_dev(rsmi_fenc *E, uint8_t *slots, int64_t S, void *stream, const CookSpec *ck);
}  // namespace

extern "C" {

int rsmi_fec_config_init(rsmi_fec_config *cfg, const char *s, int mode, int mtu, int queue_len) {
    if (!cfg || !s) return fail(RSMI_ERR_INVALID, "null config/string");
    if (mode != 0 && mode != 1) return fail(RSMI_ERR_INVALID, "mode must be 0 or 1");
    if (mtu < 1 || queue_len < 1) return fail(RSMI_ERR_INVALID, "bad mtu/queue_len");
    // rs_from_str (fec_manager.h:40-136)
    // string_to_vec(s, ",") (common.cpp:919-934) is strtok: empty tokens vanish
    std::vector<std::pair<int, int>> pv;
    std::string str(s);
    size_t pos = 0;
    while (pos <= str.size()) {
        size_t c = str.find(',', pos);
        if (c == std::string::npos) c = str.size();
        std::string tok = str.substr(pos, c - pos);
        pos = c + 1;
        if (tok.empty()) continue;
        int x, y;
        if (std::sscanf(tok.c_str(), "%d:%d", &x, &y) != 2)
            return fail(RSMI_ERR_INVALID, "failed to parse [" + tok + "]");
        if (x < 1 || y < 0 || x + y > RSMI_FEC_MAX_PACKETS)
            return fail(RSMI_ERR_INVALID, "invalid x:y in [" + tok + "]");
        pv.emplace_back(x, y);
    }
    if (pv.empty()) return fail(RSMI_ERR_INVALID, std::string("failed to parse [") + s + "]");
    for (size_t i = 1; i < pv.size(); ++i)
        if (pv[i].first <= pv[i - 1].first)
            return fail(RSMI_ERR_INVALID, "x in x:y should be in ascend order");
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->mode = mode;
    cfg->mtu = mtu;
    cfg->queue_len = queue_len;
    cfg->short_packet_optimize = 1;
    cfg->header_overhead = 40;
    for (int i = 1; i <= pv[0].first; ++i) cfg->rs_y[i - 1] = (uint8_t)pv[0].second;
    for (size_t i = 1; i < pv.size(); ++i) {
        const int now_x = pv[i].first, now_y = pv[i].second;
        const int pre_x = pv[i - 1].first, pre_y = pv[i - 1].second;
        cfg->rs_y[now_x - 1] = (uint8_t)now_y;
        for (int j = pre_x + 1; j <= now_x - 1; ++j) {
            const double distance = now_x - pre_x;
            int in_y = (int)(pre_y + (now_y - pre_y) * (j - pre_x) / distance + 0.9999);
            if (j + in_y > RSMI_FEC_MAX_PACKETS) in_y = RSMI_FEC_MAX_PACKETS - j;
            cfg->rs_y[j - 1] = (uint8_t)in_y;
        }
    }
    cfg->rs_cnt = pv.back().first;
    return RSMI_OK;
}

int rsmi_fenc_create(const rsmi_fec_config *cfg, uint32_t seq0, rsmi_fenc **out) {
    if (!cfg || !out) return fail(RSMI_ERR_INVALID, "null config/out");
    *out = nullptr;
    if ((cfg->mode != 0 && cfg->mode != 1) || cfg->rs_cnt < 1 || cfg->rs_cnt > RSMI_FEC_MAX_PACKETS ||
        cfg->mtu < 1 || cfg->queue_len < 1)
        return fail(RSMI_ERR_INVALID, "invalid fec config");
    for (int x = 1; x <= cfg->rs_cnt; ++x)
        if (x + cfg->rs_y[x - 1] > RSMI_FEC_MAX_PACKETS) return fail(RSMI_ERR_INVALID, "x + y > 255");
    rsmi_fenc *E = new rsmi_fenc();
    E->cfg = *cfg;
    E->seq = seq0;
    *out = E;  // the device is bound at the first rsmi_fenc_run_dev
    return RSMI_OK;
}

int rsmi_fenc_next_config(rsmi_fenc *E, const rsmi_fec_config *cfg) {
    if (!E || !cfg) return fail(RSMI_ERR_INVALID, "null encoder/config");
    if ((cfg->mode != 0 && cfg->mode != 1) || cfg->rs_cnt < 1 || cfg->rs_cnt > RSMI_FEC_MAX_PACKETS ||
        cfg->mtu < 1 || cfg->queue_len < 1)
        return fail(RSMI_ERR_INVALID, "invalid fec config");
    E->next_cfg = *cfg;
    E->has_next = true;
    return RSMI_OK;
}

void rsmi_fenc_destroy(rsmi_fenc *E) {
    if (!E) return;
    for (PlanSet &B : E->ps) (void)wait_set(B);
    if (E->dplan) (void)hipFree(E->dplan);
    if (E->dshadow) (void)hipFree(E->dshadow);
    if (E->depi) (void)hipFree(E->depi);
    for (int i = 0; i < 2; ++i)
        if (E->dcarry[i]) (void)hipFree(E->dcarry[i]);
    for (PlanSet &B : E->ps)
        if (B.done) (void)hipEventDestroy(B.done);
    delete E;
}

int rsmi_fenc_plan(rsmi_fenc *E, int64_t n_events, const int32_t *len, const uint64_t *in_off,
                   const uint8_t *in_base, int32_t *ret, int64_t *n_slots, int64_t *n_packets,
                   int32_t *slot_stride_min) {
    if (!E || n_events < 0 || (n_events && !len)) return fail(RSMI_ERR_INVALID, "bad fenc_plan args");
    if (E->planned && !E->plan_only && E->P->carry.size())
        return fail(RSMI_ERR_INVALID, "rsmi_fenc_plan: run the previous plan first (its carry copies)");
    bool any_packet = false;
    for (int64_t i = 0; i < n_events && !any_packet; ++i) any_packet = len[i] >= 0;
    if (!in_base && any_packet) {
        E->plan_only = true;  // decisions only; this encoder never runs on a device
    } else if (E->plan_only && any_packet) {
        return fail(RSMI_ERR_INVALID, "rsmi_fenc_plan: encoder was used plan-only (in_base NULL)");
    }
    // plan into the other set: the batch before the last one read it (its
    // upload), the last one may still be running on the GPU
    E->pcur ^= 1;
    E->P = &E->ps[E->pcur];
    int rc = wait_set(*E->P);
    if (rc) return rc;
    E->P->jobs.clear();
    E->P->max_src = 0;
    E->P->srcs.clear();
    E->P->carry.clear();
    E->P->packets.clear();
    E->P->pruns.clear();
    E->P->recs.clear();
    E->P->n_data_pk = E->P->n_par_pk = 0;
    E->P->max_fl = 0;
    E->P->n_left = 0;
    E->g_slot0.clear();
    E->g_k.clear();
    E->g_m.clear();
    E->g_len.clear();
    E->g_seq.clear();
    E->runs.clear();
    E->stack.clear();
    E->P->stale.clear();
    E->P->shadow_upd.clear();
    E->n_slots = 0;
    E->stride_min = rsmi::kSlotShard;
    for (Pending &p : E->pend) p.emitted = p.run = -1;  // sent in an earlier batch
    for (int64_t i = 0; i < n_events; ++i) {
        const bool has = len[i] >= 0;
        if (has && !in_off) return fail(RSMI_ERR_INVALID, "packet without in_off");
        const uint64_t addr = has && in_base ? (uint64_t)(uintptr_t)(in_base + in_off[i]) : 0;
        const int r = input_event(E, (int32_t)i, has, has ? len[i] : 0, addr);
        if (ret) ret[i] = r;
    }
    // mode-1 packets sent ahead of a group that is still open: a slot of their own
    for (size_t j = 0; j < E->pend.size(); ++j) {
        const Pending &p = E->pend[j];
        if (p.emitted < 0) continue;
        const int64_t slot = E->n_slots++;
        FrameGroup G{};
        G.slot0 = (uint64_t)slot;
        G.seq = E->seq;
        G.fec_len = p.len + 2;
        G.src0 = (uint32_t)E->P->srcs.size();
        G.nsrc = 1;
        G.nslots = 1;
        G.nframe = 1;
        G.mode = 1;
        G.idx0 = (uint8_t)j;
        G.nclean = G.nfr = 1;
        G.pad[0] = G.pad[1] = 0xFFFF;  // no encoder run
        E->P->srcs.push_back(FrameSrc{p.addr, p.len, 0});
        E->P->jobs.push_back(G);
        E->P->packets[(size_t)p.emitted].slot = slot;
        E->P->pruns[(size_t)p.run].slot = slot;
        E->P->pruns[(size_t)p.run].job = (int32_t)E->P->jobs.size() - 1;
        E->stride_min = std::max(E->stride_min, (int32_t)((rsmi::kSlotShard + p.len + 2 + 15) & ~15u));
    }
    shadow_update(E);
    // the open group's payloads move to the other carry buffer
    size_t cbytes = 0;
    for (const Pending &p : E->pend) cbytes += (p.len + 15) & ~15u;
    const int nxt = E->carry_cur ^ 1;
    E->carry_need = cbytes + 16;
    size_t co = 0;
    for (Pending &p : E->pend) {
        const uint64_t dst = kCarryTag | (nxt ? kCarryBuf1 : 0) | (uint64_t)co;
        if (p.len) E->P->carry.push_back(CarryCopy{p.addr, dst, p.len, 0});
        p.addr = dst;
        co += (p.len + 15) & ~15u;
    }
    E->carry_cur = nxt;
    E->planned = true;
    if (n_slots) *n_slots = E->n_slots;
    if (n_packets) *n_packets = (int64_t)E->P->packets.size();
    if (slot_stride_min) *slot_stride_min = E->stride_min;
    return RSMI_OK;
}

int rsmi_fenc_packets(const rsmi_fenc *E, rsmi_fenc_packet *out) {
    if (!E || (!out && !E->P->packets.empty())) return fail(RSMI_ERR_INVALID, "bad fenc_packets args");
    if (!E->P->packets.empty()) std::memcpy(out, E->P->packets.data(), E->P->packets.size() * sizeof(rsmi_fenc_packet));
    return RSMI_OK;
}

int rsmi_fenc_packet_runs(const rsmi_fenc *E, int64_t *n, rsmi_fenc_packet_run *out) {
    if (!E || !n) return fail(RSMI_ERR_INVALID, "bad fenc_packet_runs args");
    *n = (int64_t)E->P->pruns.size();
    static_assert(sizeof(rsmi_fenc_packet_run) == sizeof(rsmi::PacketRun), "rsmi_fenc_packet_run layout");
    if (out && *n) std::memcpy(out, E->P->pruns.data(), E->P->pruns.size() * sizeof(rsmi::PacketRun));
    return RSMI_OK;
}

int rsmi_fenc_groups(const rsmi_fenc *E, int64_t *n, int64_t *slot0, int32_t *k, int32_t *m,
                     int32_t *fec_len, uint32_t *seq) {
    if (!E) return fail(RSMI_ERR_INVALID, "null encoder");
    const size_t g = E->g_k.size();
    if (n) *n = (int64_t)g;
    if (slot0) std::copy(E->g_slot0.begin(), E->g_slot0.end(), slot0);
    if (k) std::copy(E->g_k.begin(), E->g_k.end(), k);
    if (m) std::copy(E->g_m.begin(), E->g_m.end(), m);
    if (fec_len) std::copy(E->g_len.begin(), E->g_len.end(), fec_len);
    if (seq) std::copy(E->g_seq.begin(), E->g_seq.end(), seq);
    return RSMI_OK;
}

int rsmi_fenc_run_dev(rsmi_fenc *E, uint8_t *slots, int64_t S, void *stream) {
    return run_dev(E, slots, S, stream, nullptr);
}

int rsmi_fenc_run_cooked_dev(rsmi_fenc *E, uint8_t *slots, int64_t S, const rsmi_cook_ctx *ctx,
                             uint64_t seed, uint8_t *out, int32_t *out_len, void *stream) {
    if (!ctx) return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_cooked_dev: null cook context");
    if (E && E->planned && !E->P->packets.empty() && !out_len)
        return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_cooked_dev: null out_len");
    if (out && ((uintptr_t)out & 15)) return fail(RSMI_ERR_INVALID, "cooked out must be 16-aligned");
    const CookSpec ck{ctx, seed, out, out_len, -1};
    return run_dev(E, slots, S, stream, &ck);
}

int64_t rsmi_fenc_last_parity_cooked(const rsmi_fenc *E) { return E ? E->last_epi_runs : 0; }

int rsmi_fenc_run_cooked_packed_dev(rsmi_fenc *E, uint8_t *slots, int64_t S, const rsmi_cook_ctx *ctx,
                                    uint64_t seed, uint8_t *out, int64_t out_cap, int32_t *out_len,
                                    void *stream) {
    if (!ctx) return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_cooked_packed_dev: null cook context");
    if (E && E->planned && !E->P->packets.empty() && (!out_len || !out))
        return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_cooked_packed_dev: null out / out_len");
    if (out && ((uintptr_t)out & 15)) return fail(RSMI_ERR_INVALID, "cooked out must be 16-aligned");
    if (out_cap < 0) return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_cooked_packed_dev: out_cap < 0");
    const CookSpec ck{ctx, seed, out, out_len, out_cap};
    return run_dev(E, slots, S, stream, &ck);
}

}  // extern "C"

namespace {

// Device-side preparation of a planned batch on stream s: bind the encoder to
// the current device, order s after its previous batch (which writes the
// carry area and blob buffer this one reads), grow the carry buffer the batch
// fills and create the blob buffer.
int prepare_run(rsmi_fenc *E, hipStream_t s) {
    int cur;
    if (hipGetDevice(&cur) != hipSuccess) return fail(RSMI_ERR_HIP, "fenc: no usable GPU");
    if (E->device < 0) {
        for (PlanSet &B : E->ps)
            if (hipEventCreateWithFlags(&B.done, hipEventDisableTiming) != hipSuccess)
                return fail(RSMI_ERR_HIP, "fenc: hipEventCreate");
        E->device = cur;
        // start compiling the run-time networks of the -f table's codes now, so
        // they are ready by the time those group sizes come (bitslice_rtc.cpp)
        std::vector<std::pair<int, int>> codes;
        for (int x = 1; x <= E->cfg.rs_cnt; ++x)
            if (E->cfg.rs_y[x - 1] > 0) codes.push_back({x, x + E->cfg.rs_y[x - 1]});
        rsmi::bitslice_rtc_request(codes);
    } else if (cur != E->device) {
        return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_dev on another device than the encoder's");
    }
    PlanSet &prev = E->ps[E->pcur ^ 1];
    if (prev.in_flight && prev.stream != s && hipStreamWaitEvent(s, prev.ev(), 0) != hipSuccess)
        return fail(RSMI_ERR_HIP, "fenc: hipStreamWaitEvent");
    // growing a shared device buffer frees the old one: not under the previous batch
    const bool grows = E->carry_need > E->carry_cap[E->carry_cur] || !E->dshadow;
    if (grows) {
        int rcw = wait_set(prev);
        if (rcw) return rcw;
    }
    int rc = grow(&E->dcarry[E->carry_cur], &E->carry_cap[E->carry_cur], E->carry_need, false);
    if (rc) return rc;
    if (!E->dshadow) {
        if (hipMalloc(&E->dshadow, rsmi::kBlobBufBytes) != hipSuccess)
            return fail(RSMI_ERR_NOMEM, "fenc: hipMalloc(blob buffer)");
        if (hipMemsetAsync(E->dshadow, 0, rsmi::kBlobBufBytes, s) != hipSuccess)
            return fail(RSMI_ERR_HIP, "fenc: clear blob buffer");
    }
    return RSMI_OK;
}

// RSMI_FENC_TRACE=1: run_dev's host time per stage, one stderr line a call
// (where a call's latency goes before and between its enqueues).
struct HostTrace {
    static bool enabled() {
        static const bool on = [] {
            const char *v = std::getenv("RSMI_FENC_TRACE");
            return v && *v && *v != '0';
        }();
        return on;
    }
    bool on = enabled();
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    std::string line;
    void mark(const char *stage) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        line += std::string(" ") + stage + "=" +
                std::to_string(std::chrono::duration_cast<std::chrono::microseconds>(n - t).count());
        t = n;
    }
    ~HostTrace() {
        if (on && !line.empty()) std::fprintf(stderr, "rsmi_fenc_run host us:%s\n", line.c_str());
    }
};

int run_dev(rsmi_fenc *E, uint8_t *slots, int64_t S, void *stream, const CookSpec *ck) {
    HostTrace ht;
    if (!E || !E->planned) return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_dev without a plan");
    if (E->plan_only) return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_dev on a plan-only encoder");
    if (E->n_slots && (!slots || ((uintptr_t)slots & 15)))
        return fail(RSMI_ERR_INVALID, "slots_base must be 16-aligned");
    if (S % 16 || S < E->stride_min)
        return fail(RSMI_ERR_INVALID, "slot_stride must be a multiple of 16 >= slot_stride_min (" +
                                          std::to_string(E->stride_min) + ")");
    hipStream_t s = (hipStream_t)stream;
    int rc0 = prepare_run(E, s);
    if (rc0) return rc0;
    ht.mark("prepare");
    PlanSet &prev = E->ps[E->pcur ^ 1];
    const rsmi::CarryBase carry{{E->dcarry[0], E->dcarry[1]}};
    // cooked runs: the packet list's runs go up with the plan and are expanded
    // on the device into the cook list(s)
    const size_t npk = ck ? E->P->packets.size() : 0, nrun = ck ? E->P->pruns.size() : 0;
    if (npk > (size_t)INT32_MAX) return fail(RSMI_ERR_INVALID, "fenc: more than 2^31 packets in one batch");
    // into another buffer, list A's packets (the data shards fused_shards
    // picked) are framed in one pass with the cook of the clean ones
    // (k_cook_frame), before the encoder reads their plain bytes; list B's
    // (the rest) are cooked after the encoder, in the slots.  Every list-A
    // packet must fit the kernel's bounds (it frames only those it cooks or
    // can place): else, and in place, one list in packet order, cooked after
    // the encoder.
    const int64_t cap = S - rsmi::kSlotHeader, fl = E->P->max_fl;
    const bool fuse = npk && ck->out && E->P->n_data_pk > 0 && fuse_enabled() && 8 + fl <= RSMI_COOK_MAX_LEN &&
                      16 + ((fl + 15) & ~15) - 8 <= cap &&
                      (ck->out_cap >= 0 || ((8 + fl + 4 + 33 + 8 + 15) & ~15) - 8 <= cap);
    const int64_t na = fuse ? E->P->n_data_pk : 0, nlist = fuse ? na + E->P->n_par_pk : (int64_t)npk;
    const FrameSrc *zsrc = E->P->srcs.empty() || E->P->max_src > rsmi::kFrameLdsSrc ? nullptr
                                                                                     : mapped_srcs(E->P->srcs);
    const size_t gb = E->P->jobs.size() * sizeof(FrameGroup),
                 sb = zsrc ? 0 : E->P->srcs.size() * sizeof(FrameSrc),
                 cb = E->P->carry.size() * sizeof(CarryCopy),
                 rb = E->P->stale.size() * sizeof(rsmi::ByteRun),
                 ub = E->P->shadow_upd.size() * sizeof(rsmi::ByteRun),
                 pb = nrun * sizeof(rsmi::PacketRun), xb = (size_t)nlist * sizeof(rsmi_fenc_packet);
    const bool packed = ck && ck->out_cap >= 0;
    if (packed) {  // each run's first packet's place in the packed output
        int64_t o = 0;
        for (size_t i = 0; i < nrun; ++i) {
            E->P->pruns[i].out0 = o + RSMI_FEC_COOK_LEAD;
            o += (int64_t)E->P->pruns[i].count * RSMI_FEC_COOK_SPAN(E->P->pruns[i].len);
        }
        if (o > ck->out_cap)
            return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_cooked_packed_dev: out_cap " + std::to_string(ck->out_cap) +
                                              " < packed bytes " + std::to_string(o));
    }
    // the parity packets cooked in the encoder's epilogue (RSMI_OPT_PARITY_COOK,
    // rsmi_internal.hpp EpiRec): a fused run into device memory, every encoder
    // run on a cooking split-k network
    bool epi = fuse && !packed && E->P->n_par_pk > 0 && rsmi::parity_cook_enabled();
    if (epi) {
        hipPointerAttribute_t at;
        epi = hipPointerGetAttributes(&at, ck->out) == hipSuccess && at.type == hipMemoryTypeDevice;
        (void)hipGetLastError();
    }
    E->last_epi_runs = 0;
    // per encoder run: does it have the cooking encoder (its groups' parity
    // packets are then flagged for k_cook's PREX form through FrameGroup.pad[2])
    std::vector<uint8_t> run_epi(epi ? E->runs.size() : 0, 0);
    if (epi) {
        bool any = false;
        for (size_t i = 0; i < E->runs.size(); ++i) {
            const Run &r = E->runs[i];
            run_epi[i] = rsmi::encode_cooked_ok(r.k, r.n, (int64_t)r.n * S, S, r.len, r.count) ? 1 : 0;
            any = any || run_epi[i];
            E->last_epi_runs += run_epi[i];
        }
        epi = any;
    }
    if (epi) {
        for (size_t g = 0; g < E->P->jobs.size(); ++g) {
            FrameGroup &J = E->P->jobs[g];
            const uint32_t ri = (uint32_t)J.pad[0] | (uint32_t)J.pad[1] << 16;
            J.pad[2] = ri < run_epi.size() ? run_epi[ri] : 0;
        }
    }
    if (epi) {
        // records are zero when allocated and carry the tag of the run that
        // wrote them, so a slot this run does not cook never matches
        const bool wrap = E->epi_tag == 0xFFFFFFFFu;
        if ((size_t)E->n_slots > E->epi_cap || wrap) {
            int rcw = wait_set(prev);
            if (rcw) return rcw;
            if ((size_t)E->n_slots > E->epi_cap) {
                if (E->depi) (void)hipFree(E->depi);
                E->depi = nullptr;
                E->epi_cap = 0;
                const size_t cap = (size_t)E->n_slots + (size_t)E->n_slots / 4;
                if (hipMalloc(&E->depi, cap * sizeof(rsmi::EpiRec)) != hipSuccess)
                    return fail(RSMI_ERR_NOMEM, "fenc: hipMalloc(epilogue records)");
                E->epi_cap = cap;
            }
            if (hipMemsetAsync(E->depi, 0, E->epi_cap * sizeof(rsmi::EpiRec), s) != hipSuccess)
                return fail(RSMI_ERR_HIP, "fenc: clear epilogue records");
            if (wrap) E->epi_tag = 0;
        }
        ++E->epi_tag;
    }
    const rsmi::EpiArgs epa{epi ? E->depi : nullptr, epi ? ck->out : nullptr, ck ? ck->seed : 0, E->epi_tag,
                            ck && !(rsmi::cook_ctx_flags(ck->ctx) & RSMI_COOK_NO_OBSCURE) ? 1 : 0};
    const uint32_t *zrec = fuse ? mapped(E->P->recs) : nullptr;  // read in place by k_cook_frame
    const size_t db = packed ? npk * sizeof(int64_t) : 0, jb = fuse ? (size_t)na * 2 * sizeof(int32_t) : 0;
    const size_t go = 0, so = (gb + 255) & ~size_t(255), co = (so + sb + 255) & ~size_t(255),
                 ro = (co + cb + 255) & ~size_t(255), uo = (ro + rb + 255) & ~size_t(255),
                 po = (uo + ub + 255) & ~size_t(255), xo = (po + pb + 255) & ~size_t(255),
                 dq = (xo + xb + 255) & ~size_t(255), jo = (dq + db + 255) & ~size_t(255);
    const size_t all = jo + jb + 16;
    if (all > E->plan_cap) {
        int rcw = wait_set(prev);
        if (rcw) return rcw;
    }
    int rc = grow(&E->dplan, &E->plan_cap, all, false);
    if (rc) return rc;
    ht.mark("layout");
    hipError_t e = hipSuccess;
    // (the large copies first, back to back on the copy engine)
    if (gb) e = hipMemcpyAsync(E->dplan + go, E->P->jobs.p, gb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && pb) e = hipMemcpyAsync(E->dplan + po, E->P->pruns.p, pb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && sb) e = hipMemcpyAsync(E->dplan + so, E->P->srcs.p, sb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && cb) e = hipMemcpyAsync(E->dplan + co, E->P->carry.p, cb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && rb) e = hipMemcpyAsync(E->dplan + ro, E->P->stale.p, rb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && ub)
        e = hipMemcpyAsync(E->dplan + uo, E->P->shadow_upd.p, ub, hipMemcpyHostToDevice, s);
    const FrameSrc *dsrc = zsrc ? zsrc : reinterpret_cast<const FrameSrc *>(E->dplan + so);
    ht.mark("uploads");
    if (e == hipSuccess)
        e = rsmi::launch_expand_packets(reinterpret_cast<const rsmi::PacketRun *>(E->dplan + po), (int64_t)nrun,
                                        reinterpret_cast<rsmi_fenc_packet *>(E->dplan + xo),
                                        reinterpret_cast<rsmi_fenc_packet *>(E->dplan + xo) + na,
                                        packed ? reinterpret_cast<int64_t *>(E->dplan + dq) : nullptr,
                                        fuse ? reinterpret_cast<int32_t *>(E->dplan + jo) : nullptr, s,
                                        reinterpret_cast<const FrameGroup *>(E->dplan + go), slots, S, epa);
    if (e == hipSuccess && fuse && !zrec)
        e = hipMemcpyAsync(reinterpret_cast<uint32_t *>(E->dplan + jo) + na, E->P->recs.p, (size_t)na * 4,
                           hipMemcpyHostToDevice, s);
    // (fused: k_frame only for the groups' other shards, if there are any)
    const bool frame = !fuse || E->P->n_left > 0;
    if (e == hipSuccess && frame)
        e = rsmi::launch_frame(reinterpret_cast<const FrameGroup *>(E->dplan + go), (int64_t)E->P->jobs.size(),
                               dsrc, carry, slots, S, s, fuse);
    if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("fenc frame: ") + hipGetErrorString(e));
    ht.mark(frame ? "expand+frame" : "expand");
    const int64_t *doff = packed ? reinterpret_cast<const int64_t *>(E->dplan + dq) : nullptr;
    const rsmi_fenc_packet *lists = reinterpret_cast<const rsmi_fenc_packet *>(E->dplan + xo);
    if (fuse) {  // do_cook (my_send, packet.cpp:165-168) of list A, framing it on the way
        const rsmi::FuseArgs fa{reinterpret_cast<const FrameGroup *>(E->dplan + go), dsrc, carry,
                                reinterpret_cast<const int32_t *>(E->dplan + jo),
                                zrec ? zrec : reinterpret_cast<const uint32_t *>(E->dplan + jo) + na};
        rc = rsmi::cook_frame_packets(ck->ctx, slots, S, lists, na, ck->out_len, ck->out, doff, ck->seed, fa, s);
        if (rc) return rc;
        ht.mark("cook_frame");
    }
    // stale bytes past each blob, before the parity is computed over them
    if (e == hipSuccess)
        e = rsmi::launch_byte_runs(reinterpret_cast<const rsmi::ByteRun *>(E->dplan + ro),
                                   (int64_t)E->P->stale.size(), slots, S, E->dshadow, s);
    if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("fenc frame: ") + hipGetErrorString(e));
    // parity of every group
    for (size_t ri = 0; ri < E->runs.size(); ++ri) {
        const Run &r = E->runs[ri];
        const int64_t so = r.slot0 * S + rsmi::kSlotShard;
        if (epi && run_epi[ri]) {
            const rsmi::CookEpi ce{ck->out + so, E->depi + r.slot0, rsmi::cook_ctx_ks(ck->ctx), E->epi_tag,
                                   (uint32_t)r.n};
            rc = rsmi::encode_dev_cooked(r.k, r.n, slots + so, (int64_t)r.n * S, S, r.len, r.count, ce, s);
        } else {
            rc = rsmi_encode_dev(r.k, r.n, slots + so, (int64_t)r.n * S, S, r.len, r.count, stream);
        }
        if (rc) return rc;
    }
    ht.mark(epi ? "encode+parity cook" : "encode");
    // the blob buffer as this batch leaves it (read by the next batch's stale runs)
    e = rsmi::launch_byte_runs(reinterpret_cast<const rsmi::ByteRun *>(E->dplan + uo),
                               (int64_t)E->P->shadow_upd.size(), slots, S, E->dshadow, s);
    if (e == hipSuccess)
        e = rsmi::launch_carry(reinterpret_cast<const CarryCopy *>(E->dplan + co),
                               (int64_t)E->P->carry.size(), carry, s);
    if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("fenc carry: ") + hipGetErrorString(e));
    // do_cook of the other packets (every packet in place), after the blob
    // buffer update above has read the plain shards: one launch over the
    // lists, which lie back to back.  (Cooking the data packets on a forked
    // stream beside the encoder measured no faster: the two kernels slow each
    // other down)
    if (nlist > na) {
        rc = rsmi::cook_packets(ck->ctx, slots, S, lists + na, nlist - na, ck->out_len, ck->out, doff, ck->seed, s,
                                epi);
        if (rc) return rc;
        ht.mark("tail+cook");
    }
    e = hipEventRecord(E->P->done, s);
    if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("fenc event: ") + hipGetErrorString(e));
    E->P->ext.reset();
    E->P->stream = s;
    E->P->in_flight = true;
    E->planned = false;
    return RSMI_OK;
}

}  // namespace

// ---- many managers planned at once -------------------------------------------
// A flush plans every connection's manager on its own state; they share
// nothing, so rsmi_fenc_plan_many runs rsmi_fenc_plan for each on a pool of
// host threads (host_pool.cpp).  The first failing manager's error is
// reported; the others are planned regardless.
extern "C" int rsmi_fenc_plan_many(rsmi_fenc *const *enc, int32_t n, const int64_t *ev0, const int32_t *len,
                                   const uint64_t *in_off, const uint8_t *in_base, int32_t *ret,
                                   int64_t *n_slots, int64_t *n_packets, int32_t *slot_stride_min,
                                   int32_t nthreads) {
    if (n < 0 || (n && (!enc || !ev0)) || (n && ev0[n] > ev0[0] && !len))
        return fail(RSMI_ERR_INVALID, "rsmi_fenc_plan_many: bad arguments");
    for (int i = 0; i < n; ++i) {
        if (!enc[i] || ev0[i + 1] < ev0[i]) return fail(RSMI_ERR_INVALID, "rsmi_fenc_plan_many: bad encoder or range");
        for (int j = 0; j < i; ++j)
            if (enc[j] == enc[i]) return fail(RSMI_ERR_INVALID, "rsmi_fenc_plan_many: an encoder listed twice");
    }
    std::vector<int> rcs((size_t)n, RSMI_OK);
    std::vector<std::string> errs((size_t)n);
    rsmi::host_parallel_for(n, nthreads > 0 ? nthreads : 8, [&](int i) {
        const int64_t a = ev0[i], cnt = ev0[i + 1] - ev0[i];
        int64_t ns = 0, np = 0;
        int32_t sm = 0;
        const int rc = rsmi_fenc_plan(enc[i], cnt, len ? len + a : nullptr, in_off ? in_off + a : nullptr, in_base,
                                      ret ? ret + a : nullptr, &ns, &np, &sm);
        rcs[(size_t)i] = rc;
        if (rc) {
            errs[(size_t)i] = rsmi::last_error();
            return;
        }
        if (n_slots) n_slots[i] = ns;
        if (n_packets) n_packets[i] = np;
        if (slot_stride_min) slot_stride_min[i] = sm;
    });
    for (int i = 0; i < n; ++i)
        if (rcs[(size_t)i]) return fail(rcs[(size_t)i], "encoder " + std::to_string(i) + ": " + errs[(size_t)i]);
    return RSMI_OK;
}

// ---- the collector: many managers' planned batches as one launch set --------
//
// A server keeps one fec_encode_manager_t per connection (connection.h:244-245),
// up to max_conn_num = 200 (common.h:112), each flushing on its own 8 ms timer
// (fec_manager.h:30): every flush is a handful of groups.  Run one by one,
// 200 managers cost 200 small launch sequences.  rsmi_fenc_run_many takes
// the managers' plans as they are (each planned on its own state, exactly as
// rsmi_fenc_plan does for one) and runs their byte work together: one k_frame
// over every manager's jobs, one stale-byte pass, one encode launch per
// (k, n) code over all managers' groups of that code, one blob-buffer update,
// one carry pass and one cook.  For that the managers' slots are laid out in
// one array, groups bucketed by code (so a bucket is a uniform batch for the
// bit-sliced encoders; its shard length is the bucket's longest, and a
// shorter group's parity bytes past its own fec_len are never sent), and
// every slot reference of the plans is remapped: rsmi_fenc_packets /
// rsmi_fenc_groups then report slots of the shared array.  Carry-tagged
// addresses and blob-buffer locations are resolved to absolute device
// addresses, since each manager has its own buffers.
struct rsmi_fcol {
    struct Set {
        HostArr<FrameGroup> jobs;
        HostArr<FrameSrc> srcs;
        HostArr<CarryCopy> carry;
        HostArr<rsmi::ByteRun> stale, upd;
        HostArr<rsmi::PacketRun> pruns;
        HostArr<uint32_t> recs;  // every manager's list-A records, in list-A order
        std::shared_ptr<rsmi::SharedEv> done;  // also the managers' plan sets' event (PlanSet::ext)
        bool in_flight = false;
    } set[2];
    int cur = 0;
    int device = -1;
    uint8_t *dplan[2] = {nullptr, nullptr};
    size_t plan_cap[2] = {0, 0};
};

namespace {
std::atomic<int> g_fcol_fail{0};  // rsmi_debug_fcol_fail (tests only)
}  // namespace

extern "C" {

int rsmi_debug_fcol_fail(int on) { return g_fcol_fail.exchange(on ? 1 : 0); }

int rsmi_fcol_create(rsmi_fcol **out) {
    if (!out) return fail(RSMI_ERR_INVALID, "null out");
    *out = new rsmi_fcol();
    return RSMI_OK;
}

void rsmi_fcol_destroy(rsmi_fcol *C) {
    if (!C) return;
    for (auto &B : C->set) {
        if (B.in_flight && B.done) (void)hipEventSynchronize(B.done->ev);
        B.done.reset();  // (destroyed once no manager's plan set holds it)
    }
    for (int i = 0; i < 2; ++i)
        if (C->dplan[i]) (void)hipFree(C->dplan[i]);
    delete C;
}

int rsmi_fenc_run_many(rsmi_fcol *C, rsmi_fenc *const *enc, int32_t n, uint8_t *slots, int64_t S,
                       const rsmi_cook_ctx *ctx, uint64_t seed, uint8_t *out, int32_t *out_len,
                       void *stream) {
    if (!C || n < 0 || (n && !enc)) return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_many: bad arguments");
    int64_t total_slots = 0, total_pk = 0;
    for (int i = 0; i < n; ++i) {
        rsmi_fenc *E = enc[i];
        if (!E || !E->planned) return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_many: encoder without a plan");
        if (E->plan_only) return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_many: plan-only encoder");
        for (int j = 0; j < i; ++j)
            if (enc[j] == E) return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_many: an encoder listed twice");
        if (S % 16 || S < E->stride_min)
            return fail(RSMI_ERR_INVALID, "slot_stride must be a multiple of 16 >= every encoder's "
                                          "slot_stride_min (" + std::to_string(E->stride_min) + ")");
        total_slots += E->n_slots;
        total_pk += (int64_t)E->P->packets.size();
    }
    if (total_pk > INT32_MAX) return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_many: more than 2^31 packets");
    // into another buffer, the fused framing cook as in run_dev: lists A and B
    // of every manager back to back, when every list-A packet fits its bounds
    int64_t total_a = 0, total_b = 0, n_left = 0;
    int32_t max_fl = 0;
    for (int i = 0; i < n; ++i) {
        total_a += enc[i]->P->n_data_pk;
        total_b += enc[i]->P->n_par_pk;
        n_left += enc[i]->P->n_left;
        max_fl = std::max(max_fl, enc[i]->P->max_fl);
    }
    const int64_t cap = S - rsmi::kSlotHeader;
    const bool fuse = ctx && out && total_pk && total_a > 0 && fuse_enabled() && 8 + max_fl <= RSMI_COOK_MAX_LEN &&
                      16 + ((max_fl + 15) & ~15) - 8 <= cap && ((8 + max_fl + 4 + 33 + 8 + 15) & ~15) - 8 <= cap;
    const int64_t nlist = fuse ? total_a + total_b : total_pk;
    if (total_slots && (!slots || ((uintptr_t)slots & 15)))
        return fail(RSMI_ERR_INVALID, "slots_base must be 16-aligned");
    if (ctx && total_pk && !out_len) return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_many: null out_len");
    if (out && ((uintptr_t)out & 15)) return fail(RSMI_ERR_INVALID, "cooked out must be 16-aligned");
    hipStream_t s = (hipStream_t)stream;
    int cur;
    if (hipGetDevice(&cur) != hipSuccess) return fail(RSMI_ERR_HIP, "fcol: no usable GPU");
    if (C->device < 0) {
        for (auto &B : C->set) {
            B.done = std::make_shared<rsmi::SharedEv>();
            if (hipEventCreateWithFlags(&B.done->ev, hipEventDisableTiming) != hipSuccess)
                return fail(RSMI_ERR_HIP, "fcol: hipEventCreate");
        }
        C->device = cur;
    } else if (C->device != cur) {
        return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_many on another device than the collector's");
    }
    for (int i = 0; i < n; ++i) {
        int rc = prepare_run(enc[i], s);
        if (rc) return rc;
    }
    // the other set's upload may still read its pinned arrays: refill this one
    C->cur ^= 1;
    rsmi_fcol::Set &B = C->set[C->cur];
    if (B.in_flight) {
        if (hipEventSynchronize(B.done->ev) != hipSuccess) return fail(RSMI_ERR_HIP, "fcol: wait");
        B.in_flight = false;
    }
    // ---- slot layout: every group bucketed by code, then the lone mode-1 slots
    struct Bucket {
        int k, nn, len;
        int64_t count, slot0;
    };
    std::map<int, Bucket> buckets;  // key k * 257 + n
    for (int i = 0; i < n; ++i) {
        const rsmi_fenc *E = enc[i];
        for (size_t g = 0; g < E->g_k.size(); ++g) {
            const int k = E->g_k[g], nn = k + E->g_m[g];
            Bucket &b = buckets.emplace(k * 257 + nn, Bucket{k, nn, 0, 0, 0}).first->second;
            b.count += 1;
            b.len = std::max(b.len, (int)E->g_len[g]);
        }
    }
    {
        int64_t next = 0;
        for (auto &kv : buckets) {
            kv.second.slot0 = next;
            next += kv.second.count * kv.second.nn;
        }
    }
    // From here on the plans' slot references are rewritten in place, so no
    // encoder may keep its plan past this call, whatever happens below: a
    // retried run_many (or a run_dev of one of them) would index its own
    // slot arrays with shared-array slots.  Success clears `planned` anyway.
    struct Consume {
        rsmi_fenc *const *enc;
        int n;
        ~Consume() {
            for (int i = 0; i < n; ++i) enc[i]->planned = false;
        }
    } consume{enc, n};
    std::vector<std::vector<int64_t>> smap((size_t)n);
    {
        std::map<int, int64_t> fill;
        int64_t lone = 0;
        for (auto &kv : buckets) lone += kv.second.count * kv.second.nn;
        for (int i = 0; i < n; ++i) {
            rsmi_fenc *E = enc[i];
            std::vector<int64_t> &m = smap[(size_t)i];
            m.assign((size_t)E->n_slots, -1);
            int64_t gend = 0;
            for (size_t g = 0; g < E->g_k.size(); ++g) {
                const int k = E->g_k[g], nn = k + E->g_m[g];
                const Bucket &b = buckets[k * 257 + nn];
                int64_t &f = fill[k * 257 + nn];
                const int64_t ns0 = b.slot0 + f * nn;
                f += 1;
                for (int j = 0; j < nn; ++j) m[(size_t)(E->g_slot0[g] + j)] = ns0 + j;
                gend = std::max(gend, E->g_slot0[g] + nn);
                E->g_slot0[g] = ns0;  // rsmi_fenc_groups reports the shared array
            }
            for (int64_t sl = 0; sl < E->n_slots; ++sl)
                if (m[(size_t)sl] < 0) m[(size_t)sl] = lone++;  // mode-1 packets sent ahead of a group
        }
    }
    // test hook: a failure after the remap (tests/test_fec_frame.py re-plans after it)
    if (g_fcol_fail.load(std::memory_order_relaxed))
        return fail(RSMI_ERR_INVALID, "rsmi_fenc_run_many: injected failure");
    // ---- the combined plan, every reference rewritten
    B.jobs.clear(); B.srcs.clear(); B.carry.clear(); B.stale.clear(); B.upd.clear(); B.pruns.clear();
    B.recs.clear();
    auto resolve = [](const rsmi_fenc *E, uint64_t a) -> uint64_t {
        return (a & kCarryTag) ? (uint64_t)(uintptr_t)(E->dcarry[(a & kCarryBuf1) ? 1 : 0]) + (a & rsmi::kCarryOff)
                               : a;
    };
    auto loc = [](const rsmi_fenc *E, const std::vector<int64_t> &m, uint64_t l) -> uint64_t {
        return (l & rsmi::kShadowLoc) ? (rsmi::kAbsLoc | (uint64_t)(uintptr_t)E->dshadow)
                                      : (uint64_t)m[(size_t)l];
    };
    int64_t pk_base = 0, a_base = 0, b_base = 0;
    for (int i = 0; i < n; ++i) {
        rsmi_fenc *E = enc[i];
        const std::vector<int64_t> &m = smap[(size_t)i];
        const uint32_t src0 = (uint32_t)B.srcs.size();
        const size_t job_base = B.jobs.size();
        for (size_t j = 0; j < E->P->srcs.size(); ++j) {
            FrameSrc f = E->P->srcs[j];
            f.addr = resolve(E, f.addr);
            B.srcs.push_back(f);
        }
        for (size_t j = 0; j < E->P->jobs.size(); ++j) {
            FrameGroup G = E->P->jobs[j];
            G.slot0 = (uint64_t)m[(size_t)G.slot0];  // a group's slots stay contiguous
            G.src0 += src0;
            B.jobs.push_back(G);
        }
        for (size_t j = 0; j < E->P->carry.size(); ++j) {
            CarryCopy c = E->P->carry[j];
            c.src = resolve(E, c.src);
            c.dst = resolve(E, c.dst);
            B.carry.push_back(c);
        }
        for (size_t j = 0; j < E->P->stale.size(); ++j) {
            rsmi::ByteRun r = E->P->stale[j];
            r.dst = loc(E, m, r.dst);
            r.src = loc(E, m, r.src);
            B.stale.push_back(r);
        }
        for (size_t j = 0; j < E->P->shadow_upd.size(); ++j) {
            rsmi::ByteRun r = E->P->shadow_upd[j];
            r.dst = loc(E, m, r.dst);
            r.src = loc(E, m, r.src);
            B.upd.push_back(r);
        }
        for (size_t j = 0; j < E->P->packets.size(); ++j) {
            rsmi_fenc_packet &p = E->P->packets[j];
            p.slot = m[(size_t)p.slot];  // rsmi_fenc_packets reports the shared array
        }
        for (size_t j = 0; j < E->P->pruns.size(); ++j)  // rsmi_fenc_packet_runs: shared slots too
            E->P->pruns[j].slot = m[(size_t)E->P->pruns[j].slot];  // (a run lies inside one group)
        if (ctx)
            for (size_t j = 0; j < E->P->pruns.size(); ++j) {
                rsmi::PacketRun r = E->P->pruns[j];
                r.first += (int32_t)pk_base;
                r.afirst += (int32_t)a_base;  // (fused: every list A, then every list B;
                r.bfirst += (int32_t)b_base;  // else one list in packet order)
                r.job += (int32_t)job_base;
                B.pruns.push_back(r);
            }
        if (fuse)  // (a record index is relative to its group's first source)
            for (size_t j = 0; j < E->P->recs.size(); ++j) B.recs.push_back(E->P->recs[j]);
        pk_base += (int64_t)E->P->packets.size();
        a_base += E->P->n_data_pk;
        b_base += E->P->n_par_pk;
    }
    // ---- upload + launches
    uint32_t max_src = 0;
    for (int i = 0; i < n; ++i) max_src = std::max(max_src, enc[i]->P->max_src);
    const FrameSrc *zsrc = B.srcs.empty() || max_src > rsmi::kFrameLdsSrc ? nullptr : mapped_srcs(B.srcs);
    const size_t gb = B.jobs.size() * sizeof(FrameGroup), sb = zsrc ? 0 : B.srcs.size() * sizeof(FrameSrc),
                 cb = B.carry.size() * sizeof(CarryCopy), rb = B.stale.size() * sizeof(rsmi::ByteRun),
                 ub = B.upd.size() * sizeof(rsmi::ByteRun), pb = B.pruns.size() * sizeof(rsmi::PacketRun),
                 xb = ctx ? (size_t)nlist * sizeof(rsmi_fenc_packet) : 0,
                 jb = fuse ? (size_t)total_a * 2 * sizeof(int32_t) : 0;
    const size_t go = 0, so = (gb + 255) & ~size_t(255), co = (so + sb + 255) & ~size_t(255),
                 ro = (co + cb + 255) & ~size_t(255), uo = (ro + rb + 255) & ~size_t(255),
                 po = (uo + ub + 255) & ~size_t(255), xo = (po + pb + 255) & ~size_t(255),
                 jo = (xo + xb + 255) & ~size_t(255);
    int rc = grow(&C->dplan[C->cur], &C->plan_cap[C->cur], jo + jb + 16, false);
    if (rc) return rc;
    uint8_t *dp = C->dplan[C->cur];
    hipError_t e = hipSuccess;
    if (gb) e = hipMemcpyAsync(dp + go, B.jobs.p, gb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && sb) e = hipMemcpyAsync(dp + so, B.srcs.p, sb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && cb) e = hipMemcpyAsync(dp + co, B.carry.p, cb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && rb) e = hipMemcpyAsync(dp + ro, B.stale.p, rb, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && ub) e = hipMemcpyAsync(dp + uo, B.upd.p, ub, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && pb) e = hipMemcpyAsync(dp + po, B.pruns.p, pb, hipMemcpyHostToDevice, s);
    const uint32_t *zrec = fuse ? mapped(B.recs) : nullptr;
    if (e == hipSuccess && fuse && !zrec)
        e = hipMemcpyAsync(reinterpret_cast<uint32_t *>(dp + jo) + total_a, B.recs.p, (size_t)total_a * 4,
                           hipMemcpyHostToDevice, s);
    int32_t *job_a = fuse ? reinterpret_cast<int32_t *>(dp + jo) : nullptr;
    rsmi_fenc_packet *lists = reinterpret_cast<rsmi_fenc_packet *>(dp + xo);
    if (e == hipSuccess)
        e = rsmi::launch_expand_packets(reinterpret_cast<const rsmi::PacketRun *>(dp + po), (int64_t)B.pruns.size(),
                                        lists, lists + (fuse ? total_a : 0), nullptr, job_a, s,
                                        reinterpret_cast<const FrameGroup *>(dp + go), slots, S);
    const rsmi::CarryBase none{{nullptr, nullptr}};  // every address is absolute now
    const FrameSrc *dsrc = zsrc ? zsrc : reinterpret_cast<const FrameSrc *>(dp + so);
    if (e == hipSuccess && (!fuse || n_left > 0))
        e = rsmi::launch_frame(reinterpret_cast<const FrameGroup *>(dp + go), (int64_t)B.jobs.size(), dsrc, none,
                               slots, S, s, fuse);
    if (e == hipSuccess && fuse) {  // list A framed and cooked in one pass (run_dev)
        const rsmi::FuseArgs fa{reinterpret_cast<const FrameGroup *>(dp + go), dsrc, none, job_a,
                                zrec ? zrec : reinterpret_cast<const uint32_t *>(dp + jo) + total_a};
        rc = rsmi::cook_frame_packets(ctx, slots, S, lists, total_a, out_len, out, nullptr, seed, fa, s);
        if (rc) return rc;
    }
    if (e == hipSuccess)
        e = rsmi::launch_byte_runs(reinterpret_cast<const rsmi::ByteRun *>(dp + ro), (int64_t)B.stale.size(),
                                   slots, S, nullptr, s);
    if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("fcol frame: ") + hipGetErrorString(e));
    for (auto &kv : buckets) {
        const Bucket &b = kv.second;
        if (b.nn == b.k || b.count == 0) continue;  // no parity (y = 0)
        rc = rsmi_encode_dev(b.k, b.nn, slots + b.slot0 * S + rsmi::kSlotShard, (int64_t)b.nn * S, S, b.len,
                             b.count, stream);
        if (rc) return rc;
    }
    e = rsmi::launch_byte_runs(reinterpret_cast<const rsmi::ByteRun *>(dp + uo), (int64_t)B.upd.size(), slots, S,
                               nullptr, s);
    if (e == hipSuccess)
        e = rsmi::launch_carry(reinterpret_cast<const CarryCopy *>(dp + co), (int64_t)B.carry.size(), none, s);
    if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("fcol carry: ") + hipGetErrorString(e));
    if (ctx && nlist > (fuse ? total_a : 0)) {
        rc = rsmi::cook_packets(ctx, slots, S, lists + (fuse ? total_a : 0), nlist - (fuse ? total_a : 0), out_len,
                                out, nullptr, seed, s);
        if (rc) return rc;
    }
    if (hipEventRecord(B.done->ev, s) != hipSuccess) return fail(RSMI_ERR_HIP, "fcol: event");
    B.in_flight = true;
    for (int i = 0; i < n; ++i) {  // one event for all (a record per manager cost ~5 us each)
        rsmi_fenc *E = enc[i];
        E->P->ext = B.done;
        E->P->stream = s;
        E->P->in_flight = true;
        E->planned = false;
    }
    return RSMI_OK;
}

}  // extern "C"
