// fec_dec.cpp -- receive side of the batched FEC framing (include/rsmi_fec.h,
// SURVEY §8f row f3).
//
// The planner replays fec_decode_manager_t::input (fec_manager.cpp:469-784)
// packet by packet: header checks, anti_replay_t (fec_manager.h:187-235), the
// seq -> group map with unordered_map::operator[]'s insert-on-read, the ring
// of fec_buff_num buffers whose reuse evicts old groups, and the decisions of
// when a group decodes.  None of them depends on decoded bytes, so the decodes
// of a whole batch run afterwards on the GPU (gather -> rsmi_decode_dev per
// (k,n) -> pack -> one D2H), and the outputs -- blob_decode's records (mode
// 0) or the missed data shards (mode 1), which do depend on decoded bytes --
// are resolved on the host from the copied-back rows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <cstring>
#include <map>
#include <memory>
#include <new>
#include <string>
#include <deque>
#include <unordered_map>
#include <thread>
#include <vector>

#include "rsmi_internal.hpp"
#include "../../include/rsmi_fec.h"

namespace rsmi {
void set_error(const std::string &m);
const char *last_error();
}

using rsmi::GatherCopy;
using rsmi::CarryCopy;
using rsmi::JoinCopy;

namespace {

int fail(int code, const std::string &m) {
    rsmi::set_error(m);
    return code;
}

constexpr uint32_t kAntiReplaySize = 30000;      // anti_replay_buff_size (fec_manager.h:16)
constexpr int64_t kAntiReplayTimeout = 120000;   // anti_replay_timeout, ms (fec_manager.h:185)
constexpr int kMaxBlobPackets = 30000;           // max_blob_packet_num (fec_manager.h:15)
constexpr int kMaxDataLen = 3600;                // max_data_len (common.h:102)
constexpr int kBufLen = kMaxDataLen + 200;       // buf_len (common.h:103)
constexpr int kRingBytes = (kBufLen + 15) & ~15; // carry bytes per ring slot

uint32_t rd_u32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
uint32_t rd_u16(const uint8_t *p) { return (uint32_t)p[0] << 8 | p[1]; }

// seq -> V: open addressing, linear probing, backward-shift erase (no
// tombstones), at most half full.  The planner's maps only find, insert and
// erase (nothing iterates them), so a flat table replaces the reference's
// node-based std::unordered_map without a change in behaviour, at one probe
// per lookup and no allocation per group.
template <class V>
struct SeqMap {
    struct Ent {
        uint32_t key, used;
        V val;
    };
    std::vector<Ent> t;
    size_t mask = 0, n = 0;
    uint64_t edits = 0;  // inserts + erases: a cached lookup holds while this is unchanged
    explicit SeqMap(size_t cap = 64) { rehash(cap); }
    size_t home(uint32_t k) const { return (size_t)((k * 0x9E3779B1u) ^ (k >> 16)) & mask; }
    void rehash(size_t cap) {
        size_t c = 16;
        while (c < cap) c <<= 1;
        std::vector<Ent> old(c, Ent{0, 0, V{}});
        old.swap(t);
        mask = c - 1;
        for (const Ent &e : old)
            if (e.used) {
                size_t i = home(e.key);
                while (t[i].used) i = (i + 1) & mask;
                t[i] = e;
            }
    }
    V *find(uint32_t k) {
        for (size_t i = home(k);; i = (i + 1) & mask) {
            if (!t[i].used) return nullptr;
            if (t[i].key == k) return &t[i].val;
        }
    }
    // the slot for k; inserted (value v0) if absent
    V &get(uint32_t k, const V &v0, bool *inserted = nullptr) {
        size_t i = home(k);
        for (; t[i].used; i = (i + 1) & mask)
            if (t[i].key == k) {
                if (inserted) *inserted = false;
                return t[i].val;
            }
        if (2 * (n + 1) > t.size()) {
            rehash(2 * t.size());
            return get(k, v0, inserted);
        }
        t[i] = Ent{k, 1, v0};
        ++n;
        ++edits;
        if (inserted) *inserted = true;
        return t[i].val;
    }
    bool erase(uint32_t k) {
        size_t i = home(k);
        for (;; i = (i + 1) & mask) {
            if (!t[i].used) return false;
            if (t[i].key == k) break;
        }
        // shift back the run after i: an entry moves into the hole unless its
        // home lies cyclically in (hole, its slot]
        for (size_t j = (i + 1) & mask; t[j].used; j = (j + 1) & mask) {
            const size_t h = home(t[j].key);
            const bool stays = i <= j ? (h > i && h <= j) : (h > i || h <= j);
            if (!stays) {
                t[i] = t[j];
                i = j;
            }
        }
        t[i].used = 0;
        --n;
        ++edits;
        return true;
    }
};

// anti_replay_t (fec_manager.h:187-235)
struct AntiReplay {
    struct Info {
        int64_t time;
        uint32_t index;
    };
    std::vector<int64_t> buf = std::vector<int64_t>(kAntiReplaySize, -1);
    SeqMap<Info> mp{(size_t)kAntiReplaySize * 3};
    uint32_t index = 0;
    bool valid(uint32_t seq, int64_t now) {
        Info *it = mp.find(seq);
        if (!it) return true;
        if (now - it->time > kAntiReplayTimeout) {
            buf[it->index] = -1;
            mp.erase(seq);
            return true;
        }
        return false;
    }
    void set_invalid(uint32_t seq, int64_t now) {
        if (!valid(seq, now)) return;
        if (buf[index] != -1) mp.erase((uint32_t)buf[index]);
        buf[index] = seq;
        mp.get(seq, Info{}) = Info{now, index};
        if (++index == kAntiReplaySize) index = 0;
    }
};

// inner index -> ring slot in ascending index order: the reference's
// std::map<int,int> (fec_manager.h:382), kept as one sorted vector per group
// (indices mostly arrive in order, so inserts append).
struct SlotMap {
    std::vector<std::pair<int, int>> v;
    typedef std::vector<std::pair<int, int>>::const_iterator It;
    It begin() const { return v.begin(); }
    It end() const { return v.end(); }
    size_t size() const { return v.size(); }
    It find(int key) const {
        It it = std::lower_bound(v.begin(), v.end(), key,
                                 [](const std::pair<int, int> &a, int b) { return a.first < b; });
        return it != v.end() && it->first == key ? it : v.end();
    }
    bool count(int key) const { return find(key) != v.end(); }
    void set(int key, int slot) {  // key not present (checked by the caller)
        if (v.empty()) v.reserve(32);
        if (v.empty() || v.back().first < key) {
            v.emplace_back(key, slot);
            return;
        }
        auto it = std::lower_bound(v.begin(), v.end(), key,
                                   [](const std::pair<int, int> &a, int b) { return a.first < b; });
        v.insert(it, std::make_pair(key, slot));
    }
};

struct Group {  // fec_group_t (fec_manager.h:376-384)
    int type = -1, data_num = -1, red = -1, len = -1, fec_done = 0;
    SlotMap gm;  // inner index -> ring slot
};

struct RingEnt {  // fec_data_t (fec_manager.h:366-375), bytes on the device
    bool used = false;
    uint32_t seq = 0;
    int len = 0;
    uint64_t src = 0;  // payload: device address in the batch, or carry-tagged slot
    const uint8_t *host = nullptr;  // payload in the caller's host buffer (this batch only)
    bool in_batch = false;
};

// Where the host finds data row i of a decoded group: the received packet in
// the caller's host buffer, or row `d2h` of the rows copied back.
struct RowRef {
    const uint8_t *host;
    int64_t d2h;
};

struct Job {  // one group decoded in this batch
    int type, k, n, len, inner;
    int32_t event;
    int bucket;
    int64_t row;        // group row in its bucket's staging
    int64_t rows0;      // mode 1: its k RowRefs in rsmi_fdec::rows
    int64_t lin = -1;   // mode 0: its blob (the k data rows joined on the device), in the rows copied back
};

struct Bucket {
    int k, n, len = 0;
    int64_t rows = 0, stride = 0, staging_off = 0, present_off = 0;
};

struct Out {
    int32_t event;
    int64_t job;        // -1: pass-through packet
    const uint8_t *ptr;
    int32_t len;
};

template <class T>
int dev_grow(T **p, size_t *cap, size_t need) {
    if (need <= *cap) return RSMI_OK;
    size_t c = std::max(need + need / 4, *cap * 2);  // headroom: batch sizes wander
    c = (c + 4095) & ~size_t(4095);
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc((void **)p, c) != hipSuccess) return fail(RSMI_ERR_NOMEM, "fdec device allocation failed");
    *cap = c;
    return RSMI_OK;
}

int host_grow(uint8_t **p, size_t *cap, size_t need) {
    if (need <= *cap) return RSMI_OK;
    size_t c = std::max(need + need / 4, *cap * 2);  // headroom: batch sizes wander
    c = (c + 4095) & ~size_t(4095);
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipHostMalloc((void **)p, c, hipHostMallocDefault) != hipSuccess)
        return fail(RSMI_ERR_NOMEM, "fdec pinned allocation failed");
    *cap = c;
    return RSMI_OK;
}

}  // namespace

struct Spill {
    std::vector<std::pair<std::unique_ptr<uint8_t[]>, size_t>> chunks;
    size_t chunk = 0, used = 0;
    void reset() { chunk = used = 0; }
    uint8_t *alloc(size_t n) {
        while (chunk < chunks.size() && used + n > chunks[chunk].second) {
            ++chunk;
            used = 0;
        }
        if (chunk == chunks.size()) {
            const size_t c = std::max<size_t>(n, size_t(16) << 20);
            chunks.emplace_back(std::unique_ptr<uint8_t[]>(new uint8_t[c]), c);
            used = 0;
        }
        uint8_t *p = chunks[chunk].first.get() + used;
        used += n;
        return p;
    }
};

// One batch's plan and results.  Two alternate: batch i+1 is planned on the
// host while the GPU still runs batch i, and batch i's outputs stay readable
// until the plan after that.
struct Batch {
    std::vector<Job> jobs;
    std::vector<Bucket> buckets;
    std::map<int, int> bucket_of;  // k*257+n -> bucket
    std::vector<GatherCopy> gathers;
    std::vector<std::pair<int64_t, int>> gather_ref;  // (job, shard index) of each gather
    std::vector<CarryCopy> carries;
    std::vector<Out> outs;
    std::vector<uint8_t> present;  // all buckets' present flags
    std::vector<RowRef> rows;      // k per job
    std::vector<std::pair<int64_t, int>> d2h_rows;  // (job, row; -1: the joined blob) copied back, in d2h order
    // outputs that straddle two rows are copied into bump-allocated chunks, one
    // arena per resolver thread, kept from batch to batch (fresh pages would cost
    // a fault per 4 KiB)
    std::vector<Spill> spills = std::vector<Spill>(1);
    int64_t staging_bytes = 0, d2h_bytes = 0;
    const uint8_t *host_base = nullptr;
    bool planned = false, ran = false, resolved = false;
    uint8_t *hmeta = nullptr, *hblob = nullptr;  // pinned: upload source, rows copied back
    size_t hmeta_cap = 0, hblob_cap = 0;
    // a collector run: the rows came back into the collector's pinned buffer
    // (one copy for every decoder), and its event stands for this batch's
    const uint8_t *hblob_view = nullptr;
    // ... stamped with the collector set's generation: the set is reused (its
    // buffer overwritten or freed) two runs later, or freed with the collector
    std::shared_ptr<std::atomic<uint64_t>> view_gen_src;
    uint64_t view_gen = 0;
    bool view_stale() const { return view_gen_src && view_gen_src->load() != view_gen; }
    std::shared_ptr<rsmi::SharedEv> ext;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    bool in_flight = false;
    hipEvent_t ev() const { return ext ? ext->ev : done; }
    const uint8_t *rows_back() const { return hblob_view ? hblob_view : hblob; }
};

struct EvictMemo {  // the last ring eviction (input_packet)
    bool valid = false;
    uint32_t seq = 0;
    int64_t now = 0;
    uint64_t ar_edits = 0, mp_edits = 0;
};

struct SeqMemo {  // the last packet's anti-replay check and group (input_packet)
    Group *gp = nullptr;
    uint32_t seq = 0;
    int64_t now = 0;
    uint64_t ar_edits = 0, mp_edits = 0;
};

struct rsmi_fdec {
    int buff_num = 2000;
    EvictMemo evict_memo;
    SeqMemo seq_memo;
    std::vector<std::pair<int, int>> sel;  // plan_decode's survivors
    AntiReplay ar;
    // fec_decode_manager_t::mp (fec_manager.h:388): seq -> a group in the slab
    // (stable addresses; freed groups keep their map's storage for reuse)
    SeqMap<uint32_t> mp;
    std::deque<Group> groups;
    std::vector<uint32_t> free_groups;
    std::vector<RingEnt> ring;
    int index = 0;
    bool plan_only = false;

    Batch bat[2];
    int bi = 1;               // bat[bi] is the batch planned last
    Batch *B = &bat[1];
    int out_b = -1;           // batch whose outputs rsmi_fdec_output_list reads

    // ---- device side: shared by the two batches, whose device work is ordered
    int device = -1;
    uint8_t *dcarry = nullptr;  // buff_num x kRingBytes, indexed by ring slot
    size_t dcarry_cap = 0;
    uint8_t *dstage = nullptr, *dmeta = nullptr, *dblob = nullptr;
    size_t stage_cap = 0, meta_cap = 0, blob_cap = 0;
    int32_t *dstatus = nullptr;
    size_t status_cap = 0;

    Group &group(uint32_t seq) {  // inserts, as the reference's operator[]
        bool fresh;
        uint32_t &gi = mp.get(seq, 0u, &fresh);
        if (fresh) {
            if (free_groups.empty()) {
                gi = (uint32_t)groups.size();
                groups.emplace_back();
            } else {
                gi = free_groups.back();
                free_groups.pop_back();
                Group &g = groups[gi];
                g.type = g.data_num = g.red = g.len = -1;
                g.fec_done = 0;
                g.gm.v.clear();
            }
        }
        return groups[gi];
    }
    Group *find_group(uint32_t seq) {
        uint32_t *gi = mp.find(seq);
        return gi ? &groups[*gi] : nullptr;
    }
    void erase_group(uint32_t seq) {
        uint32_t *gi = mp.find(seq);
        if (!gi) return;
        free_groups.push_back(*gi);
        mp.erase(seq);
    }
};

namespace {

int wait_batch(Batch &X) {
    if (X.in_flight) {
        hipError_t e = hipEventSynchronize(X.ev());
        X.in_flight = false;
        X.ext.reset();
        if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("fdec wait: ") + hipGetErrorString(e));
    }
    return RSMI_OK;
}

// The about_to_fec branch (fec_manager.cpp:616-757) up to the byte work:
// queue the decode job; its outputs are resolved after the run.
void plan_decode(rsmi_fdec *D, uint32_t seq, Group &g, int type, int inner, int len, int32_t event,
                 int64_t now) {
    const int k = g.data_num, m = g.red, n = k + m;
    int dlen = len;
    if (type == 1) {  // data_check (:671-695): every shard >= 2 bytes, the longest == the group's len
        int max_len = -1;
        bool ok = true;
        for (auto &kv : g.gm) {
            const int l = D->ring[(size_t)kv.second].len;
            if (l < 2) ok = false;
            max_len = std::max(max_len, l);
        }
        if (max_len != g.len) ok = false;
        if (!ok) {
            D->ar.set_invalid(seq, now);
            return;
        }
        dlen = max_len;
    }
    g.fec_done = 1;
    // rs_decode2's survivors: the first k present indices below n (rs.cpp:24-39)
    std::vector<std::pair<int, int>> &sel = D->sel;  // scratch, kept between groups
    sel.clear();
    bool bad = false;
    for (auto &kv : g.gm) {
        if (kv.first >= n) bad = true;
        else if ((int)sel.size() < k) sel.emplace_back(kv.first, kv.second);
    }
    if (bad || (int)sel.size() < k) {  // the reference aborts on its assert here
        D->ar.set_invalid(seq, now);
        return;
    }
    const int key = k * 257 + n;
    auto it = D->B->bucket_of.find(key);
    int b;
    if (it == D->B->bucket_of.end()) {
        b = (int)D->B->buckets.size();
        D->B->bucket_of[key] = b;
        Bucket B;
        B.k = k;
        B.n = n;
        D->B->buckets.push_back(B);
    } else {
        b = it->second;
    }
    Bucket &B = D->B->buckets[(size_t)b];
    B.len = std::max(B.len, dlen);
    Job J;
    J.type = type;
    J.k = k;
    J.n = n;
    J.len = dlen;
    J.inner = inner;
    J.event = event;
    J.bucket = b;
    J.row = B.rows++;
    J.rows0 = (int64_t)D->B->rows.size();
    // mode 0: the blob comes back whole, its k data rows joined on the device
    // (records straddle rows); mode 1: the rows the host reads are the received
    // packet when this batch's host buffer holds it, else the decoded (or
    // carried) row, copied back
    const int64_t job = (int64_t)D->B->jobs.size();
    if (type == 0) D->B->d2h_rows.emplace_back(job, -1);
    for (int i = 0; i < k && type != 0; ++i) {
        auto f = g.gm.find(i);
        const RingEnt *r = f != g.gm.end() ? &D->ring[(size_t)f->second] : nullptr;
        if (r && r->host && r->in_batch) {
            D->B->rows.push_back(RowRef{r->host, -1});
        } else {
            D->B->rows.push_back(RowRef{nullptr, (int64_t)D->B->d2h_rows.size()});
            D->B->d2h_rows.emplace_back(job, i);
        }
    }
    // survivor copies: dst is patched once the bucket strides are known
    for (auto &sv : sel) {
        const RingEnt &r = D->ring[(size_t)sv.second];
        GatherCopy G;
        G.src = r.src;
        G.dst = ((uint64_t)D->B->jobs.size() << 8) | (uint64_t)sv.first;  // (job, index) until patched
        G.len = (uint32_t)r.len;
        G.dst_len = 0;
        D->B->gathers.push_back(G);
    }
    D->B->outs.push_back(Out{event, (int64_t)D->B->jobs.size(), nullptr, 0});
    D->B->jobs.push_back(J);
    D->ar.set_invalid(seq, now);
}

// fec_decode_manager_t::input (fec_manager.cpp:469-784) for one packet.
int input_packet(rsmi_fdec *D, const uint8_t *s, int len, uint64_t dsrc, int32_t event, int64_t now) {
    if (len < 8) return -1;
    const uint32_t seq = rd_u32(s);
    const int type = s[4], data_num = s[5], red = s[6], inner = s[7];
    const uint8_t *pay = s + 8;
    len -= 8;
    if (type == 1) {
        if (len < 2) return -1;
        if (data_num == 0 && (int)rd_u16(pay) + 2 != len) return -1;
    }
    if (type == 0 && data_num == 0) return -1;
    if (data_num + red >= RSMI_FEC_MAX_PACKETS) return -1;
    // packets of one group mostly arrive together: the last lookup holds while
    // neither map changed and the clock stands still (a valid seq stays valid)
    SeqMemo &sm = D->seq_memo;
    Group *gp;
    if (sm.gp && sm.seq == seq && sm.now == now && sm.ar_edits == D->ar.mp.edits && sm.mp_edits == D->mp.edits) {
        gp = sm.gp;
    } else {
        if (!D->ar.valid(seq, now)) return 0;
        gp = &D->group(seq);  // inserts, as the reference's mp[seq]
        sm = SeqMemo{gp, seq, now, D->ar.mp.edits, D->mp.edits};
    }
    {
        Group &g = *gp;
        if (g.fec_done) return -1;
        if (g.gm.count(inner)) return -1;
        if (g.type == -1) g.type = type;
        else if (g.type != type) return -1;
        if (data_num != 0) {
            if (g.data_num == -1) {
                g.data_num = data_num;
                g.red = red;
                g.len = len;
            } else if (g.data_num != data_num || g.red != red || g.len != len) {
                return -1;
            }
        }
    }
    RingEnt &slot = D->ring[(size_t)D->index];
    if (slot.used) {  // ring reuse evicts the slot's group (:554-576)
        const uint32_t tmp_seq = slot.seq;
        // consecutive slots mostly hold one group: evicting it again is a no-op
        // while neither map changed since and the clock stands still
        EvictMemo &em = D->evict_memo;
        if (!(em.valid && em.seq == tmp_seq && em.now == now && em.ar_edits == D->ar.mp.edits &&
              em.mp_edits == D->mp.edits)) {
            D->ar.set_invalid(tmp_seq, now);
            D->erase_group(tmp_seq);  // other groups' references stay valid
            em = EvictMemo{true, tmp_seq, now, D->ar.mp.edits, D->mp.edits};
        }
        if (tmp_seq == seq) return -1;
    }
    slot.used = true;
    slot.seq = seq;
    slot.len = len;
    slot.src = dsrc;
    slot.host = pay;
    slot.in_batch = true;
    Group &g = *gp;
    g.gm.set(inner, D->index);
    const int size = (int)g.gm.size();
    bool about = false, end = false;
    if (type == 0) {
        if (size > data_num) {
            D->ar.set_invalid(seq, now);
            end = true;
        } else if (size == data_num) {
            about = true;
        }
    } else if (g.data_num != -1) {
        if (size > g.data_num + 1) {
            D->ar.set_invalid(seq, now);
            end = true;
        } else if (size >= g.data_num) {
            about = true;
        }
    }
    if (!end) {
        if (about) plan_decode(D, seq, g, type, inner, len, event, now);
        else if (type == 1 && data_num == 0)  // decode_fast_send (:760-776)
            D->B->outs.push_back(Out{event, -1, pay + 2, len - 2});
    }
    if (++D->index == D->buff_num) D->index = 0;
    return 0;
}

// Output records of outs[b, e) (fec_manager.cpp:97-129 and :713-755): mode 0
// from the group's blob, copied back whole; mode 1 from the rows the host holds
// and the rows copied back.
void resolve_outputs(const Batch &X, size_t b, size_t e, Spill &sp, std::vector<Out> &res) {
    for (size_t oi = b; oi < e; ++oi) {
        const Out &o = X.outs[oi];
        if (o.job < 0) {
            res.push_back(o);
            continue;
        }
        const Job &J = X.jobs[(size_t)o.job];
        const int64_t L = J.len;
        if (J.type == 0) {  // blob_decode_t::output (fec_manager.cpp:97-129)
            const uint8_t *blob = X.rows_back() + J.lin;
            const int64_t cur = (int64_t)J.k * L;  // the k data rows back to back
            if (cur < 4) continue;
            const uint32_t cnt = rd_u32(blob);
            if (cnt > (uint32_t)kMaxBlobPackets) continue;
            int64_t pos = 4;
            const size_t mark = res.size();
            bool ok = true;
            for (uint32_t i = 0; i < cnt; ++i) {
                if (pos + 2 > cur) { ok = false; break; }
                const int l = (int)rd_u16(blob + pos);
                pos += 2;
                if (pos + l > cur) { ok = false; break; }
                res.push_back(Out{o.event, o.job, blob + (l ? pos : 0), l});
                pos += l;
            }
            if (!ok) res.resize(mark);
        } else {  // mode 1 (:713-755): every data row's u16 <= max_data_len, then the missed rows
            const RowRef *rr = X.rows.data() + J.rows0;
            auto row = [&](int i) -> const uint8_t * {
                return rr[i].host ? rr[i].host : X.rows_back() + rr[i].d2h;
            };
            bool ok = true;
            for (int i = 0; i < J.k; ++i)
                if ((int)rd_u16(row(i)) > kMaxDataLen) ok = false;
            if (!ok) continue;
            // missed = rows not received + the packet that completed the group
            const Bucket &B = X.buckets[(size_t)J.bucket];
            const uint8_t *pres = X.present.data() + B.present_off + J.row * B.n;
            for (int i = 0; i < J.k; ++i) {
                if (pres[i] && i != J.inner) continue;
                const int64_t l = rd_u16(row(i));
                if (l + 2 <= L) {
                    res.push_back(Out{o.event, o.job, row(i) + 2, (int32_t)l});
                } else {  // a malformed row claims more than it holds: the reference reads
                          // stale ring-buffer bytes past it (:715-717); zeros here
                    uint8_t *buf = sp.alloc((size_t)l);
                    std::memcpy(buf, row(i) + 2, (size_t)(L - 2));
                    std::memset(buf + (L - 2), 0, (size_t)(l - (L - 2)));
                    res.push_back(Out{o.event, o.job, buf, (int32_t)l});
                }
            }
        }
    }
}

int env_int(const char *name, int dflt) {
    const char *v = std::getenv(name);
    return v && *v ? std::atoi(v) : dflt;
}

// resolver threads: RSMI_HOST_THREADS, else the hardware's, at most 16
int host_threads() {
    int t = env_int("RSMI_HOST_THREADS", 0);
    if (t <= 0) t = std::min<int>(16, (int)std::max(1u, std::thread::hardware_concurrency()));
    return t;
}

// Resolver threads, started once and kept (starting 15 threads per batch cost
// more than resolving a 30 K-packet batch).  One batch at a time: a caller
// that finds the pool busy (another connection's decoder) resolves alone.
class ResolvePool {
  public:
    static ResolvePool &get() {
        static ResolvePool *p = new ResolvePool();  // never torn down: threads are detached
        return *p;
    }
    // f(t) for t in [0, n) over the pool and the calling thread; false if busy
    bool try_run(int n, const std::function<void(int)> &f) {
        std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
        if (!busy.owns_lock()) return false;
        {
            std::lock_guard<std::mutex> lk(mu_);
            while ((int)workers_ < n - 1) {
                std::thread(&ResolvePool::loop, this).detach();
                ++workers_;
            }
            job_ = &f;
            n_ = n;
            next_.store(0);
            left_ = (int)workers_;  // every worker checks in once per job
            ++gen_;
        }
        cv_.notify_all();
        for (int t; (t = next_.fetch_add(1)) < n;) f(t);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return left_ == 0; });  // no worker still inside f
        job_ = nullptr;
        return true;
    }

  private:
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)> *f;
            int n;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                f = job_;
                n = n_;
            }
            for (int t; (t = next_.fetch_add(1)) < n;) (*f)(t);
            std::lock_guard<std::mutex> lk(mu_);
            if (--left_ == 0) done_.notify_all();
        }
    }
    std::mutex run_mu_, mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)> *job_ = nullptr;
    int n_ = 0, left_ = 0;
    std::atomic<int> next_{0};
    uint64_t gen_ = 0;
    unsigned workers_ = 0;
};

}  // namespace

extern "C" {

int rsmi_fdec_create(int32_t buff_num, rsmi_fdec **out) {
    if (!out || buff_num < 0) return fail(RSMI_ERR_INVALID, "bad fdec_create args");
    rsmi_fdec *D = new rsmi_fdec();
    if (buff_num) D->buff_num = buff_num;
    D->ring.assign((size_t)D->buff_num, RingEnt{});
    D->mp.rehash((size_t)D->buff_num * 4);
    *out = D;
    return RSMI_OK;
}

void rsmi_fdec_destroy(rsmi_fdec *D) {
    if (!D) return;
    for (Batch &X : D->bat) (void)wait_batch(X);
    for (uint8_t *p : {D->dcarry, D->dstage, D->dmeta, D->dblob}) if (p) (void)hipFree(p);
    if (D->dstatus) (void)hipFree(D->dstatus);
    for (Batch &X : D->bat) {
        for (uint8_t *p : {X.hmeta, X.hblob}) if (p) (void)hipHostFree(p);
        if (X.done) (void)hipEventDestroy(X.done);
    }
    delete D;
}

int rsmi_fdec_plan(rsmi_fdec *D, int64_t n, const int32_t *len, const uint64_t *off,
                   const uint8_t *host_base, const uint8_t *dev_base, int64_t now_ms, int32_t *ret,
                   int64_t *n_decodes) {
    if (!D || n < 0 || (n && (!len || !off || !host_base))) return fail(RSMI_ERR_INVALID, "bad fdec_plan args");
    if (D->B->planned && !D->plan_only)
        return fail(RSMI_ERR_INVALID, "rsmi_fdec_plan: run the previous plan first (its carry copies)");
    if (!dev_base) {
        D->plan_only = true;  // decisions only; this decoder never runs on a device
    } else if (D->plan_only) {
        return fail(RSMI_ERR_INVALID, "rsmi_fdec_plan: decoder was used plan-only (dev_base NULL)");
    }
    // plan into the other batch: the one before the last (its outputs, if not
    // taken yet, are dropped now); the last one may still run on the GPU
    D->bi ^= 1;
    D->B = &D->bat[D->bi];
    if (D->out_b == D->bi) D->out_b = -1;
    int rc = wait_batch(*D->B);
    if (rc) return rc;
    D->B->jobs.clear();
    D->B->buckets.clear();
    D->B->bucket_of.clear();
    D->B->gathers.clear();
    D->B->carries.clear();
    D->B->outs.clear();
    D->B->present.clear();
    D->B->rows.clear();
    D->B->d2h_rows.clear();
    for (Spill &sp : D->B->spills) sp.reset();  // the chunks are reused
    D->B->staging_bytes = D->B->d2h_bytes = 0;
    D->B->host_base = host_base;
    static const bool prof = env_int("RSMI_FDEC_PROFILE", 0) != 0;
    const auto t0 = std::chrono::steady_clock::now();
    // The headers are cold (a batch of packets is megabytes, read once): fetch
    // kAhead packets ahead, so their misses overlap instead of costing one
    // memory latency each.  mode 1 also reads the payload's u16 (bytes 8-9).
    constexpr int64_t kAhead = 16;
    for (int64_t i = 0; i < std::min(n, kAhead); ++i) __builtin_prefetch(host_base + off[i]);
    for (int64_t i = 0; i < n; ++i) {
        if (i + kAhead < n) __builtin_prefetch(host_base + off[i + kAhead]);
        int r;
        if (len[i] < 0 || len[i] + 100 >= kBufLen) {
            r = -1;  // the reference asserts len + 100 < buf_len (:471)
        } else {
            const uint64_t dsrc = dev_base ? (uint64_t)(uintptr_t)(dev_base + off[i]) + 8 : 0;
            r = input_packet(D, host_base + off[i], len[i], dsrc, (int32_t)i, now_ms);
        }
        if (ret) ret[i] = r;
    }
    const auto t1 = std::chrono::steady_clock::now();
    // staging layout per bucket: rows x n shards x stride, present flags rows x n
    int64_t so = 0, po = 0;
    for (Bucket &B : D->B->buckets) {
        B.stride = (B.len + 127) & ~127;
        B.staging_off = so;
        B.present_off = po;
        so += B.rows * B.n * B.stride;
        po += (B.rows * B.n + 15) & ~int64_t(15);
    }
    D->B->staging_bytes = so;
    D->B->present.assign((size_t)po, 0);
    D->B->gather_ref.clear();
    for (GatherCopy &G : D->B->gathers) {
        const Job &J = D->B->jobs[(size_t)(G.dst >> 8)];
        const int idx = (int)(G.dst & 0xff);
        D->B->gather_ref.push_back({(int64_t)(G.dst >> 8), idx});
        const Bucket &B = D->B->buckets[(size_t)J.bucket];
        G.dst = (uint64_t)(B.staging_off + (J.row * B.n + idx) * B.stride);  // offset; based at run time
        G.dst_len = (uint32_t)B.stride;
        D->B->present[(size_t)(B.present_off + J.row * B.n + idx)] = 1;
    }
    const auto t2 = std::chrono::steady_clock::now();
    // live shards of the batch move to the carry area, at their ring slot (:587)
    for (int sidx = 0; sidx < D->buff_num; ++sidx) {
        RingEnt &r = D->ring[(size_t)sidx];
        if (!r.used || !r.in_batch) continue;
        r.in_batch = false;
        const Group *g = D->find_group(r.seq);
        const bool live = g && !g->fec_done;
        const uint64_t dst = rsmi::kCarryTag | (uint64_t)sidx * kRingBytes;
        if (live && r.len > 0) D->B->carries.push_back(CarryCopy{r.src, dst, (uint32_t)r.len, 0});
        r.src = dst;
        r.host = nullptr;
    }
    for (auto &jr : D->B->d2h_rows) {  // byte offsets of the rows and blobs copied back
        Job &J = D->B->jobs[(size_t)jr.first];
        if (jr.second < 0) {
            J.lin = D->B->d2h_bytes;
            D->B->d2h_bytes += ((int64_t)J.k * J.len + 15) & ~int64_t(15);
        } else {
            D->B->rows[(size_t)(J.rows0 + jr.second)].d2h = D->B->d2h_bytes;
            D->B->d2h_bytes += (J.len + 15) & ~15;
        }
    }
    if (prof) {
        const auto t3 = std::chrono::steady_clock::now();
        fprintf(stderr, "fdec plan: packets %.3f ms, gathers %.3f ms, carries %.3f ms (%lld packets, %zu jobs)\n",
                std::chrono::duration<double, std::milli>(t1 - t0).count(),
                std::chrono::duration<double, std::milli>(t2 - t1).count(),
                std::chrono::duration<double, std::milli>(t3 - t2).count(), (long long)n, D->B->jobs.size());
    }
    D->B->planned = true;
    D->B->ran = D->B->resolved = false;
    if (n_decodes) *n_decodes = (int64_t)D->B->jobs.size();
    return RSMI_OK;
}

}  // extern "C"

namespace {
// Bind the decoder to the current device and order stream s after its
// previous batch, which reads and writes the shared device buffers.
int bind_dec(rsmi_fdec *D, hipStream_t s) {
    int cur;
    if (hipGetDevice(&cur) != hipSuccess) return fail(RSMI_ERR_HIP, "fdec: no usable GPU");
    if (D->device < 0) {
        for (Batch &X : D->bat)
            if (hipEventCreateWithFlags(&X.done, hipEventDisableTiming) != hipSuccess)
                return fail(RSMI_ERR_HIP, "fdec: hipEventCreate");
        D->device = cur;
    } else if (cur != D->device) {
        return fail(RSMI_ERR_INVALID, "rsmi_fdec_run_dev on another device than the decoder's");
    }
    Batch &prev = D->bat[D->bi ^ 1];
    if (prev.in_flight && prev.stream != s && hipStreamWaitEvent(s, prev.ev(), 0) != hipSuccess)
        return fail(RSMI_ERR_HIP, "fdec: hipStreamWaitEvent");
    return RSMI_OK;
}
}  // namespace

extern "C" {

// The managers of a server's connections share nothing (connection.h:244-245),
// so rsmi_fdec_plan_many runs rsmi_fdec_plan for each on the pool of host
// threads (host_pool.cpp), as rsmi_fenc_plan_many does on the send side.
int rsmi_fdec_plan_many(rsmi_fdec *const *dec, int32_t n, const int64_t *pk0, const int32_t *len,
                        const uint64_t *off, const uint8_t *const *host_base,
                        const uint8_t *const *dev_base, int64_t now_ms, int32_t *ret,
                        int64_t *n_decodes, int32_t nthreads) {
    if (n < 0 || (n && (!dec || !pk0 || !host_base)))
        return fail(RSMI_ERR_INVALID, "rsmi_fdec_plan_many: bad arguments");
    for (int i = 0; i < n; ++i) {
        if (!dec[i] || pk0[i + 1] < pk0[i]) return fail(RSMI_ERR_INVALID, "rsmi_fdec_plan_many: bad decoder or range");
        for (int j = 0; j < i; ++j)
            if (dec[j] == dec[i]) return fail(RSMI_ERR_INVALID, "rsmi_fdec_plan_many: a decoder listed twice");
    }
    std::vector<int> rcs((size_t)n, RSMI_OK);
    std::vector<std::string> errs((size_t)n);
    rsmi::host_parallel_for(n, nthreads > 0 ? nthreads : 8, [&](int i) {
        const int64_t a = pk0[i], cnt = pk0[i + 1] - pk0[i];
        int64_t nd = 0;
        const int rc = rsmi_fdec_plan(dec[i], cnt, len ? len + a : nullptr, off ? off + a : nullptr, host_base[i],
                                      dev_base ? dev_base[i] : nullptr, now_ms, ret ? ret + a : nullptr, &nd);
        rcs[(size_t)i] = rc;
        if (rc) {
            errs[(size_t)i] = rsmi::last_error();
            return;
        }
        if (n_decodes) n_decodes[i] = nd;
    });
    for (int i = 0; i < n; ++i)
        if (rcs[(size_t)i]) return fail(rcs[(size_t)i], "decoder " + std::to_string(i) + ": " + errs[(size_t)i]);
    return RSMI_OK;
}

int rsmi_fdec_run_dev(rsmi_fdec *D, void *stream) {
    if (!D || !D->B->planned) return fail(RSMI_ERR_INVALID, "rsmi_fdec_run_dev without a plan");
    if (D->plan_only) return fail(RSMI_ERR_INVALID, "rsmi_fdec_run_dev on a plan-only decoder");
    hipStream_t s = (hipStream_t)stream;
    static const bool prof = env_int("RSMI_FDEC_PROFILE", 0) != 0;
    const auto t0 = std::chrono::steady_clock::now();
    int rc0 = bind_dec(D, s);
    if (rc0) return rc0;
    Batch &prev = D->bat[D->bi ^ 1];
    int64_t max_rows = 0;
    for (const Bucket &B : D->B->buckets) max_rows = std::max(max_rows, B.rows);
    if ((size_t)D->buff_num * kRingBytes > D->dcarry_cap || (size_t)D->B->staging_bytes + 16 > D->stage_cap ||
        (size_t)D->B->d2h_bytes + 16 > D->blob_cap || (size_t)max_rows * 4 + 16 > D->status_cap) {
        int rcw = wait_batch(prev);
        if (rcw) return rcw;
    }
    int rc = dev_grow(&D->dcarry, &D->dcarry_cap, (size_t)D->buff_num * kRingBytes);
    if (!rc) rc = dev_grow(&D->dstage, &D->stage_cap, (size_t)D->B->staging_bytes + 16);
    if (!rc) rc = dev_grow(&D->dblob, &D->blob_cap, (size_t)D->B->d2h_bytes + 16);
    if (!rc) rc = host_grow(&D->B->hblob, &D->B->hblob_cap, (size_t)D->B->d2h_bytes + 16);
    if (!rc) rc = dev_grow(&D->dstatus, &D->status_cap, (size_t)max_rows * 4 + 16);
    if (rc) return rc;
    const auto ta = std::chrono::steady_clock::now();
    // metadata: gathers | present | row copies back | carries, one upload
    std::vector<JoinCopy> packs(D->B->d2h_rows.size());
    for (size_t j = 0; j < D->B->d2h_rows.size(); ++j) {
        const int i = D->B->d2h_rows[j].second;
        const Job &J = D->B->jobs[(size_t)D->B->d2h_rows[j].first];
        const Bucket &B = D->B->buckets[(size_t)J.bucket];
        const uint8_t *row = D->dstage + B.staging_off + (J.row * B.n + std::max(i, 0)) * B.stride;
        const int64_t at = i < 0 ? J.lin : D->B->rows[(size_t)(J.rows0 + i)].d2h;
        packs[j] = JoinCopy{(uint64_t)(uintptr_t)row, (uint64_t)(uintptr_t)(D->dblob + at), (uint32_t)J.len,
                            i < 0 ? (uint32_t)J.k : 1u, (uint32_t)B.stride, 0};
    }
    const size_t gb = D->B->gathers.size() * sizeof(GatherCopy), pb = D->B->present.size(),
                 kb = packs.size() * sizeof(JoinCopy), cb = D->B->carries.size() * sizeof(CarryCopy);
    const size_t go = 0, po = (gb + 255) & ~size_t(255), ko = (po + pb + 255) & ~size_t(255),
                 co = (ko + kb + 255) & ~size_t(255), all = co + cb + 16;
    if (all > D->meta_cap) {
        int rcw = wait_batch(prev);
        if (rcw) return rcw;
    }
    rc = dev_grow(&D->dmeta, &D->meta_cap, all);
    if (!rc) rc = host_grow(&D->B->hmeta, &D->B->hmeta_cap, all);
    if (rc) return rc;
    const auto tb = std::chrono::steady_clock::now();
    GatherCopy *hg = reinterpret_cast<GatherCopy *>(D->B->hmeta + go);
    for (size_t i = 0; i < D->B->gathers.size(); ++i) {
        hg[i] = D->B->gathers[i];
        hg[i].dst += (uint64_t)(uintptr_t)D->dstage;
    }
    if (pb) std::memcpy(D->B->hmeta + po, D->B->present.data(), pb);
    if (kb) std::memcpy(D->B->hmeta + ko, packs.data(), kb);
    if (cb) std::memcpy(D->B->hmeta + co, D->B->carries.data(), cb);
    const rsmi::CarryBase carry{{D->dcarry, D->dcarry}};
    const auto t1 = std::chrono::steady_clock::now();
    hipError_t e = hipMemcpyAsync(D->dmeta, D->B->hmeta, all, hipMemcpyHostToDevice, s);
    const auto t2 = std::chrono::steady_clock::now();
    if (e == hipSuccess)
        e = rsmi::launch_gather(reinterpret_cast<const GatherCopy *>(D->dmeta + go),
                                (int64_t)D->B->gathers.size(), carry, s);
    if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("fdec gather: ") + hipGetErrorString(e));
    for (const Bucket &B : D->B->buckets) {
        if (B.len == 0) continue;  // empty shards: nothing to rebuild
        rc = rsmi_decode_dev(B.k, B.n, D->dstage + B.staging_off, (int64_t)B.n * B.stride, B.stride,
                             B.len, B.rows, D->dmeta + po + B.present_off, D->dstatus, stream);
        if (rc) return rc;
    }
    e = rsmi::launch_join(reinterpret_cast<const JoinCopy *>(D->dmeta + ko), (int64_t)packs.size(), s);
    if (e == hipSuccess)
        e = rsmi::launch_carry(reinterpret_cast<const CarryCopy *>(D->dmeta + co),
                               (int64_t)D->B->carries.size(), carry, s);
    const auto t3 = std::chrono::steady_clock::now();
    if (e == hipSuccess && D->B->d2h_bytes)
        e = hipMemcpyAsync(D->B->hblob, D->dblob, (size_t)D->B->d2h_bytes, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipEventRecord(D->B->done, s);
    if (prof) {
        const auto t4 = std::chrono::steady_clock::now();
        auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
            return std::chrono::duration<double, std::milli>(b - a).count();
        };
        fprintf(stderr, "fdec run: buffers %.3f ms, packs %.3f ms, meta %.3f ms, upload %.3f ms, kernels %.3f ms, copy back %.3f ms (%zu B up, %lld B back)\n",
                ms(t0, ta), ms(ta, tb), ms(tb, t1), ms(t1, t2), ms(t2, t3), ms(t3, t4), all, (long long)D->B->d2h_bytes);
    }
    D->B->ext.reset();
    D->B->hblob_view = nullptr;
    D->B->view_gen_src.reset();
    D->B->stream = s;
    if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("fdec run: ") + hipGetErrorString(e));
    D->B->in_flight = true;
    D->B->planned = false;
    D->B->ran = true;
    return RSMI_OK;
}

int rsmi_fdec_outputs(rsmi_fdec *D, int64_t *n_out) {
    if (!D) return fail(RSMI_ERR_INVALID, "null decoder");
    // the older batch first: it ran, and batch i+1 may have been planned since
    const int xi = (D->bat[D->bi ^ 1].ran && !D->bat[D->bi ^ 1].resolved) ? (D->bi ^ 1) : D->bi;
    Batch &X = D->bat[xi];
    if (X.view_stale())
        return fail(RSMI_ERR_INVALID, "rsmi_fdec_outputs: this decoder's rows were in a collector set that "
                                      "has been reused or destroyed since (read outputs before the "
                                      "collector's second next rsmi_fdec_run_many)");
    if (!X.resolved) {
        bool any_job = !X.jobs.empty();
        if (any_job && !X.ran) return fail(RSMI_ERR_INVALID, "rsmi_fdec_outputs before rsmi_fdec_run_dev");
        static const bool prof = env_int("RSMI_FDEC_PROFILE", 0) != 0;
        const auto t0 = std::chrono::steady_clock::now();
        int rc = wait_batch(X);
        if (rc) return rc;
        const auto t1 = std::chrono::steady_clock::now();
        const size_t N = X.outs.size();
        // work ~ records, not groups: a mode-0 group yields up to k records
        size_t work = N;
        for (const Job &J : X.jobs) work += (size_t)J.k;
        int T = work >= (size_t)env_int("RSMI_FDEC_PAR_MIN", 4096) ? host_threads() : 1;
        if (T > (int)N) T = N ? (int)N : 1;
        if ((int)X.spills.size() < T) X.spills.resize((size_t)T);
        std::vector<Out> res;
        if (T == 1) {
            res.reserve(N * 2);
            resolve_outputs(X, 0, N, X.spills[0], res);
        } else {  // groups resolve independently: T contiguous ranges, joined in order
            std::vector<std::vector<Out>> part((size_t)T);
            const std::function<void(int)> range = [&X, N, T, &part](int t) {
                resolve_outputs(X, N * t / T, N * (t + 1) / T, X.spills[(size_t)t], part[(size_t)t]);
            };
            if (!ResolvePool::get().try_run(T, range))
                for (int t = 0; t < T; ++t) range(t);  // pool busy: this thread alone
            size_t tot = 0;
            for (auto &v : part) tot += v.size();
            res.reserve(tot);
            for (auto &v : part) res.insert(res.end(), v.begin(), v.end());
        }
        X.outs.swap(res);
        X.resolved = true;
        if (prof) {
            const auto t2 = std::chrono::steady_clock::now();
            fprintf(stderr, "fdec outputs: wait %.3f ms, resolve %.3f ms (%zu records, %d threads)\n",
                    std::chrono::duration<double, std::milli>(t1 - t0).count(),
                    std::chrono::duration<double, std::milli>(t2 - t1).count(), X.outs.size(), T);
        }
    }
    D->out_b = xi;
    if (n_out) *n_out = (int64_t)X.outs.size();
    return RSMI_OK;
}

int rsmi_fdec_output_list(const rsmi_fdec *D, const uint8_t **ptr, int32_t *len, int32_t *event) {
    if (!D || D->out_b < 0 || !D->bat[D->out_b].resolved)
        return fail(RSMI_ERR_INVALID, "call rsmi_fdec_outputs first");
    const Batch &X = D->bat[D->out_b];
    if (X.view_stale())
        return fail(RSMI_ERR_INVALID, "rsmi_fdec_output_list: the collector set holding these outputs has been "
                                      "reused or destroyed since rsmi_fdec_outputs");
    for (size_t i = 0; i < X.outs.size(); ++i) {
        if (ptr) ptr[i] = X.outs[i].ptr;
        if (len) len[i] = X.outs[i].len;
        if (event) event[i] = X.outs[i].event;
    }
    return RSMI_OK;
}

}  // extern "C"

// ---- the receive-side collector: many decoders' planned batches in one set --
//
// The counterpart of rsmi_fenc_run_many (fec_enc.cpp): each connection's
// fec_decode_manager_t (connection.h:244-245) plans its received packets on
// its own state; rsmi_fdec_run_many then runs their byte work together: one
// gather over every decoder's shards into a shared staging area bucketed by
// (k, n) across decoders, one decode per (k, n) code, one pass that packs the
// rows each decoder copies back and one that moves their carries, then each
// decoder's rows to its own pinned buffer.  A bucket's shard length is the
// longest of its decoders' (column-wise code: a group's rebuilt bytes below
// its own length do not depend on the bytes past it).  Carry-tagged addresses
// resolve to each decoder's own ring.
struct rsmi_fdcol {
    int device = -1;
    uint8_t *dstage = nullptr, *dmeta = nullptr;
    size_t stage_cap = 0, meta_cap = 0;
    int32_t *dstatus = nullptr;
    size_t status_cap = 0;
    uint8_t *hmeta[2] = {nullptr, nullptr};
    size_t hmeta_cap[2] = {0, 0};
    std::shared_ptr<rsmi::SharedEv> done[2];  // also the decoders' batches' event (Batch::ext)
    bool in_flight[2] = {false, false};
    int cur = 0;
    // every decoder's rows, packed on the device and copied back in one piece
    // (per set: a decoder's outputs point into the set it ran in)
    uint8_t *dback = nullptr, *hback[2] = {nullptr, nullptr};
    size_t dback_cap = 0, hback_cap[2] = {0, 0};
    // per set: bumped whenever the set's hback is about to be rewritten (and
    // at destroy), so decoders still pointing into it can tell
    std::shared_ptr<std::atomic<uint64_t>> gen[2] = {std::make_shared<std::atomic<uint64_t>>(0),
                                                     std::make_shared<std::atomic<uint64_t>>(0)};
};

extern "C" {

int rsmi_fdcol_create(rsmi_fdcol **out) {
    if (!out) return fail(RSMI_ERR_INVALID, "null out");
    *out = new rsmi_fdcol();
    return RSMI_OK;
}

void rsmi_fdcol_destroy(rsmi_fdcol *C) {
    if (!C) return;
    for (int i = 0; i < 2; ++i) {
        if (C->in_flight[i] && C->done[i]) (void)hipEventSynchronize(C->done[i]->ev);
        C->done[i].reset();  // (destroyed once no decoder's batch holds it)
        if (C->hmeta[i]) (void)hipHostFree(C->hmeta[i]);
        if (C->hback[i]) (void)hipHostFree(C->hback[i]);
        C->gen[i]->fetch_add(1);  // any decoder's view into this set is gone
    }
    for (uint8_t *p : {C->dstage, C->dmeta, C->dback}) if (p) (void)hipFree(p);
    if (C->dstatus) (void)hipFree(C->dstatus);
    delete C;
}

int rsmi_fdec_run_many(rsmi_fdcol *C, rsmi_fdec *const *dec, int32_t n, void *stream) {
    if (!C || n < 0 || (n && !dec)) return fail(RSMI_ERR_INVALID, "rsmi_fdec_run_many: bad arguments");
    for (int i = 0; i < n; ++i) {
        const rsmi_fdec *D = dec[i];
        if (!D || !D->B->planned) return fail(RSMI_ERR_INVALID, "rsmi_fdec_run_many: decoder without a plan");
        if (D->plan_only) return fail(RSMI_ERR_INVALID, "rsmi_fdec_run_many: plan-only decoder");
        for (int j = 0; j < i; ++j)
            if (dec[j] == D) return fail(RSMI_ERR_INVALID, "rsmi_fdec_run_many: a decoder listed twice");
    }
    hipStream_t s = (hipStream_t)stream;
    int cur;
    if (hipGetDevice(&cur) != hipSuccess) return fail(RSMI_ERR_HIP, "fdcol: no usable GPU");
    if (C->device < 0) {
        for (auto &ev : C->done) {
            ev = std::make_shared<rsmi::SharedEv>();
            if (hipEventCreateWithFlags(&ev->ev, hipEventDisableTiming) != hipSuccess)
                return fail(RSMI_ERR_HIP, "fdcol: hipEventCreate");
        }
        C->device = cur;
    } else if (C->device != cur) {
        return fail(RSMI_ERR_INVALID, "rsmi_fdec_run_many on another device than the collector's");
    }
    // the shared staging / metadata buffers are rewritten: after the last call
    for (int i = 0; i < 2; ++i)
        if (C->in_flight[i]) {
            if (hipEventSynchronize(C->done[i]->ev) != hipSuccess) return fail(RSMI_ERR_HIP, "fdcol: wait");
            C->in_flight[i] = false;
        }
    for (int i = 0; i < n; ++i) {
        rsmi_fdec *D = dec[i];
        int rc = bind_dec(D, s);
        if (rc) return rc;
        Batch &prev = D->bat[D->bi ^ 1];
        if ((size_t)D->buff_num * kRingBytes > D->dcarry_cap || (size_t)D->B->d2h_bytes + 16 > D->blob_cap) {
            rc = wait_batch(prev);
            if (rc) return rc;
        }
        rc = dev_grow(&D->dcarry, &D->dcarry_cap, (size_t)D->buff_num * kRingBytes);
        if (rc) return rc;
    }
    // every decoder's rows back to back in the collector's buffers
    std::vector<int64_t> boff((size_t)n + 1, 0);
    for (int i = 0; i < n; ++i) boff[(size_t)i + 1] = boff[(size_t)i] + ((dec[i]->B->d2h_bytes + 255) & ~int64_t(255));
    // ---- shared buckets: (k, n) across decoders, rows appended decoder by decoder
    struct CB {
        int k, nn, len = 0;
        int64_t rows = 0, stride = 0, off = 0, poff = 0;
    };
    std::map<int, CB> cbs;
    std::vector<std::vector<int64_t>> rowbase((size_t)n);  // per decoder bucket: first shared row
    for (int i = 0; i < n; ++i) {
        const rsmi_fdec *D = dec[i];
        for (const Bucket &B : D->B->buckets) {
            CB &c = cbs.emplace(B.k * 257 + B.n, CB{B.k, B.n}).first->second;
            rowbase[(size_t)i].push_back(c.rows);
            c.rows += B.rows;
            c.len = std::max(c.len, B.len);
        }
    }
    int64_t so = 0, po = 0, max_rows = 0;
    for (auto &kv : cbs) {
        CB &c = kv.second;
        c.stride = (c.len + 127) & ~int64_t(127);
        c.off = so;
        c.poff = po;
        so += c.rows * c.nn * c.stride;
        po += (c.rows * c.nn + 15) & ~int64_t(15);
        max_rows = std::max(max_rows, c.rows);
    }
    int rc = dev_grow(&C->dstage, &C->stage_cap, (size_t)so + 16);
    if (!rc) rc = dev_grow(&C->dstatus, &C->status_cap, (size_t)max_rows * 4 + 16);
    if (!rc)  // (the previous calls' copies out of it were waited for above)
        rc = dev_grow(&C->dback, &C->dback_cap, (size_t)boff[(size_t)n] + 16);
    if (rc) return rc;
    std::vector<GatherCopy> gathers;
    std::vector<uint8_t> present((size_t)po, 0);
    std::vector<JoinCopy> packs;
    std::vector<CarryCopy> carries;
    auto resolve = [](const rsmi_fdec *D, uint64_t a) -> uint64_t {
        return (a & rsmi::kCarryTag) ? (uint64_t)(uintptr_t)D->dcarry + (a & rsmi::kCarryOff) : a;
    };
    auto shard_at = [&](const rsmi_fdec *D, size_t di, const Job &J, int idx) -> uint64_t {
        const Bucket &B = D->B->buckets[(size_t)J.bucket];
        const CB &c = cbs[B.k * 257 + B.n];
        const int64_t row = rowbase[di][(size_t)J.bucket] + J.row;
        return (uint64_t)(uintptr_t)C->dstage + (uint64_t)(c.off + (row * c.nn + idx) * c.stride);
    };
    for (int i = 0; i < n; ++i) {
        const rsmi_fdec *D = dec[i];
        const Batch &X = *D->B;
        for (size_t g = 0; g < X.gathers.size(); ++g) {
            const Job &J = X.jobs[(size_t)X.gather_ref[g].first];
            const int idx = X.gather_ref[g].second;
            const Bucket &B = X.buckets[(size_t)J.bucket];
            const CB &c = cbs[B.k * 257 + B.n];
            GatherCopy G = X.gathers[g];
            G.src = resolve(D, G.src);
            G.dst = shard_at(D, (size_t)i, J, idx);
            G.dst_len = (uint32_t)c.stride;
            gathers.push_back(G);
            present[(size_t)(c.poff + (rowbase[(size_t)i][(size_t)J.bucket] + J.row) * c.nn + idx)] = 1;
        }
        for (const auto &jr : X.d2h_rows) {
            const Job &J = X.jobs[(size_t)jr.first];
            const Bucket &B = X.buckets[(size_t)J.bucket];
            const int64_t at = jr.second < 0 ? J.lin : X.rows[(size_t)(J.rows0 + jr.second)].d2h;
            packs.push_back(JoinCopy{shard_at(D, (size_t)i, J, std::max(jr.second, 0)),
                                     (uint64_t)(uintptr_t)(C->dback + boff[(size_t)i] + at), (uint32_t)J.len,
                                     jr.second < 0 ? (uint32_t)J.k : 1u,
                                     (uint32_t)cbs[B.k * 257 + B.n].stride, 0});
        }
        for (const CarryCopy &cc : X.carries)
            carries.push_back(CarryCopy{resolve(D, cc.src), resolve(D, cc.dst), cc.len, 0});
    }
    const size_t gb = gathers.size() * sizeof(GatherCopy), pb = present.size(),
                 kb = packs.size() * sizeof(JoinCopy), cb = carries.size() * sizeof(CarryCopy);
    const size_t go = 0, pof = (gb + 255) & ~size_t(255), ko = (pof + pb + 255) & ~size_t(255),
                 co = (ko + kb + 255) & ~size_t(255), all = co + cb + 16;
    C->cur ^= 1;
    C->gen[C->cur]->fetch_add(1);  // the set's previous views end here
    rc = dev_grow(&C->dmeta, &C->meta_cap, all);
    if (!rc) rc = host_grow(&C->hmeta[C->cur], &C->hmeta_cap[C->cur], all);
    if (!rc) rc = host_grow(&C->hback[C->cur], &C->hback_cap[C->cur], (size_t)boff[(size_t)n] + 16);
    if (rc) return rc;
    uint8_t *hm = C->hmeta[C->cur];
    if (gb) std::memcpy(hm + go, gathers.data(), gb);
    if (pb) std::memcpy(hm + pof, present.data(), pb);
    if (kb) std::memcpy(hm + ko, packs.data(), kb);
    if (cb) std::memcpy(hm + co, carries.data(), cb);
    const rsmi::CarryBase none{{nullptr, nullptr}};  // every address is absolute
    hipError_t e = hipMemcpyAsync(C->dmeta, hm, all, hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
        e = rsmi::launch_gather(reinterpret_cast<const GatherCopy *>(C->dmeta + go), (int64_t)gathers.size(),
                                none, s);
    if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("fdcol gather: ") + hipGetErrorString(e));
    for (auto &kv : cbs) {
        const CB &c = kv.second;
        if (c.len == 0 || c.rows == 0) continue;
        rc = rsmi_decode_dev(c.k, c.nn, C->dstage + c.off, (int64_t)c.nn * c.stride, c.stride, c.len, c.rows,
                             C->dmeta + pof + c.poff, C->dstatus, stream);
        if (rc) return rc;
    }
    e = rsmi::launch_join(reinterpret_cast<const JoinCopy *>(C->dmeta + ko), (int64_t)packs.size(), s);
    if (e == hipSuccess)
        e = rsmi::launch_carry(reinterpret_cast<const CarryCopy *>(C->dmeta + co), (int64_t)carries.size(), none,
                               s);
    if (e == hipSuccess && boff[(size_t)n])  // one copy for every decoder's rows
        e = hipMemcpyAsync(C->hback[C->cur], C->dback, (size_t)boff[(size_t)n], hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipEventRecord(C->done[C->cur]->ev, s);
    if (e != hipSuccess) return fail(RSMI_ERR_HIP, std::string("fdcol run: ") + hipGetErrorString(e));
    C->in_flight[C->cur] = true;
    for (int i = 0; i < n; ++i) {  // one event for all (a record per decoder cost ~5 us each)
        rsmi_fdec *D = dec[i];
        D->B->hblob_view = C->hback[C->cur] + boff[(size_t)i];
        D->B->view_gen_src = C->gen[C->cur];
        D->B->view_gen = C->gen[C->cur]->load();
        D->B->ext = C->done[C->cur];
        D->B->stream = s;
        D->B->in_flight = true;
        D->B->planned = false;
        D->B->ran = true;
    }
    return RSMI_OK;
}

}  // extern "C"
