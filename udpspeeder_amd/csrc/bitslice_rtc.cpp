// bitslice_rtc.cpp -- bit-sliced encoders for the codes that have no
// build-time network: the XOR network of fec_new(k,n)'s matrix
// (lib/fec.cpp:665-720) is emitted here, on the host, and compiled for gfx950
// with hipRTC in a background thread when the code is first made resident
// (rsmi_prepare_code / any entry point).  Until the code object is ready the
// encoders run the generic table kernel; both are bit-exact, so the switch is
// invisible in the output.  Code objects are cached on disk
// ($RSMI_RTC_CACHE, else $XDG_CACHE_HOME/rsmi, else ~/.cache/rsmi).
//
// Every code rs_from_str admits (x:y, x+y <= 255, fec_manager.h:40-136) can
// be compiled; codes with more than 10 parity rows take several passes over
// the input (8 accumulators per row, gen_bitslice.py row_blocks).  Codes
// whose k*m exceeds RSMI_RTC_MAX_COEFS (default 2048: ~25 s of compile) stay
// on the generic kernel.
//
// The emitter is a line-for-line twin of gen_bitslice.py's (the build-time
// generator); tests/test_bitslice_rtc.py checks that both print the same text.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <deque>
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
namespace {

#include "gen/bitslice_rtc_text.inc"  // kBsCoreText, kBsKernText (Makefile rule)

constexpr int kMaxRows = 10;  // gen_bitslice.MAX_ROWS
constexpr int kRing = 4;      // gen_bitslice.RING
constexpr int kSplitRows = 5;  // gen_bitslice.SPLIT_MAX_ROWS
constexpr int kMaxDev = 64;

// ---------------------------------------------------------------- emitter
struct Emitter {
    std::string out;
    int nxor = 0;
    void line(const std::string &ind, const std::string &s) {
        if (!out.empty()) out += '\n';
        out += ind;
        out += s;
    }
};

// bitmat(c)[u] as two 4-bit masks: lo = bits t<4 of row u, hi = bits t>=4
void bit_rows(uint8_t c, int lo[8], int hi[8]) {
    const GF &F = gf();
    uint8_t col[8];
    for (int t = 0; t < 8; ++t) col[t] = F.m(c, (uint8_t)(1u << t));
    for (int u = 0; u < 8; ++u) {
        lo[u] = hi[u] = 0;
        for (int t = 0; t < 4; ++t) {
            lo[u] |= ((col[t] >> u) & 1) << t;
            hi[u] |= ((col[t + 4] >> u) & 1) << t;
        }
    }
}

std::string S(long v) { return std::to_string(v); }

// Input shards j0..j1-1 through the raw-load ring into parity rows r0..r1-1
// (gen_bitslice.emit_shards).
template <class Wf>
void emit_shards(Emitter &E, Wf &w, int k, const uint8_t *par, int r0, int r1, int j0, int j1) {
    const int R = std::min(kRing, j1 - j0);
    {
        std::string s = "uint32_t ";
        for (int r = 0; r < R; ++r) s += (r ? ", rb" : "rb") + S(r) + "[8]";
        w(s + ";");
    }
    for (int r = 0; r < R; ++r) w("io.load(" + S(j0 + r) + ", rb" + S(r) + ");");
    std::vector<int> tlo((size_t)(r1 - r0) * 8), thi((size_t)(r1 - r0) * 8);
    for (int j = j0; j < j1; ++j) {
        w("{  // input shard " + S(j));
        w("    uint32_t (&p)[8] = rb" + S((j - j0) % R) + ";");
        w("    bs_transpose8(p);");
        std::vector<int> need_lo, need_hi;  // first-seen order (Python dict)
        bool seen_lo[16] = {}, seen_hi[16] = {};
        for (int i = r0; i < r1; ++i) {
            int lo[8], hi[8];
            bit_rows(par[(size_t)i * k + j], lo, hi);
            for (int u = 0; u < 8; ++u) {
                tlo[(size_t)(i - r0) * 8 + u] = lo[u];
                thi[(size_t)(i - r0) * 8 + u] = hi[u];
                if (lo[u] && !seen_lo[lo[u]]) { seen_lo[lo[u]] = true; need_lo.push_back(lo[u]); }
                if (hi[u] && !seen_hi[hi[u]]) { seen_hi[hi[u]] = true; need_hi.push_back(hi[u]); }
            }
        }
        // combination names: single planes are p[t]; multi-plane masks get a temp
        auto build = [&](std::vector<int> needed, int base, const char *tag,
                         std::string names[16]) {
            for (int t = 0; t < 4; ++t) names[1 << t] = "p[" + S(base + t) + "]";
            std::stable_sort(needed.begin(), needed.end(), [](int a, int b) {
                return __builtin_popcount(a) < __builtin_popcount(b);
            });
            // split off the highest plane; build the rest recursively
            std::function<std::string(int)> get = [&](int mm) -> std::string {
                if (!names[mm].empty()) return names[mm];
                int hb = 31 - __builtin_clz(mm);
                const std::string a = get(mm & ~(1 << hb));
                const std::string nm = std::string(tag) + S(mm);
                w("    const uint32_t " + nm + " = " + a + " ^ p[" + S(base + hb) + "];");
                E.nxor += 1;
                names[mm] = nm;
                return nm;
            };
            for (int mask : needed) get(mask);
        };
        std::string lo_names[16], hi_names[16];
        build(need_lo, 0, "l", lo_names);
        build(need_hi, 4, "h", hi_names);
        for (int i = r0; i < r1; ++i)
            for (int u = 0; u < 8; ++u) {
                const int lo = tlo[(size_t)(i - r0) * 8 + u], hi = thi[(size_t)(i - r0) * 8 + u];
                const std::string acc = "o" + S(i) + "_" + S(u);
                if (lo && hi) {
                    w("    BS_ACC3(" + acc + ", " + lo_names[lo] + ", " + hi_names[hi] + ");");
                    E.nxor += 1;
                } else if (lo || hi) {
                    w("    BS_ACC2(" + acc + ", " + (lo ? lo_names[lo] : hi_names[hi]) + ");");
                    E.nxor += 1;
                }
            }
        if (j + R < j1) w("    io.load(" + S(j + R) + ", rb" + S((j - j0) % R) + ");");
        w("}");
        w("BS_SCHED_BARRIER();");
    }
}

std::string row_list(int i) {
    std::string s;
    for (int u = 0; u < 8; ++u) s += (u ? ", o" : "o") + S(i) + "_" + S(u);
    return s;
}

template <class Wf>
void emit_acc_decl(Wf &w, int r0, int r1) {
    for (int i = r0; i < r1; ++i) {
        std::string s = "uint32_t ";
        for (int u = 0; u < 8; ++u) s += (u ? ", o" : "o") + S(i) + "_" + S(u) + " = 0";
        w(s + ";");
    }
}

template <class Wf>
void emit_store(Wf &w, int k, int i) {
    w("{");
    w("    uint32_t q[8] = {" + row_list(i) + "};");
    w("    bs_transpose8(q);");
    w("    io.store(" + S(k + i) + ", q);");
    w("}");
}

void emit_block(Emitter &E, const std::string &ind, int k, const uint8_t *par, int r0, int r1) {
    auto w = [&](const std::string &s) { E.line(ind, s); };
    emit_acc_decl(w, r0, r1);
    emit_shards(E, w, k, par, r0, r1, 0, k);
    for (int i = r0; i < r1; ++i) emit_store(w, k, i);
}

}  // namespace

// Text of bs_code_<k>_<n> exactly as gen_bitslice.emit_code prints it.
bool bitslice_emit(int k, int n, std::string &src, int *nxor) {
    std::vector<uint8_t> enc;
    if (n <= k || !build_enc_matrix(k, n, enc)) return false;
    const int m = n - k;
    const uint8_t *par = enc.data() + (size_t)k * k;
    const int nb = std::max(1, (m + kMaxRows - 1) / kMaxRows);
    const int bs = (m + nb - 1) / nb;
    std::vector<std::pair<int, int>> blocks;
    for (int b = 0; b < nb; ++b)
        if (b * bs < m) blocks.push_back({b * bs, std::min(m, (b + 1) * bs)});
    Emitter E;
    E.line("", "// RS(k=" + S(k) + ", n=" + S(n) + "): " + S(8 * m) + " output planes <- " +
                   S(8 * k) + " input planes");
    E.line("", "template <class IO>");
    E.line("", "__host__ __device__ __forceinline__ void bs_code_" + S(k) + "_" + S(n) +
                   "(IO &io) {");
    const bool multi = blocks.size() > 1;
    for (auto &b : blocks) {
        if (multi) E.line("", "    {  // parity rows " + S(b.first) + ".." + S(b.second - 1));
        emit_block(E, multi ? "        " : "    ", k, par, b.first, b.second);
        if (multi) {
            E.line("", "    }");
            E.line("", "    BS_SCHED_BARRIER();");
        }
    }
    E.line("", "}  // " + S(E.nxor) + " XOR ops");
    src.swap(E.out);
    if (nxor) *nxor = E.nxor;
    return true;
}

// gen_bitslice.split_ok: codes that get the two-wave split-k form
bool bitslice_split_ok(int k, int n) {
    const int m = n - k;
    return k >= 10 && m >= 2 && m <= 2 * kSplitRows;
}

// Text of bs_split_<k>_<n> exactly as gen_bitslice.emit_split prints it.
bool bitslice_emit_split(int k, int n, std::string &src) {
    std::vector<uint8_t> enc;
    if (!bitslice_split_ok(k, n) || !build_enc_matrix(k, n, enc)) return false;
    const int m = n - k, ka = (k + 1) / 2, mh = (m + 1) / 2;
    const uint8_t *par = enc.data() + (size_t)k * k;
    Emitter E;
    E.line("", "// RS(k=" + S(k) + ", n=" + S(n) + ") split-k: shards 0.." + S(ka - 1) + " | " +
                   S(ka) + ".." + S(k - 1) + ", rows 0.." + S(mh - 1) + " | " + S(mh) + ".." +
                   S(m - 1));
    E.line("", "template <class IO, class XCH>");
    E.line("", "__device__ __forceinline__ void bs_split_" + S(k) + "_" + S(n) +
                   "(IO &io, uint32_t h, XCH &x) {");
    for (int h = 0; h < 2; ++h) {
        const int j0 = h ? ka : 0, j1 = h ? k : ka;
        const int own0 = h ? mh : 0, own1 = h ? m : mh, oth0 = h ? 0 : mh, oth1 = h ? mh : m;
        E.line("", h == 0 ? "    if (h == 0) {" : "    } else {");
        auto w = [&](const std::string &s) { E.line("        ", s); };
        emit_acc_decl(w, 0, m);
        emit_shards(E, w, k, par, 0, m, j0, j1);
        for (int i = oth0; i < oth1; ++i) w("x.send(" + S(i - oth0) + ", " + row_list(i) + ");");
        w("x.sync();");
        for (int i = own0; i < own1; ++i) w("x.recv(" + S(i - own0) + ", " + row_list(i) + ");");
        for (int i = own0; i < own1; ++i) emit_store(w, k, i);
    }
    E.line("", "    }");
    E.line("", "}  // " + S(E.nxor) + " XOR ops + " + S(8 * m) + " exchange XORs");
    src.swap(E.out);
    return true;
}

namespace {

// ---------------------------------------------------------------- registry
enum : int { kIdle = 0, kBusy = 1, kReady = 2, kFailed = 3 };

struct Unit {  // one hipRTC program: one code (so an exit waits for one compile at most)
    std::vector<std::pair<int, int>> codes;
    // set by whoever compiles the unit (a pool worker, or a thread that waits
    // for its code before a worker took it), or by the shutdown that drops it
    std::atomic<bool> claimed{false};
    std::vector<char> co;  // code object
    std::mutex mu;         // guards mod[]
    hipModule_t mod[kMaxDev] = {};
    bool load_failed[kMaxDev] = {};
};

struct RtcCode {
    std::atomic<int> state{kIdle};
    std::shared_ptr<Unit> unit;
    std::string err;
    std::atomic<hipFunction_t> fu[kMaxDev], fr[kMaxDev], fs[kMaxDev];
    RtcCode() {
        for (int d = 0; d < kMaxDev; ++d) {
            fu[d].store(nullptr);
            fr[d].store(nullptr);
            fs[d].store(nullptr);
        }
    }
};

struct Registry {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::shared_ptr<Unit>> queue;  // units no one has claimed yet
    int workers = 0;  // pool threads alive
    int running = 0;  // threads inside compile_unit (pool workers and waiting callers)
    bool atexit_set = false;
    bool exiting = false;  // rsmi_rtc_shutdown ran: nothing new enters hipRTC
    std::atomic<RtcCode *> table[257 * 257];
    Registry() {
        for (auto &t : table) t.store(nullptr);
    }
};

Registry &reg() {
    static Registry *r = new Registry();  // never destroyed: threads may outlive main's statics
    return *r;
}

bool env_off(const char *name) {
    const char *v = getenv(name);
    return v && (!strcmp(v, "0") || !strcmp(v, "off"));
}

long max_coefs() {
    const char *v = getenv("RSMI_RTC_MAX_COEFS");
    return v && *v ? atol(v) : 2048;
}

std::string cache_dir() {
    const char *v = getenv("RSMI_RTC_CACHE");
    if (v && (!strcmp(v, "0") || !strcmp(v, "off"))) return "";
    if (v && *v) return v;
    const char *x = getenv("XDG_CACHE_HOME");
    if (x && *x) return std::string(x) + "/rsmi";
    const char *h = getenv("HOME");
    if (h && *h) return std::string(h) + "/.cache/rsmi";
    return "";
}

uint64_t fnv1a(const std::string &s, uint64_t h = 1469598103934665603ull) {
    for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
    return h;
}

void mkdirs(const std::string &d) {
    for (size_t i = 1; i <= d.size(); ++i)
        if (i == d.size() || d[i] == '/') mkdir(d.substr(0, i).c_str(), 0755);
}

bool read_file(const std::string &p, std::vector<char> &out) {
    FILE *f = fopen(p.c_str(), "rb");
    if (!f) return false;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    out.resize(sz > 0 ? (size_t)sz : 0);
    const bool ok = sz > 0 && fread(out.data(), 1, (size_t)sz, f) == (size_t)sz;
    fclose(f);
    return ok;
}

void write_file_atomic(const std::string &p, const std::vector<char> &data) {
    const std::string tmp = p + ".tmp" + std::to_string((long)getpid());
    FILE *f = fopen(tmp.c_str(), "wb");
    if (!f) return;
    const bool ok = fwrite(data.data(), 1, data.size(), f) == data.size();
    if (fclose(f) != 0 || !ok || rename(tmp.c_str(), p.c_str()) != 0) unlink(tmp.c_str());
}

const char *const kRtcOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};

#ifndef BS_RAG_XCD
#define BS_RAG_XCD 0  // bitslice_kern.hpp's default: the runtime-compiled ragged kernels must
                      // remap blocks exactly as the launcher (bitslice.hip) sizes the grid
#endif

std::string unit_source(const Unit &U) {
    std::string s =
        "typedef unsigned char uint8_t; typedef unsigned short uint16_t;\n"
        "typedef unsigned int uint32_t; typedef unsigned long uint64_t; typedef long int64_t;\n"
        "#define BS_RAG_XCD " + S(BS_RAG_XCD) + "\n";
    s += kBsCoreText;
    s += kBsKernText;
    for (auto &c : U.codes) {
        std::string src;
        bitslice_emit(c.first, c.second, src, nullptr);
        const std::string kn = S(c.first) + "_" + S(c.second);
        s += src;
        // multi-pass networks spill at 3 waves/SIMD (168 VGPRs): sized for 2
        const std::string occ = c.second - c.first > kMaxRows ? "2" : "3";
        s += "\nextern \"C\" BS_DEFINE_UNIFORM(rsmi_bs_u_" + kn + ", bs_code_" + kn + ", " + occ +
             ")\n";
        s += "extern \"C\" BS_DEFINE_RAGGED_ONE(rsmi_bs_r_" + kn + ", bs_code_" + kn + ", " + occ +
             ")\n";
        if (bitslice_emit_split(c.first, c.second, src)) {
            s += src;
            s += "\nextern \"C\" BS_DEFINE_SPLIT(rsmi_bs_s_" + kn + ", bs_split_" + kn + ", 3)\n";
        }
    }
    return s;
}

// Compile (or fetch from the disk cache) one unit; runs on a worker thread.
bool compile_unit(Unit &U, std::string &err) {
    const std::string src = unit_source(U);
    int maj = 0, mnr = 0;
    hiprtcVersion(&maj, &mnr);
    std::string key = src;
    for (const char *o : kRtcOpts) key += o;
    key += "|" + S(maj) + "." + S(mnr);
    char hex[17];
    snprintf(hex, sizeof hex, "%016llx", (unsigned long long)fnv1a(key));
    const std::string dir = cache_dir();
    const std::string path = dir.empty() ? "" : dir + "/bs-" + hex + ".co";
    if (!path.empty() && read_file(path, U.co)) return true;
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "rsmi_bitslice_rtc.hip", 0, nullptr, nullptr) !=
        HIPRTC_SUCCESS) {
        err = "hiprtcCreateProgram failed";
        return false;
    }
    const hiprtcResult r = hiprtcCompileProgram(prog, 3, kRtcOpts);
    bool ok = r == HIPRTC_SUCCESS;
    if (!ok) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n, '\0');
        if (n) hiprtcGetProgramLog(prog, &log[0]);
        err = std::string("hiprtcCompileProgram: ") + hiprtcGetErrorString(r) + "\n" +
              log.substr(0, 2000);
    } else {
        size_t n = 0;
        ok = hiprtcGetCodeSize(prog, &n) == HIPRTC_SUCCESS && n > 0;
        if (ok) {
            U.co.resize(n);
            ok = hiprtcGetCode(prog, U.co.data()) == HIPRTC_SUCCESS;
        }
        if (!ok) err = "hiprtcGetCode failed";
    }
    hiprtcDestroyProgram(&prog);
    if (ok && !path.empty()) {
        mkdirs(dir);
        write_file_atomic(path, U.co);
    }
    return ok;
}

constexpr int kMaxCompileThreads = 4;

// Compiles U (the caller has claimed it and counted itself in R.running) and
// publishes its codes' state.
void compile_and_publish(Unit &U) {
    Registry &R = reg();
    std::string err;
    const bool ok = compile_unit(U, err);
    if (!ok && getenv("RSMI_RTC_VERBOSE")) fprintf(stderr, "rsmi: runtime bit-slice compile failed: %s\n", err.c_str());
    std::lock_guard<std::mutex> lk(R.mu);
    for (auto &c : U.codes) {
        RtcCode *rc = R.table[c.first * 257 + c.second].load();
        rc->err = err;
        rc->state.store(ok ? kReady : kFailed);
    }
    --R.running;
    R.cv.notify_all();
}

// A unit that will never compile: its codes stay on the generic kernel.
// Caller holds R.mu and has claimed U.
void drop_unit_locked(Registry &R, Unit &U, const char *why) {
    for (auto &c : U.codes) {
        RtcCode *rc = R.table[c.first * 257 + c.second].load();
        rc->err = why;
        rc->state.store(kFailed);
    }
}

// Pool thread: takes queued units until the queue is empty or shutdown began.
void worker() {
    Registry &R = reg();
    std::unique_lock<std::mutex> lk(R.mu);
    while (!R.exiting && !R.queue.empty()) {
        std::shared_ptr<Unit> U = R.queue.front();
        R.queue.pop_front();
        if (U->claimed.exchange(true)) continue;  // a waiting thread compiles it
        ++R.running;
        lk.unlock();
        compile_and_publish(*U);
        lk.lock();
    }
    --R.workers;
    R.cv.notify_all();
}

// Shutdown: nothing new enters hipRTC, queued units are dropped, and the call
// returns once every compile already inside hipRTC (at most kMaxCompileThreads
// pool workers plus any waiting callers, one code each) has left it.  It must
// run before comgr/LLVM (dlopen'ed by libhiprtc on first use, so registered
// AFTER any atexit handler of ours) runs its static destructors: an exit that
// tears LLVM down under a running compile crashes or hangs the process.
void shutdown_compiles_impl() {
    Registry &R = reg();
    std::unique_lock<std::mutex> lk(R.mu);
    R.exiting = true;
    for (auto &U : R.queue)
        if (!U->claimed.exchange(true)) drop_unit_locked(R, *U, "process exiting");
    R.queue.clear();
    R.cv.notify_all();
    R.cv.wait(lk, [&] { return R.running == 0; });
}

// The exit hooks, earliest first:
//  1. the Python binding registers rsmi_rtc_shutdown with Python's atexit
//     (before interpreter finalisation);
//  2. a thread_local guard on the main thread: glibc's exit() runs the exiting
//     thread's TLS destructors before ANY atexit/__cxa_atexit handler, so this
//     runs ahead of comgr's static destructors whatever the load order;
//  3. a plain atexit handler, in case exit() is called from another thread.
struct MainThreadExitGuard {
    ~MainThreadExitGuard() { shutdown_compiles_impl(); }
};

void arm_exit_hooks_locked(Registry &R) {
    if (R.atexit_set) return;
    R.atexit_set = true;
    atexit(shutdown_compiles_impl);
}

}  // namespace

void shutdown_compiles() { shutdown_compiles_impl(); }

// Touch the guard on the thread that loads the library (the main thread, for
// a Python import or a linked program) so its destructor is registered there.
__attribute__((constructor)) static void rsmi_rtc_arm_main_guard() {
    if ((pid_t)syscall(SYS_gettid) != getpid()) return;
    static thread_local MainThreadExitGuard guard;
    (void)&guard;
}

bool bitslice_rtc_eligible(int k, int n) {
    const int m = n - k;
    return k >= 1 && m >= 1 && n <= 256 && !has_bitslice(k, n) && (long)k * m <= max_coefs() &&
           !env_off("RSMI_RTC");
}

// Queue the codes that are eligible and not yet requested (smallest k*m
// first, one code per hipRTC program) for the kMaxCompileThreads pool threads,
// and return at once.
void bitslice_rtc_request(const std::vector<std::pair<int, int>> &codes) {
    Registry &R = reg();
    std::vector<std::pair<int, int>> todo;
    std::lock_guard<std::mutex> lk(R.mu);
    for (auto &c : codes) {
        if (!bitslice_rtc_eligible(c.first, c.second)) continue;
        auto &slot = R.table[c.first * 257 + c.second];
        if (slot.load()) continue;
        RtcCode *rc = new RtcCode();
        rc->state.store(kBusy);
        slot.store(rc);
        todo.push_back(c);
    }
    if (todo.empty()) return;
    arm_exit_hooks_locked(R);
    std::stable_sort(todo.begin(), todo.end(), [](const std::pair<int, int> &a, const std::pair<int, int> &b) {
        return (long)a.first * (a.second - a.first) < (long)b.first * (b.second - b.first);
    });
    for (auto &c : todo) {
        auto U = std::make_shared<Unit>();
        U->codes.push_back(c);
        RtcCode *rc = R.table[c.first * 257 + c.second].load();
        rc->unit = U;
        if (R.exiting) {
            U->claimed.store(true);
            drop_unit_locked(R, *U, "process exiting");
            continue;
        }
        R.queue.push_back(U);
    }
    while (R.workers < kMaxCompileThreads && R.workers < (int)R.queue.size()) {
        ++R.workers;
        std::thread(worker).detach();
    }
}

// Block until every listed code's compile has finished (ready or failed).  A
// code whose unit is still queued is compiled on the calling thread instead of
// waiting its turn.
void bitslice_rtc_wait(const std::vector<std::pair<int, int>> &codes) {
    Registry &R = reg();
    for (auto &c : codes) {
        std::shared_ptr<Unit> U;
        {
            std::lock_guard<std::mutex> lk(R.mu);
            RtcCode *rc = R.table[c.first * 257 + c.second].load();
            if (rc && rc->state.load() == kBusy && !R.exiting && !rc->unit->claimed.exchange(true)) {
                U = rc->unit;
                ++R.running;
            }
        }
        if (U) compile_and_publish(*U);
    }
    std::unique_lock<std::mutex> lk(R.mu);
    R.cv.wait(lk, [&] {
        for (auto &c : codes) {
            RtcCode *rc = R.table[c.first * 257 + c.second].load();
            if (rc && rc->state.load() == kBusy) return false;
        }
        return true;
    });
}

int bitslice_rtc_state(int k, int n) {
    if (k < 1 || n > 256 || k > n) return kIdle;
    RtcCode *rc = reg().table[k * 257 + n].load();
    return rc ? rc->state.load() : kIdle;
}

// The compiled kernel for (k,n) on the current device (module loaded on first
// use), or nullptr while the code is not ready.
hipFunction_t bitslice_rtc_function(int k, int n, RtcKind kind) {
    if (k < 1 || n > 256 || k >= n) return nullptr;
    if (kind == kRtcSplit && !bitslice_split_ok(k, n)) return nullptr;
    RtcCode *rc = reg().table[k * 257 + n].load();
    if (!rc || rc->state.load(std::memory_order_acquire) != kReady) return nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return nullptr;
    std::atomic<hipFunction_t> *slot = kind == kRtcRagged ? rc->fr : (kind == kRtcSplit ? rc->fs : rc->fu);
    hipFunction_t f = slot[dev].load(std::memory_order_acquire);
    if (f) return f;
    Unit &U = *rc->unit;
    std::lock_guard<std::mutex> lk(U.mu);
    if (U.load_failed[dev]) return nullptr;
    if (!U.mod[dev] && hipModuleLoadData(&U.mod[dev], U.co.data()) != hipSuccess) {
        U.mod[dev] = nullptr;
        U.load_failed[dev] = true;
        return nullptr;
    }
    const std::string kn = S(k) + "_" + S(n);
    hipFunction_t fu = nullptr, fr = nullptr, fs = nullptr;
    if (hipModuleGetFunction(&fu, U.mod[dev], ("rsmi_bs_u_" + kn).c_str()) != hipSuccess ||
        hipModuleGetFunction(&fr, U.mod[dev], ("rsmi_bs_r_" + kn).c_str()) != hipSuccess ||
        (bitslice_split_ok(k, n) &&
         hipModuleGetFunction(&fs, U.mod[dev], ("rsmi_bs_s_" + kn).c_str()) != hipSuccess)) {
        U.load_failed[dev] = true;
        return nullptr;
    }
    rc->fu[dev].store(fu, std::memory_order_release);
    rc->fr[dev].store(fr, std::memory_order_release);
    rc->fs[dev].store(fs, std::memory_order_release);
    return kind == kRtcRagged ? fr : (kind == kRtcSplit ? fs : fu);
}

std::string bitslice_rtc_error(int k, int n) {
    Registry &R = reg();
    std::lock_guard<std::mutex> lk(R.mu);
    RtcCode *rc = R.table[k * 257 + n].load();
    return rc ? rc->err : std::string();
}

int prepare_code(int k, int n);
void set_error(const std::string &m);

}  // namespace rsmi

extern "C" void rsmi_rtc_shutdown(void) { rsmi::shutdown_compiles(); }

extern "C" int rsmi_wait_code(int k, int n) {
    int rc = rsmi::prepare_code(k, n);
    if (rc) return rc;
    rsmi::bitslice_rtc_wait({{k, n}});
    // load the module on this device now, so a later graph capture never does
    if (rsmi::bitslice_rtc_state(k, n) == rsmi::kReady) (void)rsmi::bitslice_rtc_function(k, n, rsmi::kRtcUniform);
    return RSMI_OK;
}

extern "C" int rsmi_precompile_code(int k, int n) {
    if (k < 1 || n <= k || n > 256 || !rsmi::bitslice_rtc_eligible(k, n)) {
        rsmi::set_error("no run-time network for this (k,n): built-in, n == k, over "
                        "RSMI_RTC_MAX_COEFS, or RSMI_RTC=0");
        return RSMI_ERR_INVALID;
    }
    rsmi::bitslice_rtc_request({{k, n}});
    rsmi::bitslice_rtc_wait({{k, n}});
    if (rsmi::bitslice_rtc_state(k, n) != rsmi::kReady) {
        rsmi::set_error("run-time bit-slice compile failed: " + rsmi::bitslice_rtc_error(k, n));
        return RSMI_ERR_HIP;
    }
    return RSMI_OK;
}

extern "C" int rsmi_precompile_codes_async(const int32_t *k, const int32_t *n, int count) {
    if (count < 0 || (count && (!k || !n))) {
        rsmi::set_error("rsmi_precompile_codes_async: bad arrays");
        return RSMI_ERR_INVALID;
    }
    std::vector<std::pair<int, int>> codes;
    for (int i = 0; i < count; ++i)
        if (k[i] >= 1 && n[i] > k[i] && n[i] <= 256 && rsmi::bitslice_rtc_eligible(k[i], n[i]))
            codes.push_back({k[i], n[i]});
    rsmi::bitslice_rtc_request(codes);
    return (int)codes.size();
}

extern "C" int rsmi_code_encoder(int k, int n) {
    if (k < 1 || n < k || n > 256) return RSMI_ERR_INVALID;
    if (n == k) return RSMI_ENC_NONE;
    if (rsmi::has_bitslice(k, n)) return RSMI_ENC_BITSLICE;
    switch (rsmi::bitslice_rtc_state(k, n)) {
        case rsmi::kReady: return RSMI_ENC_BITSLICE_RTC;
        case rsmi::kBusy: return RSMI_ENC_COMPILING;
        default: return RSMI_ENC_GENERIC;
    }
}

extern "C" int64_t rsmi_bitslice_source(int k, int n, char *buf, int64_t cap) {
    std::string s;
    if (k < 1 || n <= k || n > 256 || !rsmi::bitslice_emit(k, n, s, nullptr)) return RSMI_ERR_INVALID;
    if (buf && cap > 0) {
        const size_t c = std::min<size_t>((size_t)cap - 1, s.size());
        memcpy(buf, s.data(), c);
        buf[c] = '\0';
    }
    return (int64_t)s.size();
}

extern "C" int64_t rsmi_bitslice_split_source(int k, int n, char *buf, int64_t cap) {
    std::string s;
    if (k < 1 || n <= k || n > 256 || !rsmi::bitslice_emit_split(k, n, s)) return RSMI_ERR_INVALID;
    if (buf && cap > 0) {
        const size_t c = std::min((size_t)(cap - 1), s.size());
        std::memcpy(buf, s.data(), c);
        buf[c] = 0;
    }
    return (int64_t)s.size();
}
