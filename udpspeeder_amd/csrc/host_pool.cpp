// host_pool.cpp -- a small persistent pool of host threads for the planners'
// per-manager work (rsmi_fenc_plan_many / rsmi_fdec_plan_many): a flush plans
// every connection's manager, each on its own state, so they run in parallel.
// The calling thread takes items too; one parallel_for at a time.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "rsmi_internal.hpp"

namespace rsmi {
namespace {

struct Pool {
    std::mutex call_mu;  // one parallel_for at a time
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::vector<std::thread> th;
    const std::function<void(int)> *fn = nullptr;
    std::atomic<int> next{0};
    int n = 0, active = 0;
    uint64_t epoch = 0;
    bool quit = false;

    void work() {
        for (;;) {
            const int i = next.fetch_add(1);
            if (i >= n) break;
            (*fn)(i);
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return quit || epoch != seen; });
                if (quit) return;
                seen = epoch;
            }
            work();
            {
                std::lock_guard<std::mutex> lk(mu);
                --active;
            }
            done_cv.notify_all();
        }
    }
};

Pool &pool() {
    static Pool *p = new Pool();  // never destroyed: its threads may outlive static teardown
    return *p;
}

}  // namespace

void host_parallel_for(int n, int nthreads, const std::function<void(int)> &fn) {
    if (n <= 0) return;
    nthreads = std::max(1, std::min({nthreads, n, 64}));
    if (nthreads == 1) {
        for (int i = 0; i < n; ++i) fn(i);
        return;
    }
    Pool &P = pool();
    std::lock_guard<std::mutex> call(P.call_mu);
    {
        std::lock_guard<std::mutex> lk(P.mu);
        while ((int)P.th.size() < nthreads - 1) P.th.emplace_back([&P] { P.loop(); });
        P.fn = &fn;
        P.n = n;
        P.next.store(0);
        P.active = (int)P.th.size();
        ++P.epoch;
    }
    P.cv.notify_all();
    P.work();
    std::unique_lock<std::mutex> lk(P.mu);
    P.done_cv.wait(lk, [&] { return P.active == 0; });
    P.fn = nullptr;
}

}  // namespace rsmi
