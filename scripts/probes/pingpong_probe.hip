// pingpong_probe.hip -- measurement tool: the latency floor of the drop-in's
// per-call path on this box.
//  A. launch: an empty-ish kernel that raises a flag in pinned host memory,
//     the host spinning on it (launch + one posted PCIe write).
//  B. ping-pong: a resident kernel polls a doorbell in pinned host memory and
//     answers each ping with a flag write; the host times ping -> pong.
//  C. a dependent chain of 64 system-scope loads of pinned host memory, timed
//     on the GPU with s_memrealtime (PCIe read round trip).
// Build: hipcc --offload-arch=gfx950 -O3 -o pingpong_probe pingpong_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

__device__ __forceinline__ uint32_t ld_sys(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_flag(uint32_t *flag, uint32_t v) {
    if (threadIdx.x == 0) st_sys(flag, v);
}

__global__ void k_pong(uint32_t *ctl, int rounds) {  // ctl[0] ping (host), ctl[1] pong (gpu)
    if (threadIdx.x != 0) return;
    uint32_t last = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int r = 0; r < rounds;) {
        const uint32_t p = ld_sys(ctl);
        if (p != last) {
            last = p;
            st_sys(ctl + 1, p);
            ++r;
        } else if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s bound
            break;
        }
    }
}

__global__ void k_chain(const uint32_t *h, uint64_t *out) {
    if (threadIdx.x != 0) return;
    uint32_t i = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int r = 0; r < 64; ++r) i = ld_sys(h + (i & 15));
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    out[0] = t1 - t0;
    out[1] = i;
}

int main() {
    uint32_t *h = nullptr, *d = nullptr;
    (void)hipHostMalloc((void **)&h, 4096, hipHostMallocDefault);
    (void)hipHostGetDevicePointer((void **)&d, h, 0);
    for (int i = 0; i < 1024; ++i) h[i] = 0;
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    volatile uint32_t *vh = h;
    // A
    std::vector<double> ta;
    for (uint32_t i = 1; i <= 300; ++i) {
        auto t0 = std::chrono::steady_clock::now();
        k_flag<<<1, 64, 0, s>>>(d + 2, i);
        while (vh[2] != i) __builtin_ia32_pause();
        ta.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(ta.begin() + 20, ta.end());
    printf("A launch + flag: median %.2f us, p10 %.2f, p90 %.2f\n", ta[20 + 140], ta[20 + 28], ta[20 + 252]);
    (void)hipStreamSynchronize(s);
    // B
    vh[0] = 0;
    vh[1] = 0;
    const int R = 2000;
    k_pong<<<1, 64, 0, s>>>(d, R);
    std::vector<double> tb;
    for (uint32_t i = 1; i <= (uint32_t)R; ++i) {
        auto t0 = std::chrono::steady_clock::now();
        vh[0] = i;
        auto lim = t0 + std::chrono::milliseconds(500);
        while (vh[1] != i && std::chrono::steady_clock::now() < lim) __builtin_ia32_pause();
        tb.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    (void)hipStreamSynchronize(s);
    std::sort(tb.begin() + 100, tb.end());
    const size_t nb = tb.size() - 100;
    printf("B ping-pong: median %.2f us, p10 %.2f, p90 %.2f\n", tb[100 + nb / 2], tb[100 + nb / 10],
           tb[100 + nb * 9 / 10]);
    // C
    uint64_t *o = nullptr;
    (void)hipMalloc((void **)&o, 16);
    uint64_t ho[2];
    for (int rep = 0; rep < 3; ++rep) {
        k_chain<<<1, 64, 0, s>>>(d, o);
        (void)hipMemcpy(ho, o, 16, hipMemcpyDeviceToHost);
        printf("C 64 dependent pinned-host loads: %.2f us each\n", ho[0] / 100.0 / 64.0);
    }
    return 0;
}
