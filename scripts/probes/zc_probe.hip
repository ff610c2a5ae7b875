// zc_probe.hip -- measurement tool: how fast can a KERNEL read pinned host
// memory (zero-copy over PCIe) and write it, against the DMA engines
// (hipMemcpyAsync)?  Decides whether rsmi_decode_pinned can read only the k
// survivors straight from the caller's pinned buffer.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/zc zc_probe.hip && /tmp/zc
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

// rows of `row` bytes, every `stride` bytes of src, copied to dst (packed);
// one wave per row, 16 B per lane per load; AUX = buffer cache policy bits
template <int AUX_LD, int AUX_ST>
__global__ __launch_bounds__(256) void rows_copy(const uint8_t *src, uint8_t *dst, uint32_t nrows,
                                                 uint32_t row, uint32_t sstride, uint32_t dstride) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * 4;
    for (uint32_t r = blockIdx.x * 4 + (threadIdx.x >> 6); r < nrows; r += nw) {
        const uint32_t rr = __builtin_amdgcn_readfirstlane(r);
        auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src) + (uint64_t)rr * sstride, 0,
                                                    (int)row, 0x00020000);
        auto rd = __builtin_amdgcn_make_buffer_rsrc(dst + (uint64_t)rr * dstride, 0, (int)row, 0x00020000);
        for (uint32_t o = lane * 16; o < row; o += 1024) {
            u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, AUX_LD);
            __builtin_amdgcn_raw_buffer_store_b128(v, rd, o, 0, AUX_ST);
        }
    }
}

template <class F>
double time_ms(F f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) f();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    const uint32_t G = 65536, n = 30, k = 20, ss = 1280;
    const size_t bytes = (size_t)G * n * ss;  // 2.5 GB: C2's shards
    uint8_t *h = nullptr, *d = nullptr, *d2 = nullptr;
    CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    memset(h, 1, bytes);
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&d2, bytes));
    hipPointerAttribute_t at;
    CK(hipPointerGetAttributes(&at, h));
    printf("host ptr type %d device ptr %p == host %p\n", (int)at.type, at.devicePointer, (void *)h);
    const int reps = 5;
    // DMA references
    double t = time_ms([&] { (void)hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, 0); }, reps);
    printf("DMA H2D %.1f GB/s\n", bytes / t / 1e6);
    t = time_ms([&] { (void)hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, 0); }, reps);
    printf("DMA D2H %.1f GB/s\n", bytes / t / 1e6);
    // zero-copy: read k of every n rows of 1280 B (the survivors) from host into HBM
    const uint32_t nrows = G * k;
    for (int grid : {256, 1024, 4096}) {
        t = time_ms([&] { rows_copy<0, 0><<<grid, 256>>>(h, d, nrows, ss, ss * n / k * 1, ss); }, reps);
        printf("ZC read  plain     grid %5d: %.1f GB/s\n", grid, (double)nrows * ss / t / 1e6);
        t = time_ms([&] { rows_copy<3, 0><<<grid, 256>>>(h, d, nrows, ss, ss * n / k * 1, ss); }, reps);
        printf("ZC read  sc0|sc1   grid %5d: %.1f GB/s\n", grid, (double)nrows * ss / t / 1e6);
        t = time_ms([&] { rows_copy<2, 0><<<grid, 256>>>(h, d, nrows, ss, ss * n / k * 1, ss); }, reps);
        printf("ZC read  nt        grid %5d: %.1f GB/s\n", grid, (double)nrows * ss / t / 1e6);
        t = time_ms([&] { rows_copy<0, 0><<<grid, 256>>>(d, h, nrows, ss, ss, ss * n / k); }, reps);
        printf("ZC write plain     grid %5d: %.1f GB/s\n", grid, (double)nrows * ss / t / 1e6);
        t = time_ms([&] { rows_copy<0, 3><<<grid, 256>>>(d, h, nrows, ss, ss, ss * n / k); }, reps);
        printf("ZC write sc0|sc1   grid %5d: %.1f GB/s\n", grid, (double)nrows * ss / t / 1e6);
    }
    // correctness of a zero-copy read after the host rewrote the buffer
    memset(h, 7, bytes);
    rows_copy<3, 0><<<1024, 256>>>(h, d, 1024, ss, ss, ss);
    CK(hipDeviceSynchronize());
    uint8_t chk[64];
    CK(hipMemcpy(chk, d + 1000 * ss, 64, hipMemcpyDeviceToHost));
    printf("reread after host memset: %s\n", chk[0] == 7 && chk[63] == 7 ? "fresh" : "STALE");
    (void)hipFree(d);
    (void)hipFree(d2);
    (void)hipHostFree(h);
    return 0;
}
