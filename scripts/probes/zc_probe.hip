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
#include <algorithm>
#include <vector>

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

// one group's survivors (k rows of len bytes, packed) read from host memory by
// a whole workgroup, XOR-folded into one row, written to host memory: the shape
// of a one-group zero-copy decode
__global__ __launch_bounds__(256) void group_zc(const uint8_t *src, uint8_t *dst, int k, int len) {
    for (int o = threadIdx.x * 16; o < len; o += 256 * 16) {
        u32x4 acc = {0, 0, 0, 0};
        for (int j = 0; j < k; ++j) {
            auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src) + (size_t)j * len, 0,
                                                        len, 0x00020000);
            acc ^= __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 3);
        }
        auto rd = __builtin_amdgcn_make_buffer_rsrc(dst, 0, len, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(acc, rd, o, 0, 3);
    }
}

__global__ void empty_k() {}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

template <class F>
double lat_us(F f, int reps = 300) {
    for (int i = 0; i < 30; ++i) f();
    double best = 1e30, sum = 0;
    std::vector<double> v;
    for (int i = 0; i < reps; ++i) {
        double t0 = now_us();
        f();
        v.push_back(now_us() - t0);
    }
    std::sort(v.begin(), v.end());
    (void)best;
    (void)sum;
    return v[v.size() / 2];
}

int latency() {
    const int k = 20, len = 1280;
    uint8_t *hin, *hout, *din, *dout;
    CK(hipHostMalloc(&hin, k * len, hipHostMallocDefault));
    CK(hipHostMalloc(&hout, 8 * len, hipHostMallocDefault));
    CK(hipMalloc(&din, k * len));
    CK(hipMalloc(&dout, 8 * len));
    memset(hin, 3, k * len);
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    printf("latency (median us, one RS(20,10)-sized group):\n");
    printf("  empty kernel + stream sync            %.1f\n", lat_us([&] {
        empty_k<<<1, 64, 0, s>>>();
        (void)hipStreamSynchronize(s);
    }));
    printf("  H2D 25.6 KB + sync                    %.1f\n", lat_us([&] {
        (void)hipMemcpyAsync(din, hin, k * len, hipMemcpyHostToDevice, s);
        (void)hipStreamSynchronize(s);
    }));
    printf("  H2D 25.6K + kernel + D2H 4.3K + sync  %.1f\n", lat_us([&] {
        (void)hipMemcpyAsync(din, hin, k * len, hipMemcpyHostToDevice, s);
        group_zc<<<1, 256, 0, s>>>(din, dout, k, len);
        (void)hipMemcpyAsync(hout, dout, 4 * len, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
    }));
    printf("  zero-copy kernel (reads host 25.6K, writes host 1.3K) + sync %.1f\n", lat_us([&] {
        group_zc<<<1, 256, 0, s>>>(hin, hout, k, len);
        (void)hipStreamSynchronize(s);
    }));
    printf("  zero-copy kernel, one wave + sync     %.1f\n", lat_us([&] {
        group_zc<<<1, 64, 0, s>>>(hin, hout, k, len);
        (void)hipStreamSynchronize(s);
    }));
    return 0;
}

int main() {
    if (latency()) return 1;
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
