// Host harness: runs the GENERATED bit-sliced networks (gen/bitslice_codes.inc,
// the exact code the HIP kernels inline) on the CPU so tests/ can check them
// against the oracle without a GPU.  stdin: k n nchunks, then nchunks*k*32
// data bytes (chunk-major, shard-minor); stdout: nchunks*(n-k)*32 parity bytes.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define __host__
#define __device__
#define __forceinline__ inline
#define BS_ACC3(acc, a, b) ((acc) ^= (a) ^ (b))
#define BS_ACC2(acc, a) ((acc) ^= (a))
#define BS_SCHED_BARRIER() ((void)0)
#include "../udpspeeder_amd/csrc/bitslice_core.hpp"
#ifdef BS_HOST_INC
#include BS_HOST_INC  // run-time emitted networks (tests/test_bitslice_rtc.py)
#else
#include "../udpspeeder_amd/csrc/gen/bitslice_codes.inc"
#endif

struct HostIO {
    const uint8_t *in;  // k x 32
    uint8_t *out;       // m x 32
    int k;
    void load(int j, uint32_t (&p)[8]) const { std::memcpy(p, in + 32 * j, 32); }
    void store(int j, const uint32_t (&q)[8]) const { std::memcpy(out + 32 * (j - k), q, 32); }
};

int main() {
    int k, n;
    long nchunks;
    if (std::scanf("%d %d %ld", &k, &n, &nchunks) != 3) return 2;
    std::getchar();  // the newline after the header
    const int m = n - k;
    std::vector<uint8_t> in((size_t)nchunks * k * 32), out((size_t)nchunks * m * 32);
    if (std::fread(in.data(), 1, in.size(), stdin) != in.size()) return 3;
    for (long c = 0; c < nchunks; ++c) {
        HostIO io{in.data() + (size_t)c * k * 32, out.data() + (size_t)c * m * 32, k};
        switch (k * 257 + n) {
#define CASE(K, N) case K * 257 + N: bs_code_##K##_##N(io); break;
            BS_FOR_EACH_CODE(CASE)
#undef CASE
            default: return 4;
        }
    }
    std::fwrite(out.data(), 1, out.size(), stdout);
    return 0;
}
