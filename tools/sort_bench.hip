// Diagnostic: rocprim onesweep radix sort of u64 keys on a bit range, per config.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/sort_bench.hip -o build/sort_bench
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill(unsigned long long* k, size_t n, unsigned shift, unsigned long long seed) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned long long z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const unsigned long long code = (z >> 20) % 1801088541ull;
    k[i] = (code << shift) | (i & ((1ull << shift) - 1));
}

template <class Cfg>
void run(const char* name, unsigned long long* in, unsigned long long* out, size_t n, unsigned b0, unsigned b1) {
    size_t tb = 0;
    CK(rocprim::radix_sort_keys<Cfg>(nullptr, tb, in, out, n, b0, b1, 0));
    void* tmp;
    CK(hipMalloc(&tmp, tb));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 2; ++w) CK(rocprim::radix_sort_keys<Cfg>(tmp, tb, in, out, n, b0, b1, 0));
    const int reps = 10;
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) CK(rocprim::radix_sort_keys<Cfg>(tmp, tb, in, out, n, b0, b1, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    std::vector<unsigned long long> h(4096);
    CK(hipMemcpy(h.data(), out, 8 * h.size(), hipMemcpyDeviceToHost));
    bool ok = true;
    for (size_t i = 1; i < h.size(); ++i) ok &= (h[i - 1] >> b0) <= (h[i] >> b0);
    printf("%-28s n=%zu bits=[%u,%u) ms=%.3f  GB/s(16B/key)=%.0f ok=%d\n", name, n, b0, b1, ms, n * 16.0 / ms / 1e6, ok);
    CK(hipFree(tmp));
}

using namespace rocprim;
template <unsigned R, unsigned BS, unsigned IPT>
using OS = radix_sort_config<default_config, default_config,
                             radix_sort_onesweep_config<kernel_config<256, 12>, kernel_config<BS, IPT>, R>, 0>;
using DEF0 = radix_sort_config<default_config, default_config, default_config, 0>;

int main(int argc, char** argv) {
    size_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 30400000;
    unsigned shift = argc > 2 ? atoi(argv[2]) : 33;
    unsigned long long *in, *out;
    CK(hipMalloc(&in, n * 8));
    CK(hipMalloc(&out, n * 8));
    fill<<<(n + 255) / 256, 256>>>(in, n, shift, 1);
    CK(hipDeviceSynchronize());
    // bucket sort shape: 30.4M keys, 16-bit field at the top
    run<DEF0>("code default(onesweep)", in, out, n, 48, 64);
    run<OS<8, 256, 8>>("code r8 256x8", in, out, n, 48, 64);
    run<OS<8, 512, 8>>("code r8 512x8", in, out, n, 48, 64);
    run<OS<8, 1024, 4>>("code r8 1024x4", in, out, n, 48, 64);
    // pair sort shape: 5.3M keys, 34 bits
    fill<<<(n + 255) / 256, 256>>>(in, n, 0, 7);
    run<DEF0>("pairs default(onesweep)", in, out, 5300000, 0, 34);
    run<OS<9, 256, 8>>("pairs r9 256x8", in, out, 5300000, 0, 34);
    run<OS<10, 256, 8>>("pairs r10 256x8", in, out, 5300000, 0, 34);
    run<OS<12, 256, 8>>("pairs r12 256x8", in, out, 5300000, 0, 34);
    run<OS<12, 256, 4>>("pairs r12 256x4", in, out, 5300000, 0, 34);
    run<OS<9, 512, 8>>("pairs r9 512x8", in, out, 5300000, 0, 34);
    return 0;
}
