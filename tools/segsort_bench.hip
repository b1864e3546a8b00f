// Latency of one workgroup's block radix sort (rocprim, 1,024 threads x 8 keys) — the heavy path's
// whole-bucket segment sort (heavy_seg_kernel<1024, 2048, 8192>) — by key width and bit range, for
// one segment of 4,620 keys (config 1's whole buckets) padded to 8,192.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/segsort_bench.hip -o tools/segsort_bench
#include <hip/hip_runtime.h>
#include <rocprim/block/block_radix_sort.hpp>

#include <cstdio>
#include <cstdint>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                            \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

template <class K, uint32_t kThr, uint32_t kItems, uint32_t kBits = 0>
__global__ __launch_bounds__(kThr) void sort_kernel(const K* __restrict__ in, K* __restrict__ out, uint32_t n,
                                                    unsigned b0, unsigned b1) {
    using Sort = rocprim::block_radix_sort<K, kThr, kItems, rocprim::empty_type, 1, 1, kBits>;
    __shared__ typename Sort::storage_type st;
    K v[kItems];
    const K* src = in + (uint64_t)blockIdx.x * n;
#pragma unroll
    for (uint32_t e = 0; e < kItems; ++e) {
        const uint32_t i = threadIdx.x * kItems + e;
        v[e] = i < n ? src[i] : ~K(0);
    }
    Sort().sort(v, st, b0, b1);
#pragma unroll
    for (uint32_t e = 0; e < kItems; ++e) {
        const uint32_t i = threadIdx.x * kItems + e;
        if (i < n) out[(uint64_t)blockIdx.x * n + i] = v[e];
    }
}

__global__ void fill64(unsigned long long* k, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t z = i * 0x9E3779B1u;
    z ^= z >> 15;
    z *= 0x85EBCA6Bu;
    z ^= z >> 13;
    // [h (bucket bits fixed) | class | p]: 21 varying h bits, 4 class bits, 14 protein bits
    k[i] = (0x5ull << 57) | (unsigned long long)(z % 300u) << 18 | (unsigned long long)(z >> 12 & 0x3FFFFu);
}
__global__ void fill32(uint32_t* k, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t z = i * 0x9E3779B1u;
    z ^= z >> 15;
    z *= 0x85EBCA6Bu;
    z ^= z >> 13;
    k[i] = (z % 300u) << 18 | (z >> 12 & 0x3FFFFu);
}

template <class F>
float timeit(F f) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int r = 0; r < 12; ++r) {
        (void)hipEventRecord(a);
        f();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (r >= 2 && ms < best) best = ms;
    }
    return best * 1e3f;
}

int main() {
    const uint32_t n = 4620;
    unsigned long long *k64, *o64;
    uint32_t *k32, *o32;
    CK(hipMalloc(&k64, 8 * 8192));
    CK(hipMalloc(&o64, 8 * 8192));
    CK(hipMalloc(&k32, 4 * 8192));
    CK(hipMalloc(&o32, 4 * 8192));
    fill64<<<(n + 255) / 256, 256>>>(k64, n);
    fill32<<<(n + 255) / 256, 256>>>(k32, n);
    CK(hipDeviceSynchronize());
    printf("one workgroup, %u keys (padded to 8,192): best of 10 launches, us\n", n);
    printf("u64 1024x8 bits [0,64)  %7.1f\n", timeit([&] { sort_kernel<unsigned long long, 1024, 8><<<1, 1024>>>(k64, o64, n, 0, 64); }));
    printf("u64 1024x8 bits [0,39)  %7.1f\n", timeit([&] { sort_kernel<unsigned long long, 1024, 8><<<1, 1024>>>(k64, o64, n, 0, 39); }));
    printf("u64 1024x8 bits [0,32)  %7.1f\n", timeit([&] { sort_kernel<unsigned long long, 1024, 8><<<1, 1024>>>(k64, o64, n, 0, 32); }));
    printf("u64 1024x8 4-bit [0,39) %7.1f\n", timeit([&] { sort_kernel<unsigned long long, 1024, 8, 4><<<1, 1024>>>(k64, o64, n, 0, 39); }));
    printf("u64 512x16 bits [0,39)  %7.1f\n", timeit([&] { sort_kernel<unsigned long long, 512, 16><<<1, 512>>>(k64, o64, n, 0, 39); }));
    printf("u32 1024x8 bits [0,32)  %7.1f\n", timeit([&] { sort_kernel<uint32_t, 1024, 8><<<1, 1024>>>(k32, o32, n, 0, 32); }));
    printf("u32 512x16 bits [0,32)  %7.1f\n", timeit([&] { sort_kernel<uint32_t, 512, 16><<<1, 512>>>(k32, o32, n, 0, 32); }));
    printf("empty launch            %7.1f\n", timeit([&] { sort_kernel<uint32_t, 1024, 8><<<1, 1024>>>(k32, o32, 0, 0, 0); }));
    return 0;
}
