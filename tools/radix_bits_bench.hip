// radix_bits_bench.hip — rocprim onesweep with 8..12 radix bits per pass on the two postings sorts:
// 5.4M pair keys on 34 bits (pair sort) and 30.4M bucket keys on [48, 64) (bucket sort).
// hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/radix_bits_bench.hip -o tools/radix_bits_bench
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>

__global__ void gen(unsigned long long* k, uint64_t n, unsigned bits, unsigned top) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        unsigned long long x = i * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
        x ^= x >> 31;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 29;
        k[i] = top ? (x >> 1) : (x & ((1ull << bits) - 1));
    }
}

__global__ void check(const unsigned long long* k, uint64_t n, unsigned lo, unsigned hi, unsigned long long* bad) {
    const unsigned long long m = hi >= 64 ? ~0ull : ((1ull << hi) - 1);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x + 1; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (((k[i - 1] & m) >> lo) > ((k[i] & m) >> lo)) atomicAdd(bad, 1ull);
}

template <class Cfg>
void run(const char* name, unsigned long long* in, unsigned long long* out, uint64_t n, unsigned lo, unsigned hi,
         void* tmp, size_t tmp_n, unsigned long long* bad) {
    size_t t = 0;
    if (rocprim::radix_sort_keys<Cfg>(nullptr, t, in, out, (size_t)n, lo, hi) != hipSuccess || t > tmp_n) {
        printf("%-36s config error / tmp %zu\n", name, t);
        return;
    }
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    if (rocprim::radix_sort_keys<Cfg>(tmp, t, in, out, (size_t)n, lo, hi) != hipSuccess) {
        printf("%-36s launch error\n", name);
        return;
    }
    (void)hipEventRecord(a);
    for (int r = 0; r < 10; ++r) (void)rocprim::radix_sort_keys<Cfg>(tmp, t, in, out, (size_t)n, lo, hi);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipMemset(bad, 0, 8);
    check<<<2048, 256>>>(out, n, lo, hi, bad);
    unsigned long long h = 0;
    (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    printf("%-36s %7.3f ms  unsorted %llu\n", name, ms / 10, h);
}

// gfx950's tuned keys-only u64 entry is onesweep<512x12, 512x12, 8 bits, match>
template <unsigned B, unsigned BS, unsigned IPT>
using OS = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<512, 12>, rocprim::kernel_config<BS, IPT>, B,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;
using Def = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;

int main() {
    const uint64_t n1 = 5'400'000, n2 = 30'400'000;
    unsigned long long *in1, *in2, *out, *bad;
    (void)hipMalloc(&in1, n1 * 8);
    (void)hipMalloc(&in2, n2 * 8);
    (void)hipMalloc(&out, n2 * 8);
    (void)hipMalloc(&bad, 8);
    void* tmp;
    const size_t tmp_n = 512ull << 20;
    (void)hipMalloc(&tmp, tmp_n);
    gen<<<2048, 256>>>(in1, n1, 34, 0);
    gen<<<2048, 256>>>(in2, n2, 0, 1);
    run<Def>("pair 5.4M [0,34) default", in1, out, n1, 0, 34, tmp, tmp_n, bad);
    run<OS<8, 512, 12>>("pair bits8 512x12", in1, out, n1, 0, 34, tmp, tmp_n, bad);
    run<OS<9, 512, 12>>("pair bits9 512x12", in1, out, n1, 0, 34, tmp, tmp_n, bad);
    run<OS<9, 512, 8>>("pair bits9 512x8", in1, out, n1, 0, 34, tmp, tmp_n, bad);
    run<OS<9, 512, 16>>("pair bits9 512x16", in1, out, n1, 0, 34, tmp, tmp_n, bad);
    run<OS<9, 1024, 8>>("pair bits9 1024x8", in1, out, n1, 0, 34, tmp, tmp_n, bad);
    run<OS<9, 1024, 6>>("pair bits9 1024x6", in1, out, n1, 0, 34, tmp, tmp_n, bad);
    run<OS<9, 256, 24>>("pair bits9 256x24", in1, out, n1, 0, 34, tmp, tmp_n, bad);
    run<OS<9, 512, 12>>("pair bits9 512x12 (again)", in1, out, n1, 0, 34, tmp, tmp_n, bad);
    run<Def>("bucket 30.4M [48,64) default", in2, out, n2, 48, 64, tmp, tmp_n, bad);
    run<OS<8, 512, 12>>("bucket bits8 512x12", in2, out, n2, 48, 64, tmp, tmp_n, bad);
    run<OS<8, 1024, 6>>("bucket bits8 1024x6", in2, out, n2, 48, 64, tmp, tmp_n, bad);
    return 0;
}
