// Diagnostic: rocprim::radix_sort_keys on a high bit range [lo, 64) for small and large sizes;
// checks the output is sorted on that field and is a permutation (xor/sum) of the input.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/sort_check.hip -o build/sort_check
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

using OneSweep = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                            rocprim::default_config, 0>;

template <class Cfg>
void check(const char* tag, size_t n, unsigned lo, unsigned hi) {
    {
        {
            std::vector<unsigned long long> h(n);
            unsigned long long z = 12345;
            unsigned long long x0 = 0, s0 = 0;
            for (size_t i = 0; i < n; ++i) {
                z += 0x9E3779B97F4A7C15ull;
                unsigned long long v = z;
                v = (v ^ (v >> 30)) * 0xBF58476D1CE4E5B9ull;
                v ^= v >> 27;
                v &= 0x03FFFFFFFFFFFFFFull;                   // top bits zero like valid keys
                if (i % 17 == 0) v = ~0ull;                    // padding keys
                h[i] = v;
                x0 ^= v;
                s0 += v;
            }
            unsigned long long *in, *out;
            CK(hipMalloc(&in, n * 8));
            CK(hipMalloc(&out, n * 8));
            CK(hipMemcpy(in, h.data(), n * 8, hipMemcpyHostToDevice));
            size_t tb = 0;
            CK(rocprim::radix_sort_keys<Cfg>(nullptr, tb, in, out, n, lo, hi, 0));
            void* tmp;
            CK(hipMalloc(&tmp, tb));
            for (int rep = 0; rep < 2; ++rep) {
                CK(rocprim::radix_sort_keys<Cfg>(tmp, tb, in, out, n, lo, hi, 0));
                std::vector<unsigned long long> r(n);
                CK(hipMemcpy(r.data(), out, n * 8, hipMemcpyDeviceToHost));
                size_t bad = 0;
                unsigned long long x1 = 0, s1 = 0;
                for (size_t i = 0; i < n; ++i) {
                    const unsigned long long m = hi == 64 ? ~0ull : ((1ull << hi) - 1);
                    if (i && ((r[i - 1] & m) >> lo) > ((r[i] & m) >> lo)) ++bad;
                    x1 ^= r[i];
                    s1 += r[i];
                }
                printf("%s n=%zu bits=[%u,%u) rep=%d unsorted=%zu perm=%d\n", tag, n, lo, hi, rep, bad,
                       x1 == x0 && s1 == s0);
            }
            CK(hipFree(tmp));
            CK(hipFree(in));
            CK(hipFree(out));
        }
    }
}

int main() {
    const size_t sizes[] = {1000, 60000, 300000};
    const unsigned rng[][2] = {{52, 64}, {48, 64}, {33, 64}, {30, 53}, {0, 34}, {0, 64}, {20, 40}};
    for (size_t n : sizes)
        for (auto& r : rng) {
            check<rocprim::default_config>("default ", n, r[0], r[1]);
            check<OneSweep>("onesweep", n, r[0], r[1]);
        }
    return 0;
}
