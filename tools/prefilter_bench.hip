// Cost of a df = 1 prefilter ahead of level 1: every window's k-mer code
// hashed into a device-wide table, so that a second pass could drop the windows whose k-mer
// occurs once.  Measured here at config 3's size (29.4 M windows) for three table forms:
//   count32   no-return 32-bit atomicAdd per window into 2^24 counters (64 MB, MALL-sized; 32-bit
//             counters cannot wrap, so a frequent k-mer is never read back as df < 2)
//   bits2     returning atomicOr on a "seen" bitmap (2^28 bits, 32 MB), then an atomicOr on a
//             "seen twice" bitmap when the bit was already set
//   store32   plain 4-B stores to the same random addresses (the floor of any scattered table)
// plus the read-back pass the filter needs before level 1 (one random 4-B load per window, a keep
// flag written per window).
// Build: hipcc --offload-arch=gfx950 -O3 tools/prefilter_bench.hip -o /tmp/prefilter_bench
#include <hip/hip_runtime.h>

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

__device__ __forceinline__ uint32_t mix(uint32_t x) {  // a window's code -> a table hash
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

// window i's code: the synthetic batch's codes are close to uniform over 21^7; i's hash stands in
__global__ void count32_kernel(uint32_t n, uint32_t* __restrict__ tab, uint32_t mask) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&tab[mix(i * 0x9E3779B1u) & mask], 1u);
}

__global__ void bits2_kernel(uint32_t n, uint32_t* __restrict__ seen, uint32_t* __restrict__ twice, uint32_t mask) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t h = mix(i * 0x9E3779B1u) & mask, w = h >> 5, b = 1u << (h & 31);
    if (atomicOr(&seen[w], b) & b) atomicOr(&twice[w], b);
}

__global__ void store32_kernel(uint32_t n, uint32_t* __restrict__ tab, uint32_t mask) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) tab[mix(i * 0x9E3779B1u) & mask] = i;
}

__global__ void probe_kernel(uint32_t n, const uint32_t* __restrict__ tab, uint32_t mask, uint8_t* __restrict__ keep) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) keep[i] = tab[mix(i * 0x9E3779B1u) & mask] >= 2u;  // the filter's keep flag per window
}

int main() {
    const uint32_t n = 29416815u;  // config 3's windows
    const uint32_t cmask = (1u << 24) - 1, bmask = (1u << 28) - 1;
    uint32_t *tab, *seen, *twice;
    uint8_t* keep;
    CK(hipMalloc(&tab, sizeof(uint32_t) << 24));
    CK(hipMalloc(&seen, sizeof(uint32_t) << 23));
    CK(hipMalloc(&twice, sizeof(uint32_t) << 23));
    CK(hipMalloc(&keep, n));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const dim3 grid((n + 255) / 256), blk(256);
    const char* names[4] = {"count32 (no-return atomicAdd, 64 MB)", "bits2 (returning atomicOr, 2 x 32 MB)",
                            "store32 (plain random 4-B stores)", "probe (random 4-B loads, the filter's read)"};
    for (int v = 0; v < 4; ++v) {
        float best = 1e30f, sum = 0;
        const int reps = 10;
        for (int r = 0; r < reps + 2; ++r) {
            CK(hipMemsetAsync(tab, 0, sizeof(uint32_t) << 24));
            CK(hipMemsetAsync(seen, 0, sizeof(uint32_t) << 23));
            CK(hipMemsetAsync(twice, 0, sizeof(uint32_t) << 23));
            if (v == 3) count32_kernel<<<grid, blk>>>(n, tab, cmask);
            CK(hipEventRecord(a));
            if (v == 0) count32_kernel<<<grid, blk>>>(n, tab, cmask);
            if (v == 1) bits2_kernel<<<grid, blk>>>(n, seen, twice, bmask);
            if (v == 2) store32_kernel<<<grid, blk>>>(n, tab, cmask);
            if (v == 3) probe_kernel<<<grid, blk>>>(n, tab, cmask, keep);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (r >= 2) {
                sum += ms;
                best = ms < best ? ms : best;
            }
        }
        printf("%-45s %u windows: avg %.3f ms, best %.3f ms (%.2f G ops/s)\n", names[v], n, sum / reps, best,
               n / (best * 1e6));
    }
    return 0;
}
