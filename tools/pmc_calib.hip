// FETCH_SIZE / WRITE_SIZE calibration on gfx950: streaming reads and writes
// of a known byte count at 4, 8 and 16 B per lane, over a 1 GiB buffer (well past the 256 MiB
// Infinity Cache, so every byte comes from HBM).  Run under two rocprofv3 --pmc passes
// (FETCH_SIZE, then WRITE_SIZE); tools/pmc_calib.py divides each dispatch's counter by the bytes
// the kernel moves and writes the per-width factors tools/pmc_traffic.py applies.
//   hipcc --offload-arch=gfx950 -O3 -o tools/pmc_calib tools/pmc_calib.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));            \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

template <class V>
__device__ __forceinline__ uint32_t fold(const V& v);
template <>
__device__ __forceinline__ uint32_t fold(const uint32_t& v) { return v; }
template <>
__device__ __forceinline__ uint32_t fold(const uint2& v) { return v.x ^ v.y; }
template <>
__device__ __forceinline__ uint32_t fold(const uint4& v) { return v.x ^ v.y ^ v.z ^ v.w; }

// grid-stride coalesced read of n elements of V; one u32 per workgroup out (so nothing is elided)
template <class V>
__global__ __launch_bounds__(256) void read_kernel(const V* __restrict__ in, size_t n, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= fold(in[i]);
    __shared__ uint32_t s[256];
    s[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int j = 0; j < 256; ++j) t ^= s[j];
        out[blockIdx.x] = t;
    }
}

template <class V>
__device__ __forceinline__ V make(size_t i);
template <>
__device__ __forceinline__ uint32_t make(size_t i) { return (uint32_t)i; }
template <>
__device__ __forceinline__ uint2 make(size_t i) { return uint2{(uint32_t)i, (uint32_t)(i >> 32)}; }
template <>
__device__ __forceinline__ uint4 make(size_t i) { return uint4{(uint32_t)i, 1u, 2u, 3u}; }

template <class V>
__global__ __launch_bounds__(256) void write_kernel(V* __restrict__ outv, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) outv[i] = make<V>(i);
}

int main(int argc, char** argv) {
    const size_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024) << 20;  // MiB
    const int reps = argc > 2 ? atoi(argv[2]) : 3;
    void* buf = nullptr;
    uint32_t* out = nullptr;
    const int grid = 256 * 8 * 4;  // 4 workgroups of 256 per SIMD-slot group on 256 CUs
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, grid * sizeof(uint32_t)));
    CK(hipMemset(buf, 1, bytes));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](const char* name, auto launch) {
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("{\"kernel\": \"%s\", \"rep\": %d, \"bytes\": %zu, \"ms\": %.4f, \"GBs\": %.1f}\n", name, r, bytes,
                   ms, bytes / (ms * 1e6));
        }
    };
    timed("read_kernel<unsigned int>", [&] { read_kernel<uint32_t><<<grid, 256>>>((const uint32_t*)buf, bytes / 4, out); });
    timed("read_kernel<uint2>", [&] { read_kernel<uint2><<<grid, 256>>>((const uint2*)buf, bytes / 8, out); });
    timed("read_kernel<uint4>", [&] { read_kernel<uint4><<<grid, 256>>>((const uint4*)buf, bytes / 16, out); });
    timed("write_kernel<unsigned int>", [&] { write_kernel<uint32_t><<<grid, 256>>>((uint32_t*)buf, bytes / 4); });
    timed("write_kernel<uint2>", [&] { write_kernel<uint2><<<grid, 256>>>((uint2*)buf, bytes / 8); });
    timed("write_kernel<uint4>", [&] { write_kernel<uint4><<<grid, 256>>>((uint4*)buf, bytes / 16); });
    CK(hipGetLastError());
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
