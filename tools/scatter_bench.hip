// scatter_bench.hip — grouping 30M u64 keys by a 15-bit bucket: rocprim 2-pass radix sort vs
// counting scatters (DESIGN.md §4 "bucket front").  Keys are generated from their index (a
// 64-bit mix), so the scatter kernels read nothing but the histogram state.
//   B: per-workgroup 32768-bin LDS histogram -> column scan -> scatter with LDS cursors
//   C: 256 super-buckets (same scheme, 8 bits) -> per-super-bucket pass on 7 bits
// hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/scatter_bench.hip -o /tmp/scatter_bench
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <cstdio>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

constexpr uint64_t N = 30'000'000;
constexpr int BB = 15;
constexpr uint32_t NB = 1u << BB;
constexpr int SH = 49;  // bucket = key >> SH (top bit 0)

__device__ __forceinline__ unsigned long long mk(uint64_t i) {
    unsigned long long x = i * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    return x >> 1;  // top bit 0
}

template <int T>
__global__ __launch_bounds__(T) void histB(uint64_t per, uint32_t* hist) {
    __shared__ uint32_t bins[NB];
    for (uint32_t b = threadIdx.x; b < NB; b += T) bins[b] = 0;
    __syncthreads();
    const uint64_t lo = blockIdx.x * per, hi = min(N, lo + per);
    for (uint64_t i = lo + threadIdx.x; i < hi; i += T) atomicAdd(&bins[(uint32_t)(mk(i) >> SH)], 1u);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < NB; b += T) hist[(uint64_t)blockIdx.x * NB + b] = bins[b];
}

__global__ void colscan(uint32_t* hist, uint32_t G, uint32_t nb, uint32_t* tot) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    uint32_t run = 0;
    for (uint32_t g = 0; g < G; ++g) {
        const uint32_t v = hist[(uint64_t)g * nb + b];
        hist[(uint64_t)g * nb + b] = run;
        run += v;
    }
    tot[b] = run;
}

// column exclusive scan, 64 columns per 1024-thread block: 16 row groups sum their rows, LDS scan
// over the groups, second sweep writes the prefixes
__global__ __launch_bounds__(1024) void colscan2(uint32_t* hist, uint32_t G, uint32_t nb, uint32_t* tot) {
    __shared__ uint32_t part[16][65];
    const uint32_t c = blockIdx.x * 64 + (threadIdx.x & 63), r = threadIdx.x >> 6;
    const uint32_t rows = (G + 15) / 16, g0 = r * rows, g1 = min(G, g0 + rows);
    uint32_t s = 0;
    if (c < nb)
        for (uint32_t g = g0; g < g1; ++g) s += hist[(uint64_t)g * nb + c];
    part[r][threadIdx.x & 63] = s;
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (uint32_t q = 0; q < 16; ++q) {
        const uint32_t v = part[q][threadIdx.x & 63];
        before += q < r ? v : 0;
        all += v;
    }
    if (c < nb) {
        for (uint32_t g = g0; g < g1; ++g) {
            const uint32_t v = hist[(uint64_t)g * nb + c];
            hist[(uint64_t)g * nb + c] = before;
            before += v;
        }
        if (r == 0) tot[c] = all;
    }
}

template <int T>
__global__ __launch_bounds__(T) void scatB(uint64_t per, const uint32_t* hist, const uint32_t* bstart,
                                           unsigned long long* out) {
    __shared__ uint32_t cur[NB];
    for (uint32_t b = threadIdx.x; b < NB; b += T) cur[b] = bstart[b] + hist[(uint64_t)blockIdx.x * NB + b];
    __syncthreads();
    const uint64_t lo = blockIdx.x * per, hi = min(N, lo + per);
    for (uint64_t i = lo + threadIdx.x; i < hi; i += T) {
        const unsigned long long x = mk(i);
        out[atomicAdd(&cur[(uint32_t)(x >> SH)], 1u)] = x;
    }
}

// C pass 1: 256 super-buckets (top 8 bucket bits)
template <int T>
__global__ __launch_bounds__(T) void histC1(uint64_t per, uint32_t* hist) {
    __shared__ uint32_t bins[256];
    for (uint32_t b = threadIdx.x; b < 256; b += T) bins[b] = 0;
    __syncthreads();
    const uint64_t lo = blockIdx.x * per, hi = min(N, lo + per);
    for (uint64_t i = lo + threadIdx.x; i < hi; i += T) atomicAdd(&bins[(uint32_t)(mk(i) >> (SH + 7))], 1u);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < 256; b += T) hist[(uint64_t)blockIdx.x * 256 + b] = bins[b];
}
template <int T>
__global__ __launch_bounds__(T) void scatC1(uint64_t per, const uint32_t* hist, const uint32_t* bstart,
                                            unsigned long long* out) {
    __shared__ uint32_t cur[256];
    for (uint32_t b = threadIdx.x; b < 256; b += T) cur[b] = bstart[b] + hist[(uint64_t)blockIdx.x * 256 + b];
    __syncthreads();
    const uint64_t lo = blockIdx.x * per, hi = min(N, lo + per);
    for (uint64_t i = lo + threadIdx.x; i < hi; i += T) {
        const unsigned long long x = mk(i);
        out[atomicAdd(&cur[(uint32_t)(x >> (SH + 7))], 1u)] = x;
    }
}
// C pass 2: one workgroup per super-bucket: histogram sweep + scatter sweep on 7 bits
template <int T>
__global__ __launch_bounds__(T) void passC2(const unsigned long long* in, const uint32_t* sstart,
                                            unsigned long long* out, uint32_t* bstart) {
    __shared__ uint32_t bins[128];
    const uint32_t s = blockIdx.x;
    const uint32_t a = sstart[s], e = sstart[s + 1];
    if (threadIdx.x < 128) bins[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t i = a + threadIdx.x; i < e; i += T) atomicAdd(&bins[(uint32_t)(in[i] >> SH) & 127], 1u);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = a;
        for (int b = 0; b < 128; ++b) {
            const uint32_t v = bins[b];
            bins[b] = run;
            bstart[s * 128 + b] = run;
            run += v;
        }
    }
    __syncthreads();
    for (uint32_t i = a + threadIdx.x; i < e; i += T) {
        const unsigned long long x = in[i];
        out[atomicAdd(&bins[(uint32_t)(x >> SH) & 127], 1u)] = x;
    }
}

// D: one pass on 12 bits (4096 buckets of ~7.3K keys, the bucket kernel's large capacity)
template <int T, int NBD>
__global__ __launch_bounds__(T) void histD(uint64_t per, uint32_t* hist) {
    __shared__ uint32_t bins[NBD];
    constexpr int S = 64 - 1 - __builtin_ctz(NBD);
    for (uint32_t b = threadIdx.x; b < NBD; b += T) bins[b] = 0;
    __syncthreads();
    const uint64_t lo = blockIdx.x * per, hi = min(N, lo + per);
    for (uint64_t i = lo + threadIdx.x; i < hi; i += T) atomicAdd(&bins[(uint32_t)(mk(i) >> S)], 1u);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < NBD; b += T) hist[(uint64_t)blockIdx.x * NBD + b] = bins[b];
}
template <int T, int NBD>
__global__ __launch_bounds__(T) void scatD(uint64_t per, const uint32_t* hist, const uint32_t* bstart,
                                           unsigned long long* out) {
    __shared__ uint32_t cur[NBD];
    constexpr int S = 64 - 1 - __builtin_ctz(NBD);
    for (uint32_t b = threadIdx.x; b < NBD; b += T) cur[b] = bstart[b] + hist[(uint64_t)blockIdx.x * NBD + b];
    __syncthreads();
    const uint64_t lo = blockIdx.x * per, hi = min(N, lo + per);
    for (uint64_t i = lo + threadIdx.x; i < hi; i += T) {
        const unsigned long long x = mk(i);
        out[atomicAdd(&cur[(uint32_t)(x >> S)], 1u)] = x;
    }
}

// E: XCD-partitioned one pass on 12 bits.  Workgroup blockIdx = i*8 + x runs on XCD x (round-robin
// dispatch) and owns buckets [x*512, x*512+512); it generates every key of range i (of R ranges)
// and keeps its XCD's share: per XCD 32 workgroups x 512 open lines.
template <int T>
__global__ __launch_bounds__(T) void histE(uint64_t per, uint32_t R, uint32_t* hist) {
    __shared__ uint32_t bins[512];
    const uint32_t x = blockIdx.x & 7, i = blockIdx.x >> 3;
    for (uint32_t b = threadIdx.x; b < 512; b += T) bins[b] = 0;
    __syncthreads();
    const uint64_t lo = i * per, hi = min(N, lo + per);
    for (uint64_t j = lo + threadIdx.x; j < hi; j += T) {
        const uint32_t b = (uint32_t)(mk(j) >> 52);
        if ((b >> 9) == x) atomicAdd(&bins[b & 511], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < 512; b += T) hist[(uint64_t)i * 4096 + x * 512 + b] = bins[b];
}
template <int T>
__global__ __launch_bounds__(T) void scatE(uint64_t per, const uint32_t* hist, const uint32_t* bstart,
                                           unsigned long long* out) {
    __shared__ uint32_t cur[512];
    const uint32_t x = blockIdx.x & 7, i = blockIdx.x >> 3;
    for (uint32_t b = threadIdx.x; b < 512; b += T)
        cur[b] = bstart[x * 512 + b] + hist[(uint64_t)i * 4096 + x * 512 + b];
    __syncthreads();
    const uint64_t lo = i * per, hi = min(N, lo + per);
    for (uint64_t j = lo + threadIdx.x; j < hi; j += T) {
        const unsigned long long v = mk(j);
        const uint32_t b = (uint32_t)(v >> 52);
        if ((b >> 9) == x) out[atomicAdd(&cur[b & 511], 1u)] = v;
    }
}

__global__ void checkD(const unsigned long long* k, const uint32_t* bstart, unsigned long long* bad) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t b = (uint32_t)(k[i] >> 52);
        if (i < bstart[b] || i >= bstart[b + 1]) atomicAdd(bad, 1ull);
    }
}

__global__ void gen(unsigned long long* k) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x)
        k[i] = mk(i);
}

__global__ void check(const unsigned long long* k, const uint32_t* bstart, unsigned long long* bad) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t b = (uint32_t)(k[i] >> SH);
        if (i < bstart[b] || i >= bstart[b + 1]) atomicAdd(bad, 1ull);
    }
}

int main() {
    unsigned long long *keys, *out, *tmp2, *bad;
    uint32_t *hist, *tot, *bstart, *sstart;
    CK(hipMalloc(&keys, N * 8));
    CK(hipMalloc(&out, N * 8));
    CK(hipMalloc(&tmp2, N * 8));
    CK(hipMalloc(&hist, 1024ull * NB * 4));
    CK(hipMalloc(&tot, (NB + 1) * 4));
    CK(hipMalloc(&bstart, (NB + 1) * 4));
    CK(hipMalloc(&sstart, 257 * 4));
    CK(hipMalloc(&bad, 8));
    gen<<<4096, 256>>>(keys);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    size_t ts = 0, tsc = 0;
    using Cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;
    CK(rocprim::radix_sort_keys<Cfg>(nullptr, ts, keys, out, (size_t)N, SH, 64));
    CK(rocprim::exclusive_scan(nullptr, tsc, tot, bstart, 0u, (size_t)NB + 1, rocprim::plus<uint32_t>()));
    void* scratch;
    CK(hipMalloc(&scratch, std::max(ts, tsc)));
    auto timeit = [&](const char* name, auto&& f, int reps = 10) {
        f();
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        for (int r = 0; r < reps; ++r) f();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-44s %8.3f ms  (%.2f TB/s on 16 B/key)\n", name, ms / reps, 16.0 * N / (ms / reps * 1e-3) / 1e12);
    };
    timeit("rocprim radix sort [49,64)", [&] {
        size_t t = ts;
        (void)rocprim::radix_sort_keys<Cfg>(scratch, t, keys, out, (size_t)N, SH, 64);
    });
    auto planB = [&](uint32_t G, auto tag) {
        constexpr int T = decltype(tag)::value;
        const uint64_t per = (N + G - 1) / G;
        histB<T><<<G, T>>>(per, hist);
        colscan2<<<NB / 64, 1024>>>(hist, G, NB, tot);
        (void)hipMemsetAsync(tot + NB, 0, 4);
        size_t t = tsc;
        (void)rocprim::exclusive_scan(scratch, t, tot, bstart, 0u, (size_t)NB + 1, rocprim::plus<uint32_t>());
        scatB<T><<<G, T>>>(per, hist, bstart, out);
    };
    for (uint32_t G : {256u, 512u, 1024u}) {
        char nm[64];
        snprintf(nm, sizeof nm, "B: 32K-bin scatter, G=%u x1024", G);
        timeit(nm, [&] { planB(G, std::integral_constant<int, 1024>{}); });
    }
    {
        (void)hipMemset(bad, 0, 8);
        check<<<4096, 256>>>(out, bstart, bad);
        unsigned long long h = 0;
        (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
        printf("  B check: %llu misplaced\n", h);
    }
    // B phases separately at G=256
    {
        const uint32_t G = 256;
        const uint64_t per = (N + G - 1) / G;
        timeit("  B hist only (G=256)", [&] { histB<1024><<<G, 1024>>>(per, hist); });
        timeit("  B colscan only", [&] { colscan<<<NB / 256, 256>>>(hist, G, NB, tot); });
        histB<1024><<<G, 1024>>>(per, hist);
        colscan<<<NB / 256, 256>>>(hist, G, NB, tot);
        (void)hipMemsetAsync(tot + NB, 0, 4);
        size_t t = tsc;
        (void)rocprim::exclusive_scan(scratch, t, tot, bstart, 0u, (size_t)NB + 1, rocprim::plus<uint32_t>());
        timeit("  B scatter only (G=256)", [&] { scatB<1024><<<G, 1024>>>(per, hist, bstart, out); });
    }
    auto planC = [&](uint32_t G) {
        const uint64_t per = (N + G - 1) / G;
        histC1<256><<<G, 256>>>(per, hist);
        colscan<<<1, 256>>>(hist, G, 256, tot);
        (void)hipMemsetAsync(tot + 256, 0, 4);
        size_t t = tsc;
        (void)rocprim::exclusive_scan(scratch, t, tot, sstart, 0u, (size_t)257, rocprim::plus<uint32_t>());
        scatC1<256><<<G, 256>>>(per, hist, sstart, tmp2);
        passC2<1024><<<256, 1024>>>(tmp2, sstart, out, bstart);
        (void)hipMemcpyAsync(bstart + NB, sstart + 256, 4, hipMemcpyDeviceToDevice);
    };
    for (uint32_t G : {1024u, 4096u}) {
        char nm[64];
        snprintf(nm, sizeof nm, "C: 256 x 128 two-level, G=%u", G);
        timeit(nm, [&] { planC(G); });
    }
    {
        (void)hipMemset(bad, 0, 8);
        check<<<4096, 256>>>(out, bstart, bad);
        unsigned long long h = 0;
        (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
        printf("  C check: %llu misplaced\n", h);
        const uint32_t G = 4096;
        const uint64_t per = (N + G - 1) / G;
        timeit("  C pass1 scatter only", [&] { scatC1<256><<<G, 256>>>(per, hist, sstart, tmp2); });
        timeit("  C pass2 only", [&] { passC2<1024><<<256, 1024>>>(tmp2, sstart, out, bstart); });
    }
    auto planD = [&](uint32_t G, auto tagT, auto tagB) {
        constexpr int T = decltype(tagT)::value, NBD = decltype(tagB)::value;
        const uint64_t per = (N + G - 1) / G;
        histD<T, NBD><<<G, T>>>(per, hist);
        colscan2<<<(NBD + 63) / 64, 1024>>>(hist, G, NBD, tot);
        (void)hipMemsetAsync(tot + NBD, 0, 4);
        size_t t = tsc;
        (void)rocprim::exclusive_scan(scratch, t, tot, bstart, 0u, (size_t)NBD + 1, rocprim::plus<uint32_t>());
        scatD<T, NBD><<<G, T>>>(per, hist, bstart, out);
    };
    for (uint32_t G : {256u, 512u, 1024u, 2048u}) {
        char nm[64];
        snprintf(nm, sizeof nm, "D: 4096-bin one pass, G=%u x512", G);
        timeit(nm, [&] { planD(G, std::integral_constant<int, 512>{}, std::integral_constant<int, 4096>{}); });
        snprintf(nm, sizeof nm, "D: 4096-bin one pass, G=%u x1024", G);
        timeit(nm, [&] { planD(G, std::integral_constant<int, 1024>{}, std::integral_constant<int, 4096>{}); });
        snprintf(nm, sizeof nm, "D: 8192-bin one pass, G=%u x1024", G);
        timeit(nm, [&] { planD(G, std::integral_constant<int, 1024>{}, std::integral_constant<int, 8192>{}); });
    }
    {
        const uint32_t G = 512;
        const uint64_t per = (N + G - 1) / G;
        histD<1024, 4096><<<G, 1024>>>(per, hist);
        colscan2<<<64, 1024>>>(hist, G, 4096, tot);
        timeit("  D colscan2 only (G=512)", [&] { colscan2<<<64, 1024>>>(hist, G, 4096, tot); });
        histD<1024, 4096><<<G, 1024>>>(per, hist);
        colscan2<<<64, 1024>>>(hist, G, 4096, tot);
        (void)hipMemsetAsync(tot + 4096, 0, 4);
        size_t t = tsc;
        (void)rocprim::exclusive_scan(scratch, t, tot, bstart, 0u, (size_t)4097, rocprim::plus<uint32_t>());
        timeit("  D hist only (G=512 x1024)", [&] { histD<1024, 4096><<<G, 1024>>>(per, hist); });
        timeit("  D scatter only (G=512 x1024)", [&] { scatD<1024, 4096><<<G, 1024>>>(per, hist, bstart, out); });
    }
    {
        const uint32_t G = 512;
        const uint64_t per = (N + G - 1) / G;
        hipEvent_t ev[6];
        for (auto& e : ev) (void)hipEventCreate(&e);
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(ev[0]);
            histD<1024, 4096><<<G, 1024>>>(per, hist);
            (void)hipEventRecord(ev[1]);
            colscan2<<<64, 1024>>>(hist, G, 4096, tot);
            (void)hipEventRecord(ev[2]);
            (void)hipMemsetAsync(tot + 4096, 0, 4);
            (void)hipEventRecord(ev[3]);
            size_t t = tsc;
            (void)rocprim::exclusive_scan(scratch, t, tot, bstart, 0u, (size_t)4097, rocprim::plus<uint32_t>());
            (void)hipEventRecord(ev[4]);
            scatD<1024, 4096><<<G, 1024>>>(per, hist, bstart, out);
            (void)hipEventRecord(ev[5]);
            (void)hipEventSynchronize(ev[5]);
            float m[5];
            for (int i = 0; i < 5; ++i) (void)hipEventElapsedTime(&m[i], ev[i], ev[i + 1]);
            printf("  D phases: hist %.3f colscan %.3f memset %.3f scan %.3f scatter %.3f ms\n", m[0], m[1], m[2], m[3], m[4]);
            (void)hipEventRecord(ev[0]);
            scatD<1024, 4096><<<G, 1024>>>(per, hist, bstart, out);
            (void)hipEventRecord(ev[1]);
            scatD<1024, 4096><<<G, 1024>>>(per, hist, bstart, out);
            (void)hipEventRecord(ev[2]);
            (void)hipEventSynchronize(ev[2]);
            (void)hipEventElapsedTime(&m[0], ev[0], ev[1]);
            (void)hipEventElapsedTime(&m[1], ev[1], ev[2]);
            (void)hipMemset(bad, 0, 8);
            check<<<4096, 256>>>(out, bstart, bad);
            unsigned long long h = 0;
            (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
            printf("  D again: %.3f then %.3f ms; misplaced %llu\n", m[0], m[1], h);
            // a different buffer content in between: overwrite out with other data
            gen<<<4096, 256>>>(tmp2);
            (void)hipMemcpy(out, tmp2, N * 8, hipMemcpyDeviceToDevice);
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(ev[0]);
            scatD<1024, 4096><<<G, 1024>>>(per, hist, bstart, out);
            (void)hipEventRecord(ev[1]);
            (void)hipEventSynchronize(ev[1]);
            (void)hipEventElapsedTime(&m[0], ev[0], ev[1]);
            printf("  D after overwriting out: %.3f ms\n", m[0]);
        }
    }
    for (uint32_t R : {32u, 64u, 128u}) {
        const uint64_t per = (N + R - 1) / R;
        const uint32_t G = R * 8;
        hipEvent_t ev[6];
        for (auto& e : ev) (void)hipEventCreate(&e);
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(ev[0]);
            histE<1024><<<G, 1024>>>(per, R, hist);
            (void)hipEventRecord(ev[1]);
            colscan2<<<64, 1024>>>(hist, R, 4096, tot);
            (void)hipEventRecord(ev[2]);
            (void)hipMemsetAsync(tot + 4096, 0, 4);
            size_t t = tsc;
            (void)rocprim::exclusive_scan(scratch, t, tot, bstart, 0u, (size_t)4097, rocprim::plus<uint32_t>());
            (void)hipEventRecord(ev[3]);
            scatE<1024><<<G, 1024>>>(per, hist, bstart, out);
            (void)hipEventRecord(ev[4]);
            (void)hipEventSynchronize(ev[4]);
            float m[4];
            for (int i = 0; i < 4; ++i) (void)hipEventElapsedTime(&m[i], ev[i], ev[i + 1]);
            (void)hipMemset(bad, 0, 8);
            checkD<<<4096, 256>>>(out, bstart, bad);
            unsigned long long h = 0;
            (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
            printf("  E R=%u: hist %.3f colscan %.3f scan %.3f scatter %.3f = %.3f ms; misplaced %llu\n", R, m[0], m[1],
                   m[2], m[3], m[0] + m[1] + m[2] + m[3], h);
        }
    }
    return 0;
}
