// kmp_stream.hip — the summary of a streamed edge list (kmp_pairs_stream, kmerpair.h): the
// reference's counters over the edges (graph/mod.rs:545 "Number of edges now", :695 Σ w of the
// class-differing pairs, :242 w > 10 alignment candidates) plus an order-checked digest, computed
// on the device per chunk so that an edge list far larger than HBM (config 5: ~10^11 edges at
// k = 5) is summarised without ever being resident or copied whole.
//
// digest = Σ_i term(p_i, q_i, w_i, s_i, w0_i) mod 2^64 (kmp_edge_digest_term, kmerpair.h), summed
// per row segment (p * KMP_DIGEST_SEGMENTS / N) and in total.  A sum is order-free; the order is
// checked instead: every chunk must be strictly (p, q)-ascending with p < q < N and p inside the
// chunk's rows, and the chunks' rows ascend — a strictly ascending sequence is determined by its
// set, so equal digests of two ascending lists mean equal lists (up to 64-bit collisions).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "kmerpair.h"
#include "kmp_stream.hpp"

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64's finaliser
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t digest_term(uint32_t p, uint32_t q, uint32_t w, uint32_t s, uint32_t w0) {
    const uint64_t a = (uint64_t)p << 32 | q, b = (uint64_t)w << 32 | s;
    return mix64(a ^ mix64(b ^ mix64((uint64_t)w0)));
}

constexpr uint32_t kDgThreads = 256, kDgPer = 16, kDgTile = kDgThreads * kDgPer;

// one workgroup per 4,096 edges; per-thread sums for the current row segment (a tile almost never
// spans two of the 64 segments: a segment change flushes to LDS on its own), wave-reduced at the end
__global__ __launch_bounds__(kDgThreads) void edge_digest_kernel(kmp::DigestIn in, kmp::DigestAcc* __restrict__ acc) {
    __shared__ unsigned long long s_e[KMP_DIGEST_SEGMENTS], s_d[KMP_DIGEST_SEGMENTS];
    __shared__ unsigned long long s_tot[4];
    __shared__ unsigned int s_bad;
    for (uint32_t i = threadIdx.x; i < KMP_DIGEST_SEGMENTS; i += kDgThreads) s_e[i] = s_d[i] = 0;
    if (threadIdx.x < 4) s_tot[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_bad = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kDgTile;
    uint32_t seg = ~0u;
    unsigned long long ne = 0, dg = 0, sw = 0, ss = 0, na = 0, wd = 0;
    bool bad = false;
#pragma unroll 4
    for (uint32_t j = 0; j < kDgPer; ++j) {  // (unrolled: the next edges' loads issue ahead of this one's mixing)
        const uint64_t i = t0 + j * kDgThreads + threadIdx.x;
        if (i >= in.n) continue;
        const uint32_t p = in.p[i], q = in.q[i], w = in.w[i];
        const uint32_t s = in.s ? in.s[i] : w, w0 = in.w0 ? in.w0[i] : w;
        if (i > 0) {
            const uint32_t pp = in.p[i - 1], pq = in.q[i - 1];
            bad |= !(pp < p || (pp == p && pq < q));
        }
        bad |= !(p < q && q < in.n_prot && p >= in.row_lo && p < in.row_hi);
        const uint32_t g = (uint32_t)((uint64_t)min(p, in.n_prot - 1) * KMP_DIGEST_SEGMENTS / in.n_prot);
        if (g != seg) {
            if (ne) {  // rare: the tile crosses a segment boundary
                atomicAdd(&s_e[seg], ne);
                atomicAdd(&s_d[seg], dg);
            }
            seg = g;
            ne = dg = 0;
        }
        ++ne;
        dg += digest_term(p, q, w, s, w0);
        sw += w;
        ss += s;
        na += w > in.align_threshold;
        if (in.cls && in.cls[p] != in.cls[q]) wd += w;
    }
    // the last segment: wave-uniform in nearly every wave
    const uint32_t s0 = __shfl(seg, 0);
    if (__all(seg == s0 || ne == 0)) {
        for (int o = 32; o > 0; o >>= 1) {
            ne += __shfl_down(ne, o);
            dg += __shfl_down(dg, o);
        }
        if ((threadIdx.x & 63) == 0 && ne) {
            atomicAdd(&s_e[s0], ne);
            atomicAdd(&s_d[s0], dg);
        }
    } else if (ne) {
        atomicAdd(&s_e[seg], ne);
        atomicAdd(&s_d[seg], dg);
    }
    for (int o = 32; o > 0; o >>= 1) {
        sw += __shfl_down(sw, o);
        ss += __shfl_down(ss, o);
        na += __shfl_down(na, o);
        wd += __shfl_down(wd, o);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&s_tot[0], sw);
        atomicAdd(&s_tot[1], ss);
        atomicAdd(&s_tot[2], na);
        atomicAdd(&s_tot[3], wd);
    }
    if (bad) atomicOr(&s_bad, 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < KMP_DIGEST_SEGMENTS; i += kDgThreads)
        if (s_e[i]) {
            atomicAdd(&acc->seg_edges[i], s_e[i]);
            atomicAdd(&acc->seg_digest[i], s_d[i]);
        }
    if (threadIdx.x < 4 && s_tot[threadIdx.x]) atomicAdd(&acc->tot[threadIdx.x], s_tot[threadIdx.x]);
    if (threadIdx.x == 0 && s_bad) atomicOr(&acc->bad, 1u);
}

}  // namespace

namespace kmp {

hipError_t edge_digest_enqueue(const DigestIn& in, DigestAcc* acc, hipStream_t st) {
    if (in.n == 0) return hipSuccess;
    const uint64_t blocks = (in.n + kDgTile - 1) / kDgTile;
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    edge_digest_kernel<<<(uint32_t)blocks, kDgThreads, 0, st>>>(in, acc);
    return hipGetLastError();
}

}  // namespace kmp
