// kmp_edgekmers.hip — the shared k-mers of every emitted edge: the
// KmerEdgeGroup.kmers list (edge.rs:48-81; concatenated in ascending key order by combine_edges,
// mod.rs:415-417) that the postings engine reduces to its length w.
//   edge_kmers_device: one wavefront per edge intersects the repeat-filtered sets of p and q
//     (every shared k-mer is a repeat k-mer, main.rs:127-162): each lane takes one code of the
//     shorter set, binary-searches the longer one, and a ballot + popcount places the hits, so
//     the list comes out ascending.  The output range of edge i is kofs[i] .. kofs[i+1]
//     (exclusive scan of w), and a length other than w flags the edge list as foreign.
//   edge_blosum_device: the BLOSUM-weighted score of every edge over the same intersection
//     (set(p) staged in LDS per wave, set(q) streamed).
//   edge_kmers_to_ids: codes -> repeat-MPHF ids, ascending within each edge (one 64-bit sort of
//     (edge, id)), and each edge's rank in the reference's final edge order, ascending
//     (min shared id, p, q) (combine_edges with one thread).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>

#include "kmerpair.h"
#include "kmp_internal.hpp"
#include "kmp_mphf.hpp"

namespace kmp {
namespace {

constexpr uint32_t kWaves = 4;  // wavefronts (edges in flight) per 256-thread block

__global__ __launch_bounds__(256) void edge_kmers_kernel(const uint32_t* __restrict__ rep,
                                                         const uint32_t* __restrict__ rep_len,
                                                         const uint64_t* __restrict__ off,
                                                         const uint32_t* __restrict__ ep, const uint32_t* __restrict__ eq,
                                                         const uint64_t* __restrict__ kofs, uint64_t count,
                                                         uint32_t* __restrict__ out, unsigned int* __restrict__ bad) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t below = (1ull << lane) - 1;
    for (uint64_t e = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); e < count; e += (uint64_t)gridDim.x * kWaves) {
        const uint32_t a = ep[e], b = eq[e];
        const uint32_t* A = rep + set_base(off[a], a);
        const uint32_t* B = rep + set_base(off[b], b);
        uint32_t la = rep_len[a], lb = rep_len[b];
        if (la > lb) {
            const uint32_t* t = A;
            A = B;
            B = t;
            const uint32_t u = la;
            la = lb;
            lb = u;
        }
        const uint64_t o = kofs[e], w = kofs[e + 1] - o;
        uint64_t wr = 0;
        for (uint32_t c = 0; c < la; c += 64) {
            const uint32_t i = c + lane;
            bool hit = false;
            uint32_t x = 0;
            if (i < la) {
                x = A[i];
                uint32_t lo = 0, hi = lb;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (B[mid] < x) lo = mid + 1;
                    else hi = mid;
                }
                hit = lo < lb && B[lo] == x;
            }
            const uint64_t mask = __ballot(hit);
            if (hit) {
                const uint64_t pos = wr + __popcll(mask & below);
                if (pos < w) out[o + pos] = x;
            }
            wr += __popcll(mask);
        }
        if (lane == 0 && wr != w) atomicOr(bad, 1u);
    }
}

// BLOSUM62 self-scores in residue-code order (the diagonal of blosum.rs:8-30, whose rows follow
// the same C S T A G P D E Q N H R K M I L V W Y F order as AMINO_ACID_LIST); code 20 ('*' and
// unknown residues) scores 0
__constant__ int8_t c_b62_diag[21] = {9, 4, 5, 4, 6, 7, 6, 5, 5, 6, 8, 5, 5, 5, 4, 4, 4, 11, 7, 6, 0};

// BLOSUM-weighted score of every edge (a build extension, parity
// unpinned): score = Σ over the shared k-mers x of Σ_i B62[x_i][x_i] (radix-21 digits of the
// code), over the intersection of the repeat-filtered sets; hits != w flags the edge list as
// foreign.  Edges come in (p, q) order, so a wave takes 64 consecutive edges (one task), copies
// set(p) into its own LDS slice whenever p changes (~500 edges share a p at config 5), and its
// lanes walk set(q) with coalesced loads, each binary-searching the LDS copy (5e8 edges at config
// 5, k = 7).  A search in global memory (round 2's first version) cost ~9 dependent L2/HBM loads
// per code of the shorter set; here they are LDS reads.  An edge whose set(p) exceeds the slice
// searches set(p) in global memory instead.  The walk of set(q) stops once the wave has seen the
// edge's w hits (w = the shared k-mer count the pipeline computed): a list with fewer hits than its
// w is still flagged, one with extra hits only if they fall in the chunk of 64 that reaches w —
// so w must be exact (as every engine's is).  full (KMP_DEBUG set): every set(q) is walked to its
// end, and any hit count other than w flags the list as foreign.
constexpr uint32_t kBlWaves = 4, kBlSlice = 2048, kBlTask = 64;
__global__ __launch_bounds__(256) void edge_blosum_lds_kernel(const uint32_t* __restrict__ rep,
                                                              const uint32_t* __restrict__ rep_len,
                                                              const uint64_t* __restrict__ off,
                                                              const uint32_t* __restrict__ ep,
                                                              const uint32_t* __restrict__ eq,
                                                              const uint32_t* __restrict__ ew, uint64_t count, int k,
                                                              float* __restrict__ score, unsigned int* __restrict__ bad,
                                                              int full) {
    __shared__ uint32_t S[kBlWaves][kBlSlice];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t* P = S[wv];
    const uint64_t tasks = (count + kBlTask - 1) / kBlTask;
    for (uint64_t t = (uint64_t)blockIdx.x * kBlWaves + wv; t < tasks; t += (uint64_t)gridDim.x * kBlWaves) {
        uint32_t cur = 0xFFFFFFFFu, lp = 0;
        const uint64_t e1 = min(count, (t + 1) * kBlTask);
        for (uint64_t e = t * kBlTask; e < e1; ++e) {
            const uint32_t a = ep[e], b = eq[e];
            const uint32_t la = rep_len[a], lb = rep_len[b], w = ew[e];
            int sum = 0, hits = 0;
            auto add = [&](uint32_t x) {
                for (int i = 0; i < k; ++i) {
                    sum += c_b62_diag[x % kRadix];
                    x /= kRadix;
                }
                ++hits;
            };
            if (la <= kBlSlice) {
                if (a != cur) {
                    __builtin_amdgcn_wave_barrier();  // every lane is done with the previous set
                    const uint32_t* A = rep + set_base(off[a], a);
                    for (uint32_t i = lane; i < la; i += 64) P[i] = A[i];
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    cur = a;
                    lp = la;
                }
                const uint32_t* B = rep + set_base(off[b], b);
                // set(q) is sorted: the last lane's insertion point bounds the next chunk's searches
                for (uint32_t c = 0, seen = 0, base = 0; c < lb && (full || seen < w); c += 64) {
                    const uint32_t i = c + lane;
                    bool hit = false;
                    uint32_t lo = base;
                    if (i < lb) {
                        const uint32_t x = B[i];
                        uint32_t hi = lp;
                        while (lo < hi) {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (P[mid] < x) lo = mid + 1;
                            else hi = mid;
                        }
                        hit = lo < lp && P[lo] == x;
                        if (hit) add(x);
                    }
                    seen += __popcll(__ballot(hit));
                    base = __shfl(lo, (int)min(63u, lb - 1 - c));
                }
            } else {
                const uint32_t* A = rep + set_base(off[a], a);
                const uint32_t* B = rep + set_base(off[b], b);
                for (uint32_t c = 0, seen = 0; c < lb && (full || seen < w); c += 64) {
                    const uint32_t i = c + lane;
                    bool hit = false;
                    if (i < lb) {
                        const uint32_t x = B[i];
                        uint32_t lo = 0, hi = la;
                        while (lo < hi) {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (A[mid] < x) lo = mid + 1;
                            else hi = mid;
                        }
                        hit = lo < la && A[lo] == x;
                        if (hit) add(x);
                    }
                    seen += __popcll(__ballot(hit));
                }
            }
            for (int sh = 32; sh > 0; sh >>= 1) {
                sum += __shfl_down(sum, sh);
                hits += __shfl_down(hits, sh);
            }
            if (lane == 0) {
                score[e] = (float)sum;  // an integer below 2^24: exact
                if ((uint32_t)hits != w) atomicOr(bad, 1u);
            }
        }
    }
}

// (edge, id) keys: the edge owning entry j is the largest e with kofs[e] <= j
__global__ void edge_id_keys_kernel(const uint64_t* __restrict__ ids, uint64_t total, const uint64_t* __restrict__ kofs,
                                    uint64_t count, unsigned long long* __restrict__ keys) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < total; j += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t lo = 0, hi = count;
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if (kofs[mid] <= j) lo = mid;
            else hi = mid;
        }
        keys[j] = (unsigned long long)lo << 32 | (ids[j] & 0xFFFFFFFFull);
    }
}

__global__ void low_words_kernel(const unsigned long long* __restrict__ keys, uint64_t total, uint32_t* __restrict__ out) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < total; j += (uint64_t)gridDim.x * blockDim.x)
        out[j] = (uint32_t)keys[j];
}

// (min shared id, edge index): edges are in (p, q) order, so the index breaks ties as (p, q) does
__global__ void min_id_keys_kernel(const uint32_t* __restrict__ ids, const uint64_t* __restrict__ kofs, uint64_t count,
                                   unsigned long long* __restrict__ keys) {
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < count; e += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long m = kofs[e + 1] > kofs[e] ? ids[kofs[e]] : 0xFFFFFFFFull;
        keys[e] = m << 32 | e;
    }
}

__global__ void rank_scatter_kernel(const unsigned long long* __restrict__ sorted, uint64_t count,
                                    uint64_t* __restrict__ ref_key) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x)
        ref_key[sorted[i] & 0xFFFFFFFFull] = i;
}

inline uint32_t grid_for(uint64_t m) { return (uint32_t)std::min<uint64_t>((m + 255) / 256, 65536); }

template <class T>
hipError_t dmalloc(T** p, size_t n) {
    return hipMalloc(reinterpret_cast<void**>(p), std::max<size_t>(1, n) * sizeof(T));
}

}  // namespace

int edge_kmers_device(const uint32_t* d_rep, const uint32_t* d_rep_len, const uint64_t* d_off, const uint32_t* d_p,
                      const uint32_t* d_q, const uint64_t* d_kofs, uint64_t count, uint32_t* d_out, hipStream_t st) {
    if (count == 0) return KMP_OK;
    unsigned int* bad = nullptr;
    if (dmalloc(&bad, 1) != hipSuccess) return KMP_ENOMEM;
    int rc = KMP_OK;
    unsigned int h_bad = 0;
    if (hipMemsetAsync(bad, 0, 4, st) != hipSuccess) rc = KMP_EDEVICE;
    if (rc == KMP_OK) {
        const uint32_t blocks = (uint32_t)std::min<uint64_t>((count + kWaves - 1) / kWaves, 1u << 20);
        edge_kmers_kernel<<<blocks, 256, 0, st>>>(d_rep, d_rep_len, d_off, d_p, d_q, d_kofs, count, d_out, bad);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(&h_bad, bad, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            rc = KMP_EDEVICE;
    }
    (void)hipFree(bad);
    if (rc == KMP_OK && h_bad) rc = KMP_EINVAL;  // w does not match the sets: edges of another build
    return rc;
}

int edge_blosum_device(const uint32_t* d_rep, const uint32_t* d_rep_len, const uint64_t* d_off, const uint32_t* d_p,
                       const uint32_t* d_q, const uint32_t* d_w, uint64_t count, int k, float* d_score,
                       hipStream_t st) {
    if (count == 0) return KMP_OK;
    unsigned int* bad = nullptr;
    if (dmalloc(&bad, 1) != hipSuccess) return KMP_ENOMEM;
    int rc = KMP_OK;
    unsigned int h_bad = 0;
    if (hipMemsetAsync(bad, 0, 4, st) != hipSuccess) rc = KMP_EDEVICE;
    if (rc == KMP_OK) {
        const uint64_t tasks = (count + kBlTask - 1) / kBlTask;
        const uint32_t lblocks = (uint32_t)std::min<uint64_t>((tasks + kBlWaves - 1) / kBlWaves, 8192);
        edge_blosum_lds_kernel<<<lblocks, 256, 0, st>>>(d_rep, d_rep_len, d_off, d_p, d_q, d_w, count, k, d_score,
                                                         bad, getenv("KMP_DEBUG") != nullptr ? 1 : 0);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(&h_bad, bad, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            rc = KMP_EDEVICE;
    }
    (void)hipFree(bad);
    if (rc == KMP_OK && h_bad) rc = KMP_EINVAL;
    return rc;
}

int edge_kmers_to_ids(const kmp_mphf* m, const uint64_t* d_kofs, uint64_t count, uint64_t total, uint32_t* d_inout,
                      uint64_t* d_ref_key, hipStream_t st) {
    if (count == 0) return KMP_OK;
    if (count >= 0xFFFFFFFFull) return KMP_EINVAL;  // edge index must fit the high key half
    uint64_t* ids = nullptr;
    unsigned long long *ka = nullptr, *kb = nullptr;
    void* scratch = nullptr;
    const uint64_t nk = std::max(total, count);
    auto done = [&](int r) {
        for (void* q : {(void*)ids, (void*)ka, (void*)kb, scratch})
            if (q) (void)hipFree(q);
        return r;
    };
#define EB(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) return done(e_ == hipErrorOutOfMemory ? KMP_ENOMEM : KMP_EDEVICE); \
    } while (0)
    EB(dmalloc(&ids, total));
    EB(dmalloc(&ka, nk));
    EB(dmalloc(&kb, nk));
    size_t need = 0;
    EB(rocprim::radix_sort_keys(nullptr, need, ka, kb, (size_t)nk, 0u, 64u, st));
    EB(hipMalloc(&scratch, std::max<size_t>(need, 16)));
    if (total) {
        const int rc = mphf_lookup_device(m, d_inout, total, ids, st);
        if (rc != KMP_OK) return done(rc);
        edge_id_keys_kernel<<<grid_for(total), 256, 0, st>>>(ids, total, d_kofs, count, ka);
        size_t n1 = need;
        EB(rocprim::radix_sort_keys(scratch, n1, ka, kb, (size_t)total, 0u, 64u, st));
        low_words_kernel<<<grid_for(total), 256, 0, st>>>(kb, total, d_inout);
    }
    if (d_ref_key) {
        min_id_keys_kernel<<<grid_for(count), 256, 0, st>>>(d_inout, d_kofs, count, ka);
        size_t n2 = need;
        EB(rocprim::radix_sort_keys(scratch, n2, ka, kb, (size_t)count, 0u, 64u, st));
        rank_scatter_kernel<<<grid_for(count), 256, 0, st>>>(kb, count, d_ref_key);
    }
    EB(hipGetLastError());
    EB(hipStreamSynchronize(st));
#undef EB
    return done(KMP_OK);
}

}  // namespace kmp
