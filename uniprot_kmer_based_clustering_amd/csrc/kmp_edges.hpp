// kmp_edges.hpp — the library-owned edge list behind the opaque kmp_edges handle (kmp_api.cpp,
// kmp_output.cpp).
#pragma once
#include <cstdint>
#include <memory>
#include <new>
#include <utility>
#include <vector>

// Host vector whose resize leaves the new elements uninitialised: the edge arrays are filled by
// device copies right after, and at config 5 (~5e8 edges) zeroing them first cost a full extra
// pass over ~8 GB of host memory.
template <class T>
struct uninit_alloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = uninit_alloc<U>;
    };
    uninit_alloc() = default;
    template <class U>
    uninit_alloc(const uninit_alloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept {
        ::new (static_cast<void*>(p)) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};
template <class T>
using hvec = std::vector<T, uninit_alloc<T>>;

struct kmp_edges {
    hvec<uint32_t> p, q, w;  // canonical (p, q) order, p < q
    hvec<float> score;
    // shared k-mer lists (kmp_edges_kmers): edge i owns kmers[kofs[i] .. kofs[i+1])
    int kspace = -1;                // -1 none, KMP_KMERS_CODES, KMP_KMERS_IDS
    std::vector<uint64_t> kofs;
    std::vector<uint32_t> kmers;
    std::vector<uint64_t> ref_key;  // IDS only: index in the reference's final edge order
    // kmp_pairs_multi_k: the k of each merged list and the per-k weights (k-major: wk[j*count + i])
    std::vector<int> ks;
    std::vector<uint32_t> wk;
};
