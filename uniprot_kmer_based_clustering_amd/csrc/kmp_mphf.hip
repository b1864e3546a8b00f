// kmp_mphf.hip — minimal perfect hashing of u32 k-mer codes on the device, the replacement for
// boomphf's Mphf<u32> (Mphf::new(3.0, &keys), main.rs:139-140; hash(), main.rs:145,192 and
// protein.rs:154,168).  BBHash structure, as boomphf builds it:
//   level l holds a bit vector of about gamma * n_l bits; every key still unplaced hashes (a
//   seeded 64-bit mix per level) to one bit; keys alone on their bit are placed there, keys that
//   collided fall through to level l + 1;
//   id(key) = number of set bits before the key's bit over all levels (a per-word popcount
//   prefix), so the ids of n keys are exactly 0 .. n-1.
// Keys still unplaced after kMaxLevels levels go to a sorted fallback array (ids after the
// placed ones), as boomphf's fallback map does.  The ids are this build's, not boomphf's
// (boomphf hashes with wyhash and its own seeds): they are internal dense ids, unobservable in the
// edge list.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>

#include <algorithm>
#include <cmath>
#include <new>
#include <vector>

#include "kmerpair.h"
#include "kmp_internal.hpp"
#include "kmp_mphf.hpp"

using namespace kmp;

namespace {

constexpr uint32_t kMaxLevels = 32;

__device__ __forceinline__ unsigned long long fmix64(unsigned long long x) {
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 33;
    x *= 0xC4CEB9FE1A85EC53ull;
    x ^= x >> 33;
    return x;
}

// bit of `key` in level `l` of `size_bits` bits (multiply-high range reduction)
__device__ __forceinline__ uint64_t level_pos(uint32_t key, uint32_t l, uint64_t size_bits) {
    const unsigned long long h = fmix64((unsigned long long)key ^ ((unsigned long long)(l + 1) * 0x9E3779B97F4A7C15ull));
    return (uint64_t)__umul64hi(h, size_bits);
}

__global__ void mark_kernel(const uint32_t* __restrict__ keys, uint64_t m, uint32_t l, uint64_t size_bits,
                            unsigned long long* __restrict__ seen, unsigned long long* __restrict__ twice) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t pos = level_pos(keys[i], l, size_bits);
        const unsigned long long bit = 1ull << (pos & 63);
        const unsigned long long old = atomicOr(&seen[pos >> 6], bit);
        if (old & bit) atomicOr(&twice[pos >> 6], bit);
    }
}

// placed bits of the level = seen once
__global__ void settle_kernel(const unsigned long long* __restrict__ seen, const unsigned long long* __restrict__ twice,
                              uint64_t words, unsigned long long* __restrict__ bits) {
    for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < words; w += (uint64_t)gridDim.x * blockDim.x)
        bits[w] = seen[w] & ~twice[w];
}

// 1 for keys that collided (they go on to the next level)
__global__ void collided_kernel(const uint32_t* __restrict__ keys, uint64_t m, uint32_t l, uint64_t size_bits,
                                const unsigned long long* __restrict__ twice, uint8_t* __restrict__ flag) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t pos = level_pos(keys[i], l, size_bits);
        flag[i] = (twice[pos >> 6] >> (pos & 63)) & 1ull;
    }
}

__global__ void popcount_kernel(const unsigned long long* __restrict__ bits, uint64_t words,
                                unsigned long long* __restrict__ cnt) {
    for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < words; w += (uint64_t)gridDim.x * blockDim.x)
        cnt[w] = __popcll(bits[w]);
}

struct LevelTable {
    uint32_t levels;
    uint64_t size_bits[kMaxLevels];
    uint64_t word_off[kMaxLevels];
};

__global__ void lookup_kernel(const uint32_t* __restrict__ keys, uint64_t m, LevelTable t,
                              const unsigned long long* __restrict__ bits, const unsigned long long* __restrict__ rank,
                              const uint32_t* __restrict__ fallback, uint64_t n_fallback, uint64_t placed,
                              uint64_t* __restrict__ ids) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t key = keys[i];
        uint64_t id = ~0ull;
        for (uint32_t l = 0; l < t.levels; ++l) {
            const uint64_t pos = level_pos(key, l, t.size_bits[l]);
            const uint64_t w = t.word_off[l] + (pos >> 6);
            const unsigned long long word = bits[w];
            const unsigned long long bit = 1ull << (pos & 63);
            if (word & bit) {
                id = rank[w] + __popcll(word & (bit - 1));
                break;
            }
        }
        if (id == ~0ull && n_fallback) {
            uint64_t lo = 0, hi = n_fallback;
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1;
                if (fallback[mid] < key) lo = mid + 1;
                else hi = mid;
            }
            if (lo < n_fallback && fallback[lo] == key) id = placed + lo;
        }
        ids[i] = id;
    }
}

template <class T>
hipError_t dmalloc(T** p, size_t n) {
    return hipMalloc(reinterpret_cast<void**>(p), std::max<size_t>(1, n) * sizeof(T));
}

inline uint32_t grid_for(uint64_t m) { return (uint32_t)std::min<uint64_t>((m + 255) / 256, 65536); }

}  // namespace

struct kmp_mphf {
    int device = 0;
    uint64_t n = 0, placed = 0, n_fallback = 0, words = 0;
    double gamma = 3.0;
    LevelTable t{};
    unsigned long long* bits = nullptr;
    unsigned long long* rank = nullptr;
    uint32_t* fallback = nullptr;
    ~kmp_mphf() {
        if (bits) (void)hipFree(bits);
        if (rank) (void)hipFree(rank);
        if (fallback) (void)hipFree(fallback);
    }
};

namespace kmp {

int mphf_build_device(const uint32_t* d_keys, uint64_t n, double gamma, hipStream_t st, kmp_mphf** out) {
    *out = nullptr;
    if (!(gamma >= 1.0) || gamma > 100.0 || (n && !d_keys)) return KMP_EINVAL;
    kmp_mphf* m = new (std::nothrow) kmp_mphf;
    if (!m) return KMP_ENOMEM;
    (void)hipGetDevice(&m->device);
    m->n = n;
    m->gamma = gamma;
    // level sizes are only known as the build proceeds: keep each level's placed bits in its own
    // buffer, concatenate at the end
    std::vector<unsigned long long*> lvl_bits;
    uint32_t *cur = nullptr, *nxt = nullptr, *d_cnt = nullptr;
    uint8_t* flag = nullptr;
    unsigned long long *seen = nullptr, *twice = nullptr, *pc = nullptr;
    void* scratch = nullptr;
    size_t scratch_n = 0;
    auto fail = [&](int rc) {
        for (auto* b : lvl_bits) (void)hipFree(b);
        for (void* q : {(void*)cur, (void*)nxt, (void*)d_cnt, (void*)flag, (void*)seen, (void*)twice, (void*)pc, scratch})
            if (q) (void)hipFree(q);
        delete m;
        return rc;
    };
#define MB(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) return fail(e_ == hipErrorOutOfMemory ? KMP_ENOMEM : KMP_EDEVICE); \
    } while (0)
    MB(dmalloc(&cur, n));
    MB(dmalloc(&nxt, n));
    MB(dmalloc(&flag, n));
    MB(dmalloc(&d_cnt, 1));
    if (n) MB(hipMemcpyAsync(cur, d_keys, n * 4, hipMemcpyDeviceToDevice, st));
    uint64_t remaining = n, total_words = 0;
    uint32_t l = 0;
    while (remaining && l < kMaxLevels) {
        const uint64_t words = std::max<uint64_t>(1, (uint64_t)std::ceil(gamma * (double)remaining / 64.0));
        const uint64_t size_bits = words * 64;
        if (seen) (void)hipFree(seen);
        if (twice) (void)hipFree(twice);
        seen = twice = nullptr;
        MB(dmalloc(&seen, words));
        MB(dmalloc(&twice, words));
        MB(hipMemsetAsync(seen, 0, words * 8, st));
        MB(hipMemsetAsync(twice, 0, words * 8, st));
        mark_kernel<<<grid_for(remaining), 256, 0, st>>>(cur, remaining, l, size_bits, seen, twice);
        unsigned long long* b = nullptr;
        MB(dmalloc(&b, words));
        lvl_bits.push_back(b);
        settle_kernel<<<grid_for(words), 256, 0, st>>>(seen, twice, words, b);
        collided_kernel<<<grid_for(remaining), 256, 0, st>>>(cur, remaining, l, size_bits, twice, flag);
        size_t need = 0;
        MB(rocprim::select(nullptr, need, cur, flag, nxt, d_cnt, (size_t)remaining, st));
        if (need > scratch_n) {
            if (scratch) (void)hipFree(scratch);
            scratch = nullptr;
            MB(hipMalloc(&scratch, need));
            scratch_n = need;
        }
        MB(rocprim::select(scratch, need, cur, flag, nxt, d_cnt, (size_t)remaining, st));
        uint32_t h = 0;
        MB(hipMemcpyAsync(&h, d_cnt, 4, hipMemcpyDeviceToHost, st));
        MB(hipStreamSynchronize(st));
        m->t.size_bits[l] = size_bits;
        m->t.word_off[l] = total_words;
        total_words += words;
        std::swap(cur, nxt);
        remaining = h;
        ++l;
    }
    m->t.levels = l;
    m->words = total_words;
    // concatenated level bits + popcount prefix = ranks
    MB(dmalloc(&m->bits, total_words));
    MB(dmalloc(&m->rank, total_words));
    for (uint32_t i = 0; i < l; ++i)
        MB(hipMemcpyAsync(m->bits + m->t.word_off[i], lvl_bits[i], m->t.size_bits[i] / 8, hipMemcpyDeviceToDevice,
                          st));
    MB(dmalloc(&pc, total_words));
    if (total_words) {
        popcount_kernel<<<grid_for(total_words), 256, 0, st>>>(m->bits, total_words, pc);
        size_t need = 0;
        MB(rocprim::exclusive_scan(nullptr, need, pc, m->rank, 0ull, (size_t)total_words,
                                   rocprim::plus<unsigned long long>(), st));
        if (need > scratch_n) {
            if (scratch) (void)hipFree(scratch);
            scratch = nullptr;
            MB(hipMalloc(&scratch, need));
            scratch_n = need;
        }
        MB(rocprim::exclusive_scan(scratch, need, pc, m->rank, 0ull, (size_t)total_words,
                                   rocprim::plus<unsigned long long>(), st));
    }
    // fallback: the keys no level placed, sorted
    m->n_fallback = remaining;
    m->placed = n - remaining;
    MB(dmalloc(&m->fallback, remaining));
    if (remaining) {
        size_t ns = 0;
        MB(rocprim::radix_sort_keys(nullptr, ns, cur, m->fallback, (size_t)remaining, 0u, 32u, st));
        if (ns > scratch_n) {
            if (scratch) (void)hipFree(scratch);
            scratch = nullptr;
            MB(hipMalloc(&scratch, ns));
            scratch_n = ns;
        }
        MB(rocprim::radix_sort_keys(scratch, ns, cur, m->fallback, (size_t)remaining, 0u, 32u, st));
    }
    MB(hipStreamSynchronize(st));
    if (remaining) {
        // equal keys collide on every level, so duplicates can only end here
        std::vector<uint32_t> fb(remaining);
        MB(hipMemcpy(fb.data(), m->fallback, remaining * 4, hipMemcpyDeviceToHost));
        for (uint64_t i = 1; i < remaining; ++i)
            if (fb[i] == fb[i - 1]) return fail(KMP_EINVAL);
    }
#undef MB
    for (auto* b : lvl_bits) (void)hipFree(b);
    for (void* q : {(void*)cur, (void*)nxt, (void*)d_cnt, (void*)flag, (void*)seen, (void*)twice, (void*)pc, scratch})
        if (q) (void)hipFree(q);
    *out = m;
    return KMP_OK;
}

int mphf_lookup_device(const kmp_mphf* m, const uint32_t* d_keys, uint64_t n, uint64_t* d_ids, hipStream_t st) {
    if (!m || (n && (!d_keys || !d_ids))) return KMP_EINVAL;
    if (n == 0) return KMP_OK;
    lookup_kernel<<<grid_for(n), 256, 0, st>>>(d_keys, n, m->t, m->bits, m->rank, m->fallback, m->n_fallback,
                                               m->placed, d_ids);
    return hipGetLastError() == hipSuccess ? KMP_OK : KMP_EDEVICE;
}

}  // namespace kmp


namespace {

__global__ void repeat_flag_kernel(const uint32_t* __restrict__ counts, uint64_t runs, uint8_t* __restrict__ flag) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < runs; i += (uint64_t)gridDim.x * blockDim.x)
        flag[i] = counts[i] >= 2;
}

__global__ void scatter_by_id_kernel(const uint64_t* __restrict__ ids, const uint32_t* __restrict__ codes,
                                     const uint32_t* __restrict__ df, uint64_t m, uint32_t* __restrict__ code_by_id,
                                     uint32_t* __restrict__ df_by_id) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        code_by_id[ids[i]] = codes[i];
        df_by_id[ids[i]] = df[i];
    }
}

__constant__ CodeLut m_lut = make_lut();

// window codes of protein p (one block per protein), dense window order
__global__ void hk_codes_kernel(const uint8_t* __restrict__ res, const uint64_t* __restrict__ off,
                                const uint64_t* __restrict__ wofs, int k, uint32_t* __restrict__ codes) {
    const uint32_t p = blockIdx.x;
    const uint64_t base = off[p], w0 = wofs[p], nw = wofs[p + 1] - w0;
    for (uint64_t j = threadIdx.x; j < nw; j += blockDim.x) {
        uint32_t v = 0;
        for (int t = 0; t < k; ++t) v = v * kRadix + m_lut.v[res[base + j + t]];
        codes[w0 + j] = v;
    }
}

// (id, window) of every repeat window; non-members (lookup miss or a foreign key that lands on a
// set bit) sort last
__global__ void hk_keys_kernel(const uint32_t* __restrict__ codes, const uint64_t* __restrict__ ids, uint64_t W,
                               const uint32_t* __restrict__ code_by_id, uint64_t repeat,
                               unsigned long long* __restrict__ keys) {
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < W; g += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t id = ids[g];
        const bool ok = id < repeat && code_by_id[id] == codes[g];
        keys[g] = ok ? ((unsigned long long)id << 32 | g) : ~0ull;
    }
}

// protein owning dense window g: the largest p with wofs[p] <= g
__device__ __forceinline__ uint32_t protein_of(const uint64_t* __restrict__ wofs, uint32_t n, uint64_t g) {
    uint32_t lo = 0, hi = n;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (wofs[mid] <= g) lo = mid;
        else hi = mid;
    }
    return lo;
}

// first window of each (protein, id) run (modify_hash_five_mer's hash_map, protein.rs:167-172),
// re-keyed (window, id) for the position-order sort
__global__ void hk_first_kernel(const unsigned long long* __restrict__ sorted, uint64_t W,
                                const uint64_t* __restrict__ wofs, uint32_t n, unsigned long long* __restrict__ keys) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < W; i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long key = sorted[i];
        unsigned long long out = ~0ull;
        if (key != ~0ull) {
            const uint64_t id = key >> 32, g = key & 0xFFFFFFFFull;
            bool first = true;
            if (i > 0) {
                const unsigned long long prev = sorted[i - 1];
                first = (prev >> 32) != id || protein_of(wofs, n, prev & 0xFFFFFFFFull) != protein_of(wofs, n, g);
            }
            if (first) out = (unsigned long long)g << 32 | id;
        }
        keys[i] = out;
    }
}

// per-protein starts in the position-ordered keys, and the ids themselves
__global__ void hk_offsets_kernel(const unsigned long long* __restrict__ sorted, uint64_t W,
                                  const uint64_t* __restrict__ wofs, uint32_t n, uint64_t* __restrict__ out_off) {
    for (uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; p <= n; p += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long x = (unsigned long long)wofs[p] << 32;
        uint64_t lo = 0, hi = W;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (sorted[mid] < x) lo = mid + 1;
            else hi = mid;
        }
        out_off[p] = lo;
    }
}

__global__ void hk_ids_kernel(const unsigned long long* __restrict__ sorted, uint64_t m, uint32_t* __restrict__ ids) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x)
        ids[i] = (uint32_t)sorted[i];
}

}  // namespace

namespace kmp {

int repeat_mphf_build(const uint32_t* d_uniq, const uint32_t* d_counts, uint64_t runs, double gamma, hipStream_t st,
                      kmp_mphf** mphf, uint32_t** d_code_by_id, uint32_t** d_df_by_id, uint64_t* repeat) {
    *mphf = nullptr;
    *d_code_by_id = *d_df_by_id = nullptr;
    *repeat = 0;
    uint8_t* flag = nullptr;
    uint32_t *codes = nullptr, *df = nullptr, *cnt = nullptr;
    uint64_t* ids = nullptr;
    void* scratch = nullptr;
    int rc = KMP_OK;
    auto done = [&](int r) {
        for (void* q : {(void*)flag, (void*)codes, (void*)df, (void*)cnt, (void*)ids, scratch})
            if (q) (void)hipFree(q);
        return r;
    };
#define RB(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) return done(e_ == hipErrorOutOfMemory ? KMP_ENOMEM : KMP_EDEVICE); \
    } while (0)
    RB(dmalloc(&flag, runs));
    RB(dmalloc(&codes, runs));
    RB(dmalloc(&df, runs));
    RB(dmalloc(&cnt, 2));
    if (runs) repeat_flag_kernel<<<grid_for(runs), 256, 0, st>>>(d_counts, runs, flag);
    size_t need = 0;
    RB(rocprim::select(nullptr, need, d_uniq, flag, codes, cnt, (size_t)runs, st));
    RB(hipMalloc(&scratch, std::max<size_t>(need, 16)));
    RB(rocprim::select(scratch, need, d_uniq, flag, codes, cnt, (size_t)runs, st));
    RB(rocprim::select(scratch, need, d_counts, flag, df, cnt + 1, (size_t)runs, st));
    uint32_t R = 0;
    RB(hipMemcpyAsync(&R, cnt, 4, hipMemcpyDeviceToHost, st));
    RB(hipStreamSynchronize(st));
    rc = mphf_build_device(codes, R, gamma, st, mphf);
    if (rc != KMP_OK) return done(rc);
    RB(dmalloc(&ids, R));
    RB(dmalloc(d_code_by_id, R));
    RB(dmalloc(d_df_by_id, R));
    rc = mphf_lookup_device(*mphf, codes, R, ids, st);
    if (rc != KMP_OK) return done(rc);
    if (R) scatter_by_id_kernel<<<grid_for(R), 256, 0, st>>>(ids, codes, df, R, *d_code_by_id, *d_df_by_id);
    RB(hipStreamSynchronize(st));
#undef RB
    *repeat = R;
    return done(KMP_OK);
}

int hash_kmers_device(const kmp_mphf* m, const uint8_t* d_res, const uint64_t* d_off, const uint64_t* h_off,
                      uint32_t n, int k, const uint32_t* d_code_by_id, uint64_t repeat, hipStream_t st,
                      uint32_t** d_ids, std::vector<uint64_t>& h_ids_off) {
    *d_ids = nullptr;
    h_ids_off.assign((size_t)n + 1, 0);
    std::vector<uint64_t> wofs((size_t)n + 1, 0);
    for (uint32_t p = 0; p < n; ++p) {
        const uint64_t L = h_off[p + 1] - h_off[p];
        wofs[p + 1] = wofs[p] + (L >= (uint64_t)k ? L - k + 1 : 0);
    }
    const uint64_t W = wofs[n];
    if (W >= 0xFFFFFFFFull) return KMP_EINVAL;  // window index must fit the low key half
    if (W == 0 || repeat == 0) return dmalloc(d_ids, 1) == hipSuccess ? KMP_OK : KMP_ENOMEM;
    uint64_t *d_wofs = nullptr, *ids64 = nullptr, *d_ioff = nullptr;
    uint32_t* codes = nullptr;
    unsigned long long *ka = nullptr, *kb = nullptr;
    void* scratch = nullptr;
    auto done = [&](int r) {
        for (void* q : {(void*)d_wofs, (void*)ids64, (void*)d_ioff, (void*)codes, (void*)ka, (void*)kb, scratch})
            if (q) (void)hipFree(q);
        return r;
    };
#define HB(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) return done(e_ == hipErrorOutOfMemory ? KMP_ENOMEM : KMP_EDEVICE); \
    } while (0)
    HB(dmalloc(&d_wofs, n + 1));
    HB(dmalloc(&d_ioff, n + 1));
    HB(dmalloc(&codes, W));
    HB(dmalloc(&ids64, W));
    HB(dmalloc(&ka, W));
    HB(dmalloc(&kb, W));
    HB(hipMemcpyAsync(d_wofs, wofs.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
    hk_codes_kernel<<<n, 256, 0, st>>>(d_res, d_off, d_wofs, k, codes);
    int rc = mphf_lookup_device(m, codes, W, ids64, st);
    if (rc != KMP_OK) return done(rc);
    hk_keys_kernel<<<grid_for(W), 256, 0, st>>>(codes, ids64, W, d_code_by_id, repeat, ka);
    size_t need = 0;
    HB(rocprim::radix_sort_keys(nullptr, need, ka, kb, (size_t)W, 0u, 64u, st));
    HB(hipMalloc(&scratch, std::max<size_t>(need, 16)));
    HB(rocprim::radix_sort_keys(scratch, need, ka, kb, (size_t)W, 0u, 64u, st));
    hk_first_kernel<<<grid_for(W), 256, 0, st>>>(kb, W, d_wofs, n, ka);
    HB(rocprim::radix_sort_keys(scratch, need, ka, kb, (size_t)W, 0u, 64u, st));
    hk_offsets_kernel<<<grid_for(n + 1), 256, 0, st>>>(kb, W, d_wofs, n, d_ioff);
    HB(hipGetLastError());
    HB(hipMemcpyAsync(h_ids_off.data(), d_ioff, (n + 1) * 8, hipMemcpyDeviceToHost, st));
    HB(hipStreamSynchronize(st));
    const uint64_t total = h_ids_off[n];
    HB(dmalloc(d_ids, total));
    if (total) hk_ids_kernel<<<grid_for(total), 256, 0, st>>>(kb, total, *d_ids);
    HB(hipStreamSynchronize(st));
#undef HB
    return done(KMP_OK);
}

}  // namespace kmp

extern "C" {

int kmp_mphf_lookup(const kmp_mphf* m, const uint32_t* keys, uint64_t n, uint64_t* ids) {
    if (!m || (n && (!keys || !ids))) return KMP_EINVAL;
    if (n == 0) return KMP_OK;
    if (hipSetDevice(m->device) != hipSuccess) return KMP_EDEVICE;
    uint32_t* dk = nullptr;
    uint64_t* di = nullptr;
    int rc = KMP_OK;
    if (hipMalloc(&dk, n * 4) != hipSuccess || hipMalloc(&di, n * 8) != hipSuccess) rc = KMP_ENOMEM;
    if (rc == KMP_OK && hipMemcpy(dk, keys, n * 4, hipMemcpyHostToDevice) != hipSuccess) rc = KMP_EDEVICE;
    if (rc == KMP_OK) rc = kmp::mphf_lookup_device(m, dk, n, di, nullptr);
    if (rc == KMP_OK && hipMemcpy(ids, di, n * 8, hipMemcpyDeviceToHost) != hipSuccess) rc = KMP_EDEVICE;
    if (dk) (void)hipFree(dk);
    if (di) (void)hipFree(di);
    return rc;
}

int kmp_mphf_dev_lookup(const kmp_mphf* m, const uint32_t* d_keys, uint64_t n, uint64_t* d_ids, void* stream) {
    return kmp::mphf_lookup_device(m, d_keys, n, d_ids, reinterpret_cast<hipStream_t>(stream));
}

int kmp_mphf_info(const kmp_mphf* m, uint64_t* n, uint32_t* levels, uint64_t* bits, uint64_t* n_fallback) {
    if (!m) return KMP_EINVAL;
    if (n) *n = m->n;
    if (levels) *levels = m->t.levels;
    if (bits) *bits = m->words * 64;
    if (n_fallback) *n_fallback = m->n_fallback;
    return KMP_OK;
}

void kmp_mphf_free(kmp_mphf* m) { delete m; }

}  // extern "C"
