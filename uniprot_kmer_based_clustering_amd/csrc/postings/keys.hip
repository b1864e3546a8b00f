// postings/keys.hip — key layout, key chunks, the flat layout's expansion, workgroup scans.
// Part of kmp_postings.hip (included there; not a translation unit of its own).

__constant__ CodeLut c_lut = make_lut();

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

unsigned bits_for(uint64_t v) {  // bits needed for values < v
    unsigned b = 0;
    while (b < 64 && (v - 1) >> b) ++b;
    return b ? b : 1;
}

constexpr unsigned long long kNoKey = ~0ull;

// compute units of the current device (persistent grids), looked up once per device and thread
uint32_t device_cus() {
    static thread_local int dev = -1;
    static thread_local uint32_t cus = 256;
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) return cus;
    if (d != dev) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && v > 0)
            cus = (uint32_t)v;
        dev = d;
    }
    return cus;
}


// rocprim 4.2 (ROCm 7.2): with the default config, radix_sort_keys on fewer than 1M keys takes a
// merge-sort path that returns unsorted, non-permuted data for bit ranges [b, 64) with b > 0
// (tools/sort_check.hip reproduces it).  Onesweep (merge-sort limit 0) is correct for every range
// and size, so every sort here uses it.
using SortCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                           rocprim::default_config, 0>;
// Pair keys (p * N + q, 34 bits at N = 100k): 9-bit digits in 1024 x 8 workgroups take 4 onesweep
// passes instead of 5 (tools/radix_bits_bench.hip: 0.209 vs 0.269 ms for 5.4 M keys); 10-bit
// digits are slower and 11 bits exceed the LDS.  Merge-sort limit 0, as for SortCfg.
using PairSortCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<512, 12>, rocprim::kernel_config<1024, 8>, 9,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;
constexpr unsigned kClsBits = 16;

// Two key layouts (u64, kNoKey = all ones is the padding of every layout):
//   flat     [ code | class (16 bits, when it fits) | p ]       sorted on the code bits (stable)
//   bucketed [ 0 | h(code) (32) | p | class (cb bits) ]         h(code) = code * A mod 2^32 is a
//            bijection, so h identifies the k-mer; bucket = top bbits of h (equal k-mers share a
//            bucket); keys are sorted on bits [bucket .. 64): the zero top bit makes the padding
//            sort last.  cb = 31 - pbits (16 at most); a class id that does not fit sends the
//            call to the flat layout.
struct Layout {
    unsigned pbits;    // protein index bits
    unsigned cbits;    // code bits
    unsigned shift;    // flat: code starts here
    bool cls_in_key;   // flat: class bits between code and p
    bool bucketed;
    unsigned bbits;    // bucketed: bucket index bits
    unsigned clsbits;  // bucketed: class bits (bits [0, clsbits))
    unsigned hshift;   // bucketed: h(code) starts here (= pbits + clsbits)
    unsigned sort_lo, sort_hi;  // radix-sorted bit range
    uint32_t mean_keys;         // bucketed: expected keys per bucket (windows / buckets)
};

constexpr uint32_t kBucketTarget = 1024;  // mean keys per bucket
constexpr uint32_t kHashA = 0x9E3779B1u;  // odd: code -> h(code) is a bijection of u32

Layout make_layout(uint32_t n, int k, uint64_t slots, bool bucketed) {
    Layout l{};
    l.pbits = bits_for(n);
    l.cbits = bits_for(pow21(k));
    if (bucketed && l.pbits <= 30) {
        unsigned bb = 1;
        while (bb < 20 && (slots >> bb) > kBucketTarget) ++bb;  // bb + sub bits <= 32
        l.bucketed = true;
        l.bbits = bb;
        l.clsbits = std::min(16u, 31u - l.pbits);
        l.hshift = l.pbits + l.clsbits;
        l.sort_lo = l.hshift + 32 - bb;
        l.sort_hi = 64;
        // a protein's slot region (L + 4 slots and more) holds L - k + 1 windows: k + 3 slots at
        // least hold none, so this is an upper bound of the mean
        const uint64_t spare = (uint64_t)(k + 3) * n;
        l.mean_keys = (uint32_t)((slots > spare ? slots - spare : 0ull) >> bb);
        return l;
    }
    l.cls_in_key = l.pbits + kClsBits + l.cbits <= 64;
    l.shift = l.pbits + (l.cls_in_key ? kClsBits : 0);
    l.sort_lo = l.shift;
    l.sort_hi = l.shift + l.cbits;
    return l;
}

__device__ __forceinline__ unsigned long long make_key(uint32_t code, uint16_t c, uint32_t p, const Layout& l) {
    if (l.bucketed)
        return ((unsigned long long)(code * kHashA) << l.hshift) | ((unsigned long long)p << l.clsbits) |
               (c & ((1u << l.clsbits) - 1));
    unsigned long long x = ((unsigned long long)code << l.shift) | p;
    if (l.cls_in_key) x |= (unsigned long long)c << l.pbits;
    return x;
}

// class ids wider than the bucketed layout's class field -> flat layout
__device__ __forceinline__ void check_class(uint16_t c, const Layout& l, uint32_t* flags) {
    if (l.bucketed && l.clsbits < 16 && (c >> l.clsbits)) flags[1] = 1;
}

// keys of the unfiltered K(p) slots: K(p)[t] for t < |K(p)|, kNoKey for the rest of the region;
// block n fills the tail of the buffer past the last region (no memset needed)
__global__ __launch_bounds__(256) void set_keys_kernel(const uint32_t* __restrict__ set,
                                                       const uint32_t* __restrict__ set_len,
                                                       const uint64_t* __restrict__ res_off,
                                                       const uint16_t* __restrict__ cls, uint32_t n, uint64_t slots,
                                                       Layout lay, unsigned long long* __restrict__ keys,
                                                       uint32_t* __restrict__ flags) {
    const uint32_t p = blockIdx.x;
    if (p == n) {
        for (uint64_t i = set_base(res_off[n], n) + threadIdx.x; i < slots; i += 256) keys[i] = kNoKey;
        return;
    }
    const uint64_t b = set_base(res_off[p], p), e = set_base(res_off[p + 1], p + 1);
    const uint32_t len = set_len[p];
    const uint16_t c = cls[p];
    if (threadIdx.x == 0) check_class(c, lay, flags);
    for (uint64_t i = b + threadIdx.x; i < e; i += 256) {
        const uint64_t o = i - b;
        keys[i] = o < len ? make_key(set[i], c, p, lay) : kNoKey;
    }
}

// one key per window straight from the residues (Protein::new, protein.rs:82-94: window j of
// protein p is residues [j, j+k), radix-21, first residue most significant), same slot layout.
// Workgroup g owns slots [slot_begin + g*kKeyChunk, ... + kKeyChunk) of proteins
// [p_lo, p_hi) (about 13 proteins per chunk at L ~ 300).  It finds them by binary search on
// set_base, recodes just the residue span its windows need into LDS (byte -> code), and writes the
// chunk's keys coalesced; slots past a protein's windows (and past the last region) get kNoKey.
// keys[i - slot_begin] for slot i.
constexpr int kKeyThreads = 256;
constexpr uint32_t kKeyChunk = 4096;
constexpr uint32_t kKeyProtMax = kKeyChunk / 4 + 2;                // a region spans >= 4 slots
// residues a chunk can need: a protein's region is longer than its residue count, so the span is
// at most the chunk plus the last window's k - 1 residues
constexpr uint32_t kKeyResMax = kKeyChunk + 64;

// first[c] = the protein whose region holds the chunk's first slot (p_hi: the tail past the last
// region); one thread per protein writes the chunk starts that fall in its region
__global__ void chunk_first_kernel(const uint64_t* __restrict__ res_off, uint32_t p_lo, uint32_t p_hi,
                                   uint64_t slot_begin, uint64_t slot_end, uint32_t n_chunks,
                                   uint32_t* __restrict__ first) {
    const uint32_t p = p_lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (p > p_hi) return;
    const uint64_t b = set_base(res_off[p], p) - slot_begin;
    const uint64_t e = (p < p_hi ? set_base(res_off[p + 1], p + 1) : slot_end) - slot_begin;
    for (uint64_t c = (b + kKeyChunk - 1) / kKeyChunk; c * kKeyChunk < e && c < n_chunks; ++c) first[c] = p;
}

// LDS state of one key chunk: residue codes of the chunk's span and its proteins' geometry
struct KeyChunk {
    uint8_t lut[256];
    __attribute__((aligned(16))) uint8_t rc[kKeyResMax + 32];  // residue codes from a0 = r0 & ~15
    uint32_t pb[kKeyProtMax + 1];   // region start of each protein, relative to c0 (may wrap)
    int32_t pr[kKeyProtMax];        // LDS index of the protein's residue 0 (may be < 0)
    uint32_t pw[kKeyProtMax];       // window count
    uint16_t pc[kKeyProtMax];       // class
    uint32_t np;
    uint64_t r0, r1;
};

// Stage chunk [c0, c1) of proteins [first, p_hi): the proteins whose regions overlap it and the
// residue span their windows need, recoded into LDS.  Ends with a barrier.
template <uint32_t kThr = kKeyThreads>
__device__ __forceinline__ void key_chunk_load(KeyChunk& s, const uint8_t* __restrict__ res,
                                               const uint64_t* __restrict__ res_off,
                                               const uint16_t* __restrict__ cls, int k, uint32_t p_hi,
                                               uint64_t c0, uint64_t c1, uint32_t first, const Layout& lay,
                                               uint32_t* __restrict__ flags) {
    const int tid = threadIdx.x;
    if (tid < 256) s.lut[tid] = c_lut.v[tid];
    if (tid == 0) {
        s.np = 0;
        s.r0 = s.r1 = 0;
    }
    __syncthreads();
    // the chunk's proteins: first + t while its region starts before c1 (one parallel round)
    for (uint32_t t = tid; t < kKeyProtMax && first + t < p_hi; t += kThr) {
        const uint32_t p = first + t;
        const uint64_t off = res_off[p], L = res_off[p + 1] - off;
        const uint64_t b = set_base(off, p);
        if (b >= c1) break;
        const uint32_t nw = L >= (uint64_t)k ? (uint32_t)(L - k + 1) : 0u;
        s.pb[t] = (uint32_t)(b - c0);  // wraps for the first protein when it starts before c0
        s.pw[t] = nw;
        s.pc[t] = cls[p];
        check_class(s.pc[t], lay, flags);
        atomicMax(&s.np, t + 1);
        const uint64_t j0 = c0 > b ? c0 - b : 0;
        const uint64_t j1 = min<uint64_t>(nw, c1 - b);
        if (t == 0) s.r0 = off + min<uint64_t>(j0, L);
        if (j1 > j0) atomicMax((unsigned long long*)&s.r1, (unsigned long long)(off + j1 + k - 1));
    }
    __syncthreads();
    const uint32_t np = s.np;
    const uint64_t r0 = s.r0, r1 = max(s.r0, s.r1);
    // stage the span with independent 16-byte loads (byte loads where a vector would pass the end
    // of the range's residues or the base is unaligned), recoded through the LUT, one 16-byte LDS
    // store per vector
    const uint64_t a0 = r0 & ~15ull, res_end = res_off[p_hi];
    const bool vec_ok = ((uintptr_t)res & 15u) == 0;
    const uint32_t nv = (uint32_t)((r1 - a0 + 15) >> 4);
    for (uint32_t v = tid; v < nv; v += kThr) {
        const uint64_t g = a0 + 16ull * v;
        uint32_t w[4];
        if (vec_ok && g + 16 <= res_end) {
            const uint4 q = *reinterpret_cast<const uint4*>(res + g);
            w[0] = q.x, w[1] = q.y, w[2] = q.z, w[3] = q.w;
        } else {
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                w[d] = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const uint64_t i = g + 4 * d + b;
                    w[d] |= (uint32_t)(i < res_end ? res[i] : 0) << (8 * b);
                }
            }
        }
        auto code4 = [&](uint32_t x) {
            return (uint32_t)s.lut[x & 255u] | (uint32_t)s.lut[(x >> 8) & 255u] << 8 |
                   (uint32_t)s.lut[(x >> 16) & 255u] << 16 | (uint32_t)s.lut[x >> 24] << 24;
        };
        *reinterpret_cast<uint4*>(s.rc + 16 * v) =
            make_uint4(code4(w[0]), code4(w[1]), code4(w[2]), code4(w[3]));
    }
    for (uint32_t t = tid; t < np; t += kThr) s.pr[t] = (int32_t)((int64_t)res_off[first + t] - (int64_t)a0);
    __syncthreads();
}

// key of chunk slot c0 + i (kNoKey past a protein's windows)
__device__ __forceinline__ unsigned long long key_chunk_key(const KeyChunk& s, uint32_t i, int k, uint32_t first,
                                                            const Layout& lay) {
    const uint32_t np = s.np;
    if (!np) return kNoKey;
    // protein of slot c0 + i: last t with region start <= c0 + i (t = 0 may start before c0)
    uint32_t a = 0, b = np;
    while (a + 1 < b) {
        const uint32_t mid = (a + b) >> 1;
        if (s.pb[mid] <= i) a = mid;
        else b = mid;
    }
    const uint32_t j = i - s.pb[a];  // window index (pb[0] wraps: i - pb[0] = c0 + i - b0)
    if (j >= s.pw[a]) return kNoKey;
    const uint8_t* w = s.rc + (s.pr[a] + (int32_t)j);
    uint32_t v = 0;
    for (int t = 0; t < k; ++t) v = v * kRadix + w[t];
    return make_key(v, s.pc[a], first + a, lay);
}

// The kPer consecutive chunk slots i0 .. i0 + kPer - 1: one binary search, then the protein's
// state in registers (reloaded at a region start: regions are >= 4 slots, so at most one per
// slot) and the radix-21 code rolled window to window (two LDS reads instead of k).
// emit(e, valid, h, lo) per slot: h = h(code), lo = the key's p | class bits; the key is
// (u64)h << hshift | lo.  pw21 = 21^(k-1).
template <uint32_t kPer, class Emit>
__device__ __forceinline__ void key_chunk_run(const KeyChunk& s, uint32_t i0, uint32_t n_slots, int k, uint32_t pw21,
                                              uint32_t first, const Layout& lay, Emit emit) {
    const uint32_t np = s.np;
    if (!np) {
#pragma unroll
        for (uint32_t e = 0; e < kPer; ++e) emit(e, false, 0u, 0ull);
        return;
    }
    uint32_t a = 0, b = np;
    while (a + 1 < b) {
        const uint32_t mid = (a + b) >> 1;
        if (s.pb[mid] <= i0) a = mid;
        else b = mid;
    }
    const uint32_t cmask = (1u << lay.clsbits) - 1;
    uint32_t nxt = a + 1 < np ? s.pb[a + 1] : 0xFFFFFFFFu;  // first slot of protein a + 1
    uint32_t j = i0 - s.pb[a];                              // window index (pb[0] may wrap)
    uint32_t nw = s.pw[a];
    int32_t r = s.pr[a] + (int32_t)j;                       // LDS index of window j's first residue
    unsigned long long lo = ((unsigned long long)(first + a) << lay.clsbits) | (s.pc[a] & cmask);
    uint32_t v = 0;
    bool have = false;  // v holds the code of window j - 1
#pragma unroll
    for (uint32_t e = 0; e < kPer; ++e) {
        const uint32_t i = i0 + e;
        if (i == nxt) {
            ++a;
            nxt = a + 1 < np ? s.pb[a + 1] : 0xFFFFFFFFu;
            j = 0;
            nw = s.pw[a];
            r = s.pr[a];
            lo = ((unsigned long long)(first + a) << lay.clsbits) | (s.pc[a] & cmask);
            have = false;
        }
        const bool valid = j < nw && i < n_slots;
        if (valid) {
            if (have) {
                v = (v - s.rc[r - 1] * pw21) * kRadix + s.rc[r + k - 1];
            } else {
                v = 0;
                for (int t = 0; t < k; ++t) v = v * kRadix + s.rc[r + t];
            }
        }
        have = valid;
        emit(e, valid, v * kHashA, lo);
        ++j;
        ++r;
    }
}

__global__ __launch_bounds__(kKeyThreads) void residue_keys_chunk_kernel(
    const uint8_t* __restrict__ res, const uint64_t* __restrict__ res_off, const uint16_t* __restrict__ cls,
    int k, uint32_t p_hi, uint64_t slot_begin, uint64_t slot_end, const uint32_t* __restrict__ chunk_first,
    Layout lay, unsigned long long* __restrict__ keys, uint32_t* __restrict__ flags) {
    __shared__ KeyChunk s;
    const uint64_t c0 = slot_begin + (uint64_t)blockIdx.x * kKeyChunk;
    const uint64_t c1 = min(c0 + kKeyChunk, slot_end);
    const uint32_t first = chunk_first[blockIdx.x];
    key_chunk_load(s, res, res_off, cls, k, p_hi, c0, c1, first, lay, flags);
    for (uint32_t i = threadIdx.x; i < (uint32_t)(c1 - c0); i += kKeyThreads)
        keys[c0 + i - slot_begin] = key_chunk_key(s, i, k, first, lay);
}

enum : int { kStSumS, kStDistinct, kStRepeat, kStCdf2, kStMaxDf, kStHeavy, kStInc, kStN };

constexpr int kExpThreads = 256;
constexpr int kExpRounds = 8;
constexpr uint64_t kExpChunk = (uint64_t)kExpThreads * kExpRounds;  // keys per workgroup

__device__ __forceinline__ unsigned long long stat_op(int t, unsigned long long a, unsigned long long b) {
    return t == kStMaxDf ? (a > b ? a : b) : a + b;
}

// Wave64 inclusive scans on DPP (VALU only, no LDS crossbar round trips): row_shr 1/2/4/8 scan
// each 16-lane row (bound_ctrl: a source before the row start reads 0), then row_bcast 15 / 31
// carry the row totals into the later rows (rows outside the row mask keep the old value, 0).
// Every lane of the wave must be active.
template <int kCtrl, int kRowMask = 0xF>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kCtrl, kRowMask, 0xF, true);
}
__device__ __forceinline__ uint32_t wave_iscan(uint32_t x) {
    x += dpp_mov<0x111>(x);
    x += dpp_mov<0x112>(x);
    x += dpp_mov<0x114>(x);
    x += dpp_mov<0x118>(x);
    x += dpp_mov<0x142, 0xA>(x);
    x += dpp_mov<0x143, 0xC>(x);
    return x;
}
// the wave's maximum (every lane; values are unsigned, so the 0 of an invalid source is neutral)
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
    x = max(x, dpp_mov<0x111>(x));
    x = max(x, dpp_mov<0x112>(x));
    x = max(x, dpp_mov<0x114>(x));
    x = max(x, dpp_mov<0x118>(x));
    x = max(x, dpp_mov<0x142, 0xA>(x));
    x = max(x, dpp_mov<0x143, 0xC>(x));
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_iscan(x), 63);
}

// exclusive scan of one value per thread over the workgroup; returns (prefix, total)
__device__ __forceinline__ void block_scan(uint32_t v, uint32_t& excl, uint32_t& total, uint32_t* wave_tot) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t x = wave_iscan(v);
    if (lane == 63) wave_tot[w] = x;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kExpThreads / 64; ++i) {
        const uint32_t t = wave_tot[i];
        before += i < w ? t : 0;
        tot += t;
    }
    __syncthreads();
    excl = before + x - v;
    total = tot;
}

// Σ C(df,2) incidence expansion (vertex.rs:103-137) with the AMR test of mod.rs:580-587.
// Element i (a key of protein p) is the smaller protein of every pair it forms with a later,
// non-duplicate element j of its run: pair key p * N + q.  The run's extent is found by scanning
// forward while the code matches.  Workgroup b owns keys [b*kExpChunk, (b+1)*kExpChunk).
//   kWrite = false: per-key kept-partner counts, the workgroup total and, at run heads, the df
//                   statistics (per-workgroup partials, no atomics);
//   kWrite = true:  workgroup offset (scan of the totals) + in-workgroup scan of the counts,
//                   then the pair keys are written there.
template <bool kWrite, bool kClsKey>
__global__ __launch_bounds__(kExpThreads) void expand_kernel(const unsigned long long* __restrict__ k, uint64_t slots,
                                                             Layout lay, const uint16_t* __restrict__ cls,
                                                             uint32_t n_prot, int require_diff, uint32_t heavy_df,
                                                             uint32_t* __restrict__ counts,
                                                             unsigned long long* __restrict__ block_stats,
                                                             unsigned long long* __restrict__ block_tot,
                                                             const unsigned long long* __restrict__ block_off,
                                                             unsigned long long* __restrict__ out) {
    __shared__ uint32_t wave_tot[kExpThreads / 64];
    const unsigned long long pmask = (1ull << lay.pbits) - 1;
    const unsigned shift = lay.shift;
    const bool bounded = heavy_df != 0xFFFFFFFFu;
    const uint64_t base = blockIdx.x * kExpChunk;
    unsigned long long st[kStN] = {0, 0, 0, 0, 0, 0, 0};
    unsigned long long o = kWrite ? block_off[blockIdx.x] : 0ull;
    for (int r = 0; r < kExpRounds; ++r) {
        const uint64_t i = base + (uint64_t)r * kExpThreads + threadIdx.x;
        const unsigned long long x = i < slots ? k[i] : kNoKey;
        const unsigned long long prev = (i > 0 && i < slots) ? k[i - 1] : kNoKey;
        // kNoKey sorts last, so a valid key's predecessor is valid or absent (i == 0)
        const bool live = x != kNoKey && x != prev;  // not padding, not a duplicate window of p
        const unsigned long long code = x >> shift;
        const bool head = live && (i == 0 || (prev >> shift) != code);
        uint32_t c = 0;
        if (kWrite) {
            uint32_t excl, total;
            const uint32_t mine = i < slots ? counts[i] : 0u;
            block_scan(mine, excl, total, wave_tot);
            if (mine) {
                unsigned long long pos = o + excl;
                const uint32_t p = (uint32_t)(x & pmask);
                const uint32_t cp = kClsKey ? (uint32_t)((x >> lay.pbits) & 0xFFFFu) : cls[p];
                const unsigned long long row = (unsigned long long)p * n_prot;
                unsigned long long last = x;
                for (uint64_t j = i + 1; j < slots; ++j) {
                    const unsigned long long y = k[j];
                    if ((y >> shift) != code) break;
                    if (y == last) continue;
                    last = y;
                    const uint32_t q = (uint32_t)(y & pmask);
                    const uint32_t cq = kClsKey ? (uint32_t)((y >> lay.pbits) & 0xFFFFu) : cls[q];
                    if (require_diff && cq == cp) continue;
                    out[pos++] = row + q;
                }
            }
            o += total;
            continue;
        }
        if (live) {
            uint64_t f = 1;  // df of the run (exact at heads; exact everywhere when bounded)
            if (bounded && !head) {
                unsigned long long last = x;
                for (uint64_t s = i; s > 0; --s) {
                    const unsigned long long y = k[s - 1];
                    if ((y >> shift) != code) break;
                    if (y != last) ++f;
                    last = y;
                }
            }
            const uint32_t p = (uint32_t)(x & pmask);
            const uint32_t cp = kClsKey ? (uint32_t)((x >> lay.pbits) & 0xFFFFu) : cls[p];
            unsigned long long last = x;
            uint64_t after = 0;
            for (uint64_t j = i + 1; j < slots; ++j) {
                const unsigned long long y = k[j];
                if ((y >> shift) != code) break;
                if (y == last) continue;
                last = y;
                ++after;
                const uint32_t q = (uint32_t)(y & pmask);
                const uint32_t cq = kClsKey ? (uint32_t)((y >> lay.pbits) & 0xFFFFu) : cls[q];
                c += !require_diff || cq != cp;
            }
            f += after;
            if (f > heavy_df) c = 0;
            st[kStSumS] += 1;
            if (head) {
                st[kStDistinct] += 1;
                st[kStRepeat] += f >= 2;
                if (f <= heavy_df) st[kStCdf2] += f * (f - 1) / 2;
                else st[kStHeavy] += f;
                st[kStMaxDf] = f > st[kStMaxDf] ? f : st[kStMaxDf];
            }
        }
        if (i < slots) counts[i] = c;
        st[kStInc] += c;
    }
    if (kWrite) return;
    __shared__ unsigned long long red[kExpThreads / 64][kStN];
#pragma unroll
    for (int t = 0; t < kStN; ++t) {
        unsigned long long v = st[t];
        for (int s = 32; s > 0; s >>= 1) v = stat_op(t, v, __shfl_down(v, s));
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][t] = v;
    }
    __syncthreads();
    if (threadIdx.x < kStN) {
        const int t = threadIdx.x;
        unsigned long long v = red[0][t];
        for (int w = 1; w < kExpThreads / 64; ++w) v = stat_op(t, v, red[w][t]);
        block_stats[(uint64_t)blockIdx.x * kStN + t] = v;
        if (t == kStInc) block_tot[blockIdx.x] = v;
    }
}

// reduction of the per-workgroup statistics: one workgroup
__global__ __launch_bounds__(1024) void reduce_stats_kernel(const unsigned long long* __restrict__ bs, uint32_t nb,
                                                            unsigned long long* __restrict__ acc) {
    __shared__ unsigned long long red[16][kStN];
    unsigned long long v[kStN] = {0, 0, 0, 0, 0, 0, 0};
    for (uint32_t b = threadIdx.x; b < nb; b += 1024)
#pragma unroll
        for (int t = 0; t < kStN; ++t) v[t] = stat_op(t, v[t], bs[(uint64_t)b * kStN + t]);
#pragma unroll
    for (int t = 0; t < kStN; ++t) {
        for (int s = 32; s > 0; s >>= 1) v[t] = stat_op(t, v[t], __shfl_down(v[t], s));
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][t] = v[t];
    }
    __syncthreads();
    if (threadIdx.x < kStN) {
        const int t = threadIdx.x;
        unsigned long long x = red[0][t];
        for (int w = 1; w < 16; ++w) x = stat_op(t, x, red[w][t]);
        acc[t] = x;
    }
}
