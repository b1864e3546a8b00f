// kmp_internal.hpp — shared constants of libkmerpair (host + device).
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define KMP_HD __host__ __device__
#else
#define KMP_HD
#endif

namespace kmp {

// Residue alphabet of src/protein.rs:9-13; any other byte encodes as 20 (:49-54).
constexpr char kAminoAcids[21] = {'C', 'S', 'T', 'A', 'G', 'P', 'D', 'E', 'Q', 'N', 'H',
                                  'R', 'K', 'M', 'I', 'L', 'V', 'W', 'Y', 'F', '*'};
constexpr uint32_t kRadix = 21;
constexpr int kMaxK = 7;  // 21^7 - 1 = 1,801,088,540 < 2^31: every code fits u32, 0xFFFFFFFF is free

inline uint64_t pow21(int k) {
    uint64_t v = 1;
    for (int i = 0; i < k; ++i) v *= kRadix;
    return v;
}

// byte -> residue code (amino_acid_to_bits, protein.rs:49-54): unknown bytes -> 20
struct CodeLut {
    uint8_t v[256];
};
constexpr CodeLut make_lut() {
    CodeLut l{};
    for (int b = 0; b < 256; ++b) {
        l.v[b] = 20;
        for (int i = 0; i < 21; ++i)
            if ((uint8_t)kAminoAcids[i] == (uint8_t)b) {
                l.v[b] = (uint8_t)i;
                break;
            }
    }
    return l;
}

// windows j in [0, L-k] (protein.rs:114); L < k yields none (documented deviation: the
// reference wraps usize for L < 4 and panics)
inline uint64_t n_windows(uint64_t L, int k) { return L >= (uint64_t)k ? L - k + 1 : 0; }

// 16-B aligned per-protein slot of every u32 per-protein array (see kmerpair.h)
KMP_HD inline uint64_t set_base(uint64_t res_off, uint32_t p) {
    return (res_off + 4ull * p + 3ull) & ~3ull;
}

// ---- pair-kernel geometry (LDS budget per workgroup, one workgroup per CU) ----
constexpr uint32_t kPairThreads = 1024;                 // 16 waves
constexpr uint32_t kPairWaves = kPairThreads / 64;
constexpr uint32_t kTileCap = 16384;                    // row-tile k-mers (exact table: 64 KiB keys + 16 KiB rows)
constexpr uint32_t kRowsMax = 256;                      // row index fits u8
constexpr uint32_t kBloomLog2 = 12;                     // 4,096 x 64-bit Bloom blocks (32 KiB), 4 bits per key
constexpr uint32_t kBloomBlocks = 1u << kBloomLog2;
constexpr uint32_t kBuckets = kBloomBlocks;             // exact-table bucket = Bloom block of the key
constexpr uint32_t kTileSlots = kTileCap;               // reported by kmp_pair_geometry_get
constexpr uint32_t kHashMul = 0x9E3779B1u;              // block / bucket hash (top 12 bits)
constexpr uint32_t kHashMul2 = 0x85EBCA6Bu;             // bit positions inside the block
constexpr uint32_t kColRegs = 3;                        // column k-mers per lane held in registers (192 per column)
constexpr uint32_t kBatch = 8;                          // columns per register batch (two batches in flight)
constexpr uint64_t kChunkCost = 262144;                 // column k-mers per work item (one L2-shared chunk)

}  // namespace kmp
