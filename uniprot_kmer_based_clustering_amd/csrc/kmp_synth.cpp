// kmp_synth.cpp — seeded synthetic protein sets for the benchmark configs.
//
// The reference only ships uniprot_arg.fasta; configs 2–5 are synthetic. Spec (§8d):
//   * splitmix64(seed) stream, every draw in a fixed order (bit-reproducible);
//   * residues i.i.d. from the 20-aa composition of uniprot_arg.fasta;
//   * F = N/16 ancestor families; member = ancestor with per-site substitution rate
//     mu ~ U[0.05, 0.30] and indel rate 0.01; members shuffled (Fisher–Yates);
//   * class = family mod 15 for 90 % of members, else uniform in 0..14;
//   * header  SYN{idx:07}|FEATURES|SYNTH|class{c}|fam{f}  (single-line, uppercase, LF).
// Length laws: 0 = round(N(300, 30²)) clamped to [50, 2000] (configs 2–4; the normal
// deviate is Irwin–Hall(12) so no libm call decides a length), 1 = log-uniform [50, 2000]
// (config 5).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kmerpair.h"

namespace {

struct SplitMix64 {
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double u01() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
};

// residue counts of uniprot_arg.fasta, X/Z excluded
const char kLetters[20] = {'L', 'A', 'G', 'V', 'I', 'S', 'T', 'F', 'R', 'E',
                           'K', 'D', 'P', 'Q', 'N', 'Y', 'M', 'H', 'W', 'C'};
const uint32_t kCounts[20] = {377380, 336508, 269059, 258845, 257326, 206108, 194902,
                              176903, 163437, 158642, 158511, 153089, 143715, 124590,
                              118853, 101563, 92047,  64642,  54450,  26176};

struct Composition {
    uint64_t cum[20];
    uint64_t total;
    Composition() {
        total = 0;
        for (int i = 0; i < 20; ++i) { total += kCounts[i]; cum[i] = total; }
    }
    char draw(SplitMix64& r) const {
        uint64_t x = ((r.next() >> 32) * total) >> 32;
        int lo = 0, hi = 19;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (x < cum[mid]) hi = mid; else lo = mid + 1;
        }
        return kLetters[lo];
    }
};

uint32_t draw_length(SplitMix64& r, int law) {
    if (law == KMP_LEN_LOGUNIFORM) {
        double lo = std::log(50.0), hi = std::log(2000.0);
        long v = std::lround(std::exp(lo + r.u01() * (hi - lo)));
        return (uint32_t)(v < 50 ? 50 : (v > 2000 ? 2000 : v));
    }
    double s = 0.0;
    for (int i = 0; i < 12; ++i) s += r.u01();
    long v = std::lround(300.0 + 30.0 * (s - 6.0));
    return (uint32_t)(v < 50 ? 50 : (v > 2000 ? 2000 : v));
}

struct Synth {
    std::vector<char> res;
    std::vector<uint64_t> off;
    std::vector<uint16_t> cls;
    std::vector<uint32_t> fam;
};

int generate(uint32_t n, uint64_t seed, int law, Synth& out) {
    if (law != KMP_LEN_NORMAL300 && law != KMP_LEN_LOGUNIFORM) return KMP_EINVAL;
    SplitMix64 r{seed};
    Composition comp;
    const uint32_t F = n / 16 ? n / 16 : 1;
    std::vector<std::string> anc(F);
    for (uint32_t f = 0; f < F; ++f) {
        uint32_t L = draw_length(r, law);
        anc[f].resize(L);
        for (uint32_t i = 0; i < L; ++i) anc[f][i] = comp.draw(r);
    }
    std::vector<std::string> mem(n);
    std::vector<uint16_t> mcls(n);
    for (uint32_t m = 0; m < n; ++m) {
        const uint32_t f = m % F;
        const double mu = 0.05 + 0.25 * r.u01();
        const std::string& a = anc[f];
        std::string& s = mem[m];
        s.reserve(a.size() + 8);
        for (char c : a) {
            double u = r.u01();
            if (u < 0.005) continue;                          // deletion
            if (u < 0.010) s.push_back(comp.draw(r));         // insertion before the site
            s.push_back(r.u01() < mu ? comp.draw(r) : c);     // substitution / keep
        }
        if (s.empty()) s.push_back(comp.draw(r));
        mcls[m] = (uint16_t)(r.u01() < 0.9 ? f % 15 : r.below(15));
    }
    std::vector<uint32_t> perm(n);
    for (uint32_t i = 0; i < n; ++i) perm[i] = i;
    for (uint32_t i = n; i > 1; --i) {
        uint32_t j = r.below(i);
        std::swap(perm[i - 1], perm[j]);
    }
    uint64_t tot = 0;
    for (uint32_t m = 0; m < n; ++m) tot += mem[m].size();
    out.res.resize(tot);
    out.off.resize(n + 1);
    out.cls.resize(n);
    out.fam.resize(n);
    uint64_t o = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t m = perm[i];
        out.off[i] = o;
        std::memcpy(out.res.data() + o, mem[m].data(), mem[m].size());
        o += mem[m].size();
        out.cls[i] = mcls[m];
        out.fam[i] = m % F;
    }
    out.off[n] = o;
    return KMP_OK;
}

}  // namespace

extern "C" int kmp_synth_packed(uint32_t n, uint64_t seed, int length_law, uint8_t** residues,
                                uint64_t* offsets, uint16_t* class_id, uint32_t* family) {
    if (!residues || !offsets) return KMP_EINVAL;
    Synth s;
    int st = generate(n, seed, length_law, s);
    if (st != KMP_OK) return st;
    uint8_t* buf = (uint8_t*)std::malloc(s.res.size() ? s.res.size() : 1);
    if (!buf) return KMP_ENOMEM;
    std::memcpy(buf, s.res.data(), s.res.size());
    *residues = buf;
    std::memcpy(offsets, s.off.data(), sizeof(uint64_t) * (n + 1));
    if (class_id) std::memcpy(class_id, s.cls.data(), sizeof(uint16_t) * n);
    if (family) std::memcpy(family, s.fam.data(), sizeof(uint32_t) * n);
    return KMP_OK;
}

extern "C" int kmp_synth_write_fasta(const char* path, uint32_t n, uint64_t seed, int length_law) {
    if (!path) return KMP_EINVAL;
    Synth s;
    int st = generate(n, seed, length_law, s);
    if (st != KMP_OK) return st;
    FILE* f = std::fopen(path, "wb");
    if (!f) return KMP_EIO;
    std::vector<char> line;
    for (uint32_t i = 0; i < n; ++i) {
        std::fprintf(f, ">SYN%07u|FEATURES|SYNTH|class%u|fam%u\n", i, (unsigned)s.cls[i], s.fam[i]);
        std::fwrite(s.res.data() + s.off[i], 1, s.off[i + 1] - s.off[i], f);
        std::fputc('\n', f);
    }
    return std::fclose(f) == 0 ? KMP_OK : KMP_EIO;
}

extern "C" void kmp_free_host(void* p) { std::free(p); }
