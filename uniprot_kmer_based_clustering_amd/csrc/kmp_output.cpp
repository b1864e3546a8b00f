// kmp_output.cpp — the host-side consumers of the edge list:
//   kmp_write_candidates: the file side of align_and_output_pairs (mod.rs:195-319) — for every
//     edge with w > threshold (mod.rs:242), the two single-record FASTAs diamond would read
//     (mod.rs:253-261,273-280) and blastp_output.tsv's header (mod.rs:304); the diamond runs
//     themselves stay out of scope;
//   kmp_write_graph_debug: `println!("Graph right now:\n{graph_ref:#?}")` (main.rs:234) with the
//     Debug impls of Graph (mod.rs:700-708), KmerEdge (edge.rs:158-174) and ProteinVertex
//     (vertex.rs:159-165), in the reference's final edge order.
#include <ftw.h>
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "kmerpair.h"
#include "kmp_edges.hpp"
#include "kmp_threads.hpp"

namespace {

// id strings of a NUL-separated blob (kmp_read_fasta's ids)
bool split_ids(const char* ids, uint64_t bytes, uint32_t n, std::vector<std::pair<const char*, size_t>>& out) {
    out.clear();
    out.reserve(n);
    uint64_t i = 0;
    while (out.size() < n && i < bytes) {
        const char* s = ids + i;
        const void* z = std::memchr(s, 0, bytes - i);
        const size_t len = z ? (size_t)((const char*)z - s) : (size_t)(bytes - i);
        out.emplace_back(s, len);
        i += len + 1;
    }
    return out.size() == n;
}

bool make_dir(const std::string& d) { return ::mkdir(d.c_str(), 0777) == 0 || errno == EEXIST; }

// `rm -r d` (mod.rs:202-210): a missing directory is not an error, as the reference ignores rm's status
bool remove_tree(const std::string& d) {
    struct stat sb;
    if (::lstat(d.c_str(), &sb) != 0) return errno == ENOENT;
    auto rm = [](const char* path, const struct stat*, int, struct FTW*) -> int { return ::remove(path); };
    return ::nftw(d.c_str(), rm, 16, FTW_DEPTH | FTW_PHYS) == 0;
}

bool write_file(const std::string& path, const std::string& text) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = std::fwrite(text.data(), 1, text.size(), f) == text.size();
    return (std::fclose(f) == 0) && ok;
}

int threads_for(int t) { return t < 1 ? 1 : (t > 256 ? 256 : t); }

// Rust's `{:#?}` of one KmerEdge at list depth 2 (edge.rs:158-174): a single shared k-mer is
// `Single Kmer { kmer: id, .. }`, a collapsed group `Kmer Group { kmer: [ids], .. }`; size is
// vertices_key.len(), always 2
void format_edge(std::string& s, const uint32_t* k, uint64_t w) {
    if (w == 1) {
        s += "        Single Kmer {\n            kmer: ";
        s += std::to_string(k[0]);
        s += ",\n            size: 2,\n        },\n";
        return;
    }
    s += "        Kmer Group {\n            kmer: [\n";
    for (uint64_t i = 0; i < w; ++i) {
        s += "                ";
        s += std::to_string(k[i]);
        s += ",\n";
    }
    s += "            ],\n            size: 2,\n        },\n";
}

}  // namespace

extern "C" {

int kmp_write_candidates(const kmp_edges* e, const uint8_t* residues, const uint64_t* offsets, uint32_t n,
                         const char* ids, uint64_t ids_bytes, uint32_t threshold, const char* out_dir, int threads,
                         uint64_t* n_written) {
    if (!e || !offsets || !ids || !n_written) return KMP_EINVAL;
    *n_written = 0;
    std::vector<std::pair<const char*, size_t>> id;
    if (!split_ids(ids, ids_bytes, n, id)) return KMP_EINVAL;
    // the file-name prefix is id.split_once('|').0; the reference panics on an id without '|'
    std::vector<std::string> prefix(n);
    for (uint32_t p = 0; p < n; ++p) {
        const void* bar = std::memchr(id[p].first, '|', id[p].second);
        if (bar) prefix[p].assign(id[p].first, (const char*)bar - id[p].first);
    }
    std::vector<uint64_t> cand;
    for (uint64_t i = 0; i < e->p.size(); ++i) {
        if (e->w[i] <= threshold) continue;
        if (e->p[i] >= n || e->q[i] >= n) return KMP_EINVAL;
        if (!std::memchr(id[e->p[i]].first, '|', id[e->p[i]].second) ||
            !std::memchr(id[e->q[i]].first, '|', id[e->q[i]].second))
            return KMP_EINVAL;
        cand.push_back(i);
    }
    if (!cand.empty() && !residues) return KMP_EINVAL;
    const std::string root = out_dir && *out_dir ? std::string(out_dir) : std::string(".");
    const std::string fdir = root + "/fasta_files", ddir = root + "/db_files";
    // fresh directories, as the reference's rm -r + mkdir (mod.rs:202-220)
    if (!make_dir(root) || !remove_tree(fdir) || !remove_tree(ddir) || !make_dir(fdir) || !make_dir(ddir))
        return KMP_EIO;
    const bool ref_order = e->kspace == KMP_KMERS_IDS && e->ref_key.size() == e->p.size();
    std::atomic<uint64_t> next{0};
    std::atomic<int> err{KMP_OK};
    auto work = [&]() {
        std::string path, text;
        for (;;) {
            const uint64_t c = next.fetch_add(1);
            if (c >= cand.size() || err.load() != KMP_OK) return;
            const uint64_t i = cand[c];
            const uint64_t key = ref_order ? e->ref_key[i] : i;  // edge_key of mod.rs:232
            // reference file (vertices_key[0] = p) first, then the query (q): with equal prefixes the
            // query overwrites it, as in the reference
            for (uint32_t v : {e->p[i], e->q[i]}) {
                path = fdir + "/" + std::to_string(key) + "_" + prefix[v] + ".fasta";
                text.assign(">");
                text.append(id[v].first, id[v].second);
                text += '\n';
                text.append(reinterpret_cast<const char*>(residues) + offsets[v], offsets[v + 1] - offsets[v]);
                if (!write_file(path, text)) {
                    err.store(KMP_EIO);
                    return;
                }
            }
        }
    };
    const int t = threads_for(threads);
    kmp::run_parts(t, [&](int) { work(); });
    if (err.load() != KMP_OK) return err.load();
    static const char kHeader[] =
        "query id\tquery length\tsubject id\tsubject length\tquery alignment start\tquery alignment end\t"
        "subject alignment start\tsubject alignment end\talignment length\tpercent identity\tevalue\tbit score\n";
    if (!write_file(root + "/blastp_output.tsv", kHeader)) return KMP_EIO;
    *n_written = cand.size();
    return KMP_OK;
}

int kmp_write_graph_debug(const kmp_edges* e, uint32_t n, const char* path, int threads) {
    if (!e) return KMP_EINVAL;
    if (e->kspace != KMP_KMERS_IDS || e->ref_key.size() != e->p.size()) return KMP_ESTATE;
    const uint64_t count = e->p.size();
    std::vector<uint64_t> order(count);  // reference position -> edge
    for (uint64_t i = 0; i < count; ++i) {
        if (e->ref_key[i] >= count || e->p[i] >= n || e->q[i] >= n) return KMP_EINVAL;
        order[e->ref_key[i]] = i;
    }
    std::vector<uint64_t> degree(n, 0);  // ProteinVertex.edges_key.len() after the key update
    for (uint64_t i = 0; i < count; ++i) {
        ++degree[e->p[i]];
        ++degree[e->q[i]];
    }
    FILE* f = path && *path && std::strcmp(path, "-") != 0 ? std::fopen(path, "wb") : stdout;
    if (!f) return KMP_EIO;
    bool ok = true;
    auto put = [&](const std::string& s) { ok = ok && std::fwrite(s.data(), 1, s.size(), f) == s.size(); };
    put(count ? "Graph right now:\nGraph {\n    Kmers: [\n" : "Graph right now:\nGraph {\n    Kmers: [],\n");
    // format edge chunks in parallel, write them in order
    const int t = threads_for(threads);
    const uint64_t chunk = 1 << 16;
    for (uint64_t b = 0; b < count; b += chunk * t) {
        std::vector<std::string> part(t);
        kmp::run_parts(t, [&](int j) {
            const uint64_t lo = b + j * chunk, hi = std::min<uint64_t>(lo + chunk, count);
            for (uint64_t r = lo; r < hi; ++r) {
                const uint64_t i = order[r];
                format_edge(part[j], e->kmers.data() + e->kofs[i], e->kofs[i + 1] - e->kofs[i]);
            }
        });
        for (auto& s : part) put(s);
    }
    std::string s;
    if (count) s += "    ],\n";
    if (n == 0) {
        s += "    Proteins: [],\n}\n";
    } else {
        s += "    Proteins: [\n";
        for (uint32_t p = 0; p < n; ++p) {
            s += "        Protein {\n            key: ";
            s += std::to_string(p);
            s += ",\n            size: ";
            s += std::to_string(degree[p]);
            s += ",\n        },\n";
            if (s.size() > (1u << 20)) {
                put(s);
                s.clear();
            }
        }
        s += "    ],\n}\n";
    }
    put(s);
    if (f != stdout) ok = (std::fclose(f) == 0) && ok;
    else ok = (std::fflush(f) == 0) && ok;
    return ok ? KMP_OK : KMP_EIO;
}

}  // extern "C"
