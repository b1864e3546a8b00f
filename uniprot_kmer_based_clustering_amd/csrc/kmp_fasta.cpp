// kmp_fasta.cpp — FASTA ingest with the semantics the reference gets from seq_io 0.3.3
// (src/main.rs:62-72 → Protein::new, src/protein.rs:107-110):
//   * a record starts at a line beginning with '>'; the header is the rest of that line
//     without its terminator ("\n" or "\r\n");
//   * record.id() = header up to the first space;
//   * record.seq() = the raw bytes of the record's sequence lines: interior line
//     terminators are KEPT (they are not in the amino-acid list, so each encodes as 20, as
//     in the reference), only the last line's terminator is dropped;
//   * the AMR class is id.split_terminator('|')[3] (protein.rs:135-138): a trailing empty
//     field is not a field; fewer than four fields is an error (the reference panics).
// Classes are interned to u16 ids in order of first appearance.  uniprot_arg.fasta is
// single-line, LF-terminated; multi-line / CRLF inputs follow the rules above.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "kmerpair.h"
#include "kmp_threads.hpp"

namespace {

// the file mapped read-only (empty files: an empty view)
struct Mapped {
    const char* p = nullptr;
    size_t n = 0;
    bool ok = false;
    explicit Mapped(const char* path) {
        const int fd = ::open(path, O_RDONLY);
        if (fd < 0) return;
        struct stat st;
        if (::fstat(fd, &st) == 0) {
            n = (size_t)st.st_size;
            if (n == 0) {
                ok = true;
            } else {
                void* m = ::mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
                if (m != MAP_FAILED) {
                    p = static_cast<const char*>(m);
                    ok = true;
                }
            }
        }
        ::close(fd);
    }
    ~Mapped() {
        if (p) ::munmap(const_cast<char*>(p), n);
    }
};

// id.split_terminator('|')[3]
bool amr_class(std::string_view id, std::string_view& cls) {
    size_t b = 0;
    int field = 0;
    for (;;) {
        const size_t e = id.find('|', b);
        if (e == std::string_view::npos) {
            if (b < id.size() && field == 3) {  // split_terminator: no trailing ""
                cls = id.substr(b);
                return true;
            }
            return false;
        }
        if (field == 3) {
            cls = id.substr(b, e - b);
            return true;
        }
        ++field;
        b = e + 1;
    }
}

template <class T>
T* dup(const std::vector<T>& v) {
    T* p = static_cast<T*>(std::malloc(v.size() ? v.size() * sizeof(T) : 1));
    if (p && !v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
    return p;
}

// one record: its id, class and raw sequence span [s0, s1) of the text
struct Rec {
    std::string_view id, cls;
    size_t s0, s1;
};

// the records whose header line starts in [a, b) of text (a record starts at a '>' that begins a
// line); false: a record without a class field (the reference panics)
bool parse_range(const char* t, size_t N, size_t a, size_t b, std::vector<Rec>& out) {
    size_t i = a;
    while (i < b && !(t[i] == '>' && (i == 0 || t[i - 1] == '\n'))) {  // the range's first record
        const void* nl = std::memchr(t + i, '\n', N - i);
        i = nl ? (size_t)((const char*)nl - t) + 1 : N;
    }
    while (i < b) {
        const void* nl = std::memchr(t + i, '\n', N - i);
        const size_t e = nl ? (size_t)((const char*)nl - t) : N;
        size_t he = e;
        if (he > i + 1 && t[he - 1] == '\r') --he;
        std::string_view head(t + i + 1, he - (i + 1));
        const size_t sp = head.find(' ');
        Rec r;
        r.id = sp == std::string_view::npos ? head : head.substr(0, sp);
        if (!amr_class(r.id, r.cls)) return false;
        i = e < N ? e + 1 : N;
        // sequence lines up to the next header: raw bytes, the last line's terminator dropped
        r.s0 = r.s1 = i;
        while (i < N && t[i] != '>') {
            const void* ln = std::memchr(t + i, '\n', N - i);
            const size_t le = ln ? (size_t)((const char*)ln - t) : N;
            size_t ce = le;
            if (ce > i && t[ce - 1] == '\r') --ce;
            r.s1 = ce;
            i = le < N ? le + 1 : N;
        }
        out.push_back(r);
    }
    return true;
}

int threads_for(int t) {
    if (t > 0) return std::min(t, 256);
    const unsigned h = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(h ? h : 1u, 16u));
}

template <class F>
void parallel(int T, F f) {
    kmp::run_parts(T, f);
}

}  // namespace

// Multithreaded (the reference reads with parallel_fasta, main.rs:62-72): the mapped file is cut
// into `threads` byte ranges, each thread parses the records whose header starts in its range,
// classes are interned in file order of first appearance, and the residues and ids are copied in
// parallel to their prefix-summed offsets.
extern "C" int kmp_read_fasta_threads(const char* path, int threads, uint32_t* n, uint8_t** residues,
                                      uint64_t** offsets, uint16_t** class_id, char** ids, uint64_t* ids_bytes,
                                      uint32_t* n_classes) {
    if (!path || !n || !residues || !offsets || !class_id) return KMP_EINVAL;
    Mapped m(path);
    if (!m.ok) return KMP_EIO;
    const char* t = m.p;
    const size_t N = m.n;
    const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)threads_for(threads), N / (1 << 16) + 1));
    std::vector<std::vector<Rec>> recs(T);
    std::vector<char> ok(T, 1);
    parallel(T, [&](int k) { ok[k] = parse_range(t, N, N * k / T, N * (k + 1) / T, recs[k]); });
    for (int k = 0; k < T; ++k)
        if (!ok[k]) return KMP_EINVAL;
    // record offsets per thread, class ids in order of first appearance
    std::vector<size_t> rbase(T + 1, 0);
    for (int k = 0; k < T; ++k) rbase[k + 1] = rbase[k] + recs[k].size();
    const size_t R = rbase[T];
    if (R > 0xFFFFFFFFull) return KMP_EINVAL;
    std::vector<uint64_t> off(R + 1, 0), idoff(R + 1, 0);
    std::vector<uint16_t> cls(R);
    std::unordered_map<std::string_view, uint16_t> intern;
    {
        size_t r = 0;
        for (int k = 0; k < T; ++k)
            for (const Rec& x : recs[k]) {
                auto it = intern.find(x.cls);
                if (it == intern.end()) {
                    if (intern.size() >= 65535) return KMP_EINVAL;
                    it = intern.emplace(x.cls, (uint16_t)intern.size()).first;
                }
                cls[r] = it->second;
                off[r + 1] = off[r] + (x.s1 - x.s0);
                idoff[r + 1] = idoff[r] + x.id.size() + 1;
                ++r;
            }
    }
    uint8_t* res = static_cast<uint8_t*>(std::malloc(off[R] ? off[R] : 1));
    char* idb = ids ? static_cast<char*>(std::malloc(idoff[R] + 1)) : nullptr;
    if (!res || (ids && !idb)) {
        std::free(res);
        std::free(idb);
        return KMP_ENOMEM;
    }
    parallel(T, [&](int k) {
        size_t r = rbase[k];
        for (const Rec& x : recs[k]) {
            if (x.s1 > x.s0) std::memcpy(res + off[r], t + x.s0, x.s1 - x.s0);
            if (idb) {
                std::memcpy(idb + idoff[r], x.id.data(), x.id.size());
                idb[idoff[r] + x.id.size()] = '\0';
            }
            ++r;
        }
    });
    if (idb) idb[idoff[R]] = '\0';
    *n = (uint32_t)R;
    *residues = res;
    *offsets = dup(off);
    *class_id = dup(cls);
    if (ids) *ids = idb;
    if (ids_bytes) *ids_bytes = idoff[R];
    if (n_classes) *n_classes = (uint32_t)intern.size();
    if (!*offsets || !*class_id) return KMP_ENOMEM;
    return KMP_OK;
}

extern "C" int kmp_read_fasta(const char* path, uint32_t* n, uint8_t** residues, uint64_t** offsets,
                              uint16_t** class_id, char** ids, uint64_t* ids_bytes, uint32_t* n_classes) {
    return kmp_read_fasta_threads(path, 0, n, residues, offsets, class_id, ids, ids_bytes, n_classes);
}
