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
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "kmerpair.h"

namespace {

bool read_file(const char* path, std::string& out) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    char buf[1 << 16];
    size_t r;
    while ((r = std::fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, r);
    const bool ok = !std::ferror(f);
    std::fclose(f);
    return ok;
}

// id.split_terminator('|')[3]
bool amr_class(const std::string& id, std::string& cls) {
    std::vector<std::string> fields;
    size_t b = 0;
    for (;;) {
        const size_t e = id.find('|', b);
        if (e == std::string::npos) {
            if (b < id.size()) fields.push_back(id.substr(b));  // split_terminator: no trailing ""
            break;
        }
        fields.push_back(id.substr(b, e - b));
        b = e + 1;
    }
    if (fields.size() < 4) return false;
    cls = fields[3];
    return true;
}

template <class T>
T* dup(const std::vector<T>& v) {
    T* p = static_cast<T*>(std::malloc(v.size() ? v.size() * sizeof(T) : 1));
    if (p && !v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
    return p;
}

}  // namespace

extern "C" int kmp_read_fasta(const char* path, uint32_t* n, uint8_t** residues, uint64_t** offsets,
                              uint16_t** class_id, char** ids, uint64_t* ids_bytes, uint32_t* n_classes) {
    if (!path || !n || !residues || !offsets || !class_id) return KMP_EINVAL;
    std::string text;
    if (!read_file(path, text)) return KMP_EIO;
    std::vector<uint8_t> res;
    std::vector<uint64_t> off;
    std::vector<uint16_t> cls;
    std::string idbuf;
    std::unordered_map<std::string, uint16_t> intern;
    res.reserve(text.size());
    size_t i = 0;
    const size_t N = text.size();
    // skip anything before the first record header
    while (i < N && text[i] != '>') {
        const size_t e = text.find('\n', i);
        i = e == std::string::npos ? N : e + 1;
    }
    while (i < N) {
        // header line
        size_t e = text.find('\n', i);
        if (e == std::string::npos) e = N;
        size_t he = e;
        if (he > i + 1 && text[he - 1] == '\r') --he;
        const std::string head = text.substr(i + 1, he - (i + 1));
        const size_t sp = head.find(' ');
        const std::string id = sp == std::string::npos ? head : head.substr(0, sp);
        std::string c;
        if (!amr_class(id, c)) return KMP_EINVAL;
        auto it = intern.find(c);
        if (it == intern.end()) {
            if (intern.size() >= 65535) return KMP_EINVAL;
            it = intern.emplace(c, (uint16_t)intern.size()).first;
        }
        cls.push_back(it->second);
        idbuf.append(id);
        idbuf.push_back('\0');
        off.push_back(res.size());
        i = e < N ? e + 1 : N;
        // sequence lines up to the next header
        size_t s0 = i, s1 = i;
        while (i < N && text[i] != '>') {
            size_t le = text.find('\n', i);
            if (le == std::string::npos) le = N;
            size_t content_end = le;
            if (content_end > i && text[content_end - 1] == '\r') --content_end;
            s1 = content_end;  // raw bytes up to the end of the last line's content
            i = le < N ? le + 1 : N;
        }
        if (s1 > s0) res.insert(res.end(), text.begin() + s0, text.begin() + s1);
    }
    off.push_back(res.size());
    if (off.size() - 1 > 0xFFFFFFFFull) return KMP_EINVAL;
    *n = (uint32_t)(off.size() - 1);
    *residues = dup(res);
    *offsets = dup(off);
    *class_id = dup(cls);
    if (ids) {
        *ids = static_cast<char*>(std::malloc(idbuf.size() + 1));
        if (*ids) std::memcpy(*ids, idbuf.data(), idbuf.size() + 1);
    }
    if (ids_bytes) *ids_bytes = idbuf.size();
    if (n_classes) *n_classes = (uint32_t)intern.size();
    if (!*residues || !*offsets || !*class_id) return KMP_ENOMEM;
    return KMP_OK;
}
