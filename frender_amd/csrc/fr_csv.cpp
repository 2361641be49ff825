// fr_csv.cpp — the scan CSV writer (reference report_analysis,
// frender.py:482-501, which flattens the results dict and writes it with csv.DictWriter).
//
// The host's Python writer (frender_amd/scan.py) built one list of strings per unique code and fed
// csv.writer: at config-2 scale (hundreds of thousands of codes per scan) that, plus decoding every
// packed key to a Python string first, was most of an end-to-end scan's host time.  Here the rows
// are formatted straight from the arrays the GPU path already holds: the packed key of each row
// (decoded here, 3-bit fast keys and base-5 wide keys, include/frender_amd.h), its count, and its
// classification (indices into the sheet's strings).  Every string that can need CSV quoting (sheet
// entries, sample names, exotic codes' parts) arrives already formatted by Python's csv module, so
// the bytes are the excel dialect's: fields joined by ',', rows ended by "\r\n".
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/frender_amd.h"

namespace {

constexpr uint64_t WIDE_BIT = 1ull << 63;
constexpr int WIDE_MAXN = 24, WIDE_NOPLUS = 31;

// a packed key -> its code text in buf; returns the length (0: key 0, not a code)
int decode_key(uint64_t key, char* buf) {
    if (!(key & WIDE_BIT)) {
        static const char SYM[8] = {0, 'A', 'C', 'G', 'T', 'N', '+', 0};
        int n = 0;
        for (int i = 0; i < 21; ++i) {
            const char c = SYM[(key >> (3 * i)) & 7u];
            if (!c) break;
            buf[n++] = c;
        }
        return n;
    }
    // wide: lower << 62 | plus << 57 | (v + (5^nl - 1) / 4), v = sum d_k 5^k over the nl letters
    static const char UP[5] = {'A', 'C', 'G', 'T', 'N'}, LO[5] = {'a', 'c', 'g', 't', 'n'};
    const bool lower = (key >> 62) & 1u;
    const int plus = (int)((key >> 57) & 31u);
    uint64_t V = key & ((1ull << 57) - 1), off = 0, p5 = 1;
    int nl = 0;
    while (nl < WIDE_MAXN && off + p5 <= V) {  // the largest nl with (5^nl - 1) / 4 <= V
        off += p5;
        p5 *= 5;
        ++nl;
    }
    uint64_t D = V - off;
    int n = 0;
    for (int k = 0; k < nl; ++k) {
        if (k == plus) buf[n++] = '+';
        buf[n++] = (lower ? LO : UP)[D % 5];
        D /= 5;
    }
    if (plus != WIDE_NOPLUS && plus >= nl) buf[n++] = '+';
    return n;
}

struct Out {
    FILE* f;
    std::vector<char> b;
    size_t n = 0;
    bool ok = true;
    explicit Out(FILE* fp) : f(fp), b(1 << 20) {}
    void flush() {
        if (n && fwrite(b.data(), 1, n, f) != n) ok = false;
        n = 0;
    }
    void put(const char* s, size_t len) {
        if (n + len > b.size()) flush();
        if (len > b.size()) {
            if (fwrite(s, 1, len, f) != len) ok = false;
            return;
        }
        memcpy(b.data() + n, s, len);
        n += len;
    }
    void ch(char c) {
        if (n == b.size()) flush();
        b[n++] = c;
    }
    void u64(uint64_t v) {
        char t[24];
        int k = 0;
        do {
            t[k++] = (char)('0' + v % 10);
            v /= 10;
        } while (v);
        if (n + k > b.size()) flush();
        while (k) b[n++] = t[--k];
    }
};

}  // namespace

extern "C" int fr_write_scan_csv(const char* path, const char* header, uint64_t n_rows, const uint64_t* keys,
                                 const uint64_t* counts, const int16_t* m1, const int16_t* m2, const uint8_t* cls,
                                 const int16_t* row, const uint8_t* demux_ok, const char* dict,
                                 const uint64_t* dict_off, const uint32_t* dict_n, uint64_t n_exotic,
                                 const uint64_t* exo_rows, const char* exo_text, const uint64_t* exo_off) {
    if (!path || !header || (n_rows && (!keys || !counts || !m1 || !m2 || !cls || !row)) || !dict || !dict_off ||
        !dict_n || (n_exotic && (!exo_rows || !exo_text || !exo_off)))
        return FR_ERR_INVALID;
    // dictionary sections: idx1, idx2, sample names, class names (one entry each, in that order)
    const uint64_t n1 = dict_n[0], n2 = dict_n[1], ns = dict_n[2], nc = dict_n[3];
    const uint64_t b2 = n1, bs = n1 + n2, bc = n1 + n2 + ns;
    // every code must split on '+' (the reference's code.split("+")[1], frender.py:486): refuse
    // before writing anything, and the caller's own writer raises the reference's IndexError
    char code[64];
    uint64_t e = 0;
    for (uint64_t j = 0; j < n_rows; ++j) {
        if (e < n_exotic && exo_rows[e] == j) {
            ++e;
            continue;
        }
        const int len = decode_key(keys[j], code);
        if (!memchr(code, '+', (size_t)len)) return FR_ERR_INVALID;
        if ((m1[j] >= 0 && (uint64_t)m1[j] >= n1) || (m2[j] >= 0 && (uint64_t)m2[j] >= n2) ||
            (row[j] >= 0 && (uint64_t)row[j] >= ns) || cls[j] >= nc)
            return FR_ERR_INVALID;
    }
    if (e != n_exotic) return FR_ERR_INVALID;  // exotic rows must be increasing and < n_rows
    FILE* f = fopen(path, "wb");
    if (!f) return FR_ERR_IO;
    Out o(f);
    auto entry = [&](uint64_t i) { o.put(dict + dict_off[i], dict_off[i + 1] - dict_off[i]); };
    o.put(header, strlen(header));
    e = 0;
    for (uint64_t j = 0; j < n_rows; ++j) {
        if (e < n_exotic && exo_rows[e] == j) {  // "p0,p1" as Python's csv module formats them
            o.put(exo_text + exo_off[e], exo_off[e + 1] - exo_off[e]);
            ++e;
        } else {  // parts[0], parts[1] of code.split("+")
            const int len = decode_key(keys[j], code);
            const char* p = (const char*)memchr(code, '+', (size_t)len);
            const char* q = (const char*)memchr(p + 1, '+', (size_t)(code + len - (p + 1)));
            o.put(code, (size_t)(p - code));
            o.ch(',');
            o.put(p + 1, (size_t)((q ? q : code + len) - (p + 1)));
        }
        o.ch(',');
        if (m1[j] >= 0) entry((uint64_t)m1[j]);
        o.ch(',');
        if (m2[j] >= 0) entry(b2 + (uint64_t)m2[j]);
        o.ch(',');
        entry(bc + cls[j]);
        o.ch(',');
        if (row[j] >= 0) entry(bs + (uint64_t)row[j]);
        o.ch(',');
        o.u64(counts[j]);
        if (demux_ok) o.put(demux_ok[j] ? ",True" : ",False", demux_ok[j] ? 5 : 6);
        o.put("\r\n", 2);
    }
    o.flush();
    const bool ok = o.ok && fclose(f) == 0;
    return ok ? FR_OK : FR_ERR_IO;
}
