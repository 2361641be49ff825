// fr_pinflate.h — parallel DEFLATE decode of one large gzip member.
//
// The reference reads each file with gzip.open(file, "rt") (frender.py:159) in its own Pool worker
// (:189-193): one core per file.  A NovaSeq lane is one big single-member .fastq.gz, so that is one
// core for the whole lane.  A DEFLATE stream cannot be entered mid-way with zlib: a block's start is
// a bit position known only after decoding everything before it, and its back-references reach 32 KiB
// into output not decoded yet.  This decoder does what two-stage parallel gzip readers do:
//
//  1. The compressed bytes are cut into chunks.  Each chunk (in parallel) searches, from its nominal
//     start, the first bit position where a dynamic-Huffman block header parses and validates (code
//     lengths form complete prefix codes, end-of-block present) and the block decodes to its end, and
//     decodes blocks from there until the first block boundary at or past the next chunk's nominal
//     start.  Output goes to 16-bit symbols: a back-reference that reaches before the chunk's start
//     yields a MARKER (256 + its index in the unknown 32 KiB window) instead of a byte; once 32 KiB of
//     output hold no marker, no later reference can produce one and output continues as bytes.
//  2. Stitching, in order: chunk k is correct iff chunk k-1's decode ended exactly at chunk k's start
//     (a real block boundary, reached by decoding from the stream's true start).  A chunk whose start
//     was not reached (a false candidate, or a boundary the search skipped: stored / fixed-Huffman
//     blocks) is dropped and chunk k-1 decodes on until it meets a later chunk's start (or the end):
//     correctness never rests on the search.
//  3. Windows, in order (32 KiB per chunk): chunk k's window is the last 32 KiB of chunk k-1's resolved
//     output; then every chunk's markers are replaced by window bytes (in parallel).
//  4. CRC-32 (parallel, crc32_combine) and ISIZE against the member's trailer.
//
// Strictness: code-length rules follow zlib's inflate (over-subscribed codes, incomplete codes other
// than a single length-1 code, a missing end-of-block code, HLIT > 286 / HDIST > 30, repeat with no
// previous length, distances past the stream's start are all errors), and the CRC/ISIZE check closes
// the rest: any failure returns false and the caller decodes the file with zlib, which owns the exact
// error behaviour.  Only used by fr_gz.cpp.
#pragma once

#include <zlib.h>

#include <algorithm>
#include <atomic>
#ifdef FRPZ_TIMING
#include <chrono>
#include <cstdio>
#endif
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace frpz {

// vectors whose resize() leaves new elements uninitialised (every decode output is written before read)
template <class T>
struct NoInit : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInit<U>;
    };
    NoInit() = default;
    template <class U>
    NoInit(const NoInit<U>&) {}
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        if constexpr (sizeof...(A) == 0) ::new ((void*)p) U;
        else ::new ((void*)p) U(std::forward<A>(a)...);
    }
};
using U16s = std::vector<uint16_t, NoInit<uint16_t>>;

constexpr int WSIZE = 32768;
constexpr uint32_t MARK = 256;  // 16-bit output >= MARK: byte (v - MARK) of the 32 KiB window before the chunk

// ---- Huffman tables ------------------------------------------------------------------------------
// An entry: op = LIT (val = byte), BASE | extra (val = length / distance base), EOB, BAD, or SUB (val =
// subtable offset, sub = its index bits).  `len` is the whole code's length (bits consumed).
enum : uint8_t { OP_LIT = 0, OP_BASE = 16, OP_EOB = 64, OP_BAD = 128, OP_SUB = 192 };
struct Code {
    uint8_t op, len;
    uint16_t val;
};
struct Table {
    std::vector<Code> e;
    int root = 0;
};

const uint16_t LBASE[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                            31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
const uint8_t LEXTRA[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
const uint16_t DBASE[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,    65,    97,    129,
                            193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
const uint8_t DEXTRA[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

enum Kind { K_CL, K_LIT, K_DIST };

inline uint32_t rev_bits(uint32_t c, int n) {
    uint32_t r = 0;
    for (int i = 0; i < n; ++i) r |= ((c >> i) & 1u) << (n - 1 - i);
    return r;
}

// canonical Huffman decode table for lens[0..n) (zlib's acceptance rules, see the file header)
inline bool build(const uint8_t* lens, int n, int root_max, Kind kind, Table& t) {
    int count[16] = {0};
    for (int s = 0; s < n; ++s) count[lens[s]]++;
    int max = 15;
    while (max >= 1 && count[max] == 0) --max;
    const int root = std::max(1, std::min(root_max, std::max(max, 1)));
    t.root = root;
    if (max == 0) {  // no codes: every lookup is invalid (legal only while unused)
        t.e.assign((size_t)1 << root, Code{OP_BAD, 1, 0});
        return true;
    }
    int left = 1;
    for (int l = 1; l <= 15; ++l) {
        left <<= 1;
        left -= count[l];
        if (left < 0) return false;  // over-subscribed
    }
    if (left > 0 && (kind == K_CL || max != 1)) return false;  // incomplete (only one length-1 code may be)
    const int sub_bits = max > root ? max - root : 0;
    // codes in canonical order
    int next[16];
    int code = 0;
    count[0] = 0;
    for (int l = 1; l <= 15; ++l) {
        code = (code + count[l - 1]) << 1;
        next[l] = code;
    }
    t.e.assign((size_t)1 << root, Code{OP_BAD, 1, 0});
    for (int s = 0; s < n; ++s) {
        const int L = lens[s];
        if (!L) continue;
        Code c;
        c.len = (uint8_t)L;
        if (kind == K_CL) {
            c.op = OP_LIT;
            c.val = (uint16_t)s;
        } else if (kind == K_LIT) {
            if (s < 256) {
                c.op = OP_LIT;
                c.val = (uint16_t)s;
            } else if (s == 256) {
                c.op = OP_EOB;
                c.val = 0;
            } else if (s - 257 < 29) {
                c.op = (uint8_t)(OP_BASE | LEXTRA[s - 257]);
                c.val = LBASE[s - 257];
            } else {
                c.op = OP_BAD;  // 286, 287: invalid when used
                c.val = 0;
            }
        } else {
            if (s < 30) {
                c.op = (uint8_t)(OP_BASE | DEXTRA[s]);
                c.val = DBASE[s];
            } else {
                c.op = OP_BAD;
                c.val = 0;
            }
        }
        const uint32_t r = rev_bits((uint32_t)next[L]++, L);
        if (L <= root) {
            for (uint32_t j = r; j < (1u << root); j += 1u << L) t.e[j] = c;
        } else {
            const uint32_t pre = r & ((1u << root) - 1u);
            if (t.e[pre].op != OP_SUB) {
                const size_t off = t.e.size();
                t.e[pre] = Code{OP_SUB, (uint8_t)sub_bits, (uint16_t)off};
                t.e.resize(off + ((size_t)1 << sub_bits), Code{OP_BAD, (uint8_t)max, 0});
            }
            const size_t off = t.e[pre].val;
            const uint32_t rest = r >> root;
            for (uint32_t j = rest; j < (1u << sub_bits); j += 1u << (L - root)) t.e[off + j] = c;
        }
    }
    return t.e.size() <= 65535;
}

inline const Table& fixed_lit() {
    static const Table t = [] {
        uint8_t l[288];
        for (int i = 0; i < 144; ++i) l[i] = 8;
        for (int i = 144; i < 256; ++i) l[i] = 9;
        for (int i = 256; i < 280; ++i) l[i] = 7;
        for (int i = 280; i < 288; ++i) l[i] = 8;
        Table x;
        build(l, 288, 10, K_LIT, x);
        return x;
    }();
    return t;
}
inline const Table& fixed_dist() {
    static const Table t = [] {
        uint8_t l[32];
        for (int i = 0; i < 32; ++i) l[i] = 5;
        Table x;
        build(l, 32, 8, K_DIST, x);
        return x;
    }();
    return t;
}

// ---- bit input ------------------------------------------------------------------------------------
struct Bits {
    const uint8_t* s = nullptr;  // stream start
    const uint8_t* p = nullptr;  // next byte to load
    const uint8_t* end = nullptr;
    uint64_t buf = 0;
    int cnt = 0;
    size_t over = 0;  // zero bytes loaded past the end

    void init(const uint8_t* s_, size_t n, size_t bitpos) {
        s = s_;
        end = s_ + n;
        p = s_ + std::min(n, bitpos >> 3);
        buf = 0;
        cnt = 0;
        over = 0;
        refill();
        const int skip = (int)(bitpos & 7u);
        buf >>= skip;
        cnt -= skip;
    }
    inline void refill() {
        if (end - p >= 8) {
            uint64_t w;
            std::memcpy(&w, p, 8);
            buf |= w << cnt;
            p += (63 - cnt) >> 3;
            cnt |= 56;
            return;
        }
        while (cnt <= 56) {
            if (p < end) buf |= (uint64_t)*p++ << cnt;
            else ++over;
            cnt += 8;
        }
    }
    inline uint32_t peek(int n) const { return (uint32_t)(buf & ((1ull << n) - 1ull)); }
    inline void drop(int n) {
        buf >>= n;
        cnt -= n;
    }
    inline uint32_t take(int n) {
        const uint32_t v = peek(n);
        drop(n);
        return v;
    }
    size_t pos() const { return (size_t)(p - s) * 8 + over * 8 - (size_t)cnt; }  // bits consumed
    bool overrun() const { return pos() > (size_t)(end - s) * 8; }
};

inline const Code& lookup(const Table& t, uint64_t buf) {
    const Code& c = t.e[buf & ((1u << t.root) - 1u)];
    if (c.op != OP_SUB) return c;
    return t.e[c.val + ((buf >> t.root) & ((1u << c.len) - 1u))];
}

// dynamic block header after BFINAL/BTYPE: the two tables (false: not a valid header)
inline bool read_dynamic(Bits& b, Table& lit, Table& dist) {
    b.refill();
    const int hlit = (int)b.take(5) + 257, hdist = (int)b.take(5) + 1, hclen = (int)b.take(4) + 4;
    if (hlit > 286 || hdist > 30) return false;
    static const uint8_t ORD[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    uint8_t cl[19] = {0};
    for (int i = 0; i < hclen; ++i) {
        if (b.cnt < 3) b.refill();
        cl[ORD[i]] = (uint8_t)b.take(3);
    }
    Table clt;
    if (!build(cl, 19, 7, K_CL, clt)) return false;
    uint8_t lens[286 + 30];
    int i = 0;
    const int total = hlit + hdist;
    while (i < total) {
        if (b.cnt < 16) b.refill();
        const Code& c = lookup(clt, b.buf);
        if (c.op != OP_LIT) return false;
        b.drop(c.len);
        const int sym = c.val;
        if (sym < 16) {
            lens[i++] = (uint8_t)sym;
            continue;
        }
        int rep, val = 0;
        if (sym == 16) {
            if (i == 0) return false;
            val = lens[i - 1];
            rep = 3 + (int)b.take(2);
        } else if (sym == 17) {
            rep = 3 + (int)b.take(3);
        } else {
            rep = 11 + (int)b.take(7);
        }
        if (i + rep > total) return false;
        while (rep--) lens[i++] = (uint8_t)val;
    }
    if (b.overrun() || lens[256] == 0) return false;
    return build(lens, hlit, 10, K_LIT, lit) && build(lens + hlit, hdist, 8, K_DIST, dist);
}

// ---- one chunk's decoder ---------------------------------------------------------------------------
// Output positions x = 0, 1, ... of the chunk.  While a marker may still be copied, output goes to
// `head` (16-bit).  Once 32 KiB of head hold no marker, no later reference can produce one: the decoder
// switches to bytes in `tail`, a byte buffer indexed by x itself whose [H - 32 KiB, H) mirrors head's
// last 32 KiB (H = head's length at the switch) and whose [0, H - 32 KiB) is filled by the final
// resolution, so tail becomes the chunk's output buffer without a copy.  Resumable at block boundaries.
template <class Buf>
struct alignas(128) Chunk {  // (own cache lines: neighbouring chunks are decoded by other threads)
    const uint8_t* s = nullptr;  // deflate stream
    size_t n = 0;
    bool first = false;          // the stream's first chunk: no window (a reference before it is an error)
    size_t start = 0;            // bit position of the first block (SIZE_MAX: no start found)
    size_t end = 0;              // bit position after the last block decoded (a block boundary)
    bool final_seen = false;     // the final block was decoded
    bool bad = false;
    U16s head;  // sized to its capacity: head_len values are output
    size_t head_len = 0;
    Buf tail;
    size_t tail_len = 0;         // bytes mode: output length (positions [0, tail_len) of tail are defined from H - WSIZE)
    size_t last_mark = 0;        // head position + 1 of the last marker written (0: none yet)
    bool bytes = false;
    Table lit, dist;

    size_t out_len() const { return bytes ? tail_len : head_len; }

    void grow_tail(size_t need) {
        if (tail_len + need <= tail.size()) return;
        tail.resize(std::max<size_t>(tail.size() * 2, tail_len + need + (4u << 20)));
    }
    void maybe_switch() {
        if (bytes) return;
        const size_t h = head_len;
        if (h < (size_t)WSIZE || h - last_mark < (size_t)WSIZE) return;
        tail.resize(h + (16u << 20));
        for (size_t x = h - WSIZE; x < h; ++x) tail[x] = (uint8_t)head[x];
        tail_len = h;
        bytes = true;
    }

    // one block's symbols (tables set); false on a data error.  head is sized to its capacity; head_len
    // holds the output length.  Markers only ever come from copies: a copy that reads one (or reaches
    // into the window) moves last_mark to its end (conservative: the switch to bytes comes later, never
    // early).
    bool symbols16(Bits& b, const Table& L, const Table& D) {
        uint16_t* out = head.data();
        size_t o = head_len, cap = head.size(), lm = last_mark;
        struct Sync {  // locals back into the chunk on every return
            size_t &o, &lm, &head_len, &last_mark;
            ~Sync() {
                head_len = o;
                last_mark = lm;
            }
        } sync{o, lm, head_len, last_mark};
        for (;;) {
            if (o + 2 * 258 > cap) {
                head.resize(std::max<size_t>(2 * cap, o + (1u << 20)));
                out = head.data();
                cap = head.size();
            }
            if (b.cnt < 48) {
                b.refill();
                if (b.over > 8) return false;  // decoding past the data's end (a valid stream never gets here)
            }
            const Code* c = &lookup(L, b.buf);
            b.drop(c->len);
            if (c->op == OP_LIT) {
                out[o++] = c->val;
                const Code* c2 = &lookup(L, b.buf);  // a second literal without a refill (>= 33 bits left)
                if (c2->op == OP_LIT) {
                    b.drop(c2->len);
                    out[o++] = c2->val;
                }
                continue;
            }
            if (c->op == OP_EOB) break;
            if (!(c->op & OP_BASE) || (c->op & (OP_BAD | OP_EOB))) {
                return false;
            }
            const uint32_t len = c->val + b.take(c->op & 15);
            c = &lookup(D, b.buf);
            b.drop(c->len);
            if (!(c->op & OP_BASE) || (c->op & (OP_BAD | OP_EOB))) {
                return false;
            }
            const uint32_t d = c->val + b.take(c->op & 15);
            uint16_t* dst = out + o;
            if ((size_t)d > o) {
                if (first) {  // before the stream's start
                    return false;
                }
                for (uint32_t i = 0; i < len; ++i) {
                    const int64_t src = (int64_t)(o + i) - (int64_t)d;
                    dst[i] = src < 0 ? (uint16_t)(MARK + (uint32_t)(WSIZE + src)) : out[src];
                }
                lm = o + len;
            } else {
                const uint16_t* src = dst - d;
                uint16_t m = 0;
                if (d >= len) {
                    for (uint32_t i = 0; i < len; ++i) {
                        dst[i] = src[i];
                        m |= src[i];
                    }
                } else {
                    for (uint32_t i = 0; i < len; ++i) {
                        const uint16_t v = src[i];
                        dst[i] = v;
                        m |= v;
                    }
                }
                if (m >= MARK) lm = o + len;
            }
            o += len;
        }
        return !b.overrun();
    }
    bool symbols8(Bits& b, const Table& L, const Table& D) {
        grow_tail(1u << 20);
        uint8_t* out = tail.data();
        size_t o = tail_len, cap = tail.size();
        for (;;) {
            if (o + 258 * 2 > cap) {
                tail_len = o;
                grow_tail(1u << 20);
                out = tail.data();
                cap = tail.size();
            }
            if (b.cnt < 48) {
                b.refill();
                if (b.over > 8) return false;  // decoding past the data's end (a valid stream never gets here)
            }
            const Code* c = &lookup(L, b.buf);
            b.drop(c->len);
            if (c->op == OP_LIT) {
                out[o++] = (uint8_t)c->val;
                const Code* c2 = &lookup(L, b.buf);  // a second literal without a refill (>= 33 bits left)
                if (c2->op == OP_LIT) {
                    b.drop(c2->len);
                    out[o++] = (uint8_t)c2->val;
                }
                continue;
            }
            if (c->op == OP_EOB) break;
            if (!(c->op & OP_BASE) || (c->op & (OP_BAD | OP_EOB))) {
                tail_len = o;
                return false;
            }
            const uint32_t len = c->val + b.take(c->op & 15);
            c = &lookup(D, b.buf);
            b.drop(c->len);
            if (!(c->op & OP_BASE) || (c->op & (OP_BAD | OP_EOB))) {
                tail_len = o;
                return false;
            }
            const uint32_t d = c->val + b.take(c->op & 15);
            if ((size_t)d > o) {  // (never for a switched chunk: its tail holds 32 KiB before its output)
                tail_len = o;
                return false;
            }
            uint8_t* dst = out + o;
            const uint8_t* src = dst - d;
            if (d >= len) {
                std::memcpy(dst, src, len);
            } else if (d == 1) {
                std::memset(dst, *src, len);
            } else {
                for (uint32_t i = 0; i < len; ++i) dst[i] = src[i];
            }
            o += len;
        }
        tail_len = o;
        return !b.overrun();
    }

    // decode blocks from bit position `from` until a block boundary >= stop (or the final block);
    // false on an error
    bool run(size_t from, size_t stop) {
        Bits b;
        b.init(s, n, from);
        if (!bytes && head.size() < head_len + (1u << 20))  // room for about 4x the compressed span
            head.resize(head_len + std::min<size_t>(stop - std::min(stop, from), n * 8) / 2 + (1u << 20));
        for (;;) {
            b.refill();
            const size_t at = b.pos();
            if (at >= stop || final_seen) {
                end = at;
                return true;
            }
            const uint32_t bfinal = b.take(1), btype = b.take(2);
            bool ok;
            if (btype == 0) {  // stored: byte-aligned LEN, NLEN, then LEN raw bytes
                b.drop(b.cnt & 7);
                b.refill();
                const uint32_t len = b.take(16), nlen = b.take(16);
                if ((len ^ 0xFFFFu) != nlen || b.overrun()) return false;
                if ((size_t)(b.end - b.p) + (size_t)(b.cnt >> 3) < len) return false;  // past the data's end
                for (uint32_t i = 0; i < len; ++i) {
                    if (b.cnt < 8) b.refill();
                    const uint8_t v = (uint8_t)b.take(8);
                    if (bytes) {
                        grow_tail(1);
                        tail[tail_len++] = v;
                    } else {
                        if (head_len == head.size()) head.resize(std::max<size_t>(2 * head.size(), 1u << 20));
                        head[head_len++] = v;
                    }
                }
                ok = !b.overrun();
            } else if (btype == 1) {
                ok = bytes ? symbols8(b, fixed_lit(), fixed_dist()) : symbols16(b, fixed_lit(), fixed_dist());
            } else if (btype == 2) {
                if (!read_dynamic(b, lit, dist)) return false;
                ok = bytes ? symbols8(b, lit, dist) : symbols16(b, lit, dist);
            } else {
                return false;
            }
            if (!ok) return false;
            if (bfinal) final_seen = true;
            maybe_switch();
        }
    }
};

// the first plausible block start at or after bit `from` (a non-final dynamic block whose header and
// whole body decode), before bit `to`; SIZE_MAX when none
template <class Buf>
inline size_t find_start(const uint8_t* s, size_t n, size_t from, size_t to) {
    Table lit, dist;
    for (size_t bp = from; bp < to && bp + 24 < n * 8; ++bp) {
        const size_t q = bp >> 3;
        const uint32_t h = (uint32_t)(s[q] | (s[q + 1] << 8) | (s[q + 2] << 16)) >> (bp & 7);
        if ((h & 7u) != 4u) continue;                                    // BFINAL 0, BTYPE 2 (dynamic)
        if (((h >> 3) & 31u) > 29u || ((h >> 8) & 31u) > 29u) continue;  // HLIT <= 286, HDIST <= 30
        Bits b;
        b.init(s, n, bp + 3);
        if (!read_dynamic(b, lit, dist)) continue;
        Chunk<Buf> probe;  // the block body must decode too (markers allowed)
        probe.s = s;
        probe.n = n;
        if (!probe.symbols16(b, lit, dist)) continue;
        return bp;
    }
    return SIZE_MAX;
}

// ---- the member ------------------------------------------------------------------------------------
// A gzip member's deflate data starting at s[0] (the file's remaining bytes s[0, n)), decoded by
// `threads` threads in chunks of chunk_bytes compressed bytes.  Buffers in `pieces` on entry are
// reused for the chunks' output (their capacity; the caller's recycled pieces).  On success `pieces` holds the decoded
// bytes in order (each piece one chunk's output), dend = the deflate data's byte length (the trailer
// follows), crc / total = the output's CRC-32 and length.  False on any failure (the caller decodes the
// file with zlib from its start), and when the chunks' output passes max_out bytes (the caller's memory
// budget: its estimate of the decoded size was low).  member_tail: the member's 8-byte trailer must
// follow the deflate data and nothing but NUL bytes after it (a gzip file of one member), checked right
// after the stitch, before the window, resolve and CRC phases.
struct Result {
    size_t dend = 0;
    uint32_t crc = 0;
    uint64_t total = 0;
    std::string why;
};
template <class Buf>
inline bool inflate_parallel(const uint8_t* s, size_t n, int threads, size_t chunk_bytes, std::vector<Buf>& pieces,
                             Result& r, size_t max_out = SIZE_MAX, bool member_tail = false) {
    const size_t K = std::max<size_t>(1, (n + chunk_bytes - 1) / chunk_bytes);
    std::vector<Chunk<Buf>> ch(K);
    for (size_t k = 0; k < K; ++k) {
        ch[k].s = s;
        ch[k].n = n;
        ch[k].first = k == 0;
        if (k < pieces.size()) {  // a buffer the caller passed in: the chunk's output reuses its capacity
            ch[k].tail = std::move(pieces[k]);
            ch[k].tail.clear();
        }
    }
    pieces.clear();
    auto pool = [&](const std::function<void()>& fn, size_t items) {
        std::vector<std::thread> ts;
        for (int t = 1; t < (int)std::min<size_t>((size_t)std::max(threads, 1), items); ++t) ts.emplace_back(fn);
        fn();
        for (auto& t : ts) t.join();
    };
    // 1. every chunk in parallel: its start, then blocks up to the next chunk's nominal start
    std::atomic<size_t> next{0};
    std::atomic<size_t> produced{0};  // phase 1's output so far (bytes): past max_out the decode stops
    std::atomic<bool> over{false};
#ifdef FRPZ_TIMING
    auto T0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        auto t1 = std::chrono::steady_clock::now();
        fprintf(stderr, "frpz %s %.3f s\n", what, std::chrono::duration<double>(t1 - T0).count());
        T0 = t1;
    };
#else
    auto lap = [](const char*) {};
#endif
    pool(
        [&]() {
            for (size_t k; !over.load(std::memory_order_relaxed) && (k = next.fetch_add(1)) < K;) {
                auto& c = ch[k];
                const size_t stop = (k + 1) * chunk_bytes * 8;
                try {
#ifdef FRPZ_TIMING
                    auto a0 = std::chrono::steady_clock::now();
#endif
                    c.start = k == 0 ? 0 : find_start<Buf>(s, n, k * chunk_bytes * 8, std::min(stop, n * 8));
#ifdef FRPZ_TIMING
                    auto a1 = std::chrono::steady_clock::now();
#endif
                    if (c.start != SIZE_MAX && !c.run(c.start, stop)) c.bad = true;
                    // (phase 1's chunks overlap by up to a block each, and a chunk's output can carry a window
                    // prefix: a quarter and 64 MiB of slack)
                    if (max_out != SIZE_MAX &&
                        produced.fetch_add(c.out_len()) + c.out_len() > max_out + max_out / 4 + (64u << 20))
                        over = true;
#ifdef FRPZ_TIMING
                    auto a2 = std::chrono::steady_clock::now();
                    fprintf(stderr, "chunk %zu find %.1f ms (%zu bits) run %.1f ms out %zu bytes-mode %d\n", k,
                            std::chrono::duration<double>(a1 - a0).count() * 1e3, c.start - k * chunk_bytes * 8,
                            std::chrono::duration<double>(a2 - a1).count() * 1e3, c.out_len(), (int)c.bytes);
#endif
                } catch (const std::bad_alloc&) {
                    c.bad = true;
                }
            }
        },
        K);
    lap("phase 1");
    if (over) {
        r.why = "the output outgrows the budget";
        return false;
    }
    if (ch[0].bad) {
        r.why = "the first chunk does not decode";
        return false;
    }
    // 2. stitch in order: the kept chunks, each starting where the previous kept one ended
    std::vector<size_t> keep{0};
    size_t k = 0;
    try {
        while (!ch[k].final_seen) {
            size_t j = k + 1;
            while (j < K && (ch[j].start == SIZE_MAX || ch[j].bad || ch[j].start < ch[k].end)) ++j;
            if (j < K && ch[j].start == ch[k].end) {
                keep.push_back(j);
                k = j;
                continue;
            }
            // decode on from chunk k's end to chunk j's start (or the stream's end); an end past chunk
            // j's start means it was no block boundary, and the loop looks further
            const size_t target = j < K ? ch[j].start : n * 8, before = ch[k].end;
            if (!ch[k].run(before, target) || (!ch[k].final_seen && ch[k].end < target) || ch[k].end == before) {
                r.why = "the stream does not decode on";
                return false;
            }
        }
    } catch (const std::bad_alloc&) {
        r.why = "out of memory";
        return false;
    }
    lap("stitch");
    const size_t dend = (ch[k].end + 7) / 8;
    if (dend > n) {
        r.why = "the data ends inside the final block";
        return false;
    }
    if (member_tail) {  // one member: its trailer, then only NUL padding (else another member follows)
        bool tail = dend + 8 <= n;
        for (size_t q = dend + 8; tail && q < n; ++q) tail = s[q] == 0;
        if (!tail) {
            r.why = "not a single member";
            return false;
        }
    }
    if (max_out != SIZE_MAX) {  // the stitch decodes on past phase 1: the same bound on the kept chunks
        size_t tot = 0;
        for (size_t j : keep) tot += ch[j].out_len();
        if (tot > max_out + max_out / 4 + (64u << 20)) {
            r.why = "the output outgrows the budget";
            return false;
        }
    }
    // 3. windows in order: the resolved last WSIZE bytes before each kept chunk
    auto resolve = [](uint32_t v, const std::vector<uint8_t>& wv, bool& ok) -> uint8_t {
        if (v < MARK) return (uint8_t)v;
        const size_t wi = v - MARK, have = wv.size();
        if (wi < (size_t)WSIZE - have) {  // before the stream's start
            ok = false;
            return 0;
        }
        return wv[wi - ((size_t)WSIZE - have)];
    };
    std::vector<std::vector<uint8_t>> win(keep.size());
    std::vector<uint8_t> w;
    bool wok = true;
    for (size_t i = 0; i < keep.size(); ++i) {
        const auto& c = ch[keep[i]];
        win[i] = w;
        const size_t L = c.out_len(), want = std::min<size_t>(WSIZE, L);
        for (size_t x = L - want; x < L; ++x)
            w.push_back(!c.bytes ? resolve(c.head[x], win[i], wok) : c.tail[x]);
        if (w.size() > (size_t)WSIZE) w.erase(w.begin(), w.begin() + (w.size() - WSIZE));
    }
    if (!wok) {
        r.why = "a reference before the stream's start";
        return false;
    }
    lap("windows");
    // 4. every kept chunk's markers resolved, in place where it switched to bytes, and its CRC-32
    pieces.resize(keep.size());
    std::vector<uint32_t> crcs(keep.size());
    std::vector<size_t> lens(keep.size());
    std::atomic<size_t> ni{0};
    std::atomic<bool> ok{true};
    pool(
        [&]() {
            for (size_t i; (i = ni.fetch_add(1)) < keep.size();) {
                auto& c = ch[keep[i]];
                const size_t L = c.out_len();
                // head positions still to resolve: all of head, or (switched) those before its mirrored tail
                const size_t H = c.bytes ? c.head_len - WSIZE : c.head_len;
                try {
                    if (!c.bytes) c.tail.resize(L);
                } catch (const std::bad_alloc&) {
                    ok = false;
                    continue;
                }
                uint8_t* o = c.tail.data();
                bool rok = true;
                const uint16_t* hv = c.head.data();
                size_t x = 0;
                for (; x + 64 <= H; x += 64) {  // runs without a marker narrow at vector speed
                    uint16_t m = 0;
                    for (int q = 0; q < 64; ++q) m |= hv[x + q];
                    if (m < MARK) {
                        for (int q = 0; q < 64; ++q) o[x + q] = (uint8_t)hv[x + q];
                    } else {
                        for (int q = 0; q < 64; ++q) o[x + q] = resolve(hv[x + q], win[i], rok);
                    }
                }
                for (; x < H; ++x) o[x] = resolve(hv[x], win[i], rok);
                if (!rok) ok = false;
                uLong cr = crc32(0L, Z_NULL, 0);
                for (size_t q = 0; q < L;) {  // crc32 takes uInt lengths
                    const size_t m = std::min<size_t>(L - q, 1u << 30);
                    cr = crc32(cr, o + q, (uInt)m);
                    q += m;
                }
                crcs[i] = (uint32_t)cr;
                lens[i] = L;
                c.head = U16s();
                c.tail.resize(L);
                pieces[i] = std::move(c.tail);
            }
        },
        keep.size());
    lap("resolve");
    if (!ok) {
        r.why = "resolve";
        return false;
    }
    uLong crc = 0;
    uint64_t total = 0;
    for (size_t i = 0; i < keep.size(); ++i) {
        crc = i == 0 ? crcs[0] : crc32_combine(crc, crcs[i], (z_off_t)lens[i]);
        total += lens[i];
    }
    r.dend = dend;
    r.crc = (uint32_t)crc;
    r.total = total;
    return true;
}

}  // namespace frpz
