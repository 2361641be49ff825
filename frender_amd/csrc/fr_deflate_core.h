// Deflate (RFC 1951) encoder pieces shared by the GPU block encoder (fr_deflate.hip) and its host
// check build (tests/native/frd_host.cpp): code tables, Huffman code lengths, the cost-based parse of
// one lane's sub-range, the code-length header and a bit writer that ORs into zeroed words.
//
// The demux writers of the reference (frender.py:667-676) are gzip.open(..., "wb") files, i.e. zlib at
// level 9.  The GPU encoder produces other bytes than zlib (any deflate stream that inflates to the
// same text is the same file to every reader, and the reference reads only text), at a size no larger
// than zlib -9's on the demux shapes (tests/test_deflate_host.py, tests/test_gpu_deflate.py).
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define FRD_HD __host__ __device__ inline
#else
#define FRD_HD inline
#endif

namespace frd {

constexpr uint32_t BLOCK = 1u << 16;   // input bytes per deflate block (one workgroup)
constexpr uint32_t WIN = 32768;        // deflate window
constexpr uint32_t HIST = WIN;         // bytes of its stream before a block that the block may reference
#ifndef FRD_SUB
#define FRD_SUB 1024
#endif
#ifndef FRD_HBITS
#define FRD_HBITS 13
#endif
#ifndef FRD_WAYS
#define FRD_WAYS 4
#endif
constexpr uint32_t SUB = FRD_SUB;         // parse sub-range of one lane (matches end at its edge)
constexpr uint32_t NSUB = BLOCK / SUB;
constexpr uint32_t HBITS = FRD_HBITS;         // hash buckets (LDS table: 8K buckets x WAYS u16 positions)
constexpr uint32_t WAYS = FRD_WAYS;
constexpr uint32_t HLEN = 6;           // the matchfinder hashes 6 bytes (its matches are >= 6 long)
constexpr uint32_t MINM = 4;           // the parse may cut a match down to 4
constexpr uint32_t MAXM = 258;
constexpr uint32_t NLL = 286, NDIST = 30, NCL = 19;
constexpr uint32_t CF = 16;            // parse costs in 1/16 bit
constexpr uint32_t OUT_STRIDE = BLOCK + 1024;  // per-block staging bytes (stored worst case 65546)
constexpr uint32_t STAGE_MAX = BLOCK - 16;     // a dynamic block is taken only if it fits the LDS staging

// bucket of the 6 bytes at a position: lo = bytes 0..3, hi = bytes 4..7 (little-endian)
FRD_HD uint32_t hash6(uint32_t lo, uint32_t hi) {
    const uint64_t w = ((uint64_t)lo << 16) | ((uint64_t)(hi & 0xFFFF) << 48);
    return (uint32_t)((w * 0x9E3779B97F4A7C15ull) >> (64 - HBITS));
}
FRD_HD uint32_t ilog2(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

// length 3..258 -> symbol index 0..28 (symbol 257 + idx), extra bits and their value
FRD_HD void len_code(uint32_t l, uint32_t& idx, uint32_t& eb, uint32_t& ev) {
    if (l == 258) {
        idx = 28, eb = 0, ev = 0;
        return;
    }
    const uint32_t v = l - 3;
    if (v < 8) {
        idx = v, eb = 0, ev = 0;
        return;
    }
    const uint32_t e = ilog2(v) - 2;
    idx = 4 * e + 4 + ((v >> e) & 3), eb = e, ev = v & ((1u << e) - 1);
}
FRD_HD uint32_t len_ebits(uint32_t idx) { return (idx < 8 || idx == 28) ? 0 : (idx - 4) / 4; }

// distance 1..32768 -> code 0..29, extra bits and their value
FRD_HD void dist_code(uint32_t d, uint32_t& code, uint32_t& eb, uint32_t& ev) {
    const uint32_t v = d - 1;
    if (v < 4) {
        code = v, eb = 0, ev = 0;
        return;
    }
    const uint32_t e = ilog2(v) - 1;
    code = 2 * e + 2 + ((v >> e) & 1), eb = e, ev = v & ((1u << e) - 1);
}
FRD_HD uint32_t dist_ebits(uint32_t code) { return code < 4 ? 0 : code / 2 - 1; }

FRD_HD uint32_t bitrev(uint32_t v, uint32_t n) {
    uint32_t r = 0;
    for (uint32_t k = 0; k < n; ++k, v >>= 1) r = (r << 1) | (v & 1);
    return r;
}

// Huffman work area for an alphabet of up to N symbols
template <uint32_t N>
struct HuffWork {
    uint32_t key[N];   // (freq << 9) | symbol of the used symbols, ascending after the sort
    uint32_t w[2 * N];
    uint16_t parent[2 * N];
    uint32_t m;
};

// the used symbols of freq[0..n) into wk.key (unsorted); at least two symbols (a complete code)
template <uint32_t N>
FRD_HD void huff_gather(const uint32_t* freq, uint32_t n, HuffWork<N>& wk) {
    uint32_t m = 0;
    for (uint32_t i = 0; i < n; ++i)
        if (freq[i]) wk.key[m++] = (freq[i] << 9) | i;
    for (uint32_t i = 0; m < 2 && i < n; ++i)
        if (!freq[i]) wk.key[m++] = (1u << 9) | i;
    wk.m = m;
}

template <uint32_t N>
FRD_HD void huff_sort(HuffWork<N>& wk) {  // insertion sort (host build; the GPU ranks in parallel)
    for (uint32_t i = 1; i < wk.m; ++i) {
        const uint32_t k = wk.key[i];
        uint32_t j = i;
        for (; j > 0 && wk.key[j - 1] > k; --j) wk.key[j] = wk.key[j - 1];
        wk.key[j] = k;
    }
}

// code lengths <= maxlen from the sorted keys (two-queue Huffman, then the Kraft repair that moves
// codes past maxlen up: drop one maxlen code, split the longest shorter one, until the sum is 1);
// the least frequent symbols take the longest lengths
template <uint32_t N>
FRD_HD void huff_lengths(HuffWork<N>& wk, uint32_t n, uint32_t maxlen, uint8_t* len) {
    for (uint32_t i = 0; i < n; ++i) len[i] = 0;
    const uint32_t m = wk.m;
    for (uint32_t i = 0; i < m; ++i) wk.w[i] = wk.key[i] >> 9;
    uint32_t li = 0, ni = m;
    for (uint32_t k = m; k < 2 * m - 1; ++k) {
        uint32_t a, b;
        if (li < m && (ni >= k || wk.w[li] <= wk.w[ni])) a = li++; else a = ni++;
        if (li < m && (ni >= k || wk.w[li] <= wk.w[ni])) b = li++; else b = ni++;
        wk.w[k] = wk.w[a] + wk.w[b];
        wk.parent[a] = (uint16_t)k;
        wk.parent[b] = (uint16_t)k;
    }
    const uint32_t root = 2 * m - 2;
    wk.w[root] = 0;
    for (uint32_t k = root; k-- > 0;) wk.w[k] = wk.w[wk.parent[k]] + 1;
    uint32_t cnt[16];
    for (uint32_t l = 0; l < 16; ++l) cnt[l] = 0;
    for (uint32_t i = 0; i < m; ++i) cnt[wk.w[i] < maxlen ? wk.w[i] : maxlen]++;
    uint32_t total = 0;
    for (uint32_t l = 1; l <= maxlen; ++l) total += cnt[l] << (maxlen - l);
    while (total != (1u << maxlen)) {
        cnt[maxlen]--;
        for (uint32_t l = maxlen - 1; l > 0; --l)
            if (cnt[l]) {
                cnt[l]--;
                cnt[l + 1] += 2;
                break;
            }
        total--;
    }
    uint32_t i = 0;
    for (uint32_t l = maxlen; l >= 1; --l)
        for (uint32_t c = cnt[l]; c; --c) len[wk.key[i++] & 511] = (uint8_t)l;
}

// canonical codes, bit-reversed for deflate's LSB-first packing
FRD_HD void huff_codes(const uint8_t* len, uint32_t n, uint16_t* code) {
    uint32_t cnt[16], next[16];
    for (uint32_t l = 0; l < 16; ++l) cnt[l] = 0;
    for (uint32_t i = 0; i < n; ++i) cnt[len[i]]++;
    cnt[0] = 0;
    uint32_t c = 0;
    next[0] = 0;
    for (uint32_t l = 1; l < 16; ++l) {
        c = (c + cnt[l - 1]) << 1;
        next[l] = c;
    }
    for (uint32_t i = 0; i < n; ++i) code[i] = len[i] ? (uint16_t)bitrev(next[len[i]]++, len[i]) : 0;
}

// Costs of one parse pass (1/16 bit): literal byte, match length 0..258, distance code (extra bits in)
struct Costs {
    uint16_t lit[256];
    uint16_t len[MAXM + 1];
    uint16_t dist[NDIST];
};

// 16 * log2(num / den) rounded down to 1/16 bit through an integer mantissa table (num >= den > 0):
// the host build and the kernel take the same first-pass costs
FRD_HD uint32_t log2_cf(uint32_t num, uint32_t den) {
    const uint64_t x = ((uint64_t)num << 16) / den;  // >= 1 << 16
    const uint32_t e = 63u - (uint32_t)__builtin_clzll(x);
    const uint32_t frac = (uint32_t)((x << (63 - e)) >> 59) & 15;
    const uint32_t tab[16] = {0, 1, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 15};
    return CF * (e - 16) + tab[frac];
}

// pass-1 cost of a literal that occurs cnt times in a block of len bytes (1..15 bits)
FRD_HD uint16_t lit_cost0(uint32_t cnt, uint32_t len) {
    const uint32_t v = cnt ? log2_cf(len, cnt) : CF * 15;
    return (uint16_t)(v < CF ? CF : v > CF * 15 ? CF * 15 : v);
}

FRD_HD uint32_t dist_cost(const Costs& c, uint32_t d) {
    uint32_t code, eb, ev;
    dist_code(d, code, eb, ev);
    return c.dist[code];
}

// Per-position record of the matchfinder: the byte, the longest match's length (0: none) and distance
FRD_HD uint32_t mpack(uint32_t byte, uint32_t len, uint32_t dist) {
    return byte | (len << 8) | (len ? (dist - 1) << 17 : 0u);
}
FRD_HD uint32_t m_byte(uint32_t v) { return v & 255; }
FRD_HD uint32_t m_len(uint32_t v) { return (v >> 8) & 511; }
FRD_HD uint32_t m_dist(uint32_t v) { return (v >> 17) + 1; }

// The longest of the candidate matches at p (distances dds[0..nc), 0 = none; the 4 bytes at p are w),
// ties to the nearer; every surviving candidate is compared 12 bytes a step in the same round, so a
// step costs one round of independent loads (the first round also tests the 4 bytes a candidate must
// share).  ld.w12(q) = the 12 bytes at q as three little-endian words (unaligned; reads stay within 16
// bytes past the block's end).
struct W12 {
    uint32_t a, b, c;
};
template <uint32_t NC, class LD>
FRD_HD void best_match(const uint8_t* p, uint32_t w, const uint32_t* dds, uint32_t r, uint32_t maxlen, LD ld,
                       uint32_t& bl, uint32_t& bd) {
    constexpr uint32_t nc = NC;
    uint32_t len[NC];
    uint32_t alive = 0;
    // first mismatch among the 12 bytes at l (x: the xor of the two reads); 12 when none
    auto diff = [](const W12& x) -> uint32_t {
        return x.a ? (uint32_t)__builtin_ctz(x.a) >> 3
               : x.b ? 4 + ((uint32_t)__builtin_ctz(x.b) >> 3)
               : x.c ? 8 + ((uint32_t)__builtin_ctz(x.c) >> 3)
                     : 12u;
    };
    {
        const W12 pw = ld.w12(p);
        (void)w;
#pragma unroll
        for (uint32_t s = 0; s < nc; ++s) {
            len[s] = 0;
            const uint32_t dd = dds[s];
            if (dd == 0 || dd > WIN || dd > r) continue;
            const W12 cw = ld.w12(p - dd);
            const W12 x{cw.a ^ pw.a, cw.b ^ pw.b, cw.c ^ pw.c};
            if (x.a & 0xFFFFFFFFu) continue;  // the first 4 bytes differ: no match
            len[s] = diff(x);
            if (len[s] == 12) alive |= 1u << s;
        }
    }
    for (uint32_t l = 12; alive && l < maxlen; l += 12) {
        const W12 pw = ld.w12(p + l);
#pragma unroll
        for (uint32_t s = 0; s < nc; ++s) {
            if (!(alive >> s & 1)) continue;
            const W12 cw = ld.w12(p - dds[s] + l);
            const uint32_t k = diff(W12{cw.a ^ pw.a, cw.b ^ pw.b, cw.c ^ pw.c});
            len[s] = l + k;
            if (k < 12) alive &= ~(1u << s);
        }
    }
    bl = 0, bd = 0;
#pragma unroll
    for (uint32_t s = 0; s < nc; ++s) {
        const uint32_t l = len[s] < maxlen ? len[s] : maxlen;
        if (l > bl || (l == bl && l && dds[s] < bd)) bl = l, bd = dds[s];
    }
}

// Four words held in registers (a named struct, never indexed: an array indexed by a variable would
// live in scratch memory)
struct Q4 {
    uint32_t v0, v1, v2, v3;
};
FRD_HD uint32_t sel4(const Q4& a, uint32_t j) {  // by shifts: a select of fields is turned back into an index
    const uint64_t lo = (uint64_t)a.v1 << 32 | a.v0, hi = (uint64_t)a.v3 << 32 | a.v2;
    return (uint32_t)(((j & 2) ? hi : lo) >> ((j & 1) * 32));
}
FRD_HD void or4(Q4& a, uint32_t j, uint32_t v) {
    a.v0 |= j == 0 ? v : 0u;
    a.v1 |= j == 1 ? v : 0u;
    a.v2 |= j == 2 ? v : 0u;
    a.v3 |= j == 3 ? v : 0u;
}

// the compiler waits here for q's loads (an empty use of its registers)
FRD_HD void ready(const Q4& q) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" ::"v"(q.v0), "v"(q.v1), "v"(q.v2), "v"(q.v3));
#else
    (void)q;
#endif
}

// 16-byte loads and stores of the per-lane arrays (16-byte aligned chunks)
FRD_HD Q4 ld16(const void* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint4 v = *(const uint4*)p;
    return Q4{v.x, v.y, v.z, v.w};
#else
    Q4 q;
    memcpy(&q, p, 16);
    return q;
#endif
}
FRD_HD void st16(void* p, const Q4& q) {
#if defined(__HIP_DEVICE_COMPILE__)
    *(uint4*)p = make_uint4(q.v0, q.v1, q.v2, q.v3);
#else
    memcpy(p, &q, 16);
#endif
}

// The per-position arrays of a block (matchfinder records, parse choices) are laid out lane-major
// by 16-byte chunk: the chunks of one chunk index for the NSUB lanes sit side by side, so the lanes'
// loads in step are contiguous.  lane = i / SUB, k = i % SUB.
struct Lay {
    uint32_t* m;
    uint16_t* ch;
    FRD_HD uint32_t* mchunk(uint32_t i) const { return m + ((((i % SUB) >> 2) * NSUB + i / SUB) << 2); }
    FRD_HD uint16_t* cchunk(uint32_t i) const { return ch + ((((i % SUB) >> 3) * NSUB + i / SUB) << 3); }
    FRD_HD uint32_t& rec(uint32_t i) const { return mchunk(i)[i & 3]; }
};

// The parse's costs-to-end of the next 256 positions: a ring (256 words per lane; the kernel
// swizzles a lane's slots by its lane number so that lanes marching in step hit distinct LDS banks)
struct Ring {
    uint32_t* base;
    uint32_t sw;
    FRD_HD uint32_t& at(uint32_t k) const { return base[(k & 255) ^ sw]; }
};
constexpr uint32_t PARSE_MAXL = 255;  // the ring holds best[i + 1 .. i + 255]: longer matches are cut

// Backward cost-minimising parse of [a, b) (block-relative; a a multiple of 8).  m[i] = mpack record
// of i; choice[i] = 0 (literal) or the match length taken at i, written 8 at a time (a chunk past b
// is overwritten: no lane owns those positions).  Matches end at b: a lane's sub-range is parsed on
// its own.  m is read 4 positions per load, three chunks (12 positions) ahead of the one in use, into
// four register slots that keep their roles (the walk is unrolled by four chunks: rotating the slots
// by copies made every position wait for the load in flight; a store in the position loop made the
// compiler wait for every load before it).  The lengths tried at a match: all of
// 4..10, or 4..8 and the last three of a longer one (trying every length changed the FASTQ shapes'
// streams by < 0.01%).
FRD_HD void parse_range(uint32_t a, uint32_t b, const Lay& ly, const Ring& best, const Costs& c) {
    if (b <= a) return;
    best.at(b - a) = 0;
    Q4 wbuf{0, 0, 0, 0};
    const uint32_t c0 = a >> 2;
    uint32_t cc = (b - 1) >> 2, next_best = 0, i = b;
    // chunk cc - d, or the range's first chunk past it (loaded, never used: every slot loads)
    auto ldc = [&](uint32_t d) { return ld16(ly.mchunk(4 * (cc >= c0 + d ? cc - d : c0))); };
    auto pos = [&](uint32_t mi) {  // position i (already decremented) with its record mi
        const uint32_t k = i - a;
        uint32_t bc = next_best + c.lit[m_byte(mi)];  // best(k + 1) is the previous step's result
        uint32_t ch = 0;
        uint32_t L = m_len(mi);
        if (L > b - i) L = b - i;
        if (L > PARSE_MAXL) L = PARSE_MAXL;
        if (L >= MINM) {
            const uint32_t dc = dist_cost(c, m_dist(mi));
            // eight lengths in increasing order, all read at once (no per-lane loop): 4..8, then 9..11
            // (those up to L) or L-2..L
            const uint32_t up = L <= 10 ? 0u : L - 11;
            uint32_t v[8];
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) {
                const uint32_t l = 4 + q + (q >= 5 ? up : 0u);
                v[q] = c.len[l] + best.at(k + l);
            }
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q) {
                const uint32_t l = 4 + q + (q >= 5 ? up : 0u), x = v[q] + dc;
                if (l <= L && x < bc) bc = x, ch = l;
            }
        }
        best.at(k) = bc;
        next_best = bc;
        or4(wbuf, (i >> 1) & 3, ch << ((i & 1) * 16));
    };
    auto run = [&](const Q4& q) {  // the positions of chunk cc left (a loop free of memory operations)
        for (const uint32_t lo = 4 * cc; i > lo;) {
            --i;
            pos(sel4(q, i & 3));
        }
    };
    auto flush = [&]() {  // after an even chunk: the choices of its 8 positions
        st16(ly.cchunk(4 * cc), wbuf);
        wbuf = Q4{0, 0, 0, 0};
    };
    if (!(cc & 1)) {  // an even first chunk on its own: the loop below starts at an odd one
        run(ldc(0));
        flush();
        if (cc == c0) return;
        --cc;
    }
    // Chunks cc (odd) .. cc - 3 in the four slots; each slot takes the chunk four below when its chunk
    // is done.  Before a store the next two chunks' slots are waited for: a load used while a store is
    // in flight makes the compiler wait for every load, the newest ones too.
    Q4 qa = ldc(0), qb = ldc(1), qc = ldc(2), qd = ldc(3);
    while (cc >= c0 + 4) {
        run(qa), qa = ldc(4), --cc;
        run(qb), ready(qc), ready(qd), flush(), qb = ldc(4), --cc;
        run(qc), qc = ldc(4), --cc;
        run(qd), ready(qa), ready(qb), flush(), qd = ldc(4), --cc;
    }
    // the last two or four chunks (c0 is even)
    run(qa), --cc;
    run(qb), flush();
    if (cc == c0) return;
    --cc;
    run(qc), --cc;
    run(qd), flush();
}

// Forward walk of a lane's parse: sym(ch, v) for each symbol of [a, b) in order (ch the choice, v the
// record at its start; a a multiple of 8).  The walk goes through the positions in groups of 8 (two
// record chunks and one choice chunk, loaded three groups ahead) and visits the symbols that start in
// each: the next symbol's position never waits on a load (following the choices from load to load made
// every step a memory round trip).  Four group slots keep their roles, as in parse_range.
struct Grp {
    Q4 r0, r1, c;
};
template <class SYM>
FRD_HD void walk(uint32_t a, uint32_t b, const Lay& ly, SYM sym) {
    if (b <= a) return;
    const uint32_t gl = (b - 1) >> 3;
    uint32_t g = a >> 3, nxt = a;
    auto ldg = [&](uint32_t d, Grp& q) {  // group g + d, or the lane's last group past it
        const uint32_t x = 8 * (g + d <= gl ? g + d : gl);
        q.r0 = ld16(ly.mchunk(x));
        q.r1 = ld16(ly.mchunk(x + 4));
        q.c = ld16(ly.cchunk(x));
    };
    Grp ga, gb, gc, gd;
    ldg(0, ga), ldg(1, gb), ldg(2, gc), ldg(3, gd);
    auto group = [&](Grp& q) {  // the symbols that start in group g, then q takes group g + 4
        const uint32_t hi = 8 * g + 8 < b ? 8 * g + 8 : b;
        while (nxt < hi) {
            const uint32_t i = nxt;
            const uint32_t ch = (sel4(q.c, (i >> 1) & 3) >> ((i & 1) * 16)) & 0xFFFF;
            const uint32_t v0 = sel4(q.r0, i & 3), v1 = sel4(q.r1, i & 3), v = (i & 4) ? v1 : v0;
            nxt = i + (ch >= MINM ? ch : 1);
            sym(ch, v);
        }
        if (g == gl) return false;
        ldg(4, q);
        ++g;
        return true;
    };
    while (g + 4 <= gl) {  // four groups with no exit among them
        group(ga), group(gb), group(gc), group(gd);
    }
    (void)(group(ga) && group(gb) && group(gc) && group(gd));  // the last 1..4
}

// Bit writer into zeroed 32-bit words: every word is ORed in (the GPU's lanes share edge words)
struct BitW {
    uint32_t* words;
    uint64_t acc;
    uint32_t n, w;
    FRD_HD void init(uint32_t* wd, uint64_t bitoff) {
        words = wd;
        w = (uint32_t)(bitoff >> 5);
        n = (uint32_t)(bitoff & 31);
        acc = 0;
    }
    template <class OR>
    FRD_HD void put(uint32_t bits, uint32_t len, OR orf) {  // len <= 32
        acc |= (uint64_t)bits << n;
        n += len;
        if (n >= 32) {
            orf(words + w, (uint32_t)acc);
            ++w;
            acc >>= 32;
            n -= 32;
        }
    }
    template <class OR>
    FRD_HD void flush(OR orf) {
        if (n) orf(words + w, (uint32_t)acc);
    }
};

// Code lengths and codes of one block's dynamic Huffman header
struct Tables {
    uint8_t ll_len[NLL];
    uint8_t d_len[NDIST];
    uint16_t ll_code[NLL];
    uint16_t d_code[NDIST];
    uint8_t cl_len[NCL];
    uint16_t cl_code[NCL];
    uint16_t items[NLL + NDIST];  // RLE of the code lengths: symbol | extra << 5
    uint32_t n_items, hlit, hdist, hclen;
};

FRD_HD uint32_t cl_order(uint32_t k) {
    const uint8_t o[NCL] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    return o[k];
}
FRD_HD uint32_t cl_ebits(uint32_t sym) { return sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0; }

// RLE of the lit/len + distance code lengths (runs may cross between the two, RFC 1951 3.2.7)
FRD_HD void header_items(Tables& t, uint32_t* cl_freq) {
    uint32_t hlit = NLL;
    while (hlit > 257 && !t.ll_len[hlit - 1]) --hlit;
    uint32_t hdist = NDIST;
    while (hdist > 1 && !t.d_len[hdist - 1]) --hdist;
    t.hlit = hlit;
    t.hdist = hdist;
    for (uint32_t s = 0; s < NCL; ++s) cl_freq[s] = 0;
    const uint32_t N = hlit + hdist;
    uint32_t k = 0;
    auto at = [&](uint32_t i) -> uint32_t { return i < hlit ? t.ll_len[i] : t.d_len[i - hlit]; };
    auto emit = [&](uint32_t sym, uint32_t extra) {
        t.items[k++] = (uint16_t)(sym | (extra << 5));
        cl_freq[sym]++;
    };
    for (uint32_t i = 0; i < N;) {
        const uint32_t v = at(i);
        uint32_t run = 1;
        while (i + run < N && at(i + run) == v) ++run;
        uint32_t r = run;
        if (v == 0) {
            while (r >= 11) {
                const uint32_t q = r < 138 ? r : 138;
                emit(18, q - 11);
                r -= q;
            }
            if (r >= 3) {
                emit(17, r - 3);
                r = 0;
            }
            for (; r; --r) emit(0, 0);
        } else {
            emit(v, 0);
            --r;
            while (r >= 3) {
                const uint32_t q = r < 6 ? r : 6;
                emit(16, q - 3);
                r -= q;
            }
            for (; r; --r) emit(v, 0);
        }
        i += run;
    }
    t.n_items = k;
}

// header bits after the code-length code is built (t.cl_len set)
FRD_HD uint32_t header_bits(Tables& t) {
    uint32_t hclen = NCL;
    while (hclen > 4 && !t.cl_len[cl_order(hclen - 1)]) --hclen;
    t.hclen = hclen;
    uint32_t bits = 3 + 5 + 5 + 4 + 3 * hclen;
    for (uint32_t k = 0; k < t.n_items; ++k) {
        const uint32_t s = t.items[k] & 31;
        bits += t.cl_len[s] + cl_ebits(s);
    }
    return bits;
}

template <class OR>
FRD_HD void write_header(const Tables& t, bool final_block, BitW& bw, OR orf) {
    bw.put((final_block ? 1u : 0u) | (2u << 1), 3, orf);
    bw.put(t.hlit - 257, 5, orf);
    bw.put(t.hdist - 1, 5, orf);
    bw.put(t.hclen - 4, 4, orf);
    for (uint32_t k = 0; k < t.hclen; ++k) bw.put(t.cl_len[cl_order(k)], 3, orf);
    for (uint32_t k = 0; k < t.n_items; ++k) {
        const uint32_t s = t.items[k] & 31, e = t.items[k] >> 5;
        bw.put(t.cl_code[s], t.cl_len[s], orf);
        if (s >= 16) bw.put(e, cl_ebits(s), orf);
    }
}

// body bits of [a, b) under the parse in choice[] and the final tables
FRD_HD uint64_t range_bits(uint32_t a, uint32_t b, const Lay& ly, const Tables& t) {
    uint64_t bits = 0;
    walk(a, b, ly, [&](uint32_t ch, uint32_t v) {
        if (ch >= MINM) {
            uint32_t idx, eb, ev, dcode, deb, dev;
            len_code(ch, idx, eb, ev);
            dist_code(m_dist(v), dcode, deb, dev);
            bits += t.ll_len[257 + idx] + eb + t.d_len[dcode] + deb;
        } else {
            bits += t.ll_len[m_byte(v)];
        }
    });
    return bits;
}

template <class OR>
FRD_HD void write_range(uint32_t a, uint32_t b, const Lay& ly, const Tables& t, BitW& bw, OR orf) {
    walk(a, b, ly, [&](uint32_t ch, uint32_t v) {
        if (ch >= MINM) {
            uint32_t idx, eb, ev, dcode, deb, dev;
            len_code(ch, idx, eb, ev);
            dist_code(m_dist(v), dcode, deb, dev);
            bw.put(t.ll_code[257 + idx], t.ll_len[257 + idx], orf);
            if (eb) bw.put(ev, eb, orf);
            bw.put(t.d_code[dcode], t.d_len[dcode], orf);
            if (deb) bw.put(dev, deb, orf);
        } else {
            bw.put(t.ll_code[m_byte(v)], t.ll_len[m_byte(v)], orf);
        }
    });
}

// symbol counts of [a, b) under the parse in choice[]
template <class ADD>
FRD_HD void count_range(uint32_t a, uint32_t b, const Lay& ly, uint32_t* llf, uint32_t* df, ADD add) {
    walk(a, b, ly, [&](uint32_t ch, uint32_t v) {
        if (ch >= MINM) {
            uint32_t idx, eb, ev, dcode, deb, dev;
            len_code(ch, idx, eb, ev);
            dist_code(m_dist(v), dcode, deb, dev);
            add(llf + 257 + idx);
            add(df + dcode);
        } else {
            add(llf + m_byte(v));
        }
    });
}

// parse costs from code lengths (a symbol the tables do not hold costs `absent` bits)
FRD_HD void costs_from_lengths(Costs& c, const uint8_t* ll_len, const uint8_t* d_len, uint32_t absent,
                               uint32_t lo, uint32_t hi_) {  // fills lit[lo..hi_) only (lanes split it)
    for (uint32_t i = lo; i < hi_; ++i) {
        if (i < 256) c.lit[i] = (uint16_t)(CF * (ll_len[i] ? ll_len[i] : absent));
        if (i <= MAXM) {
            if (i < 3) {
                c.len[i] = 0;
            } else {
                uint32_t idx, eb, ev;
                len_code(i, idx, eb, ev);
                const uint32_t l = ll_len[257 + idx];
                c.len[i] = (uint16_t)(CF * ((l ? l : absent) + eb));
            }
        }
        if (i < NDIST) c.dist[i] = (uint16_t)(CF * ((d_len[i] ? d_len[i] : absent) + dist_ebits(i)));
    }
}

}  // namespace frd
