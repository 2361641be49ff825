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

#if defined(__HIPCC__)
#define FRD_HD __host__ __device__ inline
#else
#define FRD_HD inline
#endif

namespace frd {

constexpr uint32_t BLOCK = 1u << 16;   // input bytes per deflate block (one workgroup)
constexpr uint32_t WIN = 32768;        // deflate window: history a block may reference
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

// Backward cost-minimising parse of [a, b) (block-relative).  m[i] = longest match at i
// (len | dist << 16, len 0 when none); choice[i] = 0 (literal) or the match length taken at i.
// best[] holds b - a + 1 entries.  Matches end at b: a lane's sub-range is parsed on its own.
FRD_HD void parse_range(const uint8_t* blk, uint32_t a, uint32_t b, const uint32_t* m, uint16_t* choice,
                        uint32_t* best, const Costs& c) {
    best[b - a] = 0;
    for (uint32_t i = b; i-- > a;) {
        uint32_t bc = best[i + 1 - a] + c.lit[blk[i]];
        uint32_t ch = 0;
        const uint32_t mi = m[i];
        uint32_t L = mi & 0xFFFF;
        if (L > b - i) L = b - i;
        if (L >= MINM) {
            const uint32_t dc = dist_cost(c, mi >> 16);
            const uint32_t* bb = best + (i - a);
            if (L <= 64) {
                for (uint32_t l = MINM; l <= L; ++l) {
                    const uint32_t x = c.len[l] + dc + bb[l];
                    if (x < bc) bc = x, ch = l;
                }
            } else {
                for (uint32_t l = MINM; l <= 36; ++l) {
                    const uint32_t x = c.len[l] + dc + bb[l];
                    if (x < bc) bc = x, ch = l;
                }
                for (uint32_t l = L - 32; l <= L; ++l) {
                    const uint32_t x = c.len[l] + dc + bb[l];
                    if (x < bc) bc = x, ch = l;
                }
            }
        }
        best[i - a] = bc;
        choice[i] = (uint16_t)ch;
    }
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
FRD_HD uint64_t range_bits(const uint8_t* blk, uint32_t a, uint32_t b, const uint32_t* m, const uint16_t* choice,
                           const Tables& t) {
    uint64_t bits = 0;
    for (uint32_t i = a; i < b;) {
        const uint32_t ch = choice[i];
        if (ch >= MINM) {
            uint32_t idx, eb, ev, dcode, deb, dev;
            len_code(ch, idx, eb, ev);
            dist_code(m[i] >> 16, dcode, deb, dev);
            bits += t.ll_len[257 + idx] + eb + t.d_len[dcode] + deb;
            i += ch;
        } else {
            bits += t.ll_len[blk[i]];
            ++i;
        }
    }
    return bits;
}

template <class OR>
FRD_HD void write_range(const uint8_t* blk, uint32_t a, uint32_t b, const uint32_t* m, const uint16_t* choice,
                        const Tables& t, BitW& bw, OR orf) {
    for (uint32_t i = a; i < b;) {
        const uint32_t ch = choice[i];
        if (ch >= MINM) {
            uint32_t idx, eb, ev, dcode, deb, dev;
            len_code(ch, idx, eb, ev);
            dist_code(m[i] >> 16, dcode, deb, dev);
            bw.put(t.ll_code[257 + idx], t.ll_len[257 + idx], orf);
            if (eb) bw.put(ev, eb, orf);
            bw.put(t.d_code[dcode], t.d_len[dcode], orf);
            if (deb) bw.put(dev, deb, orf);
            i += ch;
        } else {
            bw.put(t.ll_code[blk[i]], t.ll_len[blk[i]], orf);
            ++i;
        }
    }
}

// symbol counts of [a, b) under the parse in choice[]
template <class ADD>
FRD_HD void count_range(const uint8_t* blk, uint32_t a, uint32_t b, const uint32_t* m, const uint16_t* choice,
                        uint32_t* llf, uint32_t* df, ADD add) {
    for (uint32_t i = a; i < b;) {
        const uint32_t ch = choice[i];
        if (ch >= MINM) {
            uint32_t idx, eb, ev, dcode, deb, dev;
            len_code(ch, idx, eb, ev);
            dist_code(m[i] >> 16, dcode, deb, dev);
            add(llf + 257 + idx);
            add(df + dcode);
            i += ch;
        } else {
            add(llf + blk[i]);
            ++i;
        }
    }
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
