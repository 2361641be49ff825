// Host build of the GPU block encoder's algorithm (test infrastructure: tests/test_deflate_host.py).
// It runs the shared pieces of frender_amd/csrc/fr_deflate_core.h in the order the kernel in
// frender_amd/csrc/fr_deflate.hip runs them, with the kernel's lanes as loops: the batched LDS-table
// matchfinder (a batch reads the table as the previous batches left it, then its lanes write; slot =
// the lane's wave), the per-lane sub-range parses, the passes and the block layout.  The product never
// loads this; the CPU suite uses it to check the encoder's streams with zlib and its size against zlib -9.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../frender_amd/csrc/fr_deflate_core.h"

using namespace frd;

namespace {

constexpr uint32_t TPB = 256;

uint32_t load32u(const uint8_t* p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}

struct HostLd {  // best_match's loads
    W12 w12(const uint8_t* p) const {
        W12 v;
        memcpy(&v, p, 12);
        return v;
    }
};

uint32_t crc_tab[256];
void crc_init() {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crc_tab[i] = c;
    }
}

struct Params {
    int passes;
    uint32_t len_init, dist_init;  // pass-1 symbol costs (bits) of a length / distance code
};

// one block: [start, start + len) of buf with `hist` bytes of history before it; returns bytes written
uint32_t encode_block(const uint8_t* buf, uint64_t start, uint32_t len, uint32_t hist, bool final_block, uint8_t* out,
                      const Params& P, std::vector<uint32_t>& m, std::vector<uint16_t>& choice,
                      std::vector<uint32_t>& best) {
    const uint8_t* blk = buf + start;
    const Lay ly{m.data(), choice.data()};
    const uint64_t hs = start - hist;
    const uint32_t ntot = hist + len;
    static uint16_t tab[(1u << HBITS) * WAYS];
    memset(tab, 0, sizeof tab);
    uint32_t bhist[256] = {0};
    // matchfinder: batches of TPB positions (relative to hs)
    std::vector<uint32_t> hsh(TPB);
    for (uint32_t base = 0; base < ntot; base += TPB) {
        for (uint32_t t = 0; t < TPB; ++t) {
            const uint32_t r = base + t;
            hsh[t] = ~0u;
            if (r >= ntot) continue;
            const uint64_t p = hs + r;
            if (r >= hist) bhist[buf[p]]++;
            const bool valid = r + HLEN <= ntot;
            if (!valid) {
                if (r >= hist) ly.rec(r - hist) = mpack(buf[p], 0, 0);
                continue;
            }
            const uint32_t w = load32u(buf + p);
            const uint32_t h = hash6(w, load32u(buf + p + 4));
            hsh[t] = h;
            if (r < hist) continue;
            const uint32_t maxlen = (ntot - r) < MAXM ? (ntot - r) : MAXM;
            uint32_t dds[WAYS + 1];
            for (uint32_t s = 0; s < WAYS; ++s) dds[s] = (r - tab[h * WAYS + s]) & 0xFFFF;
            dds[WAYS] = 0;
#ifndef FRD_INTRA_LO
#define FRD_INTRA_LO(t) 0
#endif
            for (uint32_t u = t; u-- > FRD_INTRA_LO(t);)  // the latest earlier lane of the batch with the same hash
                if (hsh[u] == h) {
                    dds[WAYS] = t - u;
                    break;
                }
            uint32_t bl, bd;
            best_match<WAYS + 1>(buf + p, w, dds, r, maxlen, HostLd{}, bl, bd);
            ly.rec(r - hist) = mpack(buf[p], bl >= MINM ? bl : 0, bd);
        }
        for (uint32_t t = 0; t < TPB; ++t)
            if (hsh[t] != ~0u) tab[hsh[t] * WAYS + t * WAYS / TPB] = (uint16_t)(base + t);
    }
    // CRC is folded by the caller (the whole stream); pass-1 costs
    Costs c;
    for (uint32_t b = 0; b < 256; ++b) c.lit[b] = lit_cost0(bhist[b], len);
    for (uint32_t l = 0; l <= MAXM; ++l) {
        if (l < 3) {
            c.len[l] = 0;
            continue;
        }
        uint32_t idx, eb, ev;
        len_code(l, idx, eb, ev);
        c.len[l] = (uint16_t)(CF * (P.len_init + eb));
    }
    for (uint32_t d = 0; d < NDIST; ++d) c.dist[d] = (uint16_t)(CF * (P.dist_init + dist_ebits(d)));
    const uint32_t nsub = (len + SUB - 1) / SUB;
    static Tables T;
    static HuffWork<NLL> hw;
    static HuffWork<NDIST> hwd;
    uint32_t llf[NLL], df[NDIST];
    auto add = [](uint32_t* p) { ++*p; };
    for (int pass = 0; pass < P.passes; ++pass) {
        for (uint32_t s = 0; s < nsub; ++s) {
            const uint32_t a = s * SUB, b = (s + 1) * SUB < len ? (s + 1) * SUB : len;
            parse_range(a, b, ly, Ring{best.data(), 0}, c);
        }
        memset(llf, 0, sizeof llf);
        memset(df, 0, sizeof df);
        llf[256] = 1;
        for (uint32_t s = 0; s < nsub; ++s) {
            const uint32_t a = s * SUB, b = (s + 1) * SUB < len ? (s + 1) * SUB : len;
            count_range(a, b, ly, llf, df, add);
        }
        huff_gather(llf, NLL, hw);
        huff_sort(hw);
        huff_lengths(hw, NLL, 15, T.ll_len);
        huff_gather(df, NDIST, hwd);
        huff_sort(hwd);
        huff_lengths(hwd, NDIST, 15, T.d_len);
        if (pass + 1 < P.passes) costs_from_lengths(c, T.ll_len, T.d_len, 15, 0, MAXM + 1);
    }
    huff_codes(T.ll_len, NLL, T.ll_code);
    huff_codes(T.d_len, NDIST, T.d_code);
    uint32_t clf[NCL];
    header_items(T, clf);
    static HuffWork<NCL> hwc;
    huff_gather(clf, NCL, hwc);
    huff_sort(hwc);
    huff_lengths(hwc, NCL, 7, T.cl_len);
    huff_codes(T.cl_len, NCL, T.cl_code);
    const uint32_t hdr = header_bits(T);
    uint64_t body = 0;
    for (uint32_t s = 0; s < NLL; ++s) body += (uint64_t)llf[s] * (T.ll_len[s] + (s > 256 ? len_ebits(s - 257) : 0));
    for (uint32_t s = 0; s < NDIST; ++s) body += (uint64_t)df[s] * (T.d_len[s] + dist_ebits(s));
    const uint64_t ebits = hdr + body;  // EOB counted in llf[256]
    const uint64_t dyn_bytes = final_block ? (ebits + 7) / 8 : (ebits + 3 + 7) / 8 + 4;
    const uint64_t stored_bytes = len + 5 * ((len + 65534) / 65535);
    if (dyn_bytes <= STAGE_MAX && dyn_bytes < stored_bytes) {
        uint32_t* words = (uint32_t*)out;
        memset(out, 0, (dyn_bytes + 7) & ~3ull);
        auto orf = [](uint32_t* p, uint32_t v) { *p |= v; };
        BitW bw;
        bw.init(words, 0);
        write_header(T, final_block, bw, orf);
        bw.flush(orf);
        uint64_t off = hdr;
        for (uint32_t s = 0; s < nsub; ++s) {
            const uint32_t a = s * SUB, b = (s + 1) * SUB < len ? (s + 1) * SUB : len;
            const uint64_t nb = range_bits(a, b, ly, T);
            BitW lw;
            lw.init(words, off);
            write_range(a, b, ly, T, lw, orf);
            lw.flush(orf);
            off += nb;
        }
        BitW ew;
        ew.init(words, off);
        ew.put(T.ll_code[256], T.ll_len[256], orf);
        ew.flush(orf);
        off += T.ll_len[256];
        if (off != ebits) return 0;  // accounting mismatch: the test fails on it
        if (!final_block) {
            const uint64_t q = (off + 3 + 7) / 8;
            out[q] = 0, out[q + 1] = 0, out[q + 2] = 0xFF, out[q + 3] = 0xFF;
        }
        return (uint32_t)dyn_bytes;
    }
    uint32_t o = 0;
    for (uint32_t a = 0; a < len || (a == 0 && len == 0); a += 65535) {
        const uint32_t n = len - a < 65535 ? len - a : 65535;
        const bool last = a + n >= len;
        out[o++] = (final_block && last) ? 1 : 0;
        out[o++] = n & 255, out[o++] = n >> 8, out[o++] = ~n & 255, out[o++] = (~n >> 8) & 255;
        memcpy(out + o, blk + a, n);
        o += n;
        if (len == 0) break;
    }
    return o;
}

}  // namespace

extern "C" {

// raw deflate stream of in[0, n) (blocks of BLOCK bytes, each with up to WIN bytes of history);
// returns the stream's byte count, 0 when cap is too small or the bit accounting failed
uint64_t frd_host_deflate(const uint8_t* in, uint64_t n, uint8_t* out, uint64_t cap, int passes, uint32_t len_init,
                          uint32_t dist_init, uint32_t* crc) {
    crc_init();
    uint32_t cr = 0xFFFFFFFFu;
    for (uint64_t i = 0; i < n; ++i) cr = crc_tab[(cr ^ in[i]) & 255] ^ (cr >> 8);
    *crc = ~cr;
    Params P{passes, len_init, dist_init};
    std::vector<uint32_t> m(BLOCK);
    std::vector<uint16_t> choice(BLOCK);
    std::vector<uint32_t> best(256);
    std::vector<uint8_t> padded(n + 16, 0);
    if (n) memcpy(padded.data(), in, n);
    std::vector<uint8_t> blkout(OUT_STRIDE);
    uint64_t o = 0;
    const uint64_t nb = n ? (n + BLOCK - 1) / BLOCK : 1;
    for (uint64_t b = 0; b < nb; ++b) {
        const uint64_t s = b * BLOCK;
        const uint32_t len = (uint32_t)(n - s < BLOCK ? n - s : BLOCK);
        const uint32_t hist = (uint32_t)(s < HIST ? s : HIST);
        const uint32_t k = encode_block(padded.data(), s, len, hist, b + 1 == nb, blkout.data(), P, m, choice, best);
        if (!k || o + k > cap) return 0;
        memcpy(out + o, blkout.data(), k);
        o += k;
    }
    return o;
}

}  // extern "C"
