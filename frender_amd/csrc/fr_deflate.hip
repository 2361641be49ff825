// fr_deflate.hip — the demux writers' gzip compression on the GPU (the
// gzip.open(..., "wb") writer pairs of frender.py:667-676 that every routed record goes through,
// frender.py:795-810).
//
// A window of routed bytes is already in HBM, destination-major (fr_dmx_route).  Every destination's
// range becomes one raw deflate stream: blocks of 64 KiB of input, each block one workgroup, each
// block referencing up to 32 KiB of its own destination's preceding bytes.  A non-final block ends
// with an empty stored block (the byte alignment of zlib's Z_SYNC_FLUSH), so the blocks of one
// stream simply concatenate.  Per block (deflate_blocks):
//   matchfinder   batches of 256 positions: each lane hashes the 6 bytes at its position, reads the
//                 four positions of its bucket in an LDS table (8K buckets x 4, one slot per wave)
//                 and the latest earlier lane of the batch with the same hash, extends the candidates
//                 against the block's bytes (global loads, L2-resident) and keeps the longest match
//   crc32         64 lanes over 1 KiB each, folded by the 1-KiB shift operator
//   parse         64 lanes, one 1-KiB sub-range each: backward cost-minimising parse over the
//                 longest match at every position and its shorter lengths (fr_deflate_core.h)
//   Huffman       four passes: parse, symbol counts (LDS atomics), code lengths (ranked in parallel,
//                 two-queue tree and Kraft repair on one lane), costs for the next parse
//   emit          header on lane 0, every lane's symbols ORed into an LDS staging copy at its bit
//                 offset (exclusive scan of the lanes' bit counts), copied out word by word; a block
//                 that would not shrink is stored instead
// Then the block outputs are compacted (rocprim scan + copy) and the host folds the blocks' CRCs per
// destination.  Bound: not HBM (a window is read ~3 times) but the matchfinder's dependent loads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <rocprim/rocprim.hpp>
#include <zlib.h>

#include "../../include/frender_amd.h"
#include "fr_deflate_core.h"

namespace {

using namespace frd;

constexpr uint32_t TPB = 256;
constexpr uint32_t NPASS = 3;
constexpr uint32_t NB = 1u << HBITS;
constexpr uint64_t SCR_BYTES = (uint64_t)BLOCK * 4 + (uint64_t)BLOCK * 2 + 256;
static_assert(NSUB * 256 <= NB * WAYS / 2, "the parse rings live in the matchfinder table");

struct DJob {
    uint64_t start;  // first input byte (offset into the data buffer)
    uint32_t len;    // input bytes (1..BLOCK)
    uint32_t hist;   // bytes of the same stream before start the block may reference (<= WIN)
    uint32_t last;   // 1: the stream's final block
    uint32_t pad;
};

struct DefShared {
    union {
        uint16_t tab[NB * WAYS];  // matchfinder buckets (positions mod 65536, relative to the history start)
        uint32_t stage[NB * WAYS / 2];  // then the block's output bits
    };
    alignas(8) uint16_t bh[TPB];  // this batch's hashes (0xFFFF: none)
    uint32_t seen[2][2][128];     // per batch parity: hashes (>> 1) seen once / again in the batch
    uint32_t first[256];          // per hash & 255: batch << 8 | 255 - the batch's first lane with it (max)
    uint32_t bhist[256];
    uint32_t llf[NLL];
    uint32_t df[NDIST];
    uint32_t clf[NCL];
    Costs cost;
    Tables T;
    HuffWork<NLL> hw;
    HuffWork<NDIST> hwd;
    HuffWork<NCL> hwc;
    uint32_t crc_tab[256];
    uint32_t lane_v[NSUB];
    uint32_t lane_off[NSUB];
    uint32_t misc[8];  // 0 mode (1 dynamic), 1 header bits, 2 total bytes, 3 eob bit
};

__device__ __forceinline__ uint32_t ld32u(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
    return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(a & 3));
}

#ifdef FRD_PROF
__device__ unsigned long long g_prof[12];
#define PROF_MARK(k)                                                            \
    do {                                                                        \
        if (t == 0) {                                                           \
            const unsigned long long now_ = wall_clock64();                     \
            atomicAdd(&g_prof[k], now_ - prof_t);                               \
            prof_t = now_;                                                      \
        }                                                                       \
    } while (0)
#define PROF_SUB(k) const unsigned long long k = wall_clock64()
#else
#define PROF_MARK(k) \
    do {             \
    } while (0)
#define PROF_SUB(k) \
    do {            \
    } while (0)
#endif

// best_match's loads of a block's window: one buffer load of the dwords that hold the 12 bytes at p
// (the candidates' loads are scattered, so the memory pipeline's cost is per instruction; a buffer
// load takes dword-aligned multi-dword reads, and reads past the window's 16 readable bytes return 0)
struct Ld32 {
    const uint8_t* base;
    __amdgpu_buffer_rsrc_t rs;
    __device__ Ld32(const uint8_t* b, uint32_t bytes)
        : base(b), rs(__builtin_amdgcn_make_buffer_rsrc((void*)b, (short)0, (int)bytes, 0x00020000)) {}
    __device__ W12 w12(const uint8_t* p) const {
        const uint32_t o = (uint32_t)(p - base), s = o & 3u;
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, o & ~3u, 0, 0);
        return W12{__builtin_amdgcn_alignbyte(v[1], v[0], s), __builtin_amdgcn_alignbyte(v[2], v[1], s),
                   __builtin_amdgcn_alignbyte(v[3], v[2], s)};
    }
};

struct LdsOr {
    __device__ void operator()(uint32_t* p, uint32_t v) const {
        if (v) atomicOr(p, v);
    }
};
struct LdsAdd {
    __device__ void operator()(uint32_t* p) const { atomicAdd(p, 1u); }
};

// code lengths of S.llf (all lanes: the gather and the rank sort are parallel, the tree is lane 0's)
__device__ void ll_lengths(DefShared& S, uint32_t t) {
    if (t == 0) S.hw.m = 0;
    __syncthreads();
    for (uint32_t i = t; i < NLL; i += TPB)
        if (S.llf[i]) S.hw.key[atomicAdd(&S.hw.m, 1u)] = (S.llf[i] << 9) | i;
    __syncthreads();
    if (t == 0)
        for (uint32_t i = 0; S.hw.m < 2; ++i)
            if (!S.llf[i]) S.hw.key[S.hw.m++] = (1u << 9) | i;
    __syncthreads();
    const uint32_t m = S.hw.m;
    for (uint32_t i = t; i < m; i += TPB) {
        const uint32_t k = S.hw.key[i];
        uint32_t rank = 0;
        for (uint32_t j = 0; j < m; ++j) rank += S.hw.key[j] < k;
        S.hw.w[rank] = k;
    }
    __syncthreads();
    for (uint32_t i = t; i < m; i += TPB) S.hw.key[i] = S.hw.w[i];
    __syncthreads();
    if (t == 0) huff_lengths(S.hw, NLL, 15, S.T.ll_len);
}

__global__ __launch_bounds__(TPB, 2) void deflate_blocks(const uint8_t* __restrict__ data, const DJob* __restrict__ jobs,
                                                         uint32_t n_jobs, uint8_t* __restrict__ stage_out,
                                                         uint32_t* __restrict__ out_len, uint32_t* __restrict__ out_crc,
                                                         uint8_t* __restrict__ scratch,
                                                         const uint32_t* __restrict__ crc_shift) {
    __shared__ DefShared S;
    const uint32_t t = threadIdx.x;
    {
        uint32_t c = t;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        S.crc_tab[t] = c;
    }
    uint32_t* m = (uint32_t*)(scratch + (uint64_t)blockIdx.x * SCR_BYTES);
    uint16_t* choice = (uint16_t*)(m + BLOCK);
    const Lay ly{m, choice};
#ifdef FRD_PROF
    unsigned long long prof_t = wall_clock64();
#endif
    for (uint32_t j = blockIdx.x; j < n_jobs; j += gridDim.x) {
        const DJob job = jobs[j];
        const uint32_t len = job.len, hist = job.hist, ntot = hist + len;
        const uint8_t* blk = data + job.start;
        const uint8_t* hsp = blk - hist;
        const Ld32 win(hsp, ntot + 16);  // (the data's 16 readable bytes past the end: fr_defl_run)
        for (uint32_t i = t; i < NB * WAYS / 2; i += TPB) S.stage[i] = 0;
        S.bhist[t] = 0;
        S.seen[t >> 7][0][t & 127] = 0;
        S.seen[t >> 7][1][t & 127] = 0;
        S.first[t] = 0;
        __syncthreads();
        // ---- matchfinder
#ifdef FRD_PROF
        unsigned long long ps[3] = {0, 0, 0};  // lane 0's batch segments: to the first barrier, to the second, the rest
#endif
        for (uint32_t base = 0; base < ntot; base += TPB) {
            PROF_SUB(pq0);
            const uint32_t r = base + t;
            uint32_t h = 0xFFFF, w = 0;
            if (r < ntot) {
                if (r >= hist) atomicAdd(&S.bhist[hsp[r]], 1u);
                if (r + HLEN <= ntot) {
                    w = ld32u(hsp + r);
                    h = hash6(w, ld32u(hsp + r + 4));
                }
            }
            S.bh[t] = (uint16_t)h;
            const uint32_t par = (base / TPB) & 1;
            if (h != 0xFFFF) {
                const uint32_t bit = 1u << ((h >> 1) & 31), wi = h >> 6;
                if (atomicOr(&S.seen[par][0][wi], bit) & bit) atomicOr(&S.seen[par][1][wi], bit);
                atomicMax(&S.first[h & 255], (base / TPB + 1) << 8 | (TPB - 1 - t));
            }
            __syncthreads();
            PROF_SUB(pq1);
            S.seen[par ^ 1][t >> 7][t & 127] = 0;  // the other parity's maps, for the next batch
            if (r >= hist && r < ntot) {
                uint32_t bl = 0, bd = 0;
                if (h != 0xFFFF) {
                    const uint32_t maxlen = min(MAXM, ntot - r);
                    uint32_t dds[WAYS + 1];
                    for (uint32_t s = 0; s < WAYS; ++s) dds[s] = (r - S.tab[h * WAYS + s]) & 0xFFFF;
                    dds[WAYS] = 0;
                    // the lanes of the batch with this hash are at or after the first lane with its low
                    // byte: a lane that is that first one, or whose hash the batch holds once, has none
                    const uint32_t lo = TPB - 1 - (S.first[h & 255] & 255);
                    if (lo < t && (S.seen[par][1][h >> 6] >> ((h >> 1) & 31) & 1)) {
                        // another lane of the batch may share the hash: the latest earlier one,
                        // sixteen hashes (four independent LDS reads) per step; a word's fields equal
                        // to h are found at once (zero-field flags: a flag above a zero field may be a
                        // borrow's, but a flagged word holds a zero field, its highest is the lane)
                        const uint64_t hh = (uint64_t)h * 0x0001000100010001ull;
                        const uint64_t* bw = (const uint64_t*)S.bh;
                        uint32_t u = ~0u;
                        for (int g = ((int)t - 1) >> 4; g >= (int)(lo >> 4) && u == ~0u; --g) {
                            uint64_t v[4];
#pragma unroll
                            for (int q = 0; q < 4; ++q) v[q] = bw[4 * g + q] ^ hh;
                            const int rem = (int)t - 16 * g;  // the group's lanes below t
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                const int nb = rem - 4 * q;  // fields of word q below t
                                uint64_t z = (v[q] - 0x0001000100010001ull) & ~v[q] & 0x8000800080008000ull;
                                z = nb >= 4 ? z : nb <= 0 ? 0ull : z & ((1ull << (16 * nb)) - 1ull);
                                if (z) {
                                    const uint64_t x = v[q];
                                    const uint32_t f = (nb > 3 && !(x >> 48)) ? 3u
                                                       : (nb > 2 && !((x >> 32) & 0xFFFF)) ? 2u
                                                       : (nb > 1 && !((x >> 16) & 0xFFFF)) ? 1u
                                                                                            : 0u;
                                    u = 16 * g + 4 * q + f;
                                }
                            }
                        }
                        if (u != ~0u) dds[WAYS] = t - u;
                    }
                    best_match<WAYS + 1>(hsp + r, w, dds, r, maxlen, win, bl, bd);
                }
                ly.rec(r - hist) = mpack(hsp[r], bl >= MINM ? bl : 0u, bd);
            }
            __syncthreads();
            PROF_SUB(pq2);
            if (h != 0xFFFF) S.tab[h * WAYS + (t >> 6)] = (uint16_t)r;
#ifdef FRD_PROF
            ps[0] += pq1 - pq0, ps[1] += pq2 - pq1, ps[2] += wall_clock64() - pq2;
#endif
        }
#ifdef FRD_PROF
        if (t == 0)
            for (int q = 0; q < 3; ++q) atomicAdd(&g_prof[8 + q], ps[q]);
#endif
        __syncthreads();
        PROF_MARK(0);
        // ---- crc32 of the block: 1-KiB slices, folded by lane 0
        const uint32_t nsub = (len + SUB - 1) / SUB;
        if (t < nsub) {
            const uint32_t a = t * SUB, b = min(len, a + SUB);
            uint32_t c = 0xFFFFFFFFu;
            for (uint32_t i = a; i < b; ++i) c = S.crc_tab[(c ^ blk[i]) & 255] ^ (c >> 8);
            S.lane_v[t] = ~c;
        }
        // pass-1 costs: literals from the block's byte histogram, lengths and distances flat
        {
            S.cost.lit[t] = lit_cost0(S.bhist[t], len);
            for (uint32_t l = t; l <= MAXM; l += TPB) {
                uint32_t idx = 0, eb = 0, ev;
                if (l >= 3) len_code(l, idx, eb, ev);
                S.cost.len[l] = l < 3 ? 0 : (uint16_t)(CF * (2 + eb));
            }
            if (t < NDIST) S.cost.dist[t] = (uint16_t)(CF * (2 + dist_ebits(t)));
        }
        __syncthreads();
        uint32_t crc = 0;
        if (t == 0) {
            for (uint32_t s = 0; s < nsub; ++s) {
                const uint32_t sl = min(SUB, len - s * SUB);
                if (sl == SUB) {
                    crc = crc_shift[crc & 255] ^ crc_shift[256 + ((crc >> 8) & 255)] ^
                          crc_shift[512 + ((crc >> 16) & 255)] ^ crc_shift[768 + (crc >> 24)];
                } else {
                    for (uint32_t k = 0; k < sl; ++k) crc = S.crc_tab[crc & 255] ^ (crc >> 8);
                }
                crc ^= S.lane_v[s];
            }
        }
        PROF_MARK(1);
        // ---- parse passes
        for (uint32_t pass = 0; pass < NPASS; ++pass) {
            for (uint32_t i = t; i < NLL; i += TPB) S.llf[i] = 0;
            if (t < NDIST) S.df[t] = 0;
            if (t < nsub) {
                const uint32_t a = t * SUB, b = min(len, a + SUB);
                parse_range(a, b, ly, Ring{S.stage + t * 256, t & 63}, S.cost);
            }
            __syncthreads();
            PROF_MARK(2);
            if (t == 0) S.llf[256] = 1;
            if (t < nsub) {
                const uint32_t a = t * SUB, b = min(len, a + SUB);
                count_range(a, b, ly, S.llf, S.df, LdsAdd{});
            }
            __syncthreads();
            PROF_MARK(3);
            if (t == 64) {
                huff_gather(S.df, NDIST, S.hwd);
                huff_sort(S.hwd);
                huff_lengths(S.hwd, NDIST, 15, S.T.d_len);
            }
            ll_lengths(S, t);
            __syncthreads();
            PROF_MARK(4);
            if (pass + 1 < NPASS) {
                costs_from_lengths(S.cost, S.T.ll_len, S.T.d_len, 15, t, t + 1);
                if (t + TPB <= MAXM) costs_from_lengths(S.cost, S.T.ll_len, S.T.d_len, 15, t + TPB, t + TPB + 1);
                __syncthreads();
            }
        }
        // ---- tables, header and block size (lane 0)
        if (t == 0) {
            huff_codes(S.T.ll_len, NLL, S.T.ll_code);
            huff_codes(S.T.d_len, NDIST, S.T.d_code);
            header_items(S.T, S.clf);
            huff_gather(S.clf, NCL, S.hwc);
            huff_sort(S.hwc);
            huff_lengths(S.hwc, NCL, 7, S.T.cl_len);
            huff_codes(S.T.cl_len, NCL, S.T.cl_code);
            const uint32_t hdr = header_bits(S.T);
            uint64_t body = 0;
            for (uint32_t s = 0; s < NLL; ++s)
                body += (uint64_t)S.llf[s] * (S.T.ll_len[s] + (s > 256 ? len_ebits(s - 257) : 0));
            for (uint32_t s = 0; s < NDIST; ++s) body += (uint64_t)S.df[s] * (S.T.d_len[s] + dist_ebits(s));
            const uint64_t ebits = hdr + body;
            const uint64_t dyn_bytes = job.last ? (ebits + 7) / 8 : (ebits + 3 + 7) / 8 + 4;
            const uint64_t stored_bytes = len + 5 * ((len + 65534) / 65535);
            const bool dyn = dyn_bytes <= STAGE_MAX && dyn_bytes < stored_bytes;
            S.misc[0] = dyn;
            S.misc[1] = hdr;
            S.misc[2] = (uint32_t)(dyn ? dyn_bytes : stored_bytes);
            S.misc[3] = (uint32_t)(ebits - S.T.ll_len[256]);
        }
        __syncthreads();
        PROF_MARK(5);
        uint8_t* out = stage_out + (uint64_t)j * OUT_STRIDE;
        if (S.misc[0]) {
            if (t < nsub) {
                const uint32_t a = t * SUB, b = min(len, a + SUB);
                S.lane_v[t] = (uint32_t)range_bits(a, b, ly, S.T);
            }
            __syncthreads();
            if (t == 0) {
                uint32_t off = S.misc[1];
                for (uint32_t s = 0; s < nsub; ++s) {
                    S.lane_off[s] = off;
                    off += S.lane_v[s];
                }
                // the lanes' bits must add up to the counted body; if they do not, the block is stored
                // (always a valid encoding of its bytes) and counted in out_crc[n_jobs]
                if (off != S.misc[3]) {
                    S.misc[0] = 0;
                    S.misc[2] = len + 5 * ((len + 65534) / 65535);
                    atomicAdd(&out_crc[n_jobs], 1u);
                }
            }
            __syncthreads();
        }
        const uint32_t nbytes = S.misc[2];
        if (S.misc[0]) {
            const uint32_t nw = (nbytes + 3) / 4;
            for (uint32_t i = t; i < nw + 1; i += TPB) S.stage[i] = 0;
            __syncthreads();
            if (t < nsub) {
                const uint32_t a = t * SUB, b = min(len, a + SUB);
                BitW bw;
                bw.init(S.stage, S.lane_off[t]);
                write_range(a, b, ly, S.T, bw, LdsOr{});
                bw.flush(LdsOr{});
            }
            if (t == TPB - 1) {
                BitW bw;
                bw.init(S.stage, 0);
                write_header(S.T, job.last != 0, bw, LdsOr{});
                bw.flush(LdsOr{});
                const uint32_t eob = S.misc[3];
                bw.init(S.stage, eob);
                bw.put(S.T.ll_code[256], S.T.ll_len[256], LdsOr{});
                bw.flush(LdsOr{});
                if (!job.last) {  // empty stored block: 3 zero bits, pad, LEN 0000, NLEN FFFF
                    const uint32_t q = (eob + S.T.ll_len[256] + 3 + 7) / 8;
                    LdsOr{}(&S.stage[(q + 2) >> 2], 0xFFu << (8 * ((q + 2) & 3)));
                    LdsOr{}(&S.stage[(q + 3) >> 2], 0xFFu << (8 * ((q + 3) & 3)));
                }
            }
            __syncthreads();
            uint32_t* ow = (uint32_t*)out;
            for (uint32_t i = t; i < nw; i += TPB) ow[i] = S.stage[i];
        } else {
            for (uint32_t i = t; i < len; i += TPB) out[5 * (i / 65535 + 1) + i] = blk[i];
            if (t == 0) {
                for (uint32_t a = 0; a < len; a += 65535) {
                    const uint32_t n = min(65535u, len - a);
                    uint8_t* o = out + a + 5 * (a / 65535);
                    o[0] = (job.last && a + n >= len) ? 1 : 0;
                    o[1] = n & 255, o[2] = n >> 8, o[3] = ~n & 255, o[4] = (~n >> 8) & 255;
                }
            }
        }
        if (t == 0) {
            out_len[j] = nbytes;
            out_crc[j] = crc;
        }
        __syncthreads();
        PROF_MARK(6);
    }
}

__global__ void deflate_compact(const uint8_t* __restrict__ stage_out, const uint32_t* __restrict__ out_len,
                                const uint64_t* __restrict__ boff, uint32_t n_jobs, uint8_t* __restrict__ out) {
    for (uint32_t j = blockIdx.x; j < n_jobs; j += gridDim.x) {
        const uint8_t* s = stage_out + (uint64_t)j * OUT_STRIDE;
        uint8_t* d = out + boff[j];
        const uint32_t n = out_len[j];
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) d[i] = s[i];
    }
}

// linear operator "feed n zero bytes into the raw CRC register", byte-sliced: 4 x 256 words
void crc_shift_table(uint64_t n, uint32_t* T) {
    static uint32_t tab[256];
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        tab[i] = c;
    }
    uint32_t basis[32];
    for (int b = 0; b < 32; ++b) {
        uint32_t c = 1u << b;
        for (uint64_t k = 0; k < n; ++k) c = tab[c & 255] ^ (c >> 8);
        basis[b] = c;
    }
    for (int s = 0; s < 4; ++s)
        for (uint32_t v = 0; v < 256; ++v) {
            uint32_t r = 0;
            for (int b = 0; b < 8; ++b)
                if (v >> b & 1) r ^= basis[8 * s + b];
            T[256 * s + v] = r;
        }
}

uint32_t crc_apply(const uint32_t* T, uint32_t c) {
    return T[c & 255] ^ T[256 + ((c >> 8) & 255)] ^ T[512 + ((c >> 16) & 255)] ^ T[768 + (c >> 24)];
}

}  // namespace

struct fr_defl {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::string err;
    int grid = 0;
    DJob* jobs = nullptr;
    uint32_t *blen = nullptr, *bcrc = nullptr, *shift = nullptr;
    uint64_t* boff = nullptr;
    uint8_t *stage = nullptr, *out = nullptr, *scratch = nullptr, *in = nullptr;
    void* tmp = nullptr;
    uint64_t c_jobs = 0, c_blen = 0, c_bcrc = 0, c_boff = 0, c_stage = 0, c_out = 0, c_tmp = 0, c_in = 0;
    uint64_t out_len = 0;
    uint64_t fallbacks = 0;  // blocks stored because their bit accounting did not add up (diagnostics)
    std::vector<DJob> hjobs;
    std::vector<uint32_t> hlen, hcrc;
    uint32_t shift64k[1024];
};

#define DF(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            z->err = std::string(#x) + ": " + hipGetErrorString(e_);           \
            return FR_ERR_HIP;                                                 \
        }                                                                      \
    } while (0)

template <class T>
static hipError_t grow(T** p, uint64_t& cap, uint64_t n) {
    if (n <= cap && *p) return hipSuccess;
    if (*p) {
        hipError_t e = hipFree(*p);
        if (e != hipSuccess) return e;
        *p = nullptr;
    }
    cap = std::max<uint64_t>(n + n / 4, 1024);
    return hipMalloc((void**)p, cap * sizeof(T));
}

fr_defl* fr_defl_create_on(int device, hipStream_t stream) {
    fr_defl* z = new fr_defl();
    z->device = device;
    auto fail = [&](const char* m) {
        z->err = m;
        return z;
    };
    if (hipSetDevice(device) != hipSuccess) return fail("fr_defl_create: no usable HIP device");
    if (stream) {
        z->stream = stream;
    } else {
        if (hipStreamCreateWithFlags(&z->stream, hipStreamNonBlocking) != hipSuccess)
            return fail("fr_defl_create: stream");
        z->own_stream = true;
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    z->grid = 2 * cus;
    std::vector<uint32_t> t1k(1024);
    crc_shift_table(SUB, t1k.data());
    crc_shift_table(BLOCK, z->shift64k);
    if (hipMalloc(&z->shift, 4096) != hipSuccess ||
        hipMemcpy(z->shift, t1k.data(), 4096, hipMemcpyHostToDevice) != hipSuccess ||
        hipMalloc(&z->scratch, (uint64_t)z->grid * SCR_BYTES) != hipSuccess)
        return fail("fr_defl_create: device allocation");
    return z;
}

extern "C" {

fr_defl* fr_defl_create(int device) { return fr_defl_create_on(device, nullptr); }

void fr_defl_destroy(fr_defl* z) {
    if (!z) return;
    (void)hipSetDevice(z->device);
    if (z->stream) (void)hipStreamSynchronize(z->stream);
    void* p[] = {z->jobs, z->blen, z->bcrc, z->shift, z->boff, z->stage, z->out, z->scratch, z->in, z->tmp};
    for (void* x : p)
        if (x) (void)hipFree(x);
    if (z->own_stream && z->stream) (void)hipStreamDestroy(z->stream);
    delete z;
}

const char* fr_defl_last_error(const fr_defl* z) { return z ? z->err.c_str() : "null context"; }

int fr_defl_run(fr_defl* z, const uint8_t* dev_data, const uint64_t* offsets, int n_streams, uint64_t* comp_bytes,
                uint32_t* crc32_out) {
    if (!z->scratch) return FR_ERR_HIP;
    if (n_streams < 0 || (n_streams && !offsets)) return z->err = "fr_defl_run: bad stream list", FR_ERR_INVALID;
    if (((uintptr_t)dev_data & 15u) != 0) return z->err = "fr_defl_run: data must be 16-byte aligned", FR_ERR_INVALID;
    DF(hipSetDevice(z->device));
    z->hjobs.clear();
    for (int s = 0; s < n_streams; ++s) {
        const uint64_t a = offsets[s], b = offsets[s + 1];
        if (b < a) return z->err = "fr_defl_run: offsets must not decrease", FR_ERR_INVALID;
        for (uint64_t x = a; x < b; x += BLOCK) {
            DJob j{};
            j.start = x;
            j.len = (uint32_t)std::min<uint64_t>(BLOCK, b - x);
            j.hist = (uint32_t)std::min<uint64_t>(HIST, x - a);
            j.last = x + BLOCK >= b;
            z->hjobs.push_back(j);
        }
    }
    const uint64_t nj = z->hjobs.size();
    if (nj >= 0xFFFFFFFFull) return z->err = "fr_defl_run: too many blocks", FR_ERR_CAPACITY;
    z->out_len = 0;
    if (nj) {
        DF(grow(&z->jobs, z->c_jobs, nj));
        DF(grow(&z->blen, z->c_blen, nj + 1));  // grow-only: a window's buffers serve the next ones
        DF(grow(&z->bcrc, z->c_bcrc, nj + 1));
        DF(grow(&z->boff, z->c_boff, nj + 1));
        DF(grow(&z->stage, z->c_stage, nj * OUT_STRIDE));
        DF(hipMemcpyAsync(z->jobs, z->hjobs.data(), nj * sizeof(DJob), hipMemcpyHostToDevice, z->stream));
        DF(hipMemsetAsync(z->bcrc + nj, 0, 4, z->stream));  // the kernel counts its stored fallbacks here
        const uint32_t g = (uint32_t)std::min<uint64_t>(nj, (uint64_t)z->grid);
        hipLaunchKernelGGL(deflate_blocks, dim3(g), dim3(TPB), 0, z->stream, dev_data, z->jobs, (uint32_t)nj, z->stage,
                           z->blen, z->bcrc, z->scratch, z->shift);
        DF(hipGetLastError());
#ifdef FRD_PROF
        {
            unsigned long long pr[12];
            DF(hipStreamSynchronize(z->stream));
            DF(hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_prof), sizeof pr));
            fprintf(stderr, "FRD_PROF wall ticks (100 MHz) summed over WGs: match %llu crc+cost %llu parse %llu count %llu huff %llu tables %llu emit %llu | match batches: to barrier 1 %llu, to barrier 2 %llu, rest %llu\n",
                    pr[0], pr[1], pr[2], pr[3], pr[4], pr[5], pr[6], pr[8], pr[9], pr[10]);
            unsigned long long zero[12] = {0};
            DF(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), zero, sizeof zero));
        }
#endif
        DF(hipMemsetAsync(z->blen + nj, 0, 4, z->stream));
        size_t tb = 0;
        DF(rocprim::exclusive_scan(nullptr, tb, z->blen, z->boff, (uint64_t)0, (size_t)nj + 1,
                                   rocprim::plus<uint64_t>(), z->stream));
        DF(grow((uint8_t**)&z->tmp, z->c_tmp, tb + 1));
        DF(rocprim::exclusive_scan(z->tmp, tb, z->blen, z->boff, (uint64_t)0, (size_t)nj + 1,
                                   rocprim::plus<uint64_t>(), z->stream));
        z->hlen.resize(nj);
        z->hcrc.resize(nj);
        DF(hipMemcpyAsync(z->hlen.data(), z->blen, nj * 4, hipMemcpyDeviceToHost, z->stream));
        z->hcrc.resize(nj + 1);
        DF(hipMemcpyAsync(z->hcrc.data(), z->bcrc, (nj + 1) * 4, hipMemcpyDeviceToHost, z->stream));
        DF(hipStreamSynchronize(z->stream));
        z->fallbacks += z->hcrc[nj];
        uint64_t total = 0;
        for (uint64_t k = 0; k < nj; ++k) {
            if (z->hlen[k] > OUT_STRIDE) return z->err = "fr_defl_run: a block's bit accounting failed", FR_ERR_DEVICE;
            total += z->hlen[k];
        }
        DF(grow(&z->out, z->c_out, total + 16));
        hipLaunchKernelGGL(deflate_compact, dim3((uint32_t)std::min<uint64_t>(nj, 4096)), dim3(256), 0, z->stream,
                           z->stage, z->blen, z->boff, (uint32_t)nj, z->out);
        DF(hipGetLastError());
        DF(hipStreamSynchronize(z->stream));
        z->out_len = total;
    }
    uint64_t k = 0;
    for (int s = 0; s < n_streams; ++s) {
        const uint64_t a = offsets[s], b = offsets[s + 1];
        uint64_t bytes = 0;
        uint32_t crc = 0;
        for (uint64_t x = a; x < b; x += BLOCK, ++k) {
            const uint64_t n = std::min<uint64_t>(BLOCK, b - x);
            crc = (n == BLOCK ? crc_apply(z->shift64k, crc) : (uint32_t)crc32_combine(crc, 0, (z_off_t)n)) ^ z->hcrc[k];
            bytes += z->hlen[k];
        }
        comp_bytes[s] = bytes;
        crc32_out[s] = crc;
    }
    return FR_OK;
}

int fr_defl_run_host(fr_defl* z, const uint8_t* data, uint64_t len, const uint64_t* offsets, int n_streams,
                     uint64_t* comp_bytes, uint32_t* crc32_out) {
    if (!z->scratch) return FR_ERR_HIP;
    DF(hipSetDevice(z->device));
    DF(grow(&z->in, z->c_in, len + 16));
    if (len) DF(hipMemcpyAsync(z->in, data, len, hipMemcpyHostToDevice, z->stream));
    DF(hipMemsetAsync(z->in + len, 0, 16, z->stream));
    return fr_defl_run(z, z->in, offsets, n_streams, comp_bytes, crc32_out);
}

uint64_t fr_defl_out_bytes(const fr_defl* z) { return z ? z->out_len : 0; }
uint64_t fr_defl_stored_fallbacks(const fr_defl* z) { return z ? z->fallbacks : 0; }

int fr_defl_fetch(fr_defl* z, uint8_t* out, uint64_t len) {
    if (len > z->out_len) return z->err = "fr_defl_fetch: more bytes than the last run produced", FR_ERR_INVALID;
    DF(hipSetDevice(z->device));
    if (len) DF(hipMemcpy(out, z->out, len, hipMemcpyDeviceToHost));
    return FR_OK;
}

}  // extern "C"
