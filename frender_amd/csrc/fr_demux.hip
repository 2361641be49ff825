// fr_demux.hip — SURVEY.md §8.1 row (f-1): `demux` (frender.py:733-814) on the GPU.
//
// The reference's hot loop walks R1/R2 record pairs in lockstep, takes the code after the last
// ':' of the R2 header line (frender.py:778), looks it up in the scan results and appends both
// records to the writer pair of the result's read type / sample (frender.py:779-810).  Here one
// pair of decoded files is resident in HBM and:
//   dmx_count  newline count per 16-KiB tile (HBM-bound streaming read)
//   scan       exclusive prefix of the tile counts (rocprim)
//   dmx_index  record starts (every 4th line start) and, for R2, the code -> destination lookup
//              in an open-addressing table of the results' fast codes
//   route      stable partition of the record pairs by destination (rocprim radix sort on the
//              destination, record index as payload), output offsets (rocprim scans) and a
//              gather-copy of both mates' record bytes into destination-major buffers
// The host inflates, normalises universal newlines (frender.py:776 reads in text mode), resolves
// the rare codes outside the fast alphabet, raises the reference's errors, and gzips each
// destination's bytes into its writer pair.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include <rocprim/rocprim.hpp>

#include "../../include/frender_amd.h"
#include "fr_internal.h"

namespace fr {
namespace {

constexpr int DT = 16384;        // tile bytes
constexpr int DWG = 256;         // lanes per workgroup: 64 B each
constexpr int DSEG = DT / DWG;
constexpr int DHALO = 1024;      // bytes staged past the tile for headers that cross it
constexpr int DMAXSYM = MAXSYM;  // fast key: <= 21 symbols

__device__ __forceinline__ u32 nl_mask4(u32 w) {  // exact '\n' bytes -> bits 0..3
    const u32 t = w ^ 0x0A0A0A0Au;
    const u32 z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
    return __builtin_amdgcn_udot4(z >> 7, 0x08040201u, 0u, false);
}

__device__ __forceinline__ u32 sym_byte(u32 c) {  // A1 C2 G3 T4 N5 +6, else 0
    switch (c) {
        case 'A': return 1;
        case 'C': return 2;
        case 'G': return 3;
        case 'T': return 4;
        case 'N': return 5;
        case '+': return 6;
        default: return 0;
    }
}

struct DmxTable {
    const u64* keys;  // 0 = empty
    const int32_t* vals;
    u64 mask;
};

__device__ __forceinline__ int32_t table_get(const DmxTable& t, u64 key) {
    if (!t.keys) return FR_DMX_MISSING;
    u64 h = mix64(key) & t.mask;
    for (;;) {
        const u64 k = t.keys[h];
        if (k == key) return t.vals[h];
        if (k == 0) return FR_DMX_MISSING;
        h = (h + 1) & t.mask;
    }
}

__global__ void dmx_table_insert(u64* keys, int32_t* vals, u64 mask, const u64* in_k, const int32_t* in_v, u64 n) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 key = in_k[i];
        u64 h = mix64(key) & mask;
        for (;;) {
            const u64 old = atomicCAS((unsigned long long*)&keys[h], 0ull, (unsigned long long)key);
            if (old == 0 || old == key) {
                vals[h] = in_v[i];
                break;
            }
            h = (h + 1) & mask;
        }
    }
}

// 64 bytes of lane `tid` of tile t (zeros past len) -> '\n' bitmap
__device__ __forceinline__ u64 lane_nl(const u8* buf, u64 len, u64 tile0, int tid) {
    const u64 base = tile0 + (u64)tid * DSEG;
    u64 m = 0;
    if (base + DSEG <= len) {
#pragma unroll
        for (int q = 0; q < DSEG / 16; ++q) {
            const uint4 v = *(const uint4*)(buf + base + q * 16);
            m |= (u64)(nl_mask4(v.x) | (nl_mask4(v.y) << 4) | (nl_mask4(v.z) << 8) | (nl_mask4(v.w) << 12)) << (16 * q);
        }
    } else if (base < len) {
        for (u64 j = 0; base + j < len; ++j) m |= (u64)(buf[base + j] == '\n') << j;
    }
    return m;
}

__global__ __launch_bounds__(DWG) void dmx_count(const u8* buf, u64 len, u32 ntiles, u32* tile_cnt) {
    __shared__ u32 ws[DWG / 64];
    for (u32 t = blockIdx.x; t < ntiles; t += gridDim.x) {
        u32 c = __popcll(lane_nl(buf, len, (u64)t * DT, threadIdx.x));
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
        if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
        __syncthreads();
        if (threadIdx.x == 0) tile_cnt[t] = ws[0] + ws[1] + ws[2] + ws[3];
        __syncthreads();
    }
}

__device__ __forceinline__ u32 eq_mask4(u32 w, u32 rep) {  // exact byte equality -> bits 0..3
    const u32 t = w ^ rep;
    const u32 z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
    return __builtin_amdgcn_udot4(z >> 7, 0x08040201u, 0u, false);
}

// fast key of the code bytes [s, s+n) in LDS: v_perm lookups 4 bytes per step (A1 C2 G3 T4 N5 +6);
// false when a byte is outside the fast alphabet
__device__ __forceinline__ bool encode_fast(const u8* lds, u32 s, u32 n, u64& key) {
    u64 kk = 0;
    u32 bad = 0;
    for (u32 k = 0; 4 * k < n; ++k) {
        const u32 p = s + 4 * k;
        const u32 lo = *(const u32*)(lds + (p & ~3u)), hi = *(const u32*)(lds + (p & ~3u) + 4);
        const u32 a = __builtin_amdgcn_alignbyte(hi, lo, p & 3u);
        const u32 idx = (a >> 1) & 0x07070707u;
        const u32 expect = __builtin_amdgcn_perm(0x4E002B00u, 0x47544341u, idx);
        const u32 sym = __builtin_amdgcn_perm(0x05000600u, 0x03040201u, idx);
        const u32 left = n - 4 * k;
        const u32 vm = left >= 4 ? 0xFFFFFFFFu : (0xFFFFFFFFu >> (32 - 8 * left));
        bad |= (expect ^ a) & vm;
        const u32 sv = sym & vm;
        kk |= (u64)((sv & 0x7u) | ((sv >> 5) & 0x38u) | ((sv >> 10) & 0x1C0u) | ((sv >> 15) & 0xE00u)) << (12 * k);
    }
    key = kk;
    return bad == 0;
}

// slow path: the header line runs past the staged bytes -> byte loop over global memory
__device__ __noinline__ int32_t header_dest_global(const u8* buf, u64 len, u64 p, const DmxTable& tab) {
    u64 e = p, lastc = ~0ull;
    while (e < len && buf[e] != '\n') {
        if (buf[e] == ':') lastc = e;
        ++e;
    }
    const u64 s = lastc == ~0ull ? p : lastc + 1;
    const u64 n = e - s;
    if (n == 0 || n > (u64)DMAXSYM) return FR_DMX_EXOTIC;
    u64 key = 0;
    for (u64 i = 0; i < n; ++i) {
        const u32 sy = sym_byte(buf[s + i]);
        if (!sy) return FR_DMX_EXOTIC;
        key |= (u64)sy << (3 * i);
    }
    return table_get(tab, key);
}

// the code of the header line starting at tile position q: the text after the line's last ':'
// up to its '\n' (frender.py:778) -> destination.  Word-at-a-time over the staged tile (LDS,
// zero-padded past lds_n); '\n' and ':' found with exact SWAR byte masks.
__device__ __forceinline__ int32_t header_dest(const u8* buf, u64 len, u64 tile0, u32 q, const u8* lds, u32 lds_n,
                                               const DmxTable& tab) {
    int lastc = -1, e = -1;
    u32 w = q & ~3u;
    u32 keep = (0xFu << (q & 3u)) & 0xFu;
    for (; w < lds_n; w += 4) {
        const u32 v = *(const u32*)(lds + w);
        u32 nl = eq_mask4(v, 0x0A0A0A0Au) & keep, col = eq_mask4(v, 0x3A3A3A3Au) & keep;
        keep = 0xFu;
        if (w + 4 > lds_n) {
            const u32 vm = (1u << (lds_n - w)) - 1u;
            nl &= vm;
            col &= vm;
        }
        if (nl) {
            const u32 b = __builtin_ctz(nl);
            col &= (1u << b) - 1u;
            if (col) lastc = (int)(w + 31u - __builtin_clz(col));
            e = (int)(w + b);
            break;
        }
        if (col) lastc = (int)(w + 31u - __builtin_clz(col));
    }
    if (e < 0) {
        if (tile0 + lds_n < len) return header_dest_global(buf, len, tile0 + q, tab);
        e = (int)lds_n;  // the line ends with the data
    }
    const u32 s = lastc >= 0 ? (u32)lastc + 1u : q;
    const u32 n = (u32)e - s;
    if (n == 0 || n > (u32)DMAXSYM) return FR_DMX_EXOTIC;
    u64 key;
    if (!encode_fast(lds, s, n, key)) return FR_DMX_EXOTIC;
    return table_get(tab, key);
}

__global__ __launch_bounds__(DWG) void dmx_index(const u8* buf, u64 len, u32 ntiles, const u64* tile_base,
                                                 u64* rec_start, int32_t* rec_dest, DmxTable tab) {
    __shared__ __attribute__((aligned(16))) u8 lds[DT + DHALO + 32];  // +32: zero pad for word reads
    __shared__ u32 ws[DWG / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (u32 t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const u64 tile0 = (u64)t * DT;
        const u32 lds_n = (u32)min((u64)(DT + DHALO), len - tile0);
        if (rec_dest) {
            for (u32 i = tid * 16; i < lds_n + 32; i += DWG * 16) {
                uint4 v = make_uint4(0u, 0u, 0u, 0u);
                if (i + 16 <= lds_n) {
                    v = *(const uint4*)(buf + tile0 + i);
                } else if (i < lds_n) {
                    u32 b[4] = {0u, 0u, 0u, 0u};
                    for (u32 j = i; j < lds_n; ++j) b[(j - i) >> 2] |= (u32)buf[tile0 + j] << (8 * ((j - i) & 3));
                    v = make_uint4(b[0], b[1], b[2], b[3]);
                }
                if (i < DT + DHALO + 32) *(uint4*)(lds + i) = v;
            }
        }
        const u64 m = lane_nl(buf, len, tile0, tid);
        const u32 c = __popcll(m);
        u32 x = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const u32 y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        if (lane == 63) ws[wid] = x;
        __syncthreads();
        u64 L = tile_base[t] + (x - c);
        for (int w = 0; w < wid; ++w) L += ws[w];
        // line start after each '\n' of this lane's segment: line index L + rank + 1
        u64 mm = m;
        while (mm) {
            const u32 j = __builtin_ctzll(mm);
            mm &= mm - 1;
            L += 1;
            const u64 p = tile0 + (u64)tid * DSEG + j + 1;
            if ((L & 3ull) == 0 && p < len) {
                rec_start[L >> 2] = p;
                if (rec_dest) rec_dest[L >> 2] = header_dest(buf, len, tile0, (u32)(p - tile0), lds, lds_n, tab);
            }
        }
        if (t == 0 && tid == 0 && len > 0) {  // the first line of the file
            rec_start[0] = 0;
            if (rec_dest) rec_dest[0] = header_dest(buf, len, tile0, 0u, lds, lds_n, tab);
        }
        __syncthreads();
    }
}

__global__ void dmx_first_error(const int32_t* dest, u64 n, unsigned long long* first) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x)
        if (dest[i] < 0) atomicMin(first, (unsigned long long)i);
}

__global__ void dmx_keys(const int32_t* dest, u64 n, u32* keys, u32* idx) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        keys[i] = (u32)dest[i];
        idx[i] = (u32)i;
    }
}

// lengths of both mates' records in partition order
__global__ void dmx_lengths(const u32* perm, u64 n, const u64* rs1, const u64* rs2, u64* len1, u64* len2) {
    for (u64 j = blockIdx.x * (u64)blockDim.x + threadIdx.x; j < n; j += (u64)gridDim.x * blockDim.x) {
        const u32 i = perm[j];
        len1[j] = rs1[i + 1] - rs1[i];
        len2[j] = rs2[i + 1] - rs2[i];
    }
}

// first partition position of every destination present (sorted keys: one boundary each, no atomics)
__global__ void dmx_bounds(const u32* sk, u64 n, u32* first) {
    for (u64 j = blockIdx.x * (u64)blockDim.x + threadIdx.x; j < n; j += (u64)gridDim.x * blockDim.x)
        if (j == 0 || sk[j] != sk[j - 1]) first[sk[j]] = (u32)j;
}

// byte offset of every destination's first record (n_dest entries, + the total at [n_dest])
__global__ void dmx_dest_offsets(const u32* first, int n_dest, u64 n, const u64* o1, const u64* l1, const u64* o2,
                                 const u64* l2, u64* off1, u64* off2) {
    const int d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d > n_dest) return;
    const u64 tot1 = o1[n - 1] + l1[n - 1], tot2 = o2[n - 1] + l2[n - 1];
    // an absent destination starts where the next present one does
    int e = d;
    while (e < n_dest && first[e] == 0xFFFFFFFFu) ++e;
    off1[d] = e < n_dest ? o1[first[e]] : tot1;
    off2[d] = e < n_dest ? o2[first[e]] : tot2;
}

// one wave per output record: a byte head up to the destination's 4-byte alignment, then
// aligned dword stores, each assembled from the two source dwords it straddles
// (v_alignbyte_b32), then a byte tail.  Source reads may run up to 3 bytes past the record
// inside the same aligned dword (allocations are 256-B granular).
__global__ void dmx_copy(const u32* perm, u64 n, const u64* rs, const u8* src, const u64* off, u8* dst) {
    const int lane = threadIdx.x & 63;
    const u64 waves = (u64)gridDim.x * (blockDim.x / 64);
    for (u64 j = blockIdx.x * (u64)(blockDim.x / 64) + (threadIdx.x >> 6); j < n; j += waves) {
        const u32 i = perm[j];
        const u64 s = rs[i], len = rs[i + 1] - s, o = off[j];
        const u64 head = min((u64)((4u - (u32)(o & 3u)) & 3u), len);
        if ((u64)lane < head) dst[o + lane] = src[s + lane];
        const u64 s1 = s + head, o1 = o + head, words = (len - head) >> 2;
        const u32 sh = (u32)(s1 & 3u);
        const u32* sw = (const u32*)(src + (s1 & ~3ull));
        u32* dw = (u32*)(dst + o1);
        for (u64 k = lane; k < words; k += 64) {
            const u32 lo = sw[k];
            const u32 hi = sh ? sw[k + 1] : 0u;
            dw[k] = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
        }
        const u64 t0 = head + (words << 2);
        if (t0 + lane < len) dst[o + t0 + lane] = src[s + t0 + lane];
    }
}

int grid_for(u64 n, int per = 256, int cap = 8192) {
    return (int)std::max<u64>(1, std::min<u64>((n + per - 1) / per, (u64)cap));
}

}  // namespace
}  // namespace fr

using namespace fr;

fr_defl* fr_defl_create_on(int device, hipStream_t stream);

struct fr_dmx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // results table
    u64* tkeys = nullptr;
    int32_t* tvals = nullptr;
    u64 tmask = 0;
    // per mate: data, record starts (+ sentinel), destinations (R2)
    u8* data[2] = {nullptr, nullptr};
    u64 cap[2] = {0, 0};
    const u8* src[2] = {nullptr, nullptr};  // the bytes indexed: data[m] or a caller's device buffer
    u64 len[2] = {0, 0};
    u64* rs[2] = {nullptr, nullptr};
    u64 rs_cap[2] = {0, 0};
    u64 nrec[2] = {0, 0};
    int32_t* dest = nullptr;
    u64 dest_cap = 0;
    // route temporaries (grow-only) and outputs
    u32 *k_in = nullptr, *k_out = nullptr, *i_in = nullptr, *perm = nullptr, *first_pos = nullptr;
    u64 *l1 = nullptr, *l2 = nullptr, *o1 = nullptr, *o2 = nullptr, *off1 = nullptr, *off2 = nullptr;
    u64 c_k_in = 0, c_k_out = 0, c_i_in = 0, c_perm = 0, c_first = 0, c_l1 = 0, c_l2 = 0, c_o1 = 0, c_o2 = 0,
        c_off1 = 0, c_off2 = 0;
    void* tmp = nullptr;
    u64 c_tmp = 0;
    u32* cnt = nullptr;
    u64* base = nullptr;
    u64 c_cnt = 0, c_base = 0;
    unsigned long long* fe = nullptr;
    u64 c_fe = 0;
    u8* out[2] = {nullptr, nullptr};
    u64 out_cap[2] = {0, 0};
    u64 out_len[2] = {0, 0};
    std::vector<u64> hoff[2];  // destination offsets of the routed bytes (host copy)
    fr_defl* defl[2] = {nullptr, nullptr};  // the writers' compression (fr_deflate.hip), created on first use
};

#define DK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            d->err = std::string(#x) + ": " + hipGetErrorString(e_);           \
            return FR_ERR_HIP;                                                 \
        }                                                                      \
    } while (0)

template <class T>
static hipError_t ensure(T** p, u64& cap, u64 n) {
    if (n <= cap && *p) return hipSuccess;
    if (*p) {
        hipError_t e = hipFree(*p);
        if (e != hipSuccess) return e;
        *p = nullptr;
    }
    cap = std::max<u64>(n + n / 4, 1024);
    return hipMalloc((void**)p, cap * sizeof(T));
}

extern "C" {

fr_dmx* fr_dmx_create(int device) {
    fr_dmx* d = new fr_dmx();
    d->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess)
        d->err = "fr_dmx_create: no usable HIP device";
    return d;
}

void fr_dmx_destroy(fr_dmx* d) {
    if (!d) return;
    (void)hipSetDevice(d->device);
    if (d->stream) (void)hipStreamSynchronize(d->stream);
    void* p[] = {d->tkeys, d->tvals, d->data[0], d->data[1], d->rs[0], d->rs[1], d->dest, d->out[0], d->out[1],
                 d->k_in, d->k_out, d->i_in, d->perm, d->first_pos, d->l1, d->l2, d->o1, d->o2, d->off1, d->off2,
                 d->tmp, d->cnt, d->base, d->fe};
    for (void* x : p)
        if (x) (void)hipFree(x);
    for (fr_defl* z : d->defl) fr_defl_destroy(z);
    if (d->stream) (void)hipStreamDestroy(d->stream);
    delete d;
}

const char* fr_dmx_last_error(const fr_dmx* d) { return d ? d->err.c_str() : "null context"; }

int fr_dmx_set_table(fr_dmx* d, const uint64_t* keys, const int32_t* vals, uint64_t n) {
    DK(hipSetDevice(d->device));
    if (d->tkeys) DK(hipFree(d->tkeys));
    if (d->tvals) DK(hipFree(d->tvals));
    d->tkeys = nullptr;
    d->tvals = nullptr;
    u64 slots = 1024;
    while (slots < 2 * n) slots <<= 1;
    d->tmask = slots - 1;
    DK(hipMalloc(&d->tkeys, slots * 8));
    DK(hipMalloc(&d->tvals, slots * 4));
    DK(hipMemsetAsync(d->tkeys, 0, slots * 8, d->stream));
    if (n) {
        u64* k = nullptr;
        int32_t* v = nullptr;
        DK(hipMalloc(&k, n * 8));
        DK(hipMalloc(&v, n * 4));
        DK(hipMemcpyAsync(k, keys, n * 8, hipMemcpyHostToDevice, d->stream));
        DK(hipMemcpyAsync(v, vals, n * 4, hipMemcpyHostToDevice, d->stream));
        hipLaunchKernelGGL(dmx_table_insert, dim3(grid_for(n)), dim3(256), 0, d->stream, d->tkeys, d->tvals, d->tmask,
                           k, v, n);
        DK(hipGetLastError());
        DK(hipStreamSynchronize(d->stream));
        DK(hipFree(k));
        DK(hipFree(v));
    }
    return FR_OK;
}

static int dmx_index_mate(fr_dmx* d, int mate, const u8* buf, u64 len, u64* n_records) {
    d->src[mate] = buf;
    d->len[mate] = len;
    const u32 ntiles = (u32)((len + DT - 1) / DT);
    DK(ensure(&d->cnt, d->c_cnt, (u64)ntiles + 1));
    DK(ensure(&d->base, d->c_base, (u64)ntiles + 1));
    u64 nl = 0;
    if (ntiles) {
        hipLaunchKernelGGL(dmx_count, dim3(std::min<u32>(ntiles, 8192)), dim3(DWG), 0, d->stream, buf, len, ntiles,
                           d->cnt);
        DK(hipGetLastError());
        size_t tb = 0;
        DK(rocprim::exclusive_scan(nullptr, tb, d->cnt, d->base, (u64)0, (size_t)ntiles + 1, rocprim::plus<u64>(),
                                   d->stream));
        DK(ensure((u8**)&d->tmp, d->c_tmp, tb + 1));
        DK(hipMemsetAsync(d->cnt + ntiles, 0, 4, d->stream));
        DK(rocprim::exclusive_scan(d->tmp, tb, d->cnt, d->base, (u64)0, (size_t)ntiles + 1, rocprim::plus<u64>(),
                                   d->stream));
        DK(hipMemcpyAsync(&nl, d->base + ntiles, 8, hipMemcpyDeviceToHost, d->stream));  // total '\n'
    }
    u8 lastb = '\n';
    if (len) DK(hipMemcpyAsync(&lastb, buf + len - 1, 1, hipMemcpyDeviceToHost, d->stream));
    DK(hipStreamSynchronize(d->stream));
    const u64 lines = nl + ((len && lastb != '\n') ? 1 : 0);  // a last line without '\n'
    const u64 nrec = (lines + 3) / 4;
    DK(ensure(&d->rs[mate], d->rs_cap[mate], nrec + 1));
    if (mate == 1) DK(ensure(&d->dest, d->dest_cap, nrec + 1));
    d->nrec[mate] = nrec;
    *n_records = nrec;
    DK(hipMemcpyAsync(d->rs[mate] + nrec, &d->len[mate], 8, hipMemcpyHostToDevice, d->stream));  // sentinel
    if (ntiles) {
        DmxTable tab{d->tkeys, d->tvals, d->tmask};
        hipLaunchKernelGGL(dmx_index, dim3(std::min<u32>(ntiles, 4096)), dim3(DWG), 0, d->stream, buf, len, ntiles,
                           d->base, d->rs[mate], mate == 1 ? d->dest : nullptr, tab);
        DK(hipGetLastError());
    }
    DK(hipStreamSynchronize(d->stream));
    return FR_OK;
}

int fr_dmx_load(fr_dmx* d, int mate, const uint8_t* data, uint64_t len, uint64_t* n_records) {
    if (mate < 0 || mate > 1) return d->err = "mate must be 0 (R1) or 1 (R2)", FR_ERR_INVALID;
    DK(hipSetDevice(d->device));
    DK(ensure(&d->data[mate], d->cap[mate], len + 16));
    if (len) DK(hipMemcpyAsync(d->data[mate], data, len, hipMemcpyHostToDevice, d->stream));
    return dmx_index_mate(d, mate, d->data[mate], len, n_records);
}

int fr_dmx_load_parts(fr_dmx* d, int mate, const uint8_t* const* parts, const uint64_t* lens, int n_parts,
                      uint64_t* n_records) {
    if (mate < 0 || mate > 1 || n_parts < 0) return d->err = "mate must be 0 (R1) or 1 (R2)", FR_ERR_INVALID;
    DK(hipSetDevice(d->device));
    u64 len = 0;
    for (int k = 0; k < n_parts; ++k) len += lens[k];
    DK(ensure(&d->data[mate], d->cap[mate], len + 16));
    u64 off = 0;
    for (int k = 0; k < n_parts; ++k) {
        if (lens[k]) DK(hipMemcpyAsync(d->data[mate] + off, parts[k], lens[k], hipMemcpyHostToDevice, d->stream));
        off += lens[k];
    }
    return dmx_index_mate(d, mate, d->data[mate], len, n_records);
}

int fr_dmx_load_device(fr_dmx* d, int mate, const uint8_t* dev_data, uint64_t len, uint64_t* n_records) {
    if (mate < 0 || mate > 1) return d->err = "mate must be 0 (R1) or 1 (R2)", FR_ERR_INVALID;
    if (((uintptr_t)dev_data & 15u) != 0) return d->err = "device data must be 16-byte aligned", FR_ERR_INVALID;
    DK(hipSetDevice(d->device));
    return dmx_index_mate(d, mate, dev_data, len, n_records);
}

int fr_dmx_records(fr_dmx* d, int mate, const uint64_t* recs, uint64_t n, uint64_t* starts, uint64_t* ends) {
    DK(hipSetDevice(d->device));
    std::vector<u64> all;
    for (u64 k = 0; k < n; ++k) {
        if (recs[k] >= d->nrec[mate]) return d->err = "record index out of range", FR_ERR_INVALID;
        u64 se[2];
        DK(hipMemcpy(se, d->rs[mate] + recs[k], 16, hipMemcpyDeviceToHost));
        starts[k] = se[0];
        ends[k] = se[1];
    }
    return FR_OK;
}

int fr_dmx_exotic(fr_dmx* d, uint64_t n_pairs, uint64_t* recs, uint64_t cap, uint64_t* n) {
    DK(hipSetDevice(d->device));
    n_pairs = std::min<u64>(n_pairs, d->nrec[1]);
    std::vector<int32_t> h(n_pairs);
    if (n_pairs) DK(hipMemcpy(h.data(), d->dest, n_pairs * 4, hipMemcpyDeviceToHost));
    u64 k = 0;
    for (u64 i = 0; i < n_pairs; ++i)
        if (h[i] == FR_DMX_EXOTIC) {
            if (k < cap) recs[k] = i;
            ++k;
        }
    *n = k;
    return FR_OK;
}

int fr_dmx_patch(fr_dmx* d, const uint64_t* recs, const int32_t* dest, uint64_t n) {
    DK(hipSetDevice(d->device));
    for (u64 k = 0; k < n; ++k) {
        if (recs[k] >= d->nrec[1]) return d->err = "record index out of range", FR_ERR_INVALID;
        DK(hipMemcpyAsync(d->dest + recs[k], dest + k, 4, hipMemcpyHostToDevice, d->stream));
    }
    DK(hipStreamSynchronize(d->stream));
    return FR_OK;
}

int fr_dmx_route(fr_dmx* d, int n_dest, uint64_t n_pairs, int64_t* first_error, int32_t* error_val,
                 uint64_t* bytes_r1, uint64_t* bytes_r2) {
    DK(hipSetDevice(d->device));
    const u64 P = std::min<u64>({n_pairs, d->nrec[0], d->nrec[1]});
    if (P >= 0xFFFFFFFFull) return d->err = "too many records in one file pair", FR_ERR_CAPACITY;
    *first_error = -1;
    *error_val = 0;
    for (int k = 0; k < n_dest; ++k) bytes_r1[k] = bytes_r2[k] = 0;
    d->out_len[0] = d->out_len[1] = 0;
    d->hoff[0].assign((size_t)std::max(n_dest, 0) + 1, 0);
    d->hoff[1].assign((size_t)std::max(n_dest, 0) + 1, 0);
    if (!P) return FR_OK;
    DK(ensure(&d->fe, d->c_fe, 1));
    unsigned long long* fe = d->fe;
    DK(hipMemsetAsync(fe, 0xFF, 8, d->stream));
    hipLaunchKernelGGL(dmx_first_error, dim3(grid_for(P)), dim3(256), 0, d->stream, d->dest, P, fe);
    DK(hipGetLastError());
    u64 first = 0;
    DK(hipMemcpyAsync(&first, fe, 8, hipMemcpyDeviceToHost, d->stream));
    DK(hipStreamSynchronize(d->stream));
    if (first != ~0ull) {
        int32_t v = 0;
        DK(hipMemcpy(&v, d->dest + first, 4, hipMemcpyDeviceToHost));
        *first_error = (int64_t)first;
        *error_val = v;
        return FR_OK;
    }
    // stable partition by destination (temporaries cached in the context, grow-only)
    DK(ensure(&d->k_in, d->c_k_in, P));
    DK(ensure(&d->k_out, d->c_k_out, P));
    DK(ensure(&d->i_in, d->c_i_in, P));
    DK(ensure(&d->perm, d->c_perm, P));
    DK(ensure(&d->l1, d->c_l1, P));
    DK(ensure(&d->l2, d->c_l2, P));
    DK(ensure(&d->o1, d->c_o1, P));
    DK(ensure(&d->o2, d->c_o2, P));
    DK(ensure(&d->first_pos, d->c_first, (u64)std::max(n_dest, 1)));
    DK(ensure(&d->off1, d->c_off1, (u64)n_dest + 1));
    DK(ensure(&d->off2, d->c_off2, (u64)n_dest + 1));
    u32 *k_in = d->k_in, *k_out = d->k_out, *i_in = d->i_in, *perm = d->perm, *first_pos = d->first_pos;
    u64 *l1 = d->l1, *l2 = d->l2, *o1 = d->o1, *o2 = d->o2, *off1 = d->off1, *off2 = d->off2;
    DK(hipMemsetAsync(first_pos, 0xFF, (u64)std::max(n_dest, 1) * 4, d->stream));
    hipLaunchKernelGGL(dmx_keys, dim3(grid_for(P)), dim3(256), 0, d->stream, d->dest, P, k_in, i_in);
    DK(hipGetLastError());
    int bits = 1;
    while ((1 << bits) < n_dest) ++bits;
    size_t tb = 0;
    DK(rocprim::radix_sort_pairs(nullptr, tb, k_in, k_out, i_in, perm, (size_t)P, 0, (unsigned)bits, d->stream));
    size_t tb2 = 0;
    DK(rocprim::exclusive_scan(nullptr, tb2, l1, o1, (u64)0, (size_t)P, rocprim::plus<u64>(), d->stream));
    DK(ensure((u8**)&d->tmp, d->c_tmp, std::max<size_t>(std::max(tb, tb2), 1)));
    void* tmp = d->tmp;
    DK(rocprim::radix_sort_pairs(tmp, tb, k_in, k_out, i_in, perm, (size_t)P, 0, (unsigned)bits, d->stream));
    hipLaunchKernelGGL(dmx_lengths, dim3(grid_for(P)), dim3(256), 0, d->stream, perm, P, d->rs[0], d->rs[1], l1, l2);
    DK(hipGetLastError());
    hipLaunchKernelGGL(dmx_bounds, dim3(grid_for(P)), dim3(256), 0, d->stream, k_out, P, first_pos);
    DK(hipGetLastError());
    DK(rocprim::exclusive_scan(tmp, tb2, l1, o1, (u64)0, (size_t)P, rocprim::plus<u64>(), d->stream));
    DK(rocprim::exclusive_scan(tmp, tb2, l2, o2, (u64)0, (size_t)P, rocprim::plus<u64>(), d->stream));
    hipLaunchKernelGGL(dmx_dest_offsets, dim3((n_dest + 256) / 256), dim3(256), 0, d->stream, first_pos, n_dest, P,
                       o1, l1, o2, l2, off1, off2);
    DK(hipGetLastError());
    std::vector<u64> h1(n_dest + 1), h2(n_dest + 1);
    DK(hipMemcpyAsync(h1.data(), off1, (n_dest + 1) * 8, hipMemcpyDeviceToHost, d->stream));
    DK(hipMemcpyAsync(h2.data(), off2, (n_dest + 1) * 8, hipMemcpyDeviceToHost, d->stream));
    DK(hipStreamSynchronize(d->stream));
    for (int k = 0; k < n_dest; ++k) {
        bytes_r1[k] = h1[k + 1] - h1[k];
        bytes_r2[k] = h2[k + 1] - h2[k];
    }
    const u64 s1 = h1[n_dest], s2 = h2[n_dest];
    DK(ensure(&d->out[0], d->out_cap[0], s1 + 16));
    DK(ensure(&d->out[1], d->out_cap[1], s2 + 16));
    const int cg = grid_for(P, 4, 16384);
    hipLaunchKernelGGL(dmx_copy, dim3(cg), dim3(256), 0, d->stream, perm, P, d->rs[0], d->src[0], o1, d->out[0]);
    DK(hipGetLastError());
    hipLaunchKernelGGL(dmx_copy, dim3(cg), dim3(256), 0, d->stream, perm, P, d->rs[1], d->src[1], o2, d->out[1]);
    DK(hipGetLastError());
    DK(hipStreamSynchronize(d->stream));
    d->out_len[0] = s1;
    d->out_len[1] = s2;
    d->hoff[0] = h1;
    d->hoff[1] = h2;
    return FR_OK;
}

int fr_dmx_deflate(fr_dmx* d, int mate, int n_dest, uint64_t* comp_bytes, uint32_t* crc32) {
    if (mate < 0 || mate > 1) return d->err = "mate must be 0 (R1) or 1 (R2)", FR_ERR_INVALID;
    if (n_dest < 0 || (u64)n_dest + 1 != d->hoff[mate].size())
        return d->err = "fr_dmx_deflate: n_dest differs from the last fr_dmx_route", FR_ERR_INVALID;
    DK(hipSetDevice(d->device));
    if (!d->defl[mate]) {
        d->defl[mate] = fr_defl_create_on(d->device, d->stream);
        const char* e = fr_defl_last_error(d->defl[mate]);
        if (e && *e) return d->err = std::string("fr_dmx_deflate: ") + e, FR_ERR_HIP;
    }
    const int rc = fr_defl_run(d->defl[mate], d->out[mate], d->hoff[mate].data(), n_dest, comp_bytes, crc32);
    if (rc != FR_OK) d->err = std::string("fr_dmx_deflate: ") + fr_defl_last_error(d->defl[mate]);
    return rc;
}

int fr_dmx_fetch_deflated(fr_dmx* d, int mate, uint8_t* out, uint64_t len) {
    if (mate < 0 || mate > 1 || !d->defl[mate]) return d->err = "fr_dmx_fetch_deflated: bad mate or no fr_dmx_deflate", FR_ERR_INVALID;
    const int rc = fr_defl_fetch(d->defl[mate], out, len);
    if (rc != FR_OK) d->err = std::string("fr_dmx_fetch_deflated: ") + fr_defl_last_error(d->defl[mate]);
    return rc;
}

int fr_dmx_fetch(fr_dmx* d, int mate, uint8_t* out, uint64_t len) {
    if (mate < 0 || mate > 1 || len > d->out_len[mate]) return d->err = "fr_dmx_fetch: bad mate or length", FR_ERR_INVALID;
    DK(hipSetDevice(d->device));
    if (len) DK(hipMemcpy(out, d->out[mate], len, hipMemcpyDeviceToHost));
    return FR_OK;
}

}  // extern "C"
