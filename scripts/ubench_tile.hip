// ubench_tile.hip — tile-loop structure microbenchmark for the tally kernel.
//
// Streams ~3.9 GB of 74-B FASTQ-shaped records through five loop structures with the tally
// kernel's classify (3 bitmaps + DPP line scan) and an emulated header parse (bitmap windows,
// code-byte reads from the LDS copy, LDS table atomics), to decide how the tile loop should load:
//   A  per workgroup, lane-strided 64-B segments in registers, 1 tile ahead, 2 barriers / tile (round 2)
//   B  per workgroup, coalesced LDS-DMA ring of D 16-KiB tiles, 2 barriers / tile
//   C  per wave (no barriers), coalesced register loads 1 wave-tile ahead, LDS transpose
//   D  per wave (no barriers), lane-strided register loads 1 wave-tile ahead
//   E  per wave (no barriers), coalesced LDS-DMA ring of D 4-KiB wave-tiles
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_tile.hip -o scripts/ubench_tile
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <vector>

typedef uint32_t u32;
typedef uint64_t u64;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int WG = 256, TILE = 16384, SEG = 64, WTILE = 4096;

__device__ __forceinline__ u32 classify4(u32 w) {
    const u32 lo3 = __builtin_amdgcn_perm(0x10101310u, 0x10191014u, w & 0x07070707u);
    const u32 mid3 = __builtin_amdgcn_perm(0x18101014u, 0x10101310u, (w >> 3) & 0x07070707u);
    const u32 top2 = __builtin_amdgcn_perm(0u, 0x1010000Fu, (w >> 6) & 0x03030303u);
    return lo3 & mid3 & top2;
}
template <int K>
__device__ __forceinline__ u32 gather16(u32 c0, u32 c1, u32 c2, u32 c3) {
    constexpr u32 M = 0x01010101u << K;
    u32 v = __builtin_amdgcn_udot4(c0 & M, 0x08040201u, 0u, false);
    v = __builtin_amdgcn_udot4(c1 & M, 0x80402010u, v, false);
    u32 u = __builtin_amdgcn_udot4(c2 & M, 0x08040201u, 0u, false);
    u = __builtin_amdgcn_udot4(c3 & M, 0x80402010u, u, false);
    return (v | (u << 8)) >> K;
}
struct Bits { u64 eol, sp, col; u32 c, x; };

__device__ __forceinline__ Bits classify_seg(const uint4 (&r)[4]) {
    u32 e[4], s[4], c[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const u32 c0 = classify4(r[q].x), c1 = classify4(r[q].y), c2 = classify4(r[q].z), c3 = classify4(r[q].w);
        e[q] = gather16<0>(c0, c1, c2, c3);
        s[q] = gather16<2>(c0, c1, c2, c3);
        c[q] = gather16<3>(c0, c1, c2, c3);
    }
    Bits b;
    b.eol = ((u64)(e[2] | (e[3] << 16)) << 32) | (e[0] | (e[1] << 16));
    b.sp = ((u64)(s[2] | (s[3] << 16)) << 32) | (s[0] | (s[1] << 16));
    b.col = ((u64)(c[2] | (c[3] << 16)) << 32) | (c[0] | (c[1] << 16));
    b.c = __popcll(b.eol);
    u32 x = b.c;
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xA, 0xF, false);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xC, 0xF, false);
    b.x = x;
    return b;
}

typedef __attribute__((address_space(3))) u32 lu32;
typedef __attribute__((address_space(3))) u64 lu64;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lu32x4;

__device__ __forceinline__ u32 lds_addr(const void* p) {
    return (u32)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ u64 window64(u64 x0, u64 x1, u32 b) { return (x0 >> b) | ((x1 << 1) << (63u - b)); }

// emulated header parse for the header ending this lane's segment's first line end: two bitmap
// windows, 8 code dwords from the raw copy, a v_perm encode, one LDS-table count
__device__ __forceinline__ u32 parse_emul(const lu64* bsp, const lu64* bcol, const lu32* raw, int nseg, u32 s0,
                                          u64 eol, lu32* ls, int lns_mask, int reps) {
    u32 acc = 0;
    if (!eol) return 0;
    u32 p = s0 + (u32)__builtin_ctzll(eol) + 1u;
    for (int r = 0; r < reps; ++r) {
        const u32 w = (p >> 6) % (u32)nseg, b = p & 63u;
        const u32 w1 = (w + 1) % (u32)nseg;
        const u64 se = window64(bsp[w], bsp[w1], b);
        const u32 f1 = se ? (u32)__builtin_ctzll(se) : 64u;
        const u32 q = p + f1 + 1u;
        const u32 w2 = (q >> 6) % (u32)nseg, b2 = q & 63u, w3 = (w2 + 1) % (u32)nseg;
        const u64 se2 = window64(bsp[w2], bsp[w3], b2);
        const u64 co2 = window64(bcol[w2], bcol[w3], b2);
        const u32 f2 = se2 ? (u32)__builtin_ctzll(se2) : 63u;
        const u64 cm = co2 & ((1ull << f2) - 1ull);
        const u32 cs = cm ? 64u - __builtin_clzll(cm) : 0u;
        const u32 start = (q + cs) % (u32)(nseg * 64 - 32);
        const lu32* pw = raw + (start >> 2);
        u32 wv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) wv[k] = pw[k];
        u32 bad = 0, lo = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32 x = __builtin_amdgcn_alignbyte(wv[k + 1], wv[k], start & 3u);
            const u32 idx = (x >> 1) & 0x07070707u;
            const u32 expect = __builtin_amdgcn_perm(0x4E002B00u, 0x47544341u, idx);
            const u32 sym = __builtin_amdgcn_perm(0x05000600u, 0x03040201u, idx);
            bad |= expect ^ x;
            lo ^= __builtin_amdgcn_udot4(sym, 0x00400801u, (sym >> 15) & 0xE00u, false) << (3 * k);
        }
        const u32 h = ((lo ^ bad) * 0x9E3779B1u) >> 22;
        atomicAdd((u32*)&ls[4 * (h & (u32)lns_mask) + 2], 1u);
        acc += lo + f2;
        p += 1;
    }
    return acc;
}

// ---------------------------------------------------------------------------------------------
// A: per workgroup, lane-strided registers, 1 ahead, 2 barriers
template <int LNS>
__global__ __launch_bounds__(WG) void kA(const uint8_t* __restrict__ buf, u64 ntiles, u32* sink, int reps) {
    __shared__ u32 raw[TILE / 4];
    __shared__ u32 ls[(1 << LNS) * 4];
    __shared__ u64 bsp[WG + 1], bcol[WG + 1];
    __shared__ u32 wsum[4];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (int i = tid; i < (1 << LNS) * 4; i += WG) ls[i] = 0;
    const u64 t0 = blockIdx.x * ntiles / gridDim.x, t1 = (blockIdx.x + 1) * ntiles / gridDim.x;
    uint4 r[4];
    auto load = [&](u64 t) {
        const uint4* p = (const uint4*)(buf + t * TILE + tid * SEG);
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = p[k];
    };
    u32 acc = 0;
    if (t0 < t1) load(t0);
    __syncthreads();
    for (u64 t = t0; t < t1; ++t) {
        const Bits b = classify_seg(r);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        bsp[tid] = b.sp | b.eol;
        bcol[tid] = b.col;
        if (lane == 63) wsum[wid] = b.x;
        lu32x4* dst = (lu32x4*)(lu32*)raw + tid * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) dst[k] = u32x4{r[k].x, r[k].y, r[k].z, r[k].w};
        if (t + 1 < t1) load(t + 1);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        acc += wsum[0] + b.x;
        acc += parse_emul((lu64*)bsp, (lu64*)bcol, (lu32*)raw, WG, tid * SEG, b.eol, (lu32*)ls, (1 << LNS) - 1, reps);
    }
    atomicAdd(sink, acc);
}

// B: per workgroup, LDS-DMA ring of D tiles (coalesced 1 KiB per wave-instruction), 2 barriers
__device__ __forceinline__ void glds16(const void* gsrc, u32 lds_dst) {
    u32 keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
template <int N> __device__ __forceinline__ void vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int D, int LNS>
__global__ __launch_bounds__(WG) void kB(const uint8_t* __restrict__ buf, u64 ntiles, u32* sink, int reps) {
    __shared__ __attribute__((aligned(16))) u32 ring[D][TILE / 4];
    __shared__ u32 ls[(1 << LNS) * 4];
    __shared__ u64 bsp[WG + 1], bcol[WG + 1];
    __shared__ u32 wsum[4];
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < (1 << LNS) * 4; i += WG) ls[i] = 0;
    const u64 t0 = blockIdx.x * ntiles / gridDim.x, t1 = (blockIdx.x + 1) * ntiles / gridDim.x;
    // wave wid loads the tile's 1-KiB pieces wid*4 .. wid*4+3
    auto dma = [&](u64 t) {
        const u64 tt = t < t1 ? t : t0;  // past the end: reload (keeps the wait counts uniform)
        const int slot = (int)(t % D);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int piece = wid * 4 + k;
            glds16(buf + tt * TILE + piece * 1024 + lane * 16,
                   __builtin_amdgcn_readfirstlane(lds_addr(&ring[slot][piece * 256])));
        }
    };
    u32 acc = 0;
    for (int d = 0; d < D - 1; ++d) dma(t0 + d);
    __syncthreads();
    for (u64 t = t0; t < t1; ++t) {
        vmwait<4 * (D - 2)>();  // this wave's pieces of tile t landed
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();  // B1: every piece of t landed; parse(t-1) done
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        dma(t + D - 1);
        const int slot = (int)(t % D);
        const lu32x4* src = (const lu32x4*)(lu32*)&ring[slot][0] + tid * 4;
        uint4 r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32x4 v = src[(k + (tid >> 2)) & 3];  // rotated quads: fewer bank conflicts
            r[(k + (tid >> 2)) & 3] = make_uint4(v.x, v.y, v.z, v.w);
        }
        const Bits b = classify_seg(r);
        bsp[tid] = b.sp | b.eol;
        bcol[tid] = b.col;
        if (lane == 63) wsum[wid] = b.x;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();  // B2
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        acc += wsum[0] + b.x;
        acc += parse_emul((lu64*)bsp, (lu64*)bcol, (lu32*)&ring[slot][0], WG, tid * SEG, b.eol, (lu32*)ls,
                          (1 << LNS) - 1, reps);
    }
    vmwait<0>();
    atomicAdd(sink, acc);
}

// C / D: per wave, register loads 1 wave-tile ahead, no barriers.  COAL: lane-linear 1 KiB pieces
// (then the lane reads its segment from the LDS copy); else each lane loads its own 64 B.
template <bool COAL, int LNS>
__global__ __launch_bounds__(WG) void kCD(const uint8_t* __restrict__ buf, u64 ntiles, u32* sink, int reps) {
    __shared__ __attribute__((aligned(16))) u32 raw[4][WTILE / 4];
    __shared__ u32 ls[(1 << LNS) * 4];
    __shared__ u64 bsp[4][65], bcol[4][65];
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < (1 << LNS) * 4; i += WG) ls[i] = 0;
    __syncthreads();
    const u64 nw = ntiles * (TILE / WTILE);  // wave-tiles
    const u64 g = (u64)blockIdx.x * 4 + wid, G = (u64)gridDim.x * 4;
    const u64 t0 = g * nw / G, t1 = (g + 1) * nw / G;
    uint4 r[4];
    auto load = [&](u64 t) {
        const u64 tt = t < t1 ? t : t0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4* p = COAL ? (const uint4*)(buf + tt * WTILE + k * 1024 + lane * 16)
                                  : (const uint4*)(buf + tt * WTILE + lane * SEG + k * 16);
            r[k] = *p;
        }
    };
    u32 acc = 0;
    load(t0);
    lu32* myraw = (lu32*)&raw[wid][0];
    for (u64 t = t0; t < t1; ++t) {
        uint4 s[4];
        if (COAL) {
            lu32x4* dst = (lu32x4*)myraw;
#pragma unroll
            for (int k = 0; k < 4; ++k) dst[k * 64 + lane] = u32x4{r[k].x, r[k].y, r[k].z, r[k].w};
            load(t + 1);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            const lu32x4* src = (const lu32x4*)myraw + lane * 4;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const u32x4 v = src[(k + (lane >> 2)) & 3];
                s[(k + (lane >> 2)) & 3] = make_uint4(v.x, v.y, v.z, v.w);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) s[k] = r[k];
            lu32x4* dst = (lu32x4*)myraw + lane * 4;
#pragma unroll
            for (int k = 0; k < 4; ++k) dst[k] = u32x4{r[k].x, r[k].y, r[k].z, r[k].w};
            load(t + 1);
        }
        const Bits b = classify_seg(s);
        bsp[wid][lane] = b.sp | b.eol;
        bcol[wid][lane] = b.col;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        acc += __builtin_amdgcn_readlane(b.x, 63);
        acc += parse_emul((lu64*)&bsp[wid][0], (lu64*)&bcol[wid][0], myraw, 64, lane * SEG, b.eol, (lu32*)ls,
                          (1 << LNS) - 1, reps);
    }
    atomicAdd(sink, acc);
}

// E: per wave, LDS-DMA ring of D wave-tiles, no barriers
template <int D, int LNS>
__global__ __launch_bounds__(WG) void kE(const uint8_t* __restrict__ buf, u64 ntiles, u32* sink, int reps) {
    __shared__ __attribute__((aligned(16))) u32 ring[4][D][WTILE / 4];
    __shared__ u32 ls[(1 << LNS) * 4];
    __shared__ u64 bsp[4][65], bcol[4][65];
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < (1 << LNS) * 4; i += WG) ls[i] = 0;
    __syncthreads();
    const u64 nw = ntiles * (TILE / WTILE);
    const u64 g = (u64)blockIdx.x * 4 + wid, G = (u64)gridDim.x * 4;
    const u64 t0 = g * nw / G, t1 = (g + 1) * nw / G;
    auto dma = [&](u64 t) {
        const u64 tt = t < t1 ? t : t0;
        const int slot = (int)(t % D);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            glds16(buf + tt * WTILE + k * 1024 + lane * 16,
                   __builtin_amdgcn_readfirstlane(lds_addr(&ring[wid][slot][k * 256])));
    };
    u32 acc = 0;
    for (int d = 0; d < D - 1; ++d) dma(t0 + d);
    for (u64 t = t0; t < t1; ++t) {
        vmwait<4 * (D - 2)>();
        dma(t + D - 1);  // into the slot parsed last step (this wave is done with it)
        const int slot = (int)(t % D);
        lu32* myraw = (lu32*)&ring[wid][slot][0];
        const lu32x4* src = (const lu32x4*)myraw + lane * 4;
        uint4 s[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32x4 v = src[(k + (lane >> 2)) & 3];
            s[(k + (lane >> 2)) & 3] = make_uint4(v.x, v.y, v.z, v.w);
        }
        const Bits b = classify_seg(s);
        bsp[wid][lane] = b.sp | b.eol;
        bcol[wid][lane] = b.col;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        acc += __builtin_amdgcn_readlane(b.x, 63);
        acc += parse_emul((lu64*)&bsp[wid][0], (lu64*)&bcol[wid][0], myraw, 64, lane * SEG, b.eol, (lu32*)ls,
                          (1 << LNS) - 1, reps);
    }
    vmwait<0>();
    atomicAdd(sink, acc);
}

// plain streaming read (copy-rate reference): 8 x 16 B in flight per lane
__global__ __launch_bounds__(256) void kStream(const uint4* __restrict__ p, u64 n16, u32* sink) {
    u32 acc = 0;
    const u64 stride = (u64)gridDim.x * 256;
    for (u64 i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += 8 * stride) {
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = i + k * stride < n16 ? p[i + k * stride] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= v[k].x + v[k].y + v[k].z + v[k].w;
    }
    atomicAdd(sink, acc);
}

__global__ void kFill(uint8_t* buf, u64 n) {
    const char* rec = "@SYN:1:FCX:1:1101:12345:67890 1:N:0:ACGTACGT+TTGGCCAA\nACGTACGT\n+\nFFFFFFFF\n";  // 74 B
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) buf[i] = rec[i % 74];
}

template <typename K, typename... Args>
static void run(const char* name, K kern, int occ_hint, u64 bytes, u32* sink, Args... args) {
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, WG, 0));
    if (occ_hint > 0 && occ_hint < occ) occ = occ_hint;
    const int grid = 256 * occ;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(WG), 0, 0, args...);
    CK(hipDeviceSynchronize());
    const int reps = 5;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(WG), 0, 0, args...);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    u32 s = 0;
    CK(hipMemcpy(&s, sink, 4, hipMemcpyDeviceToHost));
    printf("%-34s occ=%d grid=%5d  %8.3f ms  %6.3f TB/s  (sink %08x)\n", name, occ, grid, ms, bytes / (ms * 1e-3) / 1e12, s);
    fflush(stdout);
    CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
    const u64 ntiles = 240000;  // 3.93 GB
    const u64 bytes = ntiles * TILE;
    uint8_t* buf;
    u32* sink;
    CK(hipMalloc(&buf, bytes + 65536));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(sink, 0, 4));
    hipLaunchKernelGGL(kFill, dim3(8192), dim3(256), 0, 0, buf, bytes + 65536);
    CK(hipDeviceSynchronize());
    const char* only = argc > 1 ? argv[1] : "";
    run("stream 8x16B", kStream, 0, bytes, sink, (const uint4*)buf, bytes / 16, sink);
    for (int reps : {0, 1, 2}) {
        printf("--- parse reps %d\n", reps);
        char nm[64];
        snprintf(nm, 64, "A strided regs, WG, LNS10");  run(nm, kA<10>, 4, bytes, sink, buf, ntiles, sink, reps);
        snprintf(nm, 64, "B dma D2 WG, LNS10");  run(nm, kB<2, 10>, 4, bytes, sink, buf, ntiles, sink, reps);
        snprintf(nm, 64, "B dma D3 WG, LNS10");  run(nm, kB<3, 10>, 4, bytes, sink, buf, ntiles, sink, reps);
        snprintf(nm, 64, "B dma D2 WG, LNS9");  run(nm, kB<2, 9>, 4, bytes, sink, buf, ntiles, sink, reps);
        snprintf(nm, 64, "C wave coal regs, LNS10");  run(nm, kCD<true, 10>, 4, bytes, sink, buf, ntiles, sink, reps);
        snprintf(nm, 64, "D wave strided regs, LNS10");  run(nm, kCD<false, 10>, 4, bytes, sink, buf, ntiles, sink, reps);
        snprintf(nm, 64, "E wave dma D2, LNS10");  run(nm, kE<2, 10>, 4, bytes, sink, buf, ntiles, sink, reps);
        snprintf(nm, 64, "E wave dma D3, LNS10");  run(nm, kE<3, 10>, 4, bytes, sink, buf, ntiles, sink, reps);
        snprintf(nm, 64, "E wave dma D2, LNS9");  run(nm, kE<2, 9>, 4, bytes, sink, buf, ntiles, sink, reps);
        snprintf(nm, 64, "E wave dma D3, LNS8");  run(nm, kE<3, 8>, 4, bytes, sink, buf, ntiles, sink, reps);
    }
    (void)only;
    CK(hipFree(buf));
    return 0;
}
