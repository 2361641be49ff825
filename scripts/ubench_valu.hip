// ubench_valu.hip — wave64 VALU issue rate of the tally kernel's integer instruction mix on gfx950
// ("what bounds chunk_kernel").
//
// Each lane runs ITERS iterations of 8 independent dependency chains of one instruction kind
// (inline asm, so the instruction and its count are exact), at 1, 2, 4 and 8 waves per SIMD (one
// workgroup of 256 x W lanes per CU; W = 8 as two workgroups of 1024).  Each wave stamps
// s_memtime (shader clock) and s_memrealtime (100 MHz) around its loop.  Each configuration runs
// back to back for >= 2 s first (MI355X_MICROARCH.md, DVFS give-back item 6).  Reported per kind
// and waves/SIMD:
//   cyc/inst/wave  = the wave's loop cycles / its instructions (one wave's issue interval)
//   SIMD issue     = waves per SIMD / cyc/inst/wave  (wave64 instructions per SIMD per cycle)
//   clock          = median over waves of d(s_memtime) / d(s_memrealtime) x 100 MHz
//   overlap        = sum of the waves' loop durations (real time) / (span x 1024 SIMDs): the mean
//                    number of waves per SIMD actually running together
//   chip G inst/s  = every wave's instructions / kernel wall time (HIP events)
// The kinds are the tally loop's: v_and_b32, v_perm_b32 (the 8-entry classify lookups),
// v_dot4_u32_u8 (bitmap gathers), v_add_u32 with DPP row_shr (line-count scan), v_ffbl_b32 /
// v_ffbh_u32 (window bit search), v_lshrrev_b64 (64-bit windows), v_alignbit_b32, and "mix": the
// classify of one dword as the kernel issues it (3 AND-masks, 3 v_perm, 2 AND, 3 v_dot4).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_valu.hip -o scripts/ubench_valu
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <algorithm>
#include <vector>

typedef uint32_t u32;
typedef uint64_t u64;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

enum { K_AND, K_PERM, K_DOT4, K_DPP, K_FFBL, K_SHR64, K_ALIGN, K_MIX, K_BITOP3, K_OR3, K_LSHLOR, K_LSHR, K_CND, K_ADD,
       K_BCNT, K_MIN, K_MULLO, K_MUL24, K_ADD64, K_ALIGNB, K_N };
static const char* NAMES[K_N] = {"v_and_b32", "v_perm_b32", "v_dot4_u32_u8", "v_add_u32 dpp row_shr", "v_ffbl_b32",
                                  "v_lshrrev_b64", "v_alignbit_b32", "classify mix (11 VALU)", "v_bitop3_b32",
                                  "v_or3_b32", "v_lshl_or_b32", "v_lshrrev_b32", "v_cndmask_b32", "v_add_u32",
                                  "v_bcnt_u32_b32", "v_min_u32", "v_mul_lo_u32", "v_mul_u32_u24", "v_lshl_add_u64",
                                  "v_alignbyte_b32"};
static const int INSTS[K_N] = {1, 1, 1, 1, 1, 1, 1, 11, 1, 1, 1, 1, 2, 1, 1, 1, 1, 1, 1, 1};  // VALU instructions per chain step

template <int K>
__device__ __forceinline__ void step(u32 (&x)[8], u64 (&y)[8], u32 a, u32 b) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if constexpr (K == K_AND) {
            asm volatile("v_and_b32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
        } else if constexpr (K == K_PERM) {
            asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(x[i]) : "v"(a), "v"(b));
        } else if constexpr (K == K_DOT4) {
            asm volatile("v_dot4_u32_u8 %0, %0, %1, %0" : "+v"(x[i]) : "v"(a));
        } else if constexpr (K == K_DPP) {
            asm volatile("v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(x[i]));
        } else if constexpr (K == K_FFBL) {
            asm volatile("v_ffbl_b32 %0, %0" : "+v"(x[i]));
        } else if constexpr (K == K_SHR64) {
            asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(y[i]));
        } else if constexpr (K == K_ALIGN) {
            asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x[i]) : "v"(a));
        } else if constexpr (K == K_BITOP3) {
            asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[i]) : "v"(a), "v"(b));
        } else if constexpr (K == K_OR3) {
            asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
        } else if constexpr (K == K_LSHLOR) {
            asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(x[i]) : "v"(a));
        } else if constexpr (K == K_LSHR) {
            asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(x[i]));
        } else if constexpr (K == K_CND) {
            asm volatile("v_cmp_gt_u32 vcc, %1, %0\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[i]) : "v"(a) : "vcc");
        } else if constexpr (K == K_ADD) {
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
        } else if constexpr (K == K_BCNT) {
            asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
        } else if constexpr (K == K_MIN) {
            asm volatile("v_min_u32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
        } else if constexpr (K == K_MULLO) {
            asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
        } else if constexpr (K == K_MUL24) {
            asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[i]) : "v"(a));
        } else if constexpr (K == K_ADD64) {
            asm volatile("v_lshl_add_u64 %0, %0, 0, -1" : "+v"(y[i]));
        } else if constexpr (K == K_ALIGNB) {
            asm volatile("v_alignbyte_b32 %0, %0, %1, 3" : "+v"(x[i]) : "v"(a));
        } else {  // the classify of one dword: masks, three 8-entry lookups, two ANDs, three gathers
            u32 m0, m1, m2, l0, l1, l2;
            asm volatile(
                "v_and_b32 %0, 0x07070707, %6\n\t"
                "v_lshrrev_b32 %1, 3, %6\n\t"
                "v_and_b32 %1, 0x07070707, %1\n\t"
                "v_perm_b32 %3, %7, %8, %0\n\t"
                "v_perm_b32 %4, %8, %7, %1\n\t"
                "v_lshrrev_b32 %2, 6, %6\n\t"
                "v_perm_b32 %5, 0, %7, %2\n\t"
                "v_and_b32 %3, %3, %4\n\t"
                "v_and_b32 %3, %3, %5\n\t"
                "v_dot4_u32_u8 %6, %3, %7, %6\n\t"
                "v_dot4_u32_u8 %6, %3, %8, %6"
                : "=&v"(m0), "=&v"(m1), "=&v"(m2), "=&v"(l0), "=&v"(l1), "=&v"(l2), "+v"(x[i])
                : "v"(a), "v"(b));
        }
    }
}

template <int K>
__global__ void valu_kernel(u32* out, u64* cyc, int iters, u32 a, u32 b) {  // cyc: 4 u64 per wave
    u32 x[8];
    u64 y[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        x[i] = threadIdx.x * 7u + i;
        y[i] = ((u64)x[i] << 32) | x[i];
    }
    __syncthreads();
    const u64 r0 = __builtin_amdgcn_s_memrealtime();
    const u64 t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) step<K>(x, y, a, b);
    const u64 t1 = __builtin_amdgcn_s_memtime();
    const u64 r1 = __builtin_amdgcn_s_memrealtime();
    u32 acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= x[i] ^ (u32)y[i] ^ (u32)(y[i] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) {
        u64* c = cyc + 4 * ((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
        c[0] = t1 - t0;
        c[1] = r0;
        c[2] = r1;
        c[3] = 0;
    }
}

// Steady state (round 6): every wave spins until the common start time t0 (s_memrealtime, 100 MHz, read
// on the device by a one-lane kernel just before the launch, plus a lead for the dispatch), then runs
// blocks of 16 chain steps and checks the time after each, until t0 + window; only the instructions
// issued inside [t0, t0 + window) are counted, so launch ramps and tails are outside the measurement.
__global__ void now_kernel(u64* t) { t[0] = __builtin_amdgcn_s_memrealtime(); }

template <int K>
__global__ void valu_deadline_kernel(u32* out, u64* cnt, const u64* t0p, u64 lead, u64 window, u32 a, u32 b) {
    u32 x[8];
    u64 y[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        x[i] = threadIdx.x * 7u + i;
        y[i] = ((u64)x[i] << 32) | x[i];
    }
    const u64 t0 = t0p[0] + lead, t1 = t0 + window;
    while (__builtin_amdgcn_s_memrealtime() < t0) __builtin_amdgcn_s_sleep(1);
    const u64 c0 = __builtin_amdgcn_s_memtime();
    u64 blocks = 0;
    for (;;) {
#pragma unroll 1
        for (int it = 0; it < 16; ++it) step<K>(x, y, a, b);
        ++blocks;
        if (__builtin_amdgcn_s_memrealtime() >= t1) break;
    }
    const u64 c1 = __builtin_amdgcn_s_memtime();
    u32 acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= x[i] ^ (u32)y[i] ^ (u32)(y[i] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) {
        u64* c = cnt + 2 * ((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
        c[0] = blocks;
        c[1] = c1 - c0;
    }
}

template <int K>
static void run_steady(int wps, int ncu) {
    const int per_wg = wps >= 8 ? 1024 : 256 * wps;
    const int grid = wps >= 8 ? 2 * ncu : ncu;
    const int threads = grid * per_wg, waves = threads / 64;
    u32* out;
    u64 *cnt, *t0;
    CK(hipMalloc(&out, threads * 4));
    CK(hipMalloc(&cnt, waves * 16));
    CK(hipMalloc(&t0, 8));
    const u64 lead = 200000, window = 500000;  // 2 ms to dispatch every wave, then a 5-ms window
    for (int r = 0; r < 3; ++r) {  // the first runs warm the clock; the last is reported
        hipLaunchKernelGGL(now_kernel, dim3(1), dim3(1), 0, 0, t0);
        hipLaunchKernelGGL(valu_deadline_kernel<K>, dim3(grid), dim3(per_wg), 0, 0, out, cnt, t0, lead, window,
                           0x08040201u, 0x80402010u);
        CK(hipDeviceSynchronize());
    }
    std::vector<u64> c(2 * (size_t)waves);
    CK(hipMemcpy(c.data(), cnt, waves * 16, hipMemcpyDeviceToHost));
    double inst = 0, cyc = 0;
    for (int w = 0; w < waves; ++w) {
        inst += (double)c[2 * w] * 16 * 8 * INSTS[K];
        cyc += (double)c[2 * w + 1];
    }
    const double ghz = cyc / waves / (window * 10.0);  // shader cycles per ns of the window
    const double per_simd_cyc = inst / (4.0 * ncu) / (cyc / waves);
    printf("steady %-24s waves/SIMD %d  SIMD issue %5.3f inst/cyc  clock %.2f GHz  chip %7.1f G inst/s\n", NAMES[K], wps,
           per_simd_cyc, ghz, inst / (window * 1e-8) / 1e9);
    CK(hipFree(out));
    CK(hipFree(cnt));
    CK(hipFree(t0));
}

template <int K>
static void run(int wps, int ncu, int iters) {
    const int per_wg = wps >= 8 ? 1024 : 256 * wps;
    const int grid = wps >= 8 ? 2 * ncu : ncu;
    const int threads = grid * per_wg, waves = threads / 64;
    u32* out;
    u64* cyc;
    CK(hipMalloc(&out, threads * 4));
    CK(hipMalloc(&cyc, waves * 32));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    {  // >= 2 s of back-to-back launches first: the clock the chip holds under this load
        hipEvent_t w0, w1;
        CK(hipEventCreate(&w0));
        CK(hipEventCreate(&w1));
        float tot = 0;
        while (tot < 2000.f) {
            CK(hipEventRecord(w0));
            for (int r = 0; r < 20; ++r)
                hipLaunchKernelGGL(valu_kernel<K>, dim3(grid), dim3(per_wg), 0, 0, out, cyc, iters, 0x08040201u, 0x80402010u);
            CK(hipEventRecord(w1));
            CK(hipEventSynchronize(w1));
            float m = 0;
            CK(hipEventElapsedTime(&m, w0, w1));
            tot += m;
        }
    }
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(valu_kernel<K>, dim3(grid), dim3(per_wg), 0, 0, out, cyc, iters, 0x08040201u, 0x80402010u);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<u64> c(4 * (size_t)waves);
    CK(hipMemcpy(c.data(), cyc, waves * 32, hipMemcpyDeviceToHost));
    double mean = 0, busy = 0;
    u64 rmin = ~0ull, rmax = 0;
    std::vector<double> clk(waves);
    for (int w = 0; w < waves; ++w) {
        mean += (double)c[4 * w];
        const u64 r0 = c[4 * w + 1], r1 = c[4 * w + 2];
        rmin = std::min(rmin, r0);
        rmax = std::max(rmax, r1);
        busy += (double)(r1 - r0);
        clk[w] = r1 > r0 ? (double)c[4 * w] / (double)(r1 - r0) * 0.1 : 0.0;  // GHz
    }
    mean /= waves;
    std::sort(clk.begin(), clk.end());
    const double ghz = clk[waves / 2];
    const double overlap = busy / ((double)(rmax - rmin) * 4.0 * ncu);
    const double inst_wave = (double)iters * 8 * INSTS[K];
    const double cpi = mean / inst_wave;
    const double chip = inst_wave * waves / (ms * 1e-3) / 1e9;
    printf("%-24s waves/SIMD %d  cyc/inst/wave %6.2f  SIMD issue %5.3f inst/cyc  clock %.2f GHz  overlap %.2f  "
           "chip %7.1f G inst/s  (%.3f ms; span %.3f ms)\n",
           NAMES[K], wps, cpi, wps / cpi, ghz, overlap, chip, ms, (rmax - rmin) * 1e-5);
    CK(hipFree(out));
    CK(hipFree(cyc));
}

template <int K>
static void sweep(int ncu, int iters) {
    for (int w : {1, 2, 4, 8}) run<K>(w, ncu, iters);
    for (int w : {1, 2, 4, 8}) run_steady<K>(w, ncu);
}

template <int K>
static void quick(int ncu) { run_steady<K>(8, ncu); }

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    if (argc > 2 && argv[2][0] == 'q') {  // steady state at 8 waves/SIMD only, every kind
        hipDeviceProp_t p;
        CK(hipGetDeviceProperties(&p, 0));
        const int ncu = p.multiProcessorCount;
        quick<K_AND>(ncu); quick<K_PERM>(ncu); quick<K_DOT4>(ncu); quick<K_DPP>(ncu); quick<K_FFBL>(ncu);
        quick<K_SHR64>(ncu); quick<K_ALIGN>(ncu); quick<K_MIX>(ncu); quick<K_BITOP3>(ncu); quick<K_OR3>(ncu);
        quick<K_LSHLOR>(ncu); quick<K_LSHR>(ncu); quick<K_CND>(ncu); quick<K_ADD>(ncu); quick<K_BCNT>(ncu);
        quick<K_MIN>(ncu); quick<K_MULLO>(ncu); quick<K_MUL24>(ncu); quick<K_ADD64>(ncu); quick<K_ALIGNB>(ncu);
        return 0;
    }
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    printf("%s: %d CUs, clock %d kHz; s_memtime counts shader cycles\n", p.gcnArchName, p.multiProcessorCount,
           p.clockRate);
    const int ncu = p.multiProcessorCount;
    sweep<K_AND>(ncu, iters);
    sweep<K_PERM>(ncu, iters);
    sweep<K_DOT4>(ncu, iters);
    sweep<K_DPP>(ncu, iters);
    sweep<K_FFBL>(ncu, iters);
    sweep<K_SHR64>(ncu, iters);
    sweep<K_ALIGN>(ncu, iters);
    sweep<K_MIX>(ncu, iters / 4);
    return 0;
}
