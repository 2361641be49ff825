// ubench_l2atomic.hip — where do the tally's commit atomics execute, and what do they cost?
// (DESIGN.md §4.1, round 6).  MI355X_MICROARCH.md §"Global float atomics": device-scope atomics leave
// L2 as uncached 64-B requests and execute at the memory side.  This measures 64-bit integer atomicAdd
// (no return) on random 32-B-strided slots at three scopes/placements:
//   agent/shared : __hip_atomic_fetch_add(..., AGENT) on one table shared by the whole chip (the tally today)
//   wg/xcd       : WORKGROUP scope on a table private to the XCD the workgroup runs on (HW_REG_XCC_ID):
//                  if the XCD's L2 executes these, every workgroup of the XCD sees one coherent table
//   wg/shared    : WORKGROUP scope on the shared table (speed only: not coherent across XCDs)
// and a probe+add pattern (agent-relaxed = sc1 load of the slot, then the add) per XCD.
// Correctness of wg/xcd: each XCD's table sum must equal the adds its workgroups issued.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_l2atomic.hip -o scripts/ubench_l2atomic
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32;
typedef uint64_t u64;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ u64 mix64(u64 x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

__device__ __forceinline__ u32 xcc_id() {
    u32 x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 0xFu;
}

// mode 0 agent/shared, 1 wg/xcd, 2 wg/shared, 3 probe(sc1 load)+wg add per xcd, 4 agent/xcd
__global__ void atomic_kernel(u64* t, u32 slots_log2, u32 iters, u64 seed, int mode, u64* adds) {
    const u32 x = xcc_id();
    const u64 mask = (1ull << slots_log2) - 1ull;
    u64* base = (mode == 1 || mode == 3 || mode == 4) ? t + ((u64)x << slots_log2) * 4 : t;
    const u64 g = blockIdx.x * (u64)blockDim.x + threadIdx.x;
    u64 acc = 0;
    for (u32 i = 0; i < iters; ++i) {
        u64* p = base + (mix64(g * 0x9E3779B97F4A7C15ull + i + seed) & mask) * 4;  // 32-B slots
        if (mode == 0 || mode == 4) {
            __hip_atomic_fetch_add(p, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (mode == 3) {
            const u64 v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            acc += v;
            __hip_atomic_fetch_add(p, 1ull + (v >> 62), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            __hip_atomic_fetch_add(p, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    if (acc == 0x123456789ull) t[1] = 7;
    if (threadIdx.x == 0) atomicAdd((unsigned long long*)&adds[x], (unsigned long long)blockDim.x * iters);
}

int main(int argc, char** argv) {
    const int grid = argc > 1 ? atoi(argv[1]) : 1024;
    const u32 iters = argc > 2 ? (u32)atoi(argv[2]) : 256;
    const u32 max_log2 = 18;
    const size_t bytes = (size_t)8 * (32ull << max_log2);  // 8 XCDs x 2^18 x 32 B
    u64* t;
    u64* adds;
    CK(hipMalloc(&t, bytes));
    CK(hipMalloc(&adds, 8 * sizeof(u64)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[] = {"agent/shared", "wg/xcd", "wg/shared", "probe+wg/xcd", "agent/xcd"};
    std::vector<u64> h(bytes / 8);
    for (u32 lg : {12u, 14u, 16u, 18u}) {
        for (int mode = 0; mode < 5; ++mode) {
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                CK(hipMemset(t, 0, bytes));
                CK(hipMemset(adds, 0, 8 * sizeof(u64)));
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(atomic_kernel, dim3(grid), dim3(256), 0, 0, t, lg, iters, 77ull + rep, mode, adds);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            // correctness of the last rep: per-XCD sums (xcd modes) or the total
            CK(hipMemcpy(h.data(), t, bytes, hipMemcpyDeviceToHost));
            u64 ha[8];
            CK(hipMemcpy(ha, adds, sizeof(ha), hipMemcpyDeviceToHost));
            bool ok = true;
            u64 tot = 0, want = 0;
            for (int x = 0; x < 8; ++x) want += ha[x];
            if (mode == 1 || mode == 3 || mode == 4) {
                for (int x = 0; x < 8; ++x) {
                    u64 s = 0;
                    for (u64 i = 0; i < (1ull << lg); ++i) s += h[((u64)x << lg) * 4 + i * 4];
                    tot += s;
                    if (s != ha[x]) ok = false;
                }
            } else {
                for (u64 i = 0; i < (1ull << lg); ++i) tot += h[i * 4];
                ok = tot == want;
            }
            const double n = (double)grid * 256 * iters;
            printf("slots/table 2^%u (%6.2f MiB)  %-14s %8.3f ms  %7.2f G atomics/s  sum %s (%llu of %llu)\n", lg,
                   (32.0 * (1ull << lg)) / (1 << 20), names[mode], best, n / best / 1e6, ok ? "ok" : "WRONG",
                   (unsigned long long)tot, (unsigned long long)want);
        }
    }
    return 0;
}
