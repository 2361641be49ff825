// ubench_table.hip — calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE for the tally's table accesses
// (DESIGN.md §4.1 traffic; MI355X_MICROARCH.md §HBM: "other access widths are uncalibrated: calibrate
// on a known byte count in your own access pattern").
//
// Each kernel is its own dispatch (rocprofv3 reports per dispatch), with a known count of operations:
//   stream   : every lane reads 16 B per load, coalesced (the tile loads' pattern; the guide: reported ½)
//   probe    : random 32-B GSlot probes as resolve_batch issues them (an 8-B and a 16-B load of one slot)
//   atomic   : random 64-bit atomicAdd on a slot's count (apply_entry's fire-and-forget add)
//   atomic3  : the add plus atomicMin(first) and atomicMax(last_tag) on the same slot (a new code)
//   flush    : a 1-GiB streaming read between the table kernels, so table lines start outside the
//              256-MiB Infinity Cache as they do under the tally's 3.7-GB stream
// Table: 4 Mi slots x 32 B (128 MiB, the bench's), random slot per op from a counter hash.
// Run:  rocprofv3 --pmc FETCH_SIZE -- ./ubench_table   then   --pmc WRITE_SIZE  (separate passes)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_table.hip -o scripts/ubench_table
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef uint32_t u32;
typedef uint64_t u64;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct alignas(32) GSlot {
    u64 key, count, first;
    u32 last_tag, uidx;
};

__device__ __forceinline__ u64 mix64(u64 x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

__global__ void stream_kernel(const uint4* __restrict__ p, u64 n16, u32* out) {
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n16; i += (u64)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;  // keeps the loads
}

__global__ void probe_kernel(const GSlot* __restrict__ t, u64 mask, u64 nops, u64 seed, u32* out) {
    u32 acc = 0;
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < nops; i += (u64)gridDim.x * blockDim.x) {
        const GSlot* s = &t[mix64(i ^ seed) & mask];
        const uint2 w0 = *(const uint2*)s;
        const uint4 w1 = *((const uint4*)s + 1);
        acc ^= w0.x ^ w0.y ^ w1.x ^ w1.z;
    }
    if (acc == 0x12345678u) out[0] = 1;
}

__global__ void atomic_kernel(GSlot* t, u64 mask, u64 nops, u64 seed, int three) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < nops; i += (u64)gridDim.x * blockDim.x) {
        GSlot* s = &t[mix64(i ^ seed) & mask];
        atomicAdd((unsigned long long*)&s->count, 1ull);
        if (three) {
            atomicMin((unsigned long long*)&s->first, (unsigned long long)i);
            atomicMax(&s->last_tag, (u32)i);
        }
    }
}

int main(int argc, char** argv) {
    const u64 nops = argc > 1 ? strtoull(argv[1], nullptr, 10) : (16ull << 20);
    const u64 slots = 4ull << 20, mask = slots - 1;
    const u64 flush_bytes = 1ull << 30, stream_bytes = 1ull << 30;
    GSlot* t;
    uint4* big;
    u32* out;
    CK(hipMalloc(&t, slots * sizeof(GSlot)));
    CK(hipMalloc(&big, flush_bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(t, 0, slots * sizeof(GSlot)));
    CK(hipMemset(big, 1, flush_bytes));
    const int grid = 256 * 16, blk = 256;
    auto flush = [&]() {
        hipLaunchKernelGGL(stream_kernel, dim3(grid), dim3(blk), 0, 0, big, flush_bytes / 16, out);
    };
    printf("ops per table dispatch %llu, table %llu MiB, stream %llu MiB\n", (unsigned long long)nops,
           (unsigned long long)(slots * sizeof(GSlot) >> 20), (unsigned long long)(stream_bytes >> 20));
    printf("dispatch order: stream(calibration), flush, probe, flush, atomic, flush, atomic3\n");
    hipLaunchKernelGGL(stream_kernel, dim3(grid), dim3(blk), 0, 0, big, stream_bytes / 16, out);
    flush();
    hipLaunchKernelGGL(probe_kernel, dim3(grid), dim3(blk), 0, 0, t, mask, nops, 1ull, out);
    flush();
    hipLaunchKernelGGL(atomic_kernel, dim3(grid), dim3(blk), 0, 0, t, mask, nops, 2ull, 0);
    flush();
    hipLaunchKernelGGL(atomic_kernel, dim3(grid), dim3(blk), 0, 0, t, mask, nops, 3ull, 1);
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
