// fr_kernels.hip — gfx950 kernels for frender's scan hot path.
//
//  tally (chunk_kernel) : frender.py:154-181 scan_file + :199-205 merge, one pass over the
//                         decoded FASTQ bytes in HBM (R1-R4 of SURVEY.md §8.0)
//  classify             : frender.py:214-234 (Hamming), :237-291 (classes), :294-351 (rc)
//  table / order        : the first-occurrence-ordered merged table of :199-203
//  synth                : SYN-v1 records (frender_amd/synth.py), device side
//
// Design notes: the tally is HBM-bound byte work.  A workgroup takes a chunk of
// 4-KiB wave-tiles by ticket and each of its four waves walks a quarter of it without workgroup
// barriers: lanes classify their 64-B segments in registers (line-end / ' ' / ':' bitmaps by v_perm
// lookups and dot4 gathers), find every 4th line from the wave's line count, parse each header
// lane-owned from the bitmaps and the wave's LDS copy of the tile, pack the code 3 bits/char and
// count it in an LDS open-addressing table shared by the workgroup; each chunk's table is
// committed to the HBM table (or to the launch log) once.  Line phases are guessed per wave and
// verified per chunk and per launch (decoupled look-back over 8-B {tag, value} granules).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "fr_internal.h"

namespace fr {

#if defined(FR_STAMPS) && FR_STAMPS == 1  // diagnostic builds only: per-wave shader cycles of the chunk loop's phases (DevState::stamp)
#define FR_STAMP_DECL u64 st_[8] = {0, 0, 0, 0, 0, 0, 0, 0}; u64 tq_ = __builtin_amdgcn_s_memtime();
#define FR_STAMP(i) do { const u64 n_ = __builtin_amdgcn_s_memtime(); st_[i] += n_ - tq_; tq_ = n_; } while (0)
#define FR_STAMP_FLUSH(k0) do { st_[6] = __builtin_amdgcn_s_memtime() - (k0); \
    if ((threadIdx.x & 63) == 0) for (int i_ = 0; i_ < 8; ++i_) atomicAdd((unsigned long long*)&a.st->stamp[i_], \
        (unsigned long long)st_[i_]); } while (0)
#else
#define FR_STAMP_DECL
#define FR_STAMP(i) do { } while (0)
#define FR_STAMP_FLUSH(k0) do { } while (0)
#endif

#if defined(FR_STAMPS) && FR_STAMPS == 2  // diagnostic builds only: the commit's phases instead
#define FR_CSTAMP(i) do { const u64 n_ = __builtin_amdgcn_s_memtime(); cst_[i] += n_ - cq_; cq_ = n_; } while (0)
#else
#define FR_CSTAMP(i) do { } while (0)
#endif

#if defined(FR_STAMPS) && FR_STAMPS == 4  // diagnostic builds only: where a wave's walk time goes (walk_wave's
// steps, DevState::stamp: 0 the next tile's VMEM wait, 1 LDS copy + classify, 2 rare drain + bitmaps, 3 header
// parse, 4 walk steps counted, 5 whole-kernel wave cycles, 6 walk calls)
#define FR_WSTAMP_DECL u64 wst_[4] = {0, 0, 0, 0}; u64 wq_ = __builtin_amdgcn_s_memtime();
#define FR_WSTAMP(i) do { const u64 n_ = __builtin_amdgcn_s_memtime(); wst_[i] += n_ - wq_; wq_ = n_; } while (0)
#define FR_WSTAMP_RESET() do { wq_ = __builtin_amdgcn_s_memtime(); } while (0)
#define FR_WSTAMP_FLUSH(steps) do { if ((threadIdx.x & 63) == 0) { \
    for (int i_ = 0; i_ < 4; ++i_) atomicAdd((unsigned long long*)&a.st->stamp[i_], (unsigned long long)wst_[i_]); \
    atomicAdd((unsigned long long*)&a.st->stamp[4], (unsigned long long)(steps)); \
    atomicAdd((unsigned long long*)&a.st->stamp[6], 1ull); } } while (0)
#else
#define FR_WSTAMP_DECL
#define FR_WSTAMP(i) do { } while (0)
#define FR_WSTAMP_RESET() do { } while (0)
#define FR_WSTAMP_FLUSH(steps) do { } while (0)
#endif

#ifdef FR_DEBUG_PRINT  // diagnostic builds only: trace the tally kernel's chunk loop (workgroup 0, lane 0 of each wave)
#define FR_TRACE(...) do { if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) printf(__VA_ARGS__); } while (0)
#else
#define FR_TRACE(...) do { } while (0)
#endif

#define FR_COLD __forceinline__  // rare paths stay inline (out of line, the calls made the hot loop spill)

// Timing ablations exist only in experiment builds: scripts/build_exp.sh NAME
// "-DFR_ABLATE=<bits>" (1 no header parse, 2 no code encode, 4 no LDS insert, 8 no commit flush,
// 64 commit counts, 128 plain stores in the commit (wrong counts), 256/512/1024 launch-log passes).
// The product build has FR_ABLATE = 0: every ablation branch folds away at compile time, and nothing
// read at run time (no environment variable, no kernel argument) can select one.
#ifndef FR_ABLATE
#define FR_ABLATE 0
#endif
constexpr u32 ABLATE = FR_ABLATE;

// ------------------------------------------------------------------------------------
// small helpers
// ------------------------------------------------------------------------------------

// exact per-byte equality of w against the byte replicated in c -> 4-bit mask (byte i -> bit i)
__device__ __forceinline__ u32 eq4(u32 w, u32 c) {
    const u32 t = w ^ c;
    const u32 z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
    return (((z >> 7) * 0x00204081u) >> 21) & 0xFu;
}

__device__ __forceinline__ u32 hi4(u32 w) {  // bytes >= 0x80
    return ((((w & 0x80808080u) >> 7) * 0x00204081u) >> 21) & 0xFu;
}

// byte -> fast-key symbol (A1 C2 G3 T4 N5 +6), 0 if outside the fast alphabet
__device__ __forceinline__ u32 sym_of(u32 c) {
    const u32 i = (c >> 1) & 7u;
    const u64 expect = 0x4E002B0047544341ull;  // idx: 0 A,1 C,2 T,3 G,4 -,5 +,6 -,7 N
    const u32 symtab = 0x50603421u;
    const bool ok = ((expect >> (8 * i)) & 0xFFu) == c;
    return ok ? ((symtab >> (4 * i)) & 0xFu) : 0u;
}

// Fused byte classifier, 4 bytes per call: per byte, bit0 line end ('\n' or '\r'), bit1 '\r',
// bit2 ' ', bit3 ':', bit4 byte >= 0x80.  Three 8-entry lookups through v_perm_b32, ANDed: on bits
// [2:0], on bits [5:3], and on bits [7:6].  '\n' = 00 001 010, '\r' = 00 001 101, ' ' = 00 100 000,
// ':' = 00 111 010: each class is the one byte whose two table entries both carry its bit; bit 4 is
// in every entry of the first two tables and in the third only for bits [7:6] = 1x (checked for
// all 256 bytes).
__device__ __forceinline__ u32 classify4(u32 w) {
    const u32 lo3 = __builtin_amdgcn_perm(0x10101310u, 0x10191014u, w & 0x07070707u);
    const u32 mid3 = __builtin_amdgcn_perm(0x18101014u, 0x10101310u, (w >> 3) & 0x07070707u);
    const u32 top2 = __builtin_amdgcn_perm(0u, 0x1010000Fu, (w >> 6) & 0x03030303u);
    return lo3 & mid3 & top2;
}

// The same classes from two lookups (round 4): bits [2:0] and bits [6:3] of the byte.  The 16-entry
// lookup leans on v_perm's fixed selectors (8-11: the sign bits of table bytes 1, 3, 5, 7, all 0 here;
// 12: 0x00; 13-15: 0xFF), so bytes 0x68-0x7F would read "every class" from it: the lo-table entries
// that carry a class also carry bit 7, and a class word with bit 7 set (the ASCII bytes h j m p r u x
// z }) sends the wave-tile to classify4.  Bit 7 of the byte is not looked at: a byte >= 0x80 sends the
// wave-tile there too.  Every other ASCII byte gets exactly classify4's bits 0-3 (checked for all 128).
__device__ __forceinline__ u32 classify4_fast(u32 w) {
    const u32 lo3 = __builtin_amdgcn_perm(0x00008300u, 0x00890084u, w & 0x07070707u);
    const u32 hi4 = __builtin_amdgcn_perm(0x08000004u, 0x00000300u, (w >> 3) & 0x0F0F0F0Fu);
    return lo3 & hi4;
}

// Class K of 16 bytes (four class words, byte i of word j = position 4j + i) -> a 16-bit mask.
// v_dot4_u32_u8 gathers the flag bytes at full rate: weights 1,2,4,8 place word 0's bytes at
// bits 0-3, weights 16..128 word 1's at bits 4-7 (every product is scaled by 2^K, undone at
// the end); no quarter-rate 32-bit multiplies.
template <int K>
__device__ __forceinline__ u32 gather16(u32 c0, u32 c1, u32 c2, u32 c3) {
    constexpr u32 M = 0x01010101u << K;
    u32 v = __builtin_amdgcn_udot4(c0 & M, 0x08040201u, 0u, false);
    v = __builtin_amdgcn_udot4(c1 & M, 0x80402010u, v, false);
    u32 u = __builtin_amdgcn_udot4(c2 & M, 0x08040201u, 0u, false);
    u = __builtin_amdgcn_udot4(c3 & M, 0x80402010u, u, false);
    return (v | (u << 8)) >> K;
}

__device__ __forceinline__ u64 agent_load(const u64* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void agent_store(u64* p, u64 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ u64 wave_sum_u64(u64 v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// ------------------------------------------------------------------------------------
// HBM table insert: count add, first-occurrence min, last file tag (presence is derived per
// file by presence_scan_kernel).  One 32-B slot load decides; the count add is
// fire-and-forget and the min/max atomics run only when they can change the slot (a stale
// load only ever over-estimates `first` / under-estimates `last_tag`, so skipping is safe).
// Returns true when this call created the slot.  No global counters are touched here.
// ------------------------------------------------------------------------------------
// Home slot of a key: the TOP bits of mix64(key).  The launch-log regions (log_region) are its top
// LOG_REGION_BITS bits too, so for tables of >= LOG_NR slots each region owns one contiguous slot range
// and log_reduce_kernel's inserts stay inside it (DRAM-page and L2 locality instead of random lines).
__device__ __forceinline__ u64 table_home(u64 key, u64 mask) {
    return mask ? mix64(key) >> __builtin_clzll(mask) : 0ull;
}

__device__ bool global_insert(const Table& T, DevState* st, u64 key, u64 cnt, u64 ord, u32 tag) {
    u64 h = table_home(key, T.mask);
    for (int probe = 0; probe < GPROBE; ++probe) {
        GSlot* s = &T.slots[h];
        const uint4 w0 = *(const uint4*)s;
        const uint4 w1 = *((const uint4*)s + 1);
        u64 k = ((u64)w0.y << 32) | w0.x;
        u64 first = ((u64)w1.y << 32) | w1.x;
        u32 ltag = w1.z;
        bool created = false;
        if (k == 0) {
            const u64 old = atomicCAS((unsigned long long*)&s->key, 0ull, (unsigned long long)key);
            created = old == 0;
            k = created ? key : old;
            first = ~0ull;
            ltag = 0;
        }
        if (k == key) {
            atomicAdd((unsigned long long*)&s->count, (unsigned long long)cnt);
            if (ord < first) atomicMin((unsigned long long*)&s->first, (unsigned long long)ord);
            if (ltag < tag) atomicMax(&s->last_tag, tag);
            return created;
        }
        h = (h + 1) & T.mask;
    }
    const u64 i = atomicAdd((unsigned long long*)&st->n_overflow, 1ull);
    if (i < T.ovf_cap) {
        Overflow o;
        o.key = key;
        o.count = cnt;
        o.first = ord;
        o.tag = tag;
        o.pad = 0;
        T.ovf[i] = o;
    } else {
        atomicOr(&st->cap_flags, 2u);
    }
    return false;
}

// block-wide count of created slots -> one global add per wave
__device__ __forceinline__ void add_created(DevState* st, u32 mine) {
    u64 v = mine;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd((unsigned long long*)&st->n_keys, (unsigned long long)v);
}

// ------------------------------------------------------------------------------------
// the tally kernel (v8): per-wave walkers
//
// A workgroup takes a chunk (a contiguous run of wave-tiles) by ticket and splits it into four
// contiguous parts, one per wave.  Each wave walks its part alone: no workgroup barrier inside the
// tile loop, so a wave that waits for its next tile's loads does not hold the other three (round 2
// had two barriers per 16-KiB workgroup tile; MI355X measurements in profiles/r03a_ubench_tile.txt:
// the barrier-free walk is 8-12 % faster at equal loads and parse work).  A wave-tile is 4 KiB: lane
// L holds the 64-B segment [64 L, 64 L + 64) in registers, loaded one wave-tile ahead, classifies it
// there, and stores its ' ' / ':' / line-end bitmaps and its bytes to the wave's own LDS area, where
// the lane-owned header parse reads them.  Tiles overlap by one segment (stride TSTEP), so a
// header's bitmap window always has a successor segment.
//
// Line phase per wave: the first wave of chunk 0 starts at the range's exact line count; every
// other wave guesses its starting phase from its first wave-tile (FASTQ structure, infer_phase).
// After the walk the chunk's four counts give each wave's phase relative to the chunk start; a wave
// whose guess disagrees makes the chunk redo with the derived phases, a wave that could not guess
// walks again with its derived phase.  The chunk start itself is exact (chunk 0, or a decoupled
// look-back) or, for device feeds, the first wave's guess, committed at once and checked for the
// whole launch by verify_launch.  Correctness never depends on a guess.
// ------------------------------------------------------------------------------------
struct alignas(16) LSlot {  // one ds_read_b128 reads key, count and first offset together
    u64 key;                 // 0 = empty
    u32 cnt;
    u32 mino;                // min range offset of the code's records, ~0 = none
};

constexpr int NW = WG / 64;                  // waves per workgroup
constexpr int SEGS = TILE / SEG;             // segments per wave-tile (= lanes)
constexpr u32 RARE_WAVE = RARE_RING / NW;    // rare-event ring entries per wave

struct ScanShared {
    u32 raw[NW][TILE / 4];   // each wave's current wave-tile (the parse reads code bytes here)
    LSlot ls[NS];            // LDS hash table of this workgroup's chunk
    u64 bsp[NW][SEGS + 2];   // per wave, per 64-B segment of its staged tile: ' ' | line-end bitmap
    u64 bcol[NW][SEGS + 2];  //                                              ':' bitmap
    u64 beol[NW][SEGS + 2];  //                                              '\r' | '\n' bitmap
                             // entries SEGS, SEGS + 1 stay zero: window words past the tile
    u64 wcount[NW];          // pass 0: line terminators of each wave's part of the chunk
    int wphase[NW];          // pass 0: the phase each wave parsed with (mod 4), -1 count only
    u32 rq_tail[NW];         // rare-event ring: events pushed by each wave (monotonic)
    u64 tile_excl;
    u64 cbase;               // the chunk's first byte in the range: positions inside a chunk are u32 offsets
                             // from it (chunks are <= 512 tiles), so a range may exceed 4 GiB
    u32 chunk;
    u32 nkeys;               // occupied LDS slots
    u32 created;             // HBM slots this workgroup created (added to n_keys once, at exit)
    u32 flags;
    u32 last;                // this workgroup published the launch's last chunk count (runs verify_launch)
    u32 spec;                // side effects are buffered (a phase in use is a guess); the chunk may be redone
    u32 spec_bad;            // a speculation buffer overflowed: redo this chunk exactly
    u32 ncold;               // cold list fill
    u32 nexo;                // buffered exotic records
    u32 err_off;             // min range offset of a header without ' ' (buffered), ~0 none
    u32 log_on;              // commit: pairs this commit logs
    u32 exo_p[EXO_BUF], exo_start[EXO_BUF], exo_len[EXO_BUF];
};

typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32 lds_u32;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
typedef __attribute__((address_space(3))) u64 lds_u64;
typedef __attribute__((address_space(3))) u8 lds_u8;

// Ordinal of a record: file tag << 44 | its header's file offset rounded down to a multiple of 4.  Record
// starts are >= 4 bytes apart (four lines of >= 1 byte), so the rounding keeps every comparison of two
// records' ordinals, i.e. the first-occurrence order; it lets the launch log's fold keep a first
// occurrence in 32 bits for launches up to 16 GiB (log_reduce_kernel).  Every path rounds alike.
__device__ __forceinline__ u64 make_ord(const ScanArgs& a, u64 off_in_range) {
    return ((u64)a.file_tag << ORD_SHIFT) | ((a.file_offset + off_in_range) & ~3ull);
}

__device__ __forceinline__ u32 wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// this wave's LDS stores are complete: later reads by other lanes of the wave see them (a wave's LDS
// operations execute in order; the wait also keeps the compiler from moving reads above the stores).
// LDS only: outstanding global loads (the next tile) stay in flight.
__device__ __forceinline__ void lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// workgroup barrier that orders LDS only: outstanding global loads, stores and atomics stay in flight
// (__syncthreads() would wait for every one of them)
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ FR_COLD void direct_insert(ScanShared& sh, const ScanArgs& a, u64 key, u32 off) {
    if (global_insert(a.tabv, a.st, key, 1, make_ord(a, sh.cbase + off), a.file_tag)) atomicAdd(&sh.created, 1u);
}

__device__ __forceinline__ void rare_push(ScanShared& sh, const ScanArgs& a, u32 p, u32 kind, u32 x, u32 y);

template <bool DRAIN = false>
__device__ __forceinline__ void lds_insert(ScanShared& sh, const ScanArgs& a, u64 key, u32 off) {
    // one 32-bit multiply (keys hold <= 63 bits: fold the top down first)
    u32 h = (((u32)key ^ (u32)(key >> 27)) * 0x9E3779B1u) >> (32 - LOG_NS);
#pragma unroll 2
    for (int pr = 0; pr < LPROBE; ++pr) {
        // volatile through an explicit LDS pointer: a volatile access through a generic pointer
        // keeps its flat form (flat loads wait on vmcnt(0), i.e. on every outstanding HBM op).  The key
        // count is read in the same round as the slot (a new key's claim then costs no extra round trip)
        u32x4 sl = *(const lds_u32x4*)&sh.ls[h];
        u32 nk = *(const lds_u32*)&sh.nkeys;
        asm volatile("" : "+v"(sl), "+v"(nk) :: "memory");  // both loads in one round, not moved or reused
        u64 k = ((u64)sl.y << 32) | sl.x;
        u32 mino = sl.w;
        if (k == 0) {
            // a full LDS table stops claiming slots: the code goes to the cold list; the codes
            // already resident (the hot ones arrive first) keep aggregating here
            if (nk >= a.flush_at) break;
            const u64 old = atomicCAS((unsigned long long*)&sh.ls[h].key, 0ull, (unsigned long long)key);
            if (old == 0) {
                atomicAdd(&sh.nkeys, 1u);
                k = key;
            } else {
                k = old;
            }
            mino = 0xFFFFFFFFu;
        }
        if (k == key) {
            atomicAdd(&sh.ls[h].cnt, 1u);
            // mino only decreases, so a stale read can only cause a redundant atomic
            if (off < mino) atomicMin(&sh.ls[h].mino, off);
            return;
        }
        h = (h + 1) & (NS - 1);
    }
    // an LDS-table miss: park it in this workgroup's cold list (committed with the chunk)
    const u32 i = atomicAdd(&sh.ncold, 1u);
    if (i < a.cold_cap) {
        u64* c = a.cold + 2ull * ((u64)blockIdx.x * a.cold_cap + i);
        c[0] = key;
        c[1] = make_ord(a, sh.cbase + off);
        return;
    }
    if (sh.spec) {  // cannot insert while speculating: this chunk will be redone exactly
        atomicOr(&sh.spec_bad, 1u);
        return;
    }
    // exact phase and a full cold list: insert directly (queued out of the hot loop)
    if (DRAIN) direct_insert(sh, a, key, off);
    else rare_push(sh, a, off, 3u, (u32)key, (u32)(key >> 32));
}

// Rare events (exotic codes, headers without ' ', headers whose code leaves the bitmap window,
// direct HBM inserts, UTF-8 checks) go to the wave's ring in HBM and are handled by drain_rare at
// the wave's next tile, so their code adds no registers to the tile loop.  Entry: {chunk offset,
// kind, x, y}.  No fence here (a release would wait for the next tile's loads): drain_rare fences.
__device__ __forceinline__ void rare_push(ScanShared& sh, const ScanArgs& a, u32 p, u32 kind, u32 x, u32 y) {
    const u32 wid = wave_id();
    const u32 i = atomicAdd(&sh.rq_tail[wid], 1u);
    a.rare[(u64)blockIdx.x * RARE_RING + wid * RARE_WAVE + (i & (RARE_WAVE - 1u))] = make_uint4(p, kind, x, y);
}

// Decoupled look-back over the launch's chunk descriptors {tag = 2*epoch + inclusive, value}.
// The chunk's own aggregate was published before (chunk_kernel); this resolves its exclusive
// prefix, reading 256 predecessors per poll (4 per lane), and publishes the inclusive prefix.
// Returns the number of line terminators in chunks [0, t) of the range.
__device__ __forceinline__ u64 lookback(const ScanArgs& a, u32 t, u32 agg, int lane) {
    if (t == 0) return 0;  // chunk 0 published its inclusive value directly
    const u64 tagI = (u64)(2u * a.epoch + 1u) << 32;
    u64 excl = 0;
    i64 j = (i64)t - 1;
    u32 spins = 0;
    for (;;) {
        u64 sv[4], rdy[4], inc[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const i64 idx = j - 64 * k - lane;
            sv[k] = idx >= 0 ? agent_load(&a.tiles[idx]) : tagI;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32 tag = (u32)(sv[k] >> 32);
            const bool ready = (tag >> 1) == a.epoch;
            rdy[k] = __ballot(ready);
            inc[k] = __ballot(ready && (tag & 1u));
        }
        int kf = 4, lf = 63;
#pragma unroll
        for (int k = 3; k >= 0; --k)
            if (inc[k]) {
                kf = k;
                lf = __ffsll((long long)inc[k]) - 1;
            }
        bool ok = true;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u64 need = k < kf ? ~0ull : k == kf ? (lf == 63 ? ~0ull : ((1ull << (lf + 1)) - 1ull)) : 0ull;
            ok &= (rdy[k] & need) == need;
        }
        if (!ok) {
            if (++spins > SPIN_MAX) {
                if (lane == 0) atomicOr(&a.st->spin_fail, 1u);
                return 0;
            }
            if (spins > 2) __builtin_amdgcn_s_sleep(8);
            continue;
        }
        u64 contrib = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k < kf || (k == kf && lane <= lf)) contrib += (u32)sv[k];
        excl += wave_sum_u64(contrib);
        if (kf < 4) break;
        j -= 256;
    }
    if (lane == 0) {
        agent_store(&a.tiles[t], tagI | (u64)(u32)(excl + agg));
        if (spins) {
            atomicMax(&a.st->spin_max, spins);
            atomicAdd((unsigned long long*)&a.st->spin_total, (unsigned long long)spins);
        }
    }
    return excl;
}

// validate UTF-8 for the range bytes [s0, s0+n) (only called when a byte >= 0x80 is present);
// bytes are read from HBM (the range, and before it when readable), -1 past them.
__device__ FR_COLD bool utf8_segment_ok(const ScanArgs& a, u64 s0, u32 n) {
    auto byte_at = [&](i64 q) -> int {
        if (q < 0 && !a.pre_valid) return -1;
        if (q >= (i64)a.avail) return -1;
        return (int)a.buf[q];
    };
    for (i64 q = (i64)s0; q < (i64)s0 + (i64)n; ++q) {
        const int b = byte_at(q);
        if (b < 0x80) continue;
        if (b >= 0x80 && b <= 0xBF) {  // continuation: must be claimed by a lead
            bool claimed = false;
            for (int j = 1; j <= 3; ++j) {
                const int c = byte_at(q - j);
                if (c < 0) break;
                if (c >= 0x80 && c <= 0xBF) continue;
                const int need = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 1;
                claimed = need > j;
                break;
            }
            if (!claimed) return false;
            continue;
        }
        int need;
        if (b >= 0xC2 && b <= 0xDF) need = 2;
        else if (b >= 0xE0 && b <= 0xEF) need = 3;
        else if (b >= 0xF0 && b <= 0xF4) need = 4;
        else return false;
        for (int j = 1; j < need; ++j) {
            const int c = byte_at(q + j);
            if (c < 0x80 || c > 0xBF) return false;
            if (j == 1) {
                if (b == 0xE0 && c < 0xA0) return false;
                if (b == 0xED && c > 0x9F) return false;
                if (b == 0xF0 && c < 0x90) return false;
                if (b == 0xF4 && c > 0x8F) return false;
            }
        }
    }
    return true;
}

template <bool DRAIN = false>
__device__ __forceinline__ void count_code(ScanShared& sh, const ScanArgs& a, u32 p, u64 key) {
    if ((ABLATE & 4u) || a.exo_only) {  // ablation / exotic-only replay: skip the hash insert
        asm volatile("" ::"v"(key));
        return;
    }
    lds_insert<DRAIN>(sh, a, key, p);
}

// code bytes [q, q+n) of the range (exact byte reads) -> wide key (fr_internal.h), false when the
// code is outside the wide form.  Only called for codes that are not fast keys.
__device__ bool wide_encode(const ScanArgs& a, u64 q, u64 n, u64& key) {
    if (n < 1 || n > (u64)WIDE_MAXN + 1) return false;
    int lower = -1, plus = WIDE_NOPLUS, nl = 0;
    u64 v = 0, pw = 1;
    for (u64 k = 0; k < n; ++k) {
        const u32 c = a.buf[q + k];
        if (c == '+') {
            if (plus != WIDE_NOPLUS) return false;
            plus = nl;
            continue;
        }
        const u32 lc = c | 0x20u;
        const int d = lc == 'a' ? 0 : lc == 'c' ? 1 : lc == 'g' ? 2 : lc == 't' ? 3 : lc == 'n' ? 4 : -1;
        if (d < 0 || nl >= WIDE_MAXN) return false;
        const int isl = (c & 0x20u) ? 1 : 0;
        if (lower < 0) lower = isl;
        else if (lower != isl) return false;
        v += (u64)d * pw;
        pw *= 5;
        ++nl;
    }
    if (lower < 0) return false;  // no letter
    const int n1 = plus == WIDE_NOPLUS ? nl : plus, n2 = plus == WIDE_NOPLUS ? 0 : nl - plus;
    if (n1 > MAXSYM || n2 > MAXSYM) return false;
    key = WIDE_BIT | ((u64)lower << 62) | ((u64)plus << 57) | (v + (pw - 1) / 4);
    return true;
}

// a code the fast encoder did not take (header p: chunk offset; code [start, start + n): range offsets): exact
// fast form (defensive), wide key, or an exotic record captured verbatim (speculating: its position
// is buffered and the bytes stay resident in HBM)
__device__ void exotic_record(const ScanArgs& a, u32 p, u64 start, u64 n, ScanShared& sh) {
    {
        bool fast = n >= 1 && n <= (u64)MAXSYM;
        u64 key = 0;
        for (u64 i = 0; fast && i < n; ++i) {
            const u32 sy = sym_of(a.buf[start + i]);
            fast = sy != 0;
            key |= (u64)sy << (3 * i);
        }
        if (fast || wide_encode(a, start, n, key)) {
            count_code<true>(sh, a, p, key);
            return;
        }
    }
    if (sh.spec) {  // speculating: remember where it is; the bytes stay resident in HBM
        const u32 k = atomicAdd(&sh.nexo, 1u);
        if (k < (u32)EXO_BUF) {
            sh.exo_p[k] = p;
            sh.exo_start[k] = (u32)(start - sh.cbase);
            sh.exo_len[k] = (u32)n;
        } else {
            atomicOr(&sh.spec_bad, 1u);
        }
        return;
    }
    const u64 i = atomicAdd((unsigned long long*)&a.st->n_exotic, 1ull);
    const u64 po = atomicAdd((unsigned long long*)&a.st->exo_pool_used, (unsigned long long)n);
    if (i < a.tabv.exo_cap && po + n <= a.tabv.exo_pool_cap) {
        a.tabv.exo_ord[i] = make_ord(a, sh.cbase + p);
        a.tabv.exo_off[i] = po;
        a.tabv.exo_len[i] = (u32)n;
        for (u64 k = 0; k < n; ++k) a.tabv.exo_pool[po + k] = a.buf[start + k];
    } else {
        atomicOr(&a.st->cap_flags, 4u);
    }
}

__device__ __forceinline__ void nospace(const ScanArgs& a, u32 p, ScanShared& sh) {  // IndexError (:169)
    if (sh.spec) atomicMin(&sh.err_off, p);
    else atomicMin((unsigned long long*)&a.st->err_nospace, (unsigned long long)(a.file_offset + sh.cbase + p));
}

// slow path (rare): a header whose code does not end inside its bitmap windows, parsed byte by
// byte from HBM.  R2 (frender.py:169): the token after the first ' ' up to the next ' ' or line
// end, then its suffix after the last ':'.  p = the header's chunk offset.
__device__ FR_COLD void process_header_global(ScanShared& sh, const ScanArgs& a, u32 p) {
    const u64 eof = a.avail;
    auto rd = [&](u64 q) -> u32 { return (u32)a.buf[q]; };
    u64 q = sh.cbase + p;
    for (;;) {
        if (q >= eof) return nospace(a, p, sh);
        const u32 c = rd(q);
        if (c == ' ') break;
        if (c == '\n' || c == '\r') return nospace(a, p, sh);
        ++q;
    }
    const u64 sp1 = q++;
    i64 lc = -1;
    for (;;) {
        if (q >= eof) break;
        const u32 c = rd(q);
        if (c == ' ' || c == '\n' || c == '\r') break;
        if (c == ':') lc = (i64)q;
        ++q;
    }
    const u64 start = (lc >= 0 ? (u64)lc : sp1) + 1;
    const u64 n = q - start;
    u64 key = 0;
    bool fast = n >= 1 && n <= (u64)MAXSYM;
    for (u64 i = 0; fast && i < n; ++i) {
        const u32 sy = sym_of(rd(start + i));
        fast = sy != 0;
        key |= (u64)sy << (3 * i);
    }
    if (fast) count_code<true>(sh, a, p, key);
    else exotic_record(a, p, start, n, sh);
}

// ---- wave-tile staging: lane-contiguous segments classified straight from registers ---------
// Lane L loads its own 64-byte segment [64 L, 64 L + 64) of the wave-tile (four 16-B loads through
// a wave-uniform buffer descriptor) one tile ahead, classifies it in registers and stores it and
// its bitmaps to the wave's LDS area.  (Coalesced 1-KiB-per-instruction loads with an LDS
// transpose, and LDS-DMA rings, measured slower: profiles/r03a_ubench_tile.txt.)
struct SegRegs {
    uint4 v[SEG / 16];
    u32 nx;  // first dword of the next segment (zero past the staged bytes)
};

__device__ __forceinline__ void seg_fetch(const ScanArgs& a, u32 t, SegRegs& r, int lane, bool with_nx = false) {
    const u64 tile0 = (u64)t * TSTEP;
    const u32 nb = (u32)min((u64)TILE, a.avail - tile0);
    const u64 base = (u64)(a.buf + tile0);
    const u32 lo = __builtin_amdgcn_readfirstlane((u32)base), hi = __builtin_amdgcn_readfirstlane((u32)(base >> 32));
    const u8* ub = (const u8*)(((u64)hi << 32) | lo);
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)ub, (short)0, (int)__builtin_amdgcn_readfirstlane(nb),
                                                        0x00020000);
#pragma unroll
    for (int k = 0; k < SEG / 16; ++k) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, lane * SEG, k * 16, 0);
        r.v[k] = make_uint4(v[0], v[1], v[2], v[3]);
    }
    r.nx = with_nx ? __builtin_amdgcn_raw_buffer_load_b32(rsrc, lane * SEG + SEG, 0, 0) : 0u;  // '\r' path only
}

// the data end (a segment, or the dword after it, reaches past avail): bytewise loads, zeros past
// the staged bytes (the buffer range check is trusted only for whole vectors)
__device__ __attribute__((noinline)) SegRegs seg_load_tail(const ScanArgs& a, u32 t, int lane) {
    const u64 tile0 = (u64)t * TSTEP;
    const u32 nb = (u32)min((u64)TILE, a.avail - tile0);
    const u32 s0 = lane * SEG;
    u32 w[SEG / 4 + 1];
    for (int k = 0; k <= SEG / 4; ++k) {
        u32 v = 0;
        for (u32 q = 0; q < 4; ++q) {
            const u32 o = s0 + 4 * k + q;
            if (o < nb) v |= (u32)a.buf[tile0 + o] << (8 * q);
        }
        w[k] = v;
    }
    SegRegs r;
    for (int k = 0; k < SEG / 16; ++k) r.v[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
    r.nx = w[SEG / 4];
    return r;
}

// every lane's segment loads of wave-tile t (and the dword after them) lie inside the data
__device__ __forceinline__ bool seg_in_range(const ScanArgs& a, u32 t) {
    return (u64)t * TSTEP + (TILE + SEG + 4) <= a.avail;
}

__device__ __forceinline__ void seg_load(const ScanArgs& a, u32 t, SegRegs& r, int lane) {
    if (seg_in_range(a, t)) seg_fetch(a, t, r, lane);
    else r = seg_load_tail(a, t, lane);
}

struct SegClass {
    u64 tmask, sp, col, eol;  // terminators (own bytes), and the parse bitmaps (staged bytes)
    u32 c, x;                 // popcount(tmask), its inclusive wave scan
    u32 wtot;                 // the wave's terminators (own bytes of the wave-tile)
    bool hi;                  // a byte >= 0x80 among the own bytes (UTF-8 check, kind 4)
};

template <class Src>
__device__ __forceinline__ SegClass seg_classify_src(const ScanArgs& a, u32 t, const Src& src, int lane);

struct Cls16 {  // a segment's class bitmaps in 16-bit quarters, and the OR of its class words
    u32 eol[4], sp[4], col[4], acc;
};

// classify4 over the lane's segment, re-read from memory: the exact path of seg_classify_src
__device__ __attribute__((noinline)) Cls16 classes_exact(const ScanArgs& a, u32 t, int lane) {
    SegRegs q;
    if (seg_in_range(a, t)) seg_fetch(a, t, q, lane);
    else q = seg_load_tail(a, t, lane);
    Cls16 r;
    r.acc = 0;
#pragma unroll
    for (int qv = 0; qv < SEG / 16; ++qv) {
        const u32 c0 = classify4(q.v[qv].x), c1 = classify4(q.v[qv].y), c2 = classify4(q.v[qv].z),
                  c3 = classify4(q.v[qv].w);
        r.eol[qv] = gather16<0>(c0, c1, c2, c3);
        r.sp[qv] = gather16<2>(c0, c1, c2, c3);
        r.col[qv] = gather16<3>(c0, c1, c2, c3);
        r.acc |= c0 | c1 | c2 | c3;
    }
    return r;
}

__device__ __forceinline__ SegClass seg_classify(const ScanArgs& a, u32 t, const SegRegs& r, int lane) {
    return seg_classify_src(a, t, [&](int k) { return r.v[k]; }, lane);
}

// src(k): the segment's k-th 16 bytes (registers, or a read of the wave's LDS copy: then only one
// quarter of the segment is live at a time)
template <class Src>
__device__ __forceinline__ SegClass seg_classify_src(const ScanArgs& a, u32 t, const Src& src, int lane) {
    const u64 tile0 = (u64)t * TSTEP;
    const u32 tlen = (u32)min((u64)TSTEP, a.len - tile0);
    const u32 bl = (u32)min((u64)TILE, a.avail - tile0);
    const u32 s0 = lane * SEG;
    SegClass sc;
    sc.tmask = 0;
    sc.sp = sc.col = sc.eol = 0;
    sc.hi = false;
    if (s0 < bl) {
        u32 eol16[4], sp16[4], col16[4];
        u32 acc = 0, raw = 0;
#pragma unroll
        for (int qv = 0; qv < SEG / 16; ++qv) {  // class words live one quarter at a time
            const uint4 v = src(qv);
            const u32 c0 = classify4_fast(v.x), c1 = classify4_fast(v.y), c2 = classify4_fast(v.z),
                      c3 = classify4_fast(v.w);
            eol16[qv] = gather16<0>(c0, c1, c2, c3);
            sp16[qv] = gather16<2>(c0, c1, c2, c3);
            col16[qv] = gather16<3>(c0, c1, c2, c3);
            acc |= c0 | c1 | c2 | c3;
            raw |= v.x | v.y | v.z | v.w;
        }
        if (__ballot(((acc | raw) & 0x80808080u) != 0) != 0) {  // a wave-uniform SGPR value: a scalar branch
            // a byte >= 0x80 or a fast-table sentinel somewhere in the wave-tile: the exact classifier,
            // out of line on the segment re-read from L2 (no register of the common path is held for it)
            const Cls16 e = classes_exact(a, t, lane);
#pragma unroll
            for (int qv = 0; qv < SEG / 16; ++qv) {
                eol16[qv] = e.eol[qv];
                sp16[qv] = e.sp[qv];
                col16[qv] = e.col[qv];
            }
            acc = e.acc;
        }
        auto join = [](const u32 (&g)[4]) {
            return ((u64)(g[2] | (g[3] << 16)) << 32) | (u64)(g[0] | (g[1] << 16));
        };
        u64 eol = join(eol16), sp = join(sp16), col = join(col16);
        u64 tm = eol;
        if (__ballot((acc & 0x02020202u) != 0) != 0) {
            // '\r' somewhere in the wave (CRLF / CR files): a '\r' right before a '\n' ends no line.
            // The segment (and the byte after it) is re-read from L2 here, so no class word has to
            // stay live through the common path.
            SegRegs q;
            if (seg_in_range(a, t)) seg_fetch(a, t, q, lane, true);
            else q = seg_load_tail(a, t, lane);
            u32 cr16[4];
#pragma unroll
            for (int qv = 0; qv < SEG / 16; ++qv)
                cr16[qv] = gather16<1>(classify4(q.v[qv].x), classify4(q.v[qv].y), classify4(q.v[qv].z),
                                       classify4(q.v[qv].w));
            const u64 cr = join(cr16), nl = eol & ~cr;
            const u64 nxt = (q.nx & 0xFFu) == (u32)'\n' ? 1ull : 0ull;
            tm = eol & ~(cr & ((nl >> 1) | (nxt << 63)));
        }
        const u32 bvalid = bl - s0;
        if (bvalid < SEG) {
            const u64 vm = (1ull << bvalid) - 1ull;
            sp &= vm;
            col &= vm;
            eol &= vm;
        }
        if (s0 < tlen) {
            const u32 valid = tlen - s0;
            if (valid < SEG) tm &= (1ull << valid) - 1ull;
        } else {
            tm = 0;
        }
        sc.sp = sp;
        sc.col = col;
        sc.eol = eol;
        if (s0 < tlen) {
            sc.tmask = tm;
            sc.hi = (acc & 0x10101010u) != 0;  // exact own-byte test in drain_rare (kind 4)
        }
    }
    sc.c = __popcll(sc.tmask);
    // inclusive wave scan of c: DPP row shifts within 16-lane rows, then row broadcasts
    u32 x = sc.c;
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xF, 0xF, true);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    sc.x = x;
    sc.wtot = __builtin_amdgcn_readlane(x, 63);
    return sc;
}

__device__ FR_COLD void slow_header(ScanShared& sh, const ScanArgs& a, u32 p, int r, u32 start, u32 n);

// handle this wave's ring entries [from, to) (its lanes; the wave pushes nothing meanwhile)
__device__ __attribute__((noinline)) void drain_rare(ScanShared& sh, const ScanArgs& a, u32 wid, u32 from, u32 to,
                                                     int lane) {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // the wave's ring stores are visible to its loads
    const uint4* q = a.rare + (u64)blockIdx.x * RARE_RING + wid * RARE_WAVE;
    for (u32 i = from + lane; i - from < to - from; i += 64) {
        const uint4 e = q[i & (RARE_WAVE - 1u)];
        if (e.y == 3u) {
            direct_insert(sh, a, ((u64)e.w << 32) | e.z, e.x);
        } else if (e.y == 4u) {  // UTF-8: the segment's own bytes [e.x, e.x + e.z) of the chunk
            const u64 x = sh.cbase + e.x;
            bool hi = false;
            for (u32 k = 0; k < e.z; ++k) hi |= a.buf[x + k] >= 0x80;
            if (hi) {
                atomicOr(&sh.flags, 1u);
                if (!utf8_segment_ok(a, x, e.z)) atomicOr(&sh.flags, 2u);
            }
        } else {
            slow_header(sh, a, e.x, (int)e.y, e.z, e.w);
        }
    }
}

// phase inference bitmaps of a wave's first tile: '@' and '+' (first bytes of header / separator
// lines); exact per-byte equality, once per wave and chunk
__device__ __forceinline__ void seg_marks(const SegRegs& r, u64& at, u64& plus) {
    at = 0;
    plus = 0;
#pragma unroll
    for (int qv = 0; qv < SEG / 16; ++qv) {
        const u32 w[4] = {r.v[qv].x, r.v[qv].y, r.v[qv].z, r.v[qv].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            at |= (u64)eq4(w[k], 0x40404040u) << (qv * 16 + k * 4);
            plus |= (u64)eq4(w[k], 0x2B2B2B2Bu) << (qv * 16 + k * 4);
        }
    }
}

// Guess P = (lines before the wave-tile) mod 4 from its first PHASE_LINES complete lines: with lines
// indexed P+k+1 after the k-th terminator, a FASTQ record has a header ('@') at phase 0, '+' at
// phase 2 and equal seq/qual lengths at phases 1/3.  Exactly one consistent P -> the guess;
// otherwise -1 (unsure).  Bitmaps (staged by the caller, the wave's area): bcol = '@', beol = '+'.
// Line lengths include a '\r' of "\r\n" (equal on both lines of a consistently terminated record).
// All lanes at once (round 4; it was one lane walking the lines while the wave waited): the
// terminators e_0 .. e_PHASE_LINES of the tile go to LDS by their index in the tile (each lane writes
// its own, from the wave's terminator scan), then lane k checks line k = (e_k, e_{k+1}) against the
// four candidate phases and ballots decide.
__device__ __forceinline__ int infer_phase(ScanShared& sh, const SegClass& sc, int lane, u32 wid) {
    lds_u32* E = (lds_u32*)&sh.raw[wid][0];  // the wave's tile copy is free until its walk starts
    u32 i = sc.x - sc.c;                      // this lane's first terminator's index in the tile
    u64 m = sc.tmask;
    while (m && i <= (u32)PHASE_LINES) {
        E[i] = (u32)lane * SEG + (u32)__builtin_ctzll(m);
        m &= m - 1ull;
        ++i;
    }
    lds_fence();
    const u32 tot = __builtin_amdgcn_readlane(sc.x, 63);  // terminators in the tile
    const int K = (int)min(tot, (u32)PHASE_LINES + 1u) - 1;  // complete lines looked at
    if (K < 8) return -1;
    const bool valid = lane < K;
    int len = 0;
    bool is_at = false, is_plus = false;
    if (valid) {
        const u32 st = E[lane] + 1u;
        len = (int)E[lane + 1] - (int)st;
        is_at = len > 0 && ((sh.bcol[wid][st >> 6] >> (st & 63u)) & 1ull);
        is_plus = len > 0 && ((sh.beol[wid][st >> 6] >> (st & 63u)) & 1ull);
    }
    const int len2 = __shfl(len, lane - 2, 64);  // line k - 2: the phase-1 line before a phase-3 line
    int found = -1, nfound = 0;
#pragma unroll
    for (int P = 0; P < 4; ++P) {
        const int ph = (P + lane + 1) & 3;
        const bool bad = valid && ((ph == 0 && !is_at) || (ph == 2 && !is_plus) || (ph == 3 && lane >= 2 && len != len2));
        if (__ballot(bad) == 0) {
            found = P;
            ++nfound;
        }
    }
    return nfound == 1 ? found : -1;
}

// the line phase at wave-tile t, guessed from its content (infer_phase); -1 unsure.  Whole wave.
__device__ __attribute__((noinline)) int guess_phase(ScanShared& sh, const ScanArgs& a, u32 t, int lane, u32 wid) {
    SegRegs r;
    seg_load(a, t, r, lane);
    const SegClass sc = seg_classify(a, t, r, lane);
    u64 at, plus;
    seg_marks(r, at, plus);
    sh.bcol[wid][lane] = at;  // infer_phase: '@', '+'
    sh.beol[wid][lane] = plus;
    lds_fence();
    return infer_phase(sh, sc, lane, wid);
}

// Commit: resolve first, update last.  A wait for a load or CAS return also waits for every
// vector-memory op issued before it (vmcnt counts in order), and under the streaming load of the
// other workgroups each round trip is long; so every entry's table slot is found before any count
// is added.  resolve_batch walks CE entries per lane in rounds: the probe loads of all pending
// entries together, then the CASes that claim empty slots together; it adds nothing.  The count /
// first / tag atomics follow in apply_entry, fire-and-forget: an LDS-only barrier ends the commit.
struct Resolved {
    u32 slot;      // the key's slot; ~0: probe bound exceeded (the overflow list takes the entry)
    u32 tag;       // the slot's last_tag as loaded (0: claimed now, or unknown)
    u64 first;     // the slot's first as loaded (~0: claimed now, or unknown)
};

template <int CE>
__device__ __forceinline__ u32 resolve_batch(const ScanArgs& a, const u64 (&key)[CE], const bool (&valid)[CE],
                                             Resolved (&rs)[CE]) {
    const Table& T = a.tabv;
    bool pend[CE];
#pragma unroll
    for (int b = 0; b < CE; ++b) {
        rs[b].slot = (u32)table_home(key[b], T.mask);
        rs[b].first = ~0ull;
        rs[b].tag = 0;
        pend[b] = valid[b];
    }
    u32 made = 0;
    for (int round = 0; round < GPROBE; ++round) {
        bool any = false;
#pragma unroll
        for (int b = 0; b < CE; ++b) any |= pend[b];
        if (!any) return made;
        u64 k[CE];
#pragma unroll
        for (int b = 0; b < CE; ++b)
            if (pend[b]) {
                const GSlot* sl = &T.slots[rs[b].slot];
                const uint2 w0 = *(const uint2*)sl;
                const uint4 w1 = *((const uint4*)sl + 1);
                k[b] = ((u64)w0.y << 32) | w0.x;
                rs[b].first = ((u64)w1.y << 32) | w1.x;
                rs[b].tag = w1.z;
            }
        bool cas[CE];
#pragma unroll
        for (int b = 0; b < CE; ++b) {
            cas[b] = false;
            if (!pend[b]) continue;
            if (k[b] == key[b]) pend[b] = false;
            else if (k[b] == 0) cas[b] = true;
            else rs[b].slot = (rs[b].slot + 1u) & (u32)T.mask;
        }
        u64 old[CE];
#pragma unroll
        for (int b = 0; b < CE; ++b)
            if (cas[b]) old[b] = atomicCAS((unsigned long long*)&T.slots[rs[b].slot].key, 0ull, (unsigned long long)key[b]);
#pragma unroll
        for (int b = 0; b < CE; ++b) {
            if (!cas[b]) continue;
            if (old[b] == 0 || old[b] == key[b]) {  // claimed now, or by another workgroup meanwhile
                made += old[b] == 0 ? 1u : 0u;
                rs[b].first = ~0ull;
                rs[b].tag = 0;
                pend[b] = false;
            } else {
                rs[b].slot = (rs[b].slot + 1u) & (u32)T.mask;
            }
        }
    }
#pragma unroll
    for (int b = 0; b < CE; ++b)
        if (pend[b]) rs[b].slot = ~0u;
    return made;
}

// the fire-and-forget update of one resolved entry (or its overflow-list entry)
__device__ __forceinline__ void apply_entry(const ScanArgs& a, const Resolved& r, u64 key, u32 cnt, u64 ord) {
    const Table& T = a.tabv;
    if (r.slot == ~0u) {  // probe bound exceeded: the overflow list (reinserted after a rehash)
        const u64 i = atomicAdd((unsigned long long*)&a.st->n_overflow, 1ull);
        if (i < T.ovf_cap) {
            Overflow o;
            o.key = key;
            o.count = cnt;
            o.first = ord;
            o.tag = a.file_tag;
            o.pad = 0;
            T.ovf[i] = o;
        } else {
            atomicOr(&a.st->cap_flags, 2u);
        }
        return;
    }
    GSlot* sl = &T.slots[r.slot];
    if (ABLATE & 128u) {  // timing ablation: plain stores instead of atomics (wrong counts)
        sl->count = cnt;
        return;
    }
    atomicAdd((unsigned long long*)&sl->count, (unsigned long long)cnt);
    if (ord < r.first) atomicMin((unsigned long long*)&sl->first, (unsigned long long)ord);
    if (r.tag < a.file_tag) atomicMax(&sl->last_tag, a.file_tag);
}

struct Geom {  // the launch's chunk geometry (ScanArgs' normal or heavy set, chosen at the kernel start)
    u32 chunk_tiles, mid_chunks, num_chunks, down_g;
};
// After a chunk's commit (one lane): the launch's last commit decides the next launch's geometry
// from the device's own counters (no host snapshot): heavy when at least a quarter of the chunks
// since the reset sent their commits to the launch log.  Exotic-only replays leave it alone.
__device__ __forceinline__ void note_commit(const ScanArgs& a, const Geom& g, bool hv) {
    if (a.exo_only) return;
    // relaxed: the decision is a performance heuristic (a stale log_commits only delays a switch), and
    // a release here would write back the XCD's L2 once per chunk (MI355X_MICROARCH.md fence table)
    const u32 prev = __hip_atomic_fetch_add(&a.st->commits_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev != g.num_chunks - 1u) return;
    const u64 tot = __hip_atomic_load(&a.st->chunks_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + g.num_chunks;
    const u64 lc = __hip_atomic_load(&a.st->log_commits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&a.st->chunks_total, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&a.st->heavy[a.par ^ 1u], (lc && lc * 4 >= tot) ? 1u : 0u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    if (hv) __hip_atomic_fetch_add(&a.st->heavy_launches, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&a.st->commits_done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// publish the LDS table and the cold list / buffered side effects into HBM (all threads): resolve
// every entry's slot, then add (resolve_batch / apply_entry), or append them to the launch log.
__device__ __attribute__((noinline)) void commit_buffers(ScanShared& sh, const ScanArgs& a, int tid, const Geom& g,
                                                        bool hv) {
#if defined(FR_STAMPS) && FR_STAMPS == 2
    u64 cst_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    u64 cq_ = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();
    FR_CSTAMP(0);
    u32 made = 0;
    if (ABLATE & 64u) {  // diag: flushed LDS slots and cold entries per commit
        u32 live = 0;
        for (int i = tid; i < NS; i += WG) live += sh.ls[i].key != 0;
        if (live) atomicAdd((unsigned long long*)&a.st->stamp[4], (unsigned long long)live);
        if (tid == 0) atomicAdd((unsigned long long*)&a.st->stamp[5], (unsigned long long)min(sh.ncold, a.cold_cap));
        if (tid == 0) atomicAdd((unsigned long long*)&a.st->stamp[6], 1ull);
    }
    const bool flush = !(ABLATE & 8u);  // ablation 8: no HBM flush of the LDS table / cold list
    const u64 cb = sh.cbase;  // LDS offsets are chunk offsets
    const u32 nc = flush ? min(sh.ncold, a.cold_cap) : 0u;
    const u32 nl = flush ? sh.nkeys : 0u;  // claimed LDS slots = the live ones
    // heavy commits (at least log_min pairs: many distinct codes per chunk) go to the launch log,
    // aggregated after the launch; lighter ones insert straight into the table
    bool logged = false;
    const u64* cl = a.cold + 2ull * (u64)blockIdx.x * a.cold_cap;
    // LDS scratch of the logged commit (the walks are done): per-region run counters
    u32* rcnt = &sh.raw[0][0];
    u32* rcur = rcnt + LOG_NB;
    u32* rbase = rcur + LOG_NB;  // each bucket's run start in its part of the log
    static_assert(3 * LOG_NB * 4 <= sizeof(sh.raw), "log bucket scratch");
    u32* bcur = LOG_DIRECT ? a.st->log_scur : a.st->log_rcur;  // the buckets' cursors (sub-regions or regions)
    constexpr int CB = 8;  // cold entries per lane with their loads in flight together
    // a logged commit sends its hot codes (chunk count >= log_hot: few per chunk, their slots L2-warm)
    // straight to the table; the tail goes to the log, one run per region appended to the region's part
    if (a.log && nl + nc && nl + nc >= a.log_min) {
        for (int i = tid; i < LOG_NB; i += WG) rcnt[i] = rcur[i] = 0;
        __syncthreads();
        for (int i = tid; i < NS; i += WG) {
            const LSlot e = sh.ls[i];
            if (e.key && e.cnt < a.log_hot) atomicAdd(&rcnt[log_bucket(e.key)], 1u);
        }
        for (u32 i0 = tid; i0 < nc; i0 += CB * WG) {
            u64 k[CB];
#pragma unroll
            for (int q = 0; q < CB; ++q) k[q] = i0 + q * WG < nc ? cl[2 * (i0 + q * WG)] : 0ull;
#pragma unroll
            for (int q = 0; q < CB; ++q)
                if (i0 + q * WG < nc) atomicAdd(&rcnt[log_bucket(k[q])], 1u);
        }
        if (tid == 0) sh.log_on = 0;
        __syncthreads();
        FR_CSTAMP(1);
        {  // one claim per region with a run, all in flight together
            constexpr int PR = (LOG_NB + WG - 1) / WG;
            u32 n[PR], base[PR], tot = 0;
#pragma unroll
            for (int j = 0; j < PR; ++j) {
                const int r = tid + j * WG;
                n[j] = r < LOG_NB ? rcnt[r] : 0u;
                tot += n[j];
            }
#pragma unroll
            for (int j = 0; j < PR; ++j) base[j] = n[j] ? atomicAdd(&bcur[tid + j * WG], n[j]) : 0u;
#pragma unroll
            for (int j = 0; j < PR; ++j)
                if (tid + j * WG < LOG_NB) rbase[tid + j * WG] = base[j];
            if (tot) atomicAdd(&sh.log_on, tot);
        }
        __syncthreads();
        FR_CSTAMP(2);
        if (tid == 0 && sh.log_on) {
            atomicAdd((unsigned long long*)&a.st->log_n, (unsigned long long)sh.log_on);
            atomicAdd((unsigned long long*)&a.st->log_commits, 1ull);
        }
        logged = sh.log_on != 0;  // else (nothing but hot codes) every pair inserts directly
    } else if (!a.log && !a.exo_only && tid == 0 && nl + nc && nl + nc >= a.log_min) {
        // a launch without a log (fr_tuning log = 0): count the commit that would have logged (note_commit's
        // heavy-geometry decision sees it)
        atomicAdd((unsigned long long*)&a.st->log_commits, 1ull);
    }
    if (logged) {
        constexpr int CL = NS / WG;
        const u64 ord0 = make_ord(a, 0);
        // a pair past its region's end inserts directly (the region's claimed range up to its end is
        // always written: the aggregation reads min(cursor, log_rcap) entries)
        auto put = [&](u64 k, u64 off, u32 cnt) {
            const u32 r = log_bucket(k);
            const u64 pos = (u64)rbase[r] + atomicAdd(&rcur[r], 1u);
            const bool fits = cnt <= LOG_CNT_MAX;  // (a chunk holds fewer records unless its geometry is extreme)
            if (pos < a.log_rcap) a.log[(u64)r * a.log_rcap + pos] = fits ? LogEntry{k, log_pack(off, cnt)} : LogEntry{0, 0};
            if (pos >= a.log_rcap || !fits) {  // (a zero key is skipped by the aggregation)
                const u64 k1[1] = {k};
                const bool v1[1] = {true};
                Resolved r1[1];
                made += resolve_batch<1>(a, k1, v1, r1);
                apply_entry(a, r1[0], k, cnt, make_ord(a, off));  // (off: a launch offset, or a multiple of 4 past ord0)
            }
        };
        u64 hk[CL];
        bool hv[CL];
#pragma unroll
        for (int b = 0; b < CL; ++b) {
            const LSlot e = sh.ls[tid + b * WG];
            hv[b] = e.key && e.cnt >= a.log_hot;
            hk[b] = e.key;
            if (e.key && !hv[b]) put(e.key, cb + e.mino, e.cnt);  // launch offsets (a logged range may exceed 4 GiB)
        }
        for (u32 i0 = tid; i0 < nc; i0 += CB * WG) {
            u64 k[CB], o[CB];
#pragma unroll
            for (int q = 0; q < CB; ++q) {
                const u32 i = i0 + q * WG;
                k[q] = i < nc ? cl[2 * i] : 0ull;
                o[q] = i < nc ? cl[2 * i + 1] : 0ull;
            }
#pragma unroll
            for (int q = 0; q < CB; ++q)
                if (i0 + q * WG < nc) put(k[q], o[q] - ord0, 1u);
        }
        Resolved rh[CL];
        made += resolve_batch<CL>(a, hk, hv, rh);
#pragma unroll
        for (int b = 0; b < CL; ++b) {
            if (!hv[b]) continue;
            const LSlot e = sh.ls[tid + b * WG];
            apply_entry(a, rh[b], e.key, e.cnt, make_ord(a, cb + e.mino));
        }
    } else if (flush) {
        constexpr int CL = NS / WG;  // LDS slots per lane; also cold entries per lane per batch
        Resolved* park = (Resolved*)&sh.raw[0][0];  // the walks are done: the tile area holds NS resolutions
        static_assert(sizeof(Resolved) * NS <= sizeof(sh.raw), "resolution parking");
        // the first cold batch's HBM reads lead: they land while the LDS slots resolve
        u64 ck[CL], co[CL];
        bool cv[CL];
#pragma unroll
        for (int b = 0; b < CL; ++b) {
            const u32 i = tid + b * WG;
            cv[b] = i < nc;
            ck[b] = cv[b] ? cl[2 * i] : 0;
            co[b] = cv[b] ? cl[2 * i + 1] : 0;
        }
        Resolved rc[CL];
#if defined(FR_COMMIT_JOINT)  // the LDS slots and the first cold batch resolved in one set of rounds
        {
            u64 jk[2 * CL];
            bool jv[2 * CL];
            Resolved jr[2 * CL];
#pragma unroll
            for (int b = 0; b < CL; ++b) {
                jk[b] = sh.ls[tid + b * WG].key;
                jv[b] = jk[b] != 0;
                jk[CL + b] = ck[b];
                jv[CL + b] = cv[b];
            }
            made += resolve_batch<2 * CL>(a, jk, jv, jr);
#pragma unroll
            for (int b = 0; b < CL; ++b) {
                park[tid + b * WG] = jr[b];
                rc[b] = jr[CL + b];
            }
        }
        FR_CSTAMP(1);
        FR_CSTAMP(2);
#else
        {
            u64 lk[CL];
            bool lv[CL];
            Resolved rs[CL];
#pragma unroll
            for (int b = 0; b < CL; ++b) {
                lk[b] = sh.ls[tid + b * WG].key;
                lv[b] = lk[b] != 0;
            }
            made += resolve_batch<CL>(a, lk, lv, rs);
#pragma unroll
            for (int b = 0; b < CL; ++b) park[tid + b * WG] = rs[b];
        }
        FR_CSTAMP(1);
        made += resolve_batch<CL>(a, ck, cv, rc);
        FR_CSTAMP(2);
#endif
        // every slot is known: the updates, none waited for
#pragma unroll
        for (int b = 0; b < CL; ++b) {
            const LSlot e = sh.ls[tid + b * WG];
            if (e.key) apply_entry(a, park[tid + b * WG], e.key, e.cnt, make_ord(a, cb + e.mino));
        }
#pragma unroll
        for (int b = 0; b < CL; ++b)
            if (cv[b]) apply_entry(a, rc[b], ck[b], 1u, co[b]);
        // a cold list of more than NS entries: further batches, each resolved, then applied
        for (u32 c0 = CL * WG; c0 < nc; c0 += CL * WG) {
#pragma unroll
            for (int b = 0; b < CL; ++b) {
                const u32 i = c0 + tid + b * WG;
                cv[b] = i < nc;
                ck[b] = cv[b] ? cl[2 * i] : 0;
                co[b] = cv[b] ? cl[2 * i + 1] : 0;
            }
            made += resolve_batch<CL>(a, ck, cv, rc);
#pragma unroll
            for (int b = 0; b < CL; ++b)
                if (cv[b]) apply_entry(a, rc[b], ck[b], 1u, co[b]);
        }
    }
    if (made) atomicAdd(&sh.created, made);
    // buffered exotic records and the first "no space" error
    const u32 ne = min(sh.nexo, (u32)EXO_BUF);
    for (u32 k = tid; k < ne; k += WG) {
        const u64 n = sh.exo_len[k];
        const u64 i = atomicAdd((unsigned long long*)&a.st->n_exotic, 1ull);
        const u64 po = atomicAdd((unsigned long long*)&a.st->exo_pool_used, (unsigned long long)n);
        if (i < a.tabv.exo_cap && po + n <= a.tabv.exo_pool_cap) {
            a.tabv.exo_ord[i] = make_ord(a, cb + sh.exo_p[k]);
            a.tabv.exo_off[i] = po;
            a.tabv.exo_len[i] = (u32)n;
            for (u64 q = 0; q < n; ++q) a.tabv.exo_pool[po + q] = a.buf[cb + sh.exo_start[k] + q];
        } else {
            atomicOr(&a.st->cap_flags, 4u);
        }
    }
    if (tid == 0 && sh.err_off != 0xFFFFFFFFu)
        atomicMin((unsigned long long*)&a.st->err_nospace, (unsigned long long)(a.file_offset + cb + sh.err_off));
    // (in here, not in the chunk loop: lane-divergent code at the loop's end made the structurizer move
    // it out of the loop, past the ticket barrier, for one lane)
    if (tid == 0) note_commit(a, g, hv);
    FR_CSTAMP(3);
    // LDS-only barriers from here: the commit's count atomics, log entries and exotic bytes stay in
    // flight (no later read in this launch needs them), while the LDS table is reset for the next chunk
    lds_barrier();
    FR_CSTAMP(4);
    for (int i = tid; i < NS; i += WG) sh.ls[i] = LSlot{0, 0, 0xFFFFFFFFu};
    if (tid == 0) {
        sh.nkeys = 0;
        sh.ncold = 0;
        sh.nexo = 0;
        sh.err_off = 0xFFFFFFFFu;
        sh.spec_bad = 0;
    }
    lds_barrier();
#if defined(FR_STAMPS) && FR_STAMPS == 2
    FR_CSTAMP(5);
    cst_[6] = nl;
    cst_[7] = nc;
    if ((tid & 63) == 0)
        for (int i_ = 0; i_ < 8; ++i_) atomicAdd((unsigned long long*)&a.st->stamp[i_], (unsigned long long)cst_[i_]);
#endif
}

// drop everything buffered (a redone chunk)
__device__ __forceinline__ void discard_buffers(ScanShared& sh, int tid) {
    __syncthreads();
    for (int i = tid; i < NS; i += WG) sh.ls[i] = LSlot{0, 0, 0xFFFFFFFFu};
    if (tid == 0) {
        sh.nkeys = 0;
        sh.ncold = 0;
        sh.nexo = 0;
        sh.err_off = 0xFFFFFFFFu;
        sh.spec_bad = 0;
    }
    __syncthreads();
}

__device__ __forceinline__ bool uniform_flag(u32 v) { return __builtin_amdgcn_readfirstlane(v) != 0; }

// code bytes at [start, start + n) of the wave's LDS copy -> fast key with v_perm SWAR, 4 bytes per
// step (false if outside the fast alphabet).  Byte index i = (c >> 1) & 7 selects the expected
// byte (A C T G - + - N) and its symbol (A1 C2 G3 T4 N5 +6); a byte is valid iff it equals the
// expected one.  Eight dwords from start & ~3 (bytes past the tile read the next area; masked off).
__device__ __forceinline__ void encode_load_lds(const ScanShared& sh, u32 wid, u32 start, u32 (&w)[8]) {
    const lds_u32* p = (const lds_u32*)(&sh.raw[wid][0]) + (start >> 2);
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = p[k];
}

__device__ __forceinline__ bool encode_pack(const u32 (&w)[8], u32 start, u32 n, u64& key) {
    if (n < 1 || n > (u32)MAXSYM) return false;
    const u32 sh = start & 3u;
    u64 kk = 0;
    u32 bad = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const u32 x = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);  // code bytes 4k .. 4k+3
        const u32 idx = (x >> 1) & 0x07070707u;
        const u32 expect = __builtin_amdgcn_perm(0x4E002B00u, 0x47544341u, idx);
        const u32 sym = __builtin_amdgcn_perm(0x05000600u, 0x03040201u, idx);
        const int left = (int)n - 4 * k;  // bytes of the code in this word
        const u32 vm = left >= 4 ? 0xFFFFFFFFu : left <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * left));
        bad |= (expect ^ x) & vm;
        const u32 sv = sym & vm;
        const u32 packed = __builtin_amdgcn_udot4(sv, 0x00400801u, (sv >> 15) & 0xE00u, false);
        kk |= (u64)packed << (12 * k);
    }
    key = kk;
    return bad == 0;
}

// the rare header outcomes (chunk offsets): word-scan fallback, no ' ' (IndexError), or an exotic code
__device__ FR_COLD void slow_header(ScanShared& sh, const ScanArgs& a, u32 p, int r, u32 start, u32 n) {
    if (r == 2) process_header_global(sh, a, p);
    else if (r == 1) nospace(a, p, sh);
    else exotic_record(a, p, sh.cbase + start, n, sh);
}

// ---- header parse: two 64-bit bitmap windows, wave-uniform code length encode ---------------
// v_ffbl / v_ffbh return ~0 for 0, which the min tricks below rely on; the builtins add a
// compare and select per word (or make the zero case undefined).
__device__ __forceinline__ u32 ffbl32(u32 x) {
    u32 r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ u32 ffbh32(u32 x) {
    u32 r;
    asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ u32 ctz64x(u64 x) { return min(ffbl32((u32)x), ffbl32((u32)(x >> 32)) | 32u); }  // ~0: none
// index of the highest set bit; negative (-64) when none
__device__ __forceinline__ int hsb64x(u64 x) { return (int)(min(ffbh32((u32)(x >> 32)), ffbh32((u32)x) | 32u) ^ 63u); }

// bits [b, b + 64) of the 128-bit (x0, x1), b in [0, 63]
__device__ __forceinline__ u64 window64(u64 x0, u64 x1, u32 b) { return (x0 >> b) | ((x1 << 1) << (63u - b)); }

// R2 on the wave-tile's bitmaps in two 64-bit windows: from the line start p the first ' ' or line
// end f1 (a line end first: no ' ', IndexError); from the token start q = f1 + 1 the token end f2
// and the last ':' before it.  0: code at [start, start + n) (tile offsets); 1: no ' '; 2: word-scan
// fallback (the first ' ' or the token end lies 64 or more bytes on, or the token starts past the
// staged bytes).
__device__ __forceinline__ int locate_code(const ScanShared& sh, u32 wid, u32 p, u32 bl, u32& start, u32& n) {
    // One LDS round for both windows: the token start q < p + 64 lies in word w or w + 1, so words w .. w + 2
    // hold everything either window reads (the loads go out together, before any branch; w <= 63 keeps
    // w + 2 inside the SEGS + 2 words).  Round 4 read the second window's words after the first window's
    // test: two dependent LDS round trips per header, each a bitmap pair at a time (four waits).
    const u32 w = min(p >> 6, (u32)SEGS - 1u), b = p & 63u;
    const lds_u64* S = (const lds_u64*)&sh.bsp[wid][w];
    const lds_u64* E = (const lds_u64*)&sh.beol[wid][w];
    const lds_u64* C = (const lds_u64*)&sh.bcol[wid][w];
    u64 s0 = S[0], s1 = S[1], s2 = S[2], e0 = E[0], e1 = E[1], c0 = C[0], c1 = C[1], c2 = C[2];
    // all eight in registers here: the compiler would otherwise sink each load into the branch that uses
    // it (one wait per load again)
    asm volatile("" : "+v"(s0), "+v"(s1), "+v"(s2), "+v"(e0), "+v"(e1), "+v"(c0), "+v"(c1), "+v"(c2));
    if (p >= bl) return 2;
    const u64 se = window64(s0, s1, b);
    const u64 eo = window64(e0, e1, b);
    const u32 f1 = ctz64x(se);
    const u32 q = p + f1 + 1u;
    if (f1 >= 64u) return 2;
    if (ctz64x(eo) == f1) return 1;
    if (q >= bl) return 2;
    const bool nxt = (q >> 6) != w;  // the token starts in word w + 1
    const u32 b2 = q & 63u;
    const u64 se2 = window64(nxt ? s1 : s0, nxt ? s2 : s1, b2);
    const u64 co2 = window64(nxt ? c1 : c0, nxt ? c2 : c1, b2);
    const u32 f2 = ctz64x(se2);
    if (f2 >= 64u) return 2;
    const int hc = hsb64x(co2 & ((1ull << f2) - 1ull));  // the last ':' of the token, < 0 none
    const u32 cs = (u32)max(hc + 1, 0);
    start = q + cs;
    n = f2 - cs;
    return 0;
}

// code bytes [start, start + n) from the wave's LDS copy -> fast key, n wave-uniform (nu): the
// per-word byte masks are scalars and only the words the code reaches are packed
__device__ __forceinline__ bool encode_uniform(const ScanShared& sh, u32 wid, u32 start, u32 nu, u64& key) {
    u32 w[8];
    encode_load_lds(sh, wid, start, w);
    const u32 al = start & 3u;
    u32 bad = 0, lo = 0, hi = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        if ((u32)(4 * k) >= nu) break;  // uniform
        const u32 x = __builtin_amdgcn_alignbyte(w[k + 1], w[k], al);
        const u32 idx = (x >> 1) & 0x07070707u;
        const u32 expect = __builtin_amdgcn_perm(0x4E002B00u, 0x47544341u, idx);
        u32 sym = __builtin_amdgcn_perm(0x05000600u, 0x03040201u, idx);
        const u32 left = nu - 4u * k;
        if (left >= 4u) {
            bad |= expect ^ x;
        } else {
            const u32 vm = 0xFFFFFFFFu >> (32u - 8u * left);  // uniform
            bad |= (expect ^ x) & vm;
            sym &= vm;
        }
        const u32 packed = __builtin_amdgcn_udot4(sym, 0x00400801u, (sym >> 15) & 0xE00u, false);
        if (k == 0) lo = packed;
        else if (k == 1) lo |= packed << 12;
        else if (k == 2) { lo |= packed << 24; hi = packed >> 8; }
        else hi |= packed << (12 * k - 32);
    }
    key = ((u64)hi << 32) | lo;
    return bad == 0;
}

// R2 from the line start p in ONE window of the ' ' | line-end bitmap and one of the ':' bitmap (round 6):
// f1 = the first ' ' or line end, the token end = the next one (the window's second set bit), the code
// start = one past the last ':' before the token end, or the token start when the token has none.  The
// byte at f1 tells a ' ' from a line end (IndexError), read from the wave's tile copy with the code.
// Branch-free: 0 code at [start, start + n) (tile offsets); 2 word-scan fallback (the line starts past the
// staged bytes, or no ' ' / line end within 64 bytes); 3 the token ends past the window (a first token of
// 40-odd bytes: Illumina instrument headers), which locate_code finishes from the token start.
__device__ __forceinline__ int locate_near(const ScanShared& sh, u32 wid, u32 p, u32 bl, u32& start, u32& n, u32& f1) {
    const u32 w = min(p >> 6, (u32)SEGS - 1u), b = p & 63u;
    const lds_u64* S = (const lds_u64*)&sh.bsp[wid][w];
    const lds_u64* C = (const lds_u64*)&sh.bcol[wid][w];
    u64 s0 = S[0], s1 = S[1], c0 = C[0], c1 = C[1];
    asm volatile("" : "+v"(s0), "+v"(s1), "+v"(c0), "+v"(c1));  // one LDS round, before any use
    const u64 se = window64(s0, s1, b);
    const u64 co = window64(c0, c1, b);
    const u64 se1 = se & (se - 1ull);
    f1 = ctz64x(se);
    const u32 f2 = ctz64x(se1);
    const int hc = hsb64x(co & ((1ull << (f2 & 63u)) - 1ull));  // the last ':' before the token end (< 0: none)
    const u32 cs = (u32)max(hc, (int)f1) + 1u;                  // a ':' of the first token does not count
    start = p + cs;
    n = f2 - cs;
    return (p >= bl || se == 0ull) ? 2 : (se1 == 0ull ? 3 : 0);
}

__device__ __forceinline__ void parse_header(ScanShared& sh, const ScanArgs& a, u32 wid, u32 tile0, u32 p, u32 bl) {
    u32 start = 0, n = 0, f1 = 0;
    int r = locate_near(sh, wid, p, bl, start, n, f1);
    if (__ballot(r == 3) != 0) {  // uniform: some lane's token ends past its first window
        if (r == 3) {
            r = locate_code(sh, wid, p, bl, start, n);  // decides "no ' '" itself
            f1 = 0xFFFFFFFFu;
        }
    }
    // the first delimiter's byte (in the staged bytes whenever r == 0 and f1 < 64): not a ' ' -> a line end
    const u32 dch = *((const lds_u8*)&sh.raw[wid][0] + min(p + f1, (u32)TILE - 1u));
    if (ABLATE & 2u) {
        asm volatile("" ::"v"(start), "v"(n), "v"(r), "v"(dch));
        return;
    }
    u64 key = 0;
    bool fast = false;
    if (r == 0 && n >= 1u && n <= (u32)MAXSYM) {
        const u32 nu = __builtin_amdgcn_readfirstlane(n);
        if (__ballot(n != nu) == 0) {
            fast = encode_uniform(sh, wid, start, nu, key);  // the common case
        } else {
            u32 w[8];
            encode_load_lds(sh, wid, start, w);
            fast = encode_pack(w, start, n, key);
        }
    }
    if (r == 0 && f1 < 64u && dch != (u32)' ') {  // the line ends before any ' ': IndexError (:169)
        r = 1;
        fast = false;
    }
    if (fast) count_code(sh, a, tile0 + p, key);
    else rare_push(sh, a, tile0 + p, (u32)r, tile0 + start, n);
}

// The line starts after every 4th terminator (lines == 0 mod 4) in this lane's segment, parsed
// where they lie.  L0 = lines before the wave-tile (absolute with -s, else mod 4 suffices).  The
// first header needs the skip-th set bit of the terminator mask; a second one in the same segment
// (records shorter than 64 B) takes the loop at the end.
template <bool LIM>
__device__ __forceinline__ void parse_own_headers(ScanShared& sh, const ScanArgs& a, u32 t, u32 ct,
                                                  const SegClass& sc, u64 L0, int lane, u32 wid) {
    const u64 tile0 = (u64)t * TSTEP;
    const u32 tile0c = (t - ct) * TSTEP;  // the tile's chunk offset (ct: the chunk's first tile)
    const u32 bl = (u32)min((u64)TILE, a.avail - tile0);
    const u64 rem64 = a.len - tile0;  // line starts p < pend are this launch's (uniform)
    const u32 pend = rem64 >= 0xFFFFFFFFull ? 0xFFFFFFFFu : (u32)rem64 + ((a.own_end && a.len < a.avail) ? 1u : 0u);
    const u32 lb = (u32)L0 + (sc.x - sc.c);  // terminators before this segment (low bits)
    const u32 skip = (3u - lb) & 3u;
    const u32 s0 = lane * SEG;
    u64 m = sc.tmask;
#pragma unroll
    for (u32 q = 0; q < 3; ++q) {
        const u64 d = m & (m - 1ull);
        m = q < skip ? d : m;
    }
    constexpr bool limited = LIM;  // -s (a.max_records > 0): the kernel instance's, so the common one has no record limit
    u64 rec = 0;
    if (limited) rec = (L0 + (sc.x - sc.c) + skip + 1u) >> 2;
    // the range's own first line start (position 0): lane 0 of the range's first tile; the rest is wave-uniform
    const bool own0s = t == 0 && a.own_start && (L0 & 3ull) == 0 && a.avail > 0 &&
                       (!limited || (i64)(L0 >> 2) < a.max_records);
    const bool own0 = own0s && lane == 0;
    // m's lowest set bit: the first header terminator.  own0's header at position 0 comes first.
    const u32 p = own0 ? 0u : s0 + ctz64x(m) + 1u;
    const bool ok = own0 || (m != 0 && p < pend && (!limited || (i64)rec < a.max_records));
    if (ok) parse_header(sh, a, wid, tile0c, p, bl);
    // another header in this segment (records shorter than 64 B; never at R=8's 74 B): uniform check
    bool more = ok && (own0 ? m != 0 : __popcll(m) > 4);
    if (!__ballot(more)) return;
    if (!own0) {
        m &= m - 1ull;
        m &= m - 1ull;
        m &= m - 1ull;
        m &= m - 1ull;
        ++rec;
    }
    while (__ballot(more)) {
        if (more) {
            const u32 pn = s0 + ctz64x(m) + 1u;
            more = pn < pend && (!limited || (i64)rec < a.max_records);
            if (more) parse_header(sh, a, wid, tile0c, pn, bl);
            ++rec;
            m &= m - 1ull;
            m &= m - 1ull;
            m &= m - 1ull;
            m &= m - 1ull;
            more = more && m != 0;
        }
    }
}

// One wave walks wave-tiles [tb, te) of the range; L0 = lines before tile tb (absolute, or only
// mod 4 without -s).  parse = false: count only.  Returns the line terminators in [tb, te).  No
// workgroup barrier: every LDS area the walk writes is this wave's.  Per step: the tile's bytes
// (in registers since the previous step) go to the wave's LDS copy first, so the registers take the
// next tile's loads at once and those stay in flight through this tile's classify AND its parse;
// the classify reads the lane's segment back from LDS.
template <bool LIM>
__device__ __forceinline__ u64 walk_wave(ScanShared& sh, const ScanArgs& a0, u32 ct, u32 tb, u32 te, u64 L0,
                                         bool parse, int lane, u32 wid) {
    const ScanArgs& a = a0;
    u64 lines = 0;
    u32 done = *(const volatile lds_u32*)&sh.rq_tail[wid];
    SegRegs r;
    if (tb < te) seg_load(a, tb, r, lane);
    lds_u32x4* mine = (lds_u32x4*)(&sh.raw[wid][0]) + lane * (SEG / 16);
    FR_WSTAMP_DECL
    for (u32 t = tb; t < te; ++t) {
#if defined(FR_STAMPS) && FR_STAMPS == 4
        FR_WSTAMP_RESET();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        FR_WSTAMP(0);
#endif
        // the previous tile's parse is done with the LDS copy (program order)
#pragma unroll
        for (int k = 0; k < SEG / 16; ++k) {
            u32x4 v;
            v.x = r.v[k].x; v.y = r.v[k].y; v.z = r.v[k].z; v.w = r.v[k].w;
            mine[k] = v;
        }
        if (t + 1 < te) seg_load(a, t + 1, r, lane);
        // volatile: a real LDS read, one quarter of the segment at a time inside the classify
        const SegClass sc = seg_classify_src(a, t, [&](int k) {
            const u32x4 v = *(const volatile lds_u32x4*)&mine[k];
            return make_uint4(v.x, v.y, v.z, v.w);
        }, lane);
        FR_WSTAMP(1);
        if (sc.hi) rare_push(sh, a, (t - ct) * TSTEP + lane * SEG, 4u,
                             min((u32)min((u64)TSTEP, a.len - (u64)t * TSTEP) - lane * SEG, (u32)SEG), 0u);
        const u32 tail = *(const volatile lds_u32*)&sh.rq_tail[wid];
        if (tail != done) {  // uniform: the previous tile's rare events (and this tile's UTF-8 checks)
            drain_rare(sh, a, wid, done, tail, lane);
            done = tail;
        }
        sh.bsp[wid][lane] = sc.sp | sc.eol;  // token ends: ' ' or line end
        sh.bcol[wid][lane] = sc.col;
        sh.beol[wid][lane] = sc.eol;
        lds_fence();
        // (a speculation buffer that overflowed mid-walk, sh.spec_bad, is not checked per tile: the chunk is
        // redone exactly and everything its walk buffered is discarded, so parsing on is harmless; the check
        // was an LDS round trip per tile)
        FR_WSTAMP(2);
        if (parse && !(ABLATE & 1u)) parse_own_headers<LIM>(sh, a, t, ct, sc, L0 + lines, lane, wid);
        lines += sc.wtot;
        FR_WSTAMP(3);
    }
    FR_WSTAMP_FLUSH(te > tb ? te - tb : 0u);
    lds_fence();
    const u32 tail = *(const volatile lds_u32*)&sh.rq_tail[wid];
    if (tail != done) drain_rare(sh, a, wid, done, tail, lane);
    return lines;
}

// Tiles [tb, te) of chunk c.  Uniform: chunk_tiles each.  Ramped (ramp_g = G > 0, C = chunk_tiles,
// s = the ramp's smallest chunk): R_s(j) = s j + floor((C-s) j (j+1) / 2G) tiles precede ramp-up
// chunk j, so chunk j holds s + ~(C-s)(j+1)/G tiles and the G first chunks, all taken at once, finish
// in ticket order; mid_chunks full chunks follow; the last Gd = ramp_down_g chunks shrink the same way
// (over Gd chunks, smallest ramp_down_s), so every workgroup runs out of work at about the same time.  fr_api only ramps
// ranges of >= R_up(G) + R_down(G) + C tiles (ramp_prefix in fr_internal.h, shared with the host).
__device__ __forceinline__ u64 ramp_prefix(const Geom& g, u64 G, u64 j, u32 s0) {
    return ramp_tiles_before(g.chunk_tiles, G, s0, j);
}

// Run by the workgroup that finishes the launch's last chunk: the exact line prefix of every chunk
// (exclusive scan of the published counts), checked against the phase each committed speculative
// chunk guessed; writes the range's line total for the next launch.
__device__ __attribute__((noinline)) void verify_launch(ScanShared& sh, const ScanArgs& a, u32 n, u64 base_lines,
                                                       int tid) {
    const u32 per = (n + WG - 1) / WG;
    const u32 lo = min(tid * per, n), hi = min(lo + per, n);
    u64 sum = 0;
    for (u32 c = lo; c < hi; ++c) sum += (u32)agent_load(&a.chunk_info[c]);
    // block exclusive scan of the per-thread sums (the wave counts are free scratch here)
    u64 x = sum;
    const int lane = tid & 63, wid = tid >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const u64 y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) sh.wcount[wid] = x;
    __syncthreads();
    u64 before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const u64 v = sh.wcount[w];
        before += w < wid ? v : 0ull;
        total += v;
    }
    u64 run = base_lines + before + (x - sum);
    bool bad = false;
    for (u32 c = lo; c < hi; ++c) {
        const u64 info = agent_load(&a.chunk_info[c]);
        const u32 f = (u32)(info >> 32);
        if ((f & 1u) && ((f >> 1) & 3u) != (u32)(run & 3ull)) bad = true;
        run += (u32)info;
    }
    if (bad) atomicOr(&a.st->spec_fail, 1u);
    if (tid == 0) a.st->lines[a.par ^ 1u] = base_lines + total;
    __syncthreads();
}

__device__ __forceinline__ void chunk_bounds(const ScanArgs& a, const Geom& g, u32 c, u32& tb, u32& te) {
    if (a.ramp_g == 0) {
        tb = min(c * g.chunk_tiles, a.num_tiles);
        te = min(tb + g.chunk_tiles, a.num_tiles);
        return;
    }
    const u32 su = min(a.ramp_up_s, g.chunk_tiles), sd = min(a.ramp_down_s, g.chunk_tiles);
    const u64 G = a.ramp_g, Gd = g.down_g;
    const u64 rg = ramp_prefix(g, G, G, su), mid_end = (u64)a.num_tiles - ramp_prefix(g, Gd, Gd, sd);
    if (c < G) {
        tb = (u32)ramp_prefix(g, G, c, su);
        te = (u32)ramp_prefix(g, G, c + 1, su);
    } else if (c < G + g.mid_chunks) {
        const u64 b = rg + (u64)(c - G) * g.chunk_tiles;
        tb = (u32)b;
        te = (u32)min(b + g.chunk_tiles, mid_end);
    } else {
        const u64 j = c - G - g.mid_chunks;  // 0 .. Gd-1: shrinking
        tb = (u32)((u64)a.num_tiles - ramp_prefix(g, Gd, Gd - j, sd));
        te = (u32)((u64)a.num_tiles - ramp_prefix(g, Gd, Gd - j - 1, sd));
    }
}

#if defined(FR_STAMPS) && FR_STAMPS == 3  // diagnostic builds only: a timeline of every chunk and workgroup
constexpr u32 TRACE_CHUNKS = 1u << 14;  // per launch parity
constexpr u32 TRACE_WGS = 4096;
__device__ u64 g_chunk_trace[2 * TRACE_CHUNKS * 4];  // per ticket: {wg | xcc << 16 | tiles << 32, ticket, walked, committed}
__device__ u64 g_wg_trace[2 * TRACE_WGS * 2];        // per workgroup: {entry, exit} (s_memrealtime, 100 MHz)
__device__ __forceinline__ u32 xcc_id() {
    u32 x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 0xFu;
}
extern "C" int fr_trace_read(u64* chunks, u64* wgs) {
    if (hipMemcpyFromSymbol(chunks, HIP_SYMBOL(g_chunk_trace), sizeof(g_chunk_trace)) != hipSuccess) return 1;
    if (hipMemcpyFromSymbol(wgs, HIP_SYMBOL(g_wg_trace), sizeof(g_wg_trace)) != hipSuccess) return 1;
    return 0;
}
extern "C" int fr_trace_clear() {
    static u64 zero[2 * TRACE_CHUNKS * 4];
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_chunk_trace), zero, sizeof(g_chunk_trace)) != hipSuccess) return 1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_wg_trace), zero, sizeof(g_wg_trace)) != hipSuccess) return 1;
    return 0;
}
#endif

#ifndef FR_OCC
#define FR_OCC 4  // workgroups (= waves per SIMD) per CU: ~39 KB of LDS per workgroup (the wave-tile copies
                  // and the LDS table) fit 4 in a CU's 160 KB; fr_api sizes the grid with chunk_occupancy()
#endif
// LIM: -s (a.max_records > 0), the launch's instance (launch_chunk_scan): the record limit's checks are not in the
// common instance's tile loop
template <bool LIM>
__global__ __launch_bounds__(WG, FR_OCC) void chunk_kernel(ScanArgs args) {
    // every helper reads the arguments where they lie (the kernarg segment): the out-of-line
    // helpers take them by reference without a scratch copy of the struct
    (void)args;
    const ScanArgs& a = *(const ScanArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    __shared__ ScanShared sh;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const u32 wid = wave_id();  // wave-uniform: LDS addresses by wave stay scalar
    for (int i = tid; i < NS; i += WG) sh.ls[i] = LSlot{0, 0, 0xFFFFFFFFu};
    if (lane == 0) {
        sh.bsp[wid][SEGS] = sh.bsp[wid][SEGS + 1] = 0;
        sh.bcol[wid][SEGS] = sh.bcol[wid][SEGS + 1] = 0;
        sh.beol[wid][SEGS] = sh.beol[wid][SEGS + 1] = 0;
        sh.rq_tail[wid] = 0;
    }
    if (tid == 0) {
        sh.nkeys = 0;
        sh.created = 0;
        sh.flags = 0;
        sh.spec = 0;
        sh.spec_bad = 0;
        sh.ncold = 0;
        sh.nexo = 0;
        sh.err_off = 0xFFFFFFFFu;
    }
#if defined(FR_STAMPS) && FR_STAMPS == 3
    if (tid == 0 && blockIdx.x < TRACE_WGS) g_wg_trace[(a.par * TRACE_WGS + blockIdx.x) * 2] = __builtin_amdgcn_s_memrealtime();
    u64 tl_t0 = 0;
#endif
    const u64 base_lines = a.st->lines[a.par];
    // the geometry: heavy when the previous launch said so (ramped launches that have a heavy set)
    const bool hv = a.num_chunks_h != 0 &&
                    __builtin_amdgcn_readfirstlane(__hip_atomic_load(&a.st->heavy[a.par], __ATOMIC_RELAXED,
                                                                     __HIP_MEMORY_SCOPE_AGENT)) != 0;
    const Geom g = hv ? Geom{a.chunk_tiles_h, a.mid_chunks_h, a.num_chunks_h, a.ramp_down_g_h}
                      : Geom{a.chunk_tiles, a.mid_chunks, a.num_chunks, a.ramp_down_g};
    constexpr bool limited = LIM;
#if defined(FR_STAMPS) && (FR_STAMPS == 1 || FR_STAMPS == 4)
    const u64 k0_ = __builtin_amdgcn_s_memtime();
#endif
    FR_STAMP_DECL
    for (;;) {
        if (tid == 0) {
            // every chunk goes by ticket, the first too: the chunk a look-back waits on is then always
            // held by a workgroup that is already running.  (Round 4 gave each workgroup its own index
            // as its first chunk; a resident workgroup could then wait on a chunk whose workgroup was not
            // dispatched yet -- a grid larger than the free CUs, or another process's kernels holding
            // them -- for a 0.2 % shorter launch head.)
            const u32 cn = atomicAdd(&a.st->ticket, 1u);
            sh.chunk = cn;
            if (cn < g.num_chunks) {  // the chunk's base for its offsets (published by the barrier)
                u32 tb0, te0;
                chunk_bounds(a, g, cn, tb0, te0);
                sh.cbase = (u64)tb0 * TSTEP;
            }
            sh.spec = 1u;  // pass 0 runs on guessed phases: side effects are buffered
        }
        __syncthreads();
        const u32 c = sh.chunk;
        FR_TRACE("w%d ticket %u of %u\n", (int)wid, c, g.num_chunks);
        if (c >= g.num_chunks) break;
        u32 tb, te;
        chunk_bounds(a, g, c, tb, te);
#if defined(FR_STAMPS) && FR_STAMPS == 3
        if (tid == 0) tl_t0 = __builtin_amdgcn_s_memrealtime();
#endif
        const u32 per = (te - tb + NW - 1) / NW;  // this wave's part of the chunk: [wb, we)
        const u32 wb = min(tb + wid * per, te), we = min(wb + per, te);
        // ---- pass 0: chunk 0's first wave starts at the range's exact line count; every other
        // wave guesses its phase (count only when unsure, and with -s or an exotic-only replay) --
        u64 L0 = 0;
        bool parse = false;
        FR_STAMP(3);
        if (wb < we) {
            if (c == 0 && wid == 0) {
                L0 = base_lines;
                parse = true;
            } else if (!limited && !a.exo_only) {
                const int P = guess_phase(sh, a, wb, lane, wid);
                parse = P >= 0;
                L0 = (u64)max(P, 0);
            }
        }
        FR_STAMP(0);
#if defined(FR_STAMPS) && FR_STAMPS == 1
        st_[7] += 1;
#endif
        // One walk site, several passes.  Pass 0 as above.  Then each wave's start follows from the
        // chunk start and the earlier waves' pass-0 counts: a wave that parsed on another phase (or a
        // buffer that overflowed) makes every wave redo; a wave that only counted walks again.  The
        // chunk start is exact (chunk 0, or a decoupled look-back) or, for a device feed, the first
        // wave's guess, committed at once (verify_launch checks it); a speculation buffer that
        // overflows on a guessed start sends the chunk to the look-back and an exact redo.
        bool run = wb < we, exact = true, force = false;
        u64 base = base_lines;
        for (int pass = 0;; ++pass) {
            FR_TRACE("w%d pass %d run %d [%u,%u) parse %d\n", (int)wid, pass, (int)run, wb, we, (int)parse);
            const u64 n = run ? walk_wave<LIM>(sh, a, tb, wb, we, L0, parse, lane, wid) : 0ull;
            FR_TRACE("w%d walked %llu\n", (int)wid, (unsigned long long)n);
            FR_STAMP(pass == 0 ? 1 : 4);
            if (pass == 0) {
                if (lane == 0) {
                    sh.wcount[wid] = n;
                    sh.wphase[wid] = run && parse ? (int)(L0 & 3ull) : -1;
                }
                __syncthreads();
                FR_STAMP(2);
                u64 total = 0;
#pragma unroll
                for (int w = 0; w < NW; ++w) total += sh.wcount[w];
                const int p0 = sh.wphase[0];
                const bool fast = a.spec_commit && c != 0 && p0 >= 0 && !uniform_flag(sh.spec_bad);
                if (tid == 0) {  // publish the chunk's line count
                    agent_store(&a.tiles[c], ((u64)(2u * a.epoch + (c == 0 ? 1u : 0u)) << 32) | (u32)total);
                    const u32 f = fast ? (1u | ((u32)p0 << 1)) : 0u;
                    agent_store(&a.chunk_info[c], ((u64)f << 32) | (u32)total);
                    // the sc1 (agent) stores drain before the count that signals them; verify_launch reads
                    // chunk_info with sc1 loads only (MI355X_MICROARCH.md, valid hand-off forms): no
                    // release fence, which would write back the XCD's L2 once per chunk
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    const u32 prev = __hip_atomic_fetch_add(&a.st->chunks_done, 1u, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
                    sh.last = prev == g.num_chunks - 1u;
                }
                exact = !fast;
                if (fast) {
                    base = (u64)p0;
                } else if (c != 0) {
                    if (wid == 0) {
                        const u64 ex = lookback(a, c, (u32)total, lane);
                        if (lane == 0) sh.tile_excl = ex;
                    }
                    __syncthreads();
                    base = base_lines + sh.tile_excl;
                }
            } else {
                __syncthreads();
                if (exact || !uniform_flag(sh.spec_bad)) break;
                // a speculation buffer overflowed on the guessed chunk start: look back, redo exactly
                u64 total = 0;
#pragma unroll
                for (int w = 0; w < NW; ++w) total += sh.wcount[w];
                if (wid == 0) {
                    const u64 ex = lookback(a, c, (u32)total, lane);
                    if (lane == 0) sh.tile_excl = ex;
                }
                __syncthreads();
                base = base_lines + sh.tile_excl;
                exact = true;
                force = true;
            }
            // plan the next pass from the pass-0 counts and phases (LDS: nothing held across the walk)
            u64 D = base;
            bool bad = force || uniform_flag(sh.spec_bad);
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                const int pw = sh.wphase[w];
                if (w == (int)wid) L0 = D;
                if (pw >= 0 && (u64)pw != (D & 3ull)) bad = true;
                D += sh.wcount[w];
            }
            run = wb < we && (bad || sh.wphase[wid] < 0);
            parse = true;
            if (bad) discard_buffers(sh, tid);
            if (tid == 0) sh.spec = exact ? 0u : 1u;
            __syncthreads();
        }
        FR_TRACE("w%d commit\n", (int)wid);
        FR_STAMP(3);
#if defined(FR_STAMPS) && FR_STAMPS == 3
        const u64 tl_t1 = __builtin_amdgcn_s_memrealtime();
#endif
        commit_buffers(sh, a, tid, g, hv);  // starts and ends with a barrier: sh.last is visible
#if defined(FR_STAMPS) && FR_STAMPS == 3
        if (tid == 0 && c < TRACE_CHUNKS) {
            u64* e = &g_chunk_trace[(a.par * TRACE_CHUNKS + c) * 4];
            e[0] = (u64)blockIdx.x | ((u64)xcc_id() << 16) | ((u64)(te - tb) << 32);
            e[1] = tl_t0;
            e[2] = tl_t1;
            e[3] = __builtin_amdgcn_s_memrealtime();
        }
#endif
        FR_TRACE("w%d committed last %u\n", (int)wid, sh.last);
        if (sh.last) {  // once per launch: the acquire is cheap here (chunk_info is read with sc1 loads anyway)
            __atomic_thread_fence(__ATOMIC_ACQUIRE);
            verify_launch(sh, a, g.num_chunks, base_lines, tid);
        }
        FR_STAMP(5);
    }
#if defined(FR_STAMPS) && FR_STAMPS == 1
    FR_STAMP_FLUSH(k0_);
#endif
#if defined(FR_STAMPS) && FR_STAMPS == 4
    if ((threadIdx.x & 63) == 0)
        atomicAdd((unsigned long long*)&a.st->stamp[5], (unsigned long long)(__builtin_amdgcn_s_memtime() - k0_));
#endif
#if defined(FR_STAMPS) && FR_STAMPS == 3
    if (tid == 0 && blockIdx.x < TRACE_WGS) g_wg_trace[(a.par * TRACE_WGS + blockIdx.x) * 2 + 1] = __builtin_amdgcn_s_memrealtime();
#endif
    __syncthreads();
    if (tid == 0) {
        if (sh.created) atomicAdd((unsigned long long*)&a.st->n_keys, (unsigned long long)sh.created);
        if (sh.flags & 1u) atomicOr(&a.st->nonascii, 1u);
        if (sh.flags & 2u) atomicOr(&a.st->utf8_bad, 1u);
        // every workgroup has taken its last ticket: the last one out zeroes the launch's counters
        // for the next launch (stream order makes the plain stores visible to it)
        if (atomicAdd(&a.st->exits, 1u) == gridDim.x - 1u) {
            a.st->ticket = 0;
            a.st->chunks_done = 0;
            a.st->exits = 0;
        }
    }
}

int chunk_occupancy() { return FR_OCC; }

hipError_t launch_chunk_scan(const ScanArgs& a, int grid, hipStream_t s) {
    if (a.max_records > 0) hipLaunchKernelGGL(chunk_kernel<true>, dim3(grid), dim3(WG), 0, s, a);
    else hipLaunchKernelGGL(chunk_kernel<false>, dim3(grid), dim3(WG), 0, s, a);
    return hipGetLastError();
}


// ------------------------------------------------------------------------------------
// table maintenance
// ------------------------------------------------------------------------------------
__global__ void table_init_kernel(GSlot* slots, u64 n) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        GSlot g;
        g.key = 0;
        g.count = 0;
        g.first = ~0ull;
        g.last_tag = 0;
        g.uidx = 0;
        slots[i] = g;
    }
}

hipError_t launch_table_init(GSlot* slots, u64 n, hipStream_t s) {
    const int grid = (int)std::min<u64>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(table_init_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, slots, n);
    return hipGetLastError();
}

// re-insert overflow entries (after the table has grown); presence is re-derived
__global__ void reinsert_kernel(Table t, DevState* st, const Overflow* src, u64 n) {
    u32 made = 0;
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const Overflow o = src[i];
        made += global_insert(t, st, o.key, o.count, o.first, o.tag) ? 1u : 0u;
    }
    add_created(st, made);
}

hipError_t launch_reinsert_overflow(Table t, DevState* st, const Overflow* src, u64 n, hipStream_t s) {
    if (!n) return hipSuccess;
    const int grid = (int)std::min<u64>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(reinsert_kernel, dim3(grid), dim3(256), 0, s, t, st, src, n);
    return hipGetLastError();
}

// move every live slot of an old table into a bigger one (keeps count/first/last_tag)
__global__ void rehash_kernel(Table t, const GSlot* src, u64 nsrc) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < nsrc; i += (u64)gridDim.x * blockDim.x) {
        const GSlot g = src[i];
        if (!g.key) continue;
        u64 h = table_home(g.key, t.mask);
        for (;;) {
            const u64 old = atomicCAS((unsigned long long*)&t.slots[h].key, 0ull, (unsigned long long)g.key);
            if (old == 0) {
                t.slots[h].count = g.count;
                t.slots[h].first = g.first;
                t.slots[h].last_tag = g.last_tag;
                break;
            }
            h = (h + 1) & t.mask;
        }
    }
}

hipError_t launch_rehash(Table dst, DevState* st, const GSlot* src, u64 nsrc, hipStream_t s) {
    (void)st;
    const int grid = (int)std::min<u64>((nsrc + 255) / 256, 8192);
    hipLaunchKernelGGL(rehash_kernel, dim3(grid), dim3(256), 0, s, dst, src, nsrc);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// launch-log aggregation: the tally kernel's heavy commits append their (code, count, first) pairs to
// the launch log's regions (commit_buffers) instead of inserting each into the HBM table (one
// dependent slot load plus memory-side atomics per pair).  After the launch the workgroups of each
// sub-region fold its codes in LDS and only the distinct codes reach the HBM table -- batched, with
// every slot load in flight at once, and with plain stores: the sub-regions partition the codes.
// ------------------------------------------------------------------------------------
// this block is the last of the grid to pass here (counter ctr, reset for the next launch); every
// block's earlier global writes are visible to the last one
__device__ __forceinline__ bool last_block(u32* ctr) {
    __shared__ u32 last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        const u32 prev = atomicAdd(ctr, 1u);
        last = prev == gridDim.x - 1u;
        if (last) {
            *ctr = 0;
            __threadfence();
        }
    }
    __syncthreads();
    return last != 0;
}

constexpr int AGG_PROBE = 256;  // (64 let ~20 of a 7.4-GB launch's 11M entries overflow a fold at load 0.69)
constexpr int CLAIM_WORDS = 1024;  // a reduce workgroup's claim bitmap: sub-regions of up to 32K slots (4 KB; tables of up to 16 Mi slots)
struct alignas(16) AggSlot {
    u64 key;
    u32 mino, cnt;  // min launch offset (logged launches are <= RANGE_FIRST_MAX: u32), records
};

// distinct (key, count, first, last tag) rows into the HBM table in rounds: every pending row's probe
// slot is loaded together, hits take fire-and-forget atomics, empty slots are claimed by CASes issued
// together (a lane waits for max-probe-depth round trips, not the sum over its rows)
// EXCL: no other thread touches these keys' slots while this kernel runs (log_reduce_kernel's buckets
// partition the keys and nothing else updates the table): a found or claimed slot takes plain stores of
// the updated count / first / tag instead of three memory-side atomics.
// A reduce workgroup's claim zone: slots [lo, hi) of its sub-region's home range (base = the range's
// first slot) that no other workgroup's probe can reach -- every insert gives up after GPROBE probes, so
// a key homed before the range reaches at most GPROBE - 1 slots into it.  There an empty slot is claimed
// through the workgroup's LDS bitmap and written with plain stores instead of a memory-side CAS (one
// round trip and one atomic fewer per new code); elsewhere CAS as usual.  bits == nullptr: no zone.
struct ClaimZone {
    u32* bits;
    u64 base, lo, hi;
};

template <int B, bool EXCL = false>
__device__ __forceinline__ u32 insert_rows(const Table& T, DevState* st, const u64 (&key)[B], const u32 (&cnt)[B],
                                           const u64 (&ord)[B], const u32 (&tag)[B], const bool (&valid)[B],
                                           const ClaimZone& cz = ClaimZone{nullptr, 0, 0, 0}) {
    u32 h[B];
    bool pend[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
        h[b] = (u32)table_home(key[b], T.mask);
        pend[b] = valid[b];
    }
    u32 made = 0;
    for (int round = 0; round < GPROBE; ++round) {
        bool any = false;
#pragma unroll
        for (int b = 0; b < B; ++b) any |= pend[b];
        if (!any) break;
        uint4 w0[B], w1[B];
#pragma unroll
        for (int b = 0; b < B; ++b)
            if (pend[b]) {
                const GSlot* sl = &T.slots[h[b]];
                w0[b] = *(const uint4*)sl;
                w1[b] = *((const uint4*)sl + 1);
            }
        bool cas[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            cas[b] = false;
            if (!pend[b]) continue;
            const u64 k = ((u64)w0[b].y << 32) | w0[b].x;
            if (k == key[b]) {
                GSlot* sl = &T.slots[h[b]];
                const u64 first = ((u64)w1[b].y << 32) | w1[b].x;
                if (EXCL) {
                    const u64 c = (((u64)w0[b].w << 32) | w0[b].z) + cnt[b];
                    const u64 f = min(first, ord[b]);
                    *((uint4*)sl) = make_uint4(w0[b].x, w0[b].y, (u32)c, (u32)(c >> 32));
                    *((uint4*)sl + 1) = make_uint4((u32)f, (u32)(f >> 32), max(w1[b].z, tag[b]), w1[b].w);
                } else {
                    atomicAdd((unsigned long long*)&sl->count, (unsigned long long)cnt[b]);
                    if (ord[b] < first) atomicMin((unsigned long long*)&sl->first, (unsigned long long)ord[b]);
                    if (w1[b].z < tag[b]) atomicMax(&sl->last_tag, tag[b]);
                }
                pend[b] = false;
            } else if (k == 0) {
                if (EXCL && cz.bits && h[b] >= cz.lo && h[b] < cz.hi) {
                    const u32 bit = (u32)(h[b] - cz.base), m = 1u << (bit & 31u);
                    if (!(atomicOr(&cz.bits[bit >> 5], m) & m)) {  // ours: the whole slot, plain stores
                        GSlot* sl = &T.slots[h[b]];
                        *((uint4*)sl) = make_uint4((u32)key[b], (u32)(key[b] >> 32), cnt[b], 0u);
                        *((uint4*)sl + 1) = make_uint4((u32)ord[b], (u32)(ord[b] >> 32), tag[b], w1[b].w);
                        made += 1;
                        pend[b] = false;
                    } else {  // another lane of this workgroup took it meanwhile
                        h[b] = (u32)((h[b] + 1ull) & T.mask);
                    }
                } else {
                    cas[b] = true;
                }
            } else {
                h[b] = (u32)((h[b] + 1ull) & T.mask);
            }
        }
        u64 old[B];
#pragma unroll
        for (int b = 0; b < B; ++b)
            if (cas[b]) old[b] = atomicCAS((unsigned long long*)&T.slots[h[b]].key, 0ull, (unsigned long long)key[b]);
#pragma unroll
        for (int b = 0; b < B; ++b) {
            if (!cas[b]) continue;
            if (old[b] == 0 || old[b] == key[b]) {
                GSlot* sl = &T.slots[h[b]];
                made += old[b] == 0 ? 1u : 0u;
                if (cz.bits && old[b] == 0 && h[b] >= cz.lo && h[b] < cz.hi) {  // (a fold overflow's claim)
                    const u32 bit = (u32)(h[b] - cz.base);
                    atomicOr(&cz.bits[bit >> 5], 1u << (bit & 31u));
                }
                if (EXCL && old[b] == 0) {  // claimed an initialised slot (count 0, first ~0, tag 0): ours alone
                    *((u64*)&sl->count) = cnt[b];
                    *((uint4*)sl + 1) = make_uint4((u32)ord[b], (u32)(ord[b] >> 32), tag[b], w1[b].w);
                } else {
                    atomicAdd((unsigned long long*)&sl->count, (unsigned long long)cnt[b]);
                    atomicMin((unsigned long long*)&sl->first, (unsigned long long)ord[b]);
                    atomicMax(&sl->last_tag, tag[b]);
                }
                pend[b] = false;
            } else {
                h[b] = (u32)((h[b] + 1ull) & T.mask);
            }
        }
    }
#pragma unroll
    for (int b = 0; b < B; ++b) {
        if (!pend[b]) continue;  // probe bound exceeded: the overflow list
        const u64 i = atomicAdd((unsigned long long*)&st->n_overflow, 1ull);
        if (i < T.ovf_cap) {
            Overflow o;
            o.key = key[b];
            o.count = cnt[b];
            o.first = ord[b];
            o.tag = tag[b];
            o.pad = 0;
            T.ovf[i] = o;
        } else {
            atomicOr(&st->cap_flags, 2u);
        }
    }
    return made;
}

// Split pass: every region's part of the log counting-sorted by sub-region into the sub-region parts.
// SPLIT_WGS workgroups per region take 2048-entry tiles of its part (each wave a contiguous 512-entry
// slab: coalesced loads); wave ballots rank each entry among its wave's entries of the same sub-region,
// one cursor atomic per (tile, sub-region) places the tile's run, and the stores go out as runs of
// ~256 consecutive entries.  A sub-region part that is full takes the rest directly into the table.
constexpr int SPLIT_PER = 8;
constexpr int SPLIT_TILE = SPLIT_PER * 256;
#ifndef FR_SPLIT_WGS
#define FR_SPLIT_WGS 64
#endif
constexpr int SPLIT_WGS = FR_SPLIT_WGS;
__global__ __launch_bounds__(256) void log_split_kernel(Table t, DevState* st, const LogEntry* log, u32 rcap,
                                                        LogEntry* sub, u32 scap, u32 file_tag, u64 ord0) {
    if (st->log_n == 0) return;
    const u32 r = blockIdx.x / SPLIT_WGS, j = blockIdx.x % SPLIT_WGS;
    const u32 n = min(st->log_rcur[r], rcap);
    const LogEntry* part = log + (u64)r * rcap;
    __shared__ u32 wcnt[4][LOG_SUBS];
    __shared__ u32 sbase[4][LOG_SUBS];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u64 lt = (1ull << lane) - 1ull;
    u32 made = 0;
    for (u32 t0 = j * SPLIT_TILE; t0 < n; t0 += SPLIT_WGS * SPLIT_TILE) {
        LogEntry e[SPLIT_PER];
        u32 sb[SPLIT_PER], rank[SPLIT_PER];
        u32 run[LOG_SUBS];
#pragma unroll
        for (int s = 0; s < LOG_SUBS; ++s) run[s] = 0;
#pragma unroll
        for (int q = 0; q < SPLIT_PER; ++q) {
            const u32 i = t0 + w * 64 * SPLIT_PER + q * 64 + lane;
            e[q] = i < n ? part[i] : LogEntry{0, 0};
        }
#pragma unroll
        for (int q = 0; q < SPLIT_PER; ++q) {
            sb[q] = e[q].key ? log_subregion(e[q].key) : (u32)LOG_SUBS;
            rank[q] = 0;
#pragma unroll
            for (int s = 0; s < LOG_SUBS; ++s) {
                const u64 m = __ballot(sb[q] == (u32)s);
                if (sb[q] == (u32)s) rank[q] = run[s] + (u32)__popcll(m & lt);
                run[s] += (u32)__popcll(m);
            }
        }
        if (lane == 0) {
#pragma unroll
            for (int s = 0; s < LOG_SUBS; ++s) wcnt[w][s] = run[s];
        }
        __syncthreads();
        if (tid < LOG_SUBS) {
            u32 tot = 0;
#pragma unroll
            for (int v = 0; v < 4; ++v) tot += wcnt[v][tid];
            u32 b = tot ? atomicAdd(&st->log_scur[r * LOG_SUBS + tid], tot) : 0u;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                sbase[v][tid] = b;
                b += wcnt[v][tid];
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < SPLIT_PER; ++q) {
            if (sb[q] >= (u32)LOG_SUBS) continue;
            const u32 pos = sbase[w][sb[q]] + rank[q];
            if (pos < scap) {
                sub[(u64)(r * LOG_SUBS + sb[q]) * scap + pos] = e[q];
            } else {
                const u64 key1[1] = {e[q].key};
                const u32 cnt1[1] = {log_cnt(e[q].oc)};
                const u64 ord1[1] = {(ord0 + log_off(e[q].oc)) & ~3ull};  // make_ord's rounding
                const u32 tag1[1] = {file_tag};
                const bool v1[1] = {true};
                made += insert_rows<1>(t, st, key1, cnt1, ord1, tag1, v1);
            }
        }
        __syncthreads();  // wcnt / sbase are reused by the next tile
    }
    add_created(st, made);
}

// One workgroup per sub-region: its part of the log (coalesced, eight entries in flight per thread)
// folded in LDS (records summed, min offset), then its distinct codes inserted into the HBM table with
// the launch's ordinal base and file tag.  The sub-regions partition the codes, so found and claimed
// slots take plain stores (insert_rows EXCL).  The last workgroup empties the log for the next launch.
// RED_WG threads (round 6: 512, was 256): the fold's LDS table (64 KB) allows two workgroups per CU, and
// with 256 threads that left 2 waves per SIMD to cover the entry loads' and the inserts' round trips (1 024
// threads need 114 VGPRs: one workgroup per CU, and the 512 sub-regions would run in two rounds).
#ifndef FR_RED_WG
#define FR_RED_WG 512
#endif
constexpr int RED_WG = FR_RED_WG;
constexpr int RED_FB = RED_WG >= 512 ? 4 : 8;  // distinct codes per thread per insert batch (4: <= 128 VGPRs, two workgroups per CU)
__global__ __launch_bounds__(RED_WG) void log_reduce_kernel(Table t, DevState* st, const LogEntry* sub, u32 scap,
                                                         u32 file_tag, u64 ord0) {
    if (st->log_n == 0) return;
    __shared__ AggSlot ls[AGG_LNS];
    __shared__ u32 zone_bits[CLAIM_WORDS];
    __shared__ u16 occ[AGG_LNS];  // the occupied slots of ls, listed for the inserts
    __shared__ u32 occ_n;
    u32 made = 0;
    for (int i = threadIdx.x; i < AGG_LNS; i += RED_WG) ls[i] = AggSlot{0, 0xFFFFFFFFu, 0};
    // this sub-region's home range: slots [blockIdx.x n, (blockIdx.x + 1) n) of the table (table_home's top
    // bits are the region and sub-region bits); its claim zone skips the first GPROBE slots
    const u64 nslots = t.mask + 1ull, rn = nslots >= (u64)LOG_NSUB ? nslots / LOG_NSUB : 0ull;
    ClaimZone cz{nullptr, 0, 0, 0};
    if (rn > 2ull * GPROBE && rn <= 32ull * CLAIM_WORDS && !(ABLATE & 2048u)) {
        cz = ClaimZone{zone_bits, (u64)blockIdx.x * rn, (u64)blockIdx.x * rn + GPROBE, (u64)(blockIdx.x + 1) * rn};
        for (u32 i = threadIdx.x; i < (u32)(rn / 32); i += RED_WG) zone_bits[i] = 0;
    }
    __syncthreads();
    const u32 n = min(st->log_scur[blockIdx.x], scap);
    const LogEntry* part = sub + (u64)blockIdx.x * scap;
    // a first occurrence folds as v = its ordinal's offset / 4 - the launch base's (make_ord's rounding): 32 bits
    // for launches up to 16 GiB; the ordinal is tag | (base4 + v) << 2
    const u64 base4 = (ord0 & ((1ull << ORD_SHIFT) - 1ull)) >> 2, tagpart = ord0 & ~((1ull << ORD_SHIFT) - 1ull);
    u64 sink = 0;
    constexpr int LB = 8;  // entries per thread per batch; the next batch's loads fly during this one's fold
    const u32 nn = (ABLATE & 512u) ? 0u : n;  // 512: timing ablation
    // unconditional loads (a clamped index, the key zeroed past the end): exec-masked loads made the compiler wait
    // for every outstanding load (vmcnt(0)) right after issuing the next batch, so no batch flew during a fold
    LogEntry nx[LB];
    if (nn) {
#pragma unroll
        for (int q = 0; q < LB; ++q) nx[q] = part[min(threadIdx.x + q * RED_WG, nn - 1u)];
    }
    for (u32 i0 = threadIdx.x; i0 < nn; i0 += LB * RED_WG) {
        LogEntry ev[LB];
#pragma unroll
        for (int q = 0; q < LB; ++q) {
            ev[q] = nx[q];
            nx[q] = part[min(i0 + (LB + q) * RED_WG, nn - 1u)];  // (past the end: the last entry again, skipped)
        }
#pragma unroll
        for (int q = 0; q < LB; ++q) {
            const LogEntry e = ev[q];
            if (i0 + q * RED_WG >= nn || !e.key) continue;
            if (ABLATE & 1024u) {  // timing ablation: loads only
                sink ^= e.key;
                continue;
            }
            const u32 eoff = (u32)((((ord0 & ((1ull << ORD_SHIFT) - 1ull)) + log_off(e.oc)) >> 2) - base4);
            const u32 ecnt = log_cnt(e.oc);
            // the fold's slot and probe step (double hashing: a wave waits for its lanes' longest probe chain,
            // and linear probing's clusters at the fold's ~0.7 load made that chain long); two 32-bit
            // multiplies (a sub-region's keys share mix64's top bits, not these)
            u32 h = (u32)e.key * 0x9E3779B1u ^ (u32)(e.key >> 32) * 0x85EBCA6Bu;
            const u32 hstep = ((h >> 7) & (AGG_LNS - 1)) | 1u;
            h = (h ^ (h >> 15)) & (AGG_LNS - 1);
            bool done = false;
            for (int pr = 0; pr < AGG_PROBE && !done; ++pr) {
                const AggSlot sl = ls[h];  // key, first and count in one LDS read
                u64 k = sl.key;
                u32 mino = sl.mino;
                if (k == 0) {
                    const u64 old = atomicCAS((unsigned long long*)&ls[h].key, 0ull, (unsigned long long)e.key);
                    k = old == 0 ? e.key : old;
                    mino = old == 0 ? 0xFFFFFFFFu : ls[h].mino;
                }
                if (k == e.key) {
                    atomicAdd(&ls[h].cnt, ecnt);  // (fire-and-forget LDS atomics: no wait in the fold's chain)
                    if (eoff < mino) atomicMin(&ls[h].mino, eoff);
                    done = true;
                    break;
                }
                h = (h + hstep) & (AGG_LNS - 1);
            }
            if (!done) {  // a full LDS table: this row goes in on its own
                const u64 key1[1] = {e.key};
                const u32 cnt1[1] = {ecnt};
                const u64 ord1[1] = {tagpart | ((base4 + eoff) << 2)};
                const u32 tag1[1] = {file_tag};
                const bool v1[1] = {true};
                made += insert_rows<1>(t, st, key1, cnt1, ord1, tag1, v1, cz);
                atomicAdd(&st->log_fold_over, 1u);  // the fold was full: the next feeds keep smaller logged launches
            }
        }
    }
    if (sink == 1) atomicAdd((unsigned long long*)&st->stamp[7], 1ull);  // keeps the ablation's loads
    __syncthreads();
    // the distinct codes into the table: the occupied slots listed first (LDS), then FB of them per thread in
    // flight -- one batch of probe loads covers RED_WG * FB codes, instead of one batch per FB slots scanned
    // (half of them empty at the fold's usual load)
    if (threadIdx.x == 0) occ_n = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < AGG_LNS; i += RED_WG)
        if (ls[i].key) occ[atomicAdd(&occ_n, 1u)] = (u16)i;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&st->log_fold_max, occ_n);  // the feed's fullest fold (fr_feed_device's launch size)
    constexpr int FB = RED_FB;
    const u32 nocc = (ABLATE & 256u) ? 0u : occ_n;  // 256: timing ablation
    for (u32 i0 = threadIdx.x; i0 < nocc; i0 += FB * RED_WG) {
        u64 key[FB], ord[FB];
        u32 cnt[FB], tag[FB];
        bool v[FB];
#pragma unroll
        for (int b = 0; b < FB; ++b) {
            const u32 j = i0 + b * RED_WG;
            v[b] = j < nocc;
            const AggSlot e = v[b] ? ls[occ[j]] : AggSlot{0, 0, 0};
            key[b] = e.key;
            cnt[b] = e.cnt;
            ord[b] = tagpart | ((base4 + e.mino) << 2);
            tag[b] = file_tag;
        }
        made += insert_rows<FB, true>(t, st, key, cnt, ord, tag, v, cz);
    }
    add_created(st, made);
    // every workgroup has read log_n and its cursor (the split pass read the region cursors before
    // this launch): the last one empties the log
    if (last_block(&st->log_red_done)) {
        for (int i = threadIdx.x; i < LOG_NR; i += RED_WG)
            __hip_atomic_store(&st->log_rcur[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int i = threadIdx.x; i < LOG_NSUB; i += RED_WG)
            __hip_atomic_store(&st->log_scur[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (threadIdx.x == 0) __hip_atomic_store(&st->log_n, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

size_t log_aggregate_temp_bytes() { return 0; }

hipError_t launch_log_aggregate(Table t, DevState* st, const LogEntry* log, u32 rcap, LogEntry* sub, u32 scap,
                                u32 file_tag, u64 file_offset, hipStream_t s) {
    // reads log_n on the device and returns at once when no commit logged (the usual case for
    // low-cardinality runs: only commits of at least ScanArgs::log_min pairs log)
    const u64 ord0 = ((u64)file_tag << ORD_SHIFT) | file_offset;
    if (!LOG_DIRECT)  // (direct logging: the commits wrote the sub-region parts)
        hipLaunchKernelGGL(log_split_kernel, dim3(LOG_NR * SPLIT_WGS), dim3(256), 0, s, t, st, log, rcap, sub, scap,
                           file_tag, ord0);
    hipLaunchKernelGGL(log_reduce_kernel, dim3(LOG_NSUB), dim3(RED_WG), 0, s, t, st, sub, scap, file_tag, ord0);
    return hipGetLastError();  // log_reduce_kernel's last block emptied the log
}

// Stream compaction of table slots with one atomic per workgroup (single-address atomics
// serialise at ~11 ns each: a per-wave append over a 4 Mi-slot table costs ~0.8 ms).  Each
// workgroup owns a contiguous slot range: pass 1 counts its hits and reserves one output
// range, pass 2 re-reads the (L2-warm) range and writes hits in slot order.
constexpr int CWG = 256;

template <class Pred>
__device__ __forceinline__ u64 block_reserve(u64 lo, u64 hi, Pred pred, u64* counter, u32* red) {
    const int tid = threadIdx.x;
    u32 mine = 0;
    for (u64 i = lo + tid; i < hi; i += CWG) mine += pred(i) ? 1u : 0u;
    for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = mine;
    __syncthreads();
    if (tid == 0) {
        const u32 tot = red[0] + red[1] + red[2] + red[3];
        *(u64*)&red[4] = tot ? atomicAdd((unsigned long long*)counter, (unsigned long long)tot) : 0ull;
    }
    __syncthreads();
    return *(const u64*)&red[4];
}

// calls emit(out_index, slot_index) for every hit of [lo, hi), in slot order
template <class Pred, class Emit>
__device__ __forceinline__ void block_emit(u64 lo, u64 hi, u64 base, Pred pred, Emit emit, u32* wc) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    for (u64 b = lo; b < hi; b += CWG) {
        const u64 i = b + tid;
        const bool hit = i < hi && pred(i);
        const u64 m = __ballot(hit);
        if (lane == 0) wc[wid] = (u32)__popcll(m);
        __syncthreads();
        u32 before = 0, tot = 0;
        for (int w = 0; w < CWG / 64; ++w) {
            before += w < wid ? wc[w] : 0u;
            tot += wc[w];
        }
        if (hit) emit(base + before + (u64)__popcll(m & ((1ull << lane) - 1ull)), i);
        base += tot;
        __syncthreads();
    }
}

__device__ __forceinline__ void block_range(u64 n, u64& lo, u64& hi) {
    const u64 per = (n + gridDim.x - 1) / gridDim.x;
    lo = min(n, (u64)blockIdx.x * per);
    hi = min(n, lo + per);
}

__global__ __launch_bounds__(CWG) void compact_kernel(const GSlot* slots, u64 nslots, u64* keys, u64* counts,
                                                      u64* first, u32* pos, u64* counter) {
    __shared__ u32 red[8];
    u64 lo, hi;
    block_range(nslots, lo, hi);
    auto pred = [&](u64 i) { return slots[i].key != 0; };
    const u64 base = block_reserve(lo, hi, pred, counter, red);
    block_emit(lo, hi, base, pred, [&](u64 p, u64 i) {
        const GSlot g = slots[i];
        keys[p] = g.key;
        counts[p] = g.count;
        first[p] = g.first;
        pos[p] = (u32)p;
    }, red);
}

hipError_t launch_compact(const GSlot* slots, u64 nslots, u64* keys, u64* counts, u64* first, u32* pos,
                          u64* counter, hipStream_t s) {
    const int grid = (int)std::max<u64>(1, std::min<u64>((nslots + 4095) / 4096, 2048));
    hipLaunchKernelGGL(compact_kernel, dim3(grid), dim3(CWG), 0, s, slots, nslots, keys, counts, first, pos,
                       counter);
    return hipGetLastError();
}

hipError_t launch_order(const u64* first_in, const u32* pos_in, u64 n, u64* first_out, u32* perm_out, void* temp,
                        size_t* temp_bytes, int begin_bit, int end_bit, hipStream_t s) {
    return rocprim::radix_sort_pairs(temp, *temp_bytes, first_in, first_out, pos_in, perm_out, (size_t)n,
                                     (unsigned)begin_bit, (unsigned)end_bit, s);
}

__global__ void gather_kernel(const u32* perm, u64 n, const u64* keys, const u64* counts, u64* keys_o,
                              u64* counts_o, u32* rank) {
    for (u64 j = blockIdx.x * (u64)blockDim.x + threadIdx.x; j < n; j += (u64)gridDim.x * blockDim.x) {
        const u32 p = perm[j];
        keys_o[j] = keys[p];
        counts_o[j] = counts[p];
        rank[p] = (u32)j;
    }
}

hipError_t launch_gather(const u32* perm, u64 n, const u64* keys, const u64* counts, u64* keys_o, u64* counts_o,
                         u32* rank, hipStream_t s) {
    if (!n) return hipSuccess;
    const int grid = (int)std::min<u64>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(gather_kernel, dim3(grid), dim3(256), 0, s, perm, n, keys, counts, keys_o, counts_o, rank);
    return hipGetLastError();
}

__device__ __forceinline__ const GSlot* table_find(const GSlot* slots, u64 mask, u64 key) {
    u64 h = table_home(key, mask);
    for (u64 probe = 0; probe <= mask; ++probe) {
        const GSlot* s = &slots[h];
        if (s->key == key) return s;
        if (s->key == 0) return nullptr;
        h = (h + 1) & mask;
    }
    return nullptr;
}

// write each live slot's sorted index into slot.uidx (keys in sorted order)
__global__ void set_uidx_kernel(GSlot* slots, u64 mask, const u64* keys, u64 n) {
    for (u64 j = blockIdx.x * (u64)blockDim.x + threadIdx.x; j < n; j += (u64)gridDim.x * blockDim.x) {
        GSlot* s = const_cast<GSlot*>(table_find(slots, mask, keys[j]));
        if (s) s->uidx = (u32)j;
    }
}

hipError_t launch_set_uidx(GSlot* slots, u64 mask, const u64* keys, u64 n, const u32* rank_of_pos, hipStream_t s) {
    (void)rank_of_pos;
    if (!n) return hipSuccess;
    const int grid = (int)std::min<u64>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(set_uidx_kernel, dim3(grid), dim3(256), 0, s, slots, mask, keys, n);
    return hipGetLastError();
}

__global__ void presence_map_kernel(const GSlot* slots, u64 mask, const Presence* pres, u64 n, u32* uidx,
                                    u32* file_idx, u64* snap) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const Presence p = pres[i];
        const GSlot* s = table_find(slots, mask, p.key);
        uidx[i] = s ? s->uidx : 0xFFFFFFFFu;
        file_idx[i] = (u32)(p.tc & ((1u << PRES_TAG_BITS) - 1u)) - 1u;
        snap[i] = p.tc >> PRES_TAG_BITS;
    }
}

// The presence pairs of a scan of one file (fr_finalize when fr_end_file deferred that file's scan):
// every finalized code, in final order, present in that file with its whole count -- what
// presence_scan_kernel + presence_map_kernel would give, without the two passes over the table.
__global__ void presence_one_file_kernel(const u64* counts, u64 n, u32 tag, u32* uidx, u32* file_idx, u64* snap) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        uidx[i] = (u32)i;
        file_idx[i] = tag - 1u;
        snap[i] = counts[i] & ((1ull << (64 - PRES_TAG_BITS)) - 1ull);
    }
}

hipError_t launch_presence_one_file(const u64* counts, u64 n, u32 tag, u32* uidx, u32* file_idx, u64* snap,
                                    hipStream_t s) {
    if (!n) return hipSuccess;
    const int grid = (int)std::min<u64>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(presence_one_file_kernel, dim3(grid), dim3(256), 0, s, counts, n, tag, uidx, file_idx, snap);
    return hipGetLastError();
}

hipError_t launch_presence_map(const GSlot* slots, u64 mask, const Presence* pres, u64 n, u32* uidx,
                               u32* file_idx, u64* snap, hipStream_t s) {
    if (!n) return hipSuccess;
    const int grid = (int)std::min<u64>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(presence_map_kernel, dim3(grid), dim3(256), 0, s, slots, mask, pres, n, uidx, file_idx, snap);
    return hipGetLastError();
}

// ---- first-occurrence order by binning (fr_finalize, one context's own ordinals) -------------
// An ordinal is a record start; records are four terminated lines, so two ordinals of one file
// are >= 4 bytes apart and a bin of 2^shift bytes holds at most 2^(shift-2) codes (twice that
// where a bin straddles two files).  Count per bin (each slot keeps its arrival index in uidx),
// exclusive scan, scatter by bin, then each code's rank inside its bin gives its final index: the
// table is read twice and nothing is sorted globally.
__device__ __forceinline__ u64 ord_bin(const BinMap& m, u64 ord) {
    const u64 tag = ord >> ORD_SHIFT, off = ord & ((1ull << ORD_SHIFT) - 1ull);
    return min(((tag - m.first_tag) * m.span + off) >> m.shift, m.nbins - 1ull);  // clamp: never out of bounds
}

// One slot (one 32-B sector) per lane, the whole table in one grid.  Every store here is a whole
// sector or part of a coalesced run: a random 4- or 8-B store is a partial-sector write, which HBM
// turns into a read-modify-write (the first version of these kernels stored into table slots and
// ran at half the speed).
__global__ __launch_bounds__(256) void fin_hist_kernel(const GSlot* slots, u64 n, BinMap m, u32* cnt, u32* arr) {
    const u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 w0 = *(const uint4*)&slots[i];
    const uint4 w1 = *((const uint4*)&slots[i] + 1);
    u32 v = 0xFFFFFFFFu;
    if ((w0.x | w0.y) != 0u) v = atomicAdd(&cnt[ord_bin(m, ((u64)w1.y << 32) | w1.x)], 1u);
    arr[i] = v;  // arrival index in the bin (coalesced: every lane stores)
}

// each live slot's row {ordinal, key, count, slot} to its bin's run, one 32-B sector per row
__global__ __launch_bounds__(256) void fin_scatter_kernel(const GSlot* slots, u64 n, BinMap m, const u32* base,
                                                          const u32* arr, FinRow* rows) {
    const u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 k = arr[i];
    if (k == 0xFFFFFFFFu) return;
    const uint4 w0 = *(const uint4*)&slots[i];
    const uint4 w1 = *((const uint4*)&slots[i] + 1);
    const u64 first = ((u64)w1.y << 32) | w1.x;
    const u32 q = base[ord_bin(m, first)] + k;
    if (q < m.cap) {
        typedef u32 u32x4 __attribute__((ext_vector_type(4)));
        u32x4* d = (u32x4*)&rows[q];
        d[0] = u32x4{w1.x, w1.y, w0.x, w0.y};
        d[1] = u32x4{w0.z, w0.w, (u32)i, 0u};
    }
}

// final index = the bin's base + the codes of the bin with a smaller ordinal (ties: slot index,
// never met for one context's ordinals); the row goes there and the slot's uidx becomes that index
__global__ __launch_bounds__(256) void fin_rank_kernel(GSlot* slots, u64 nk, BinMap m, const u32* base,
                                                       const FinRow* rows, u64* keys_o, u64* counts_o, u64* first_o,
                                                       int set_uidx) {
    const u64 q = blockIdx.x * (u64)blockDim.x + threadIdx.x;
    if (q >= nk) return;
    const FinRow row = rows[q];
    const u64 b = ord_bin(m, row.first);
    const u32 lo = base[b], hi = (u32)min((u64)base[b + 1], m.cap);
    u32 r = 0;
    for (u32 j = lo; j < hi; ++j) {
        const u64 fj = rows[j].first;
        r += (fj < row.first || (fj == row.first && rows[j].slot < row.slot)) ? 1u : 0u;
    }
    const u32 out = lo + r;
    if (out >= nk) return;  // only when the live count disagrees with n_keys (fr_finalize fails then)
    keys_o[out] = row.key;
    counts_o[out] = row.count;
    first_o[out] = row.first;
    if (set_uidx) slots[row.slot].uidx = out;  // read only by presence_map_kernel (a random partial-sector store)
}

static unsigned lane_grid(u64 n) { return (unsigned)std::max<u64>(1, (n + 255) / 256); }

hipError_t launch_fin_hist(const GSlot* slots, u64 nslots, const BinMap& m, u32* cnt, u32* arr, hipStream_t s) {
    hipLaunchKernelGGL(fin_hist_kernel, dim3(lane_grid(nslots)), dim3(256), 0, s, slots, nslots, m, cnt, arr);
    return hipGetLastError();
}

// exclusive scan of cnt[0, n) into base[0, n) (temp = nullptr: size query)
hipError_t launch_fin_scan(const u32* cnt, u32* base, u64 n, void* temp, size_t* temp_bytes, hipStream_t s) {
    return rocprim::exclusive_scan(temp, *temp_bytes, cnt, base, 0u, (size_t)n, rocprim::plus<u32>(), s);
}

hipError_t launch_fin_scatter(const GSlot* slots, u64 nslots, const BinMap& m, const u32* base, const u32* arr,
                              FinRow* rows, hipStream_t s) {
    hipLaunchKernelGGL(fin_scatter_kernel, dim3(lane_grid(nslots)), dim3(256), 0, s, slots, nslots, m, base, arr, rows);
    return hipGetLastError();
}

hipError_t launch_fin_rank(GSlot* slots, u64 nk, const BinMap& m, const u32* base, const FinRow* rows, u64* keys_o,
                           u64* counts_o, u64* first_o, bool set_uidx, hipStream_t s) {
    if (!nk) return hipSuccess;
    hipLaunchKernelGGL(fin_rank_kernel, dim3(lane_grid(nk)), dim3(256), 0, s, slots, nk, m, base, rows, keys_o,
                       counts_o, first_o, set_uidx ? 1 : 0);
    return hipGetLastError();
}

// merge another GPU's compacted table into this one (count +, first min); presence of
// remote keys travels separately (fr_get_presence on each rank)
__global__ void merge_kernel(Table t, DevState* st, const u64* keys, const u64* counts, const u64* first, u64 n) {
    u32 made = 0;
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x)
        made += global_insert(t, st, keys[i], counts[i], first[i], 0u) ? 1u : 0u;
    add_created(st, made);
}

// the multi-GPU merge's send side: the finalized rows (key, count, first) partitioned by owner rank
// (owner = the top 24 bits of key * 0x9E3779B97F4A7C15 mod world, frender_amd/dist.py owner_of), row-major,
// owner blocks contiguous.  Pass 1 counts per owner (an LDS histogram per workgroup, one atomic per
// (workgroup, owner)); pass 2 gives each workgroup's rows of an owner a run claimed from that owner's cursor
// (cursors start at the owners' exclusive prefix).  Order inside a block is not fixed: the merge is commutative.
constexpr int PART_MAX = 1024;  // ranks
__device__ __forceinline__ u32 owner_rank(u64 key, u32 world) {
    return (u32)(((key * 0x9E3779B97F4A7C15ull) >> 40) & 0xFFFFFFull) % world;
}
__global__ __launch_bounds__(256) void part_count_kernel(const u64* keys, u64 n, u32 world, u64* counts) {
    __shared__ u32 h[PART_MAX];
    for (u32 i = threadIdx.x; i < world; i += 256) h[i] = 0;
    __syncthreads();
    for (u64 i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (u64)gridDim.x * 256ull) atomicAdd(&h[owner_rank(keys[i], world)], 1u);
    __syncthreads();
    for (u32 i = threadIdx.x; i < world; i += 256)
        if (h[i]) atomicAdd((unsigned long long*)&counts[i], (unsigned long long)h[i]);
}
__global__ __launch_bounds__(256) void part_scatter_kernel(const u64* keys, const u64* counts_in, const u64* first,
                                                          u64 n, u32 world, const u64* counts, u64* cursor, u64* rows) {
    __shared__ u32 h[PART_MAX];
    __shared__ u64 base[PART_MAX];
    for (u32 i = threadIdx.x; i < world; i += 256) h[i] = 0;
    __syncthreads();
    const u64 stride = (u64)gridDim.x * 256ull;
    for (u64 i = blockIdx.x * 256ull + threadIdx.x; i < n; i += stride) atomicAdd(&h[owner_rank(keys[i], world)], 1u);
    __syncthreads();
    if (threadIdx.x == 0) {  // cursors start at the exclusive prefix of the counts (the first claim of each sets it)
        u64 pre = 0;
        for (u32 r = 0; r < world; ++r) {
            base[r] = h[r] ? pre + atomicAdd((unsigned long long*)&cursor[r], (unsigned long long)h[r]) : 0ull;
            pre += counts[r];
            h[r] = 0;
        }
    }
    __syncthreads();
    for (u64 i = blockIdx.x * 256ull + threadIdx.x; i < n; i += stride) {
        const u64 k = keys[i];
        const u32 r = owner_rank(k, world);
        const u64 at = base[r] + atomicAdd(&h[r], 1u);
        rows[3 * at] = k;
        rows[3 * at + 1] = counts_in[i];
        rows[3 * at + 2] = first[i];
    }
}
// merge rows (key, count, first), row-major, into the table (count +, first min)
__global__ void merge_rows_kernel(Table t, DevState* st, const u64* rows, u64 n) {
    u32 made = 0;
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x)
        made += global_insert(t, st, rows[3 * i], rows[3 * i + 1], rows[3 * i + 2], 0u) ? 1u : 0u;
    add_created(st, made);
}
hipError_t launch_partition_rows(const u64* keys, const u64* counts_in, const u64* first, u64 n, u32 world,
                                 u64* counts, u64* cursor, u64* rows, hipStream_t s) {
    if (world < 1 || world > (u32)PART_MAX) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(counts, 0, 2ull * world * sizeof(u64), s);  // counts and cursors (adjacent)
    if (e != hipSuccess || !n) return e;
    const int grid = (int)std::min<u64>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(part_count_kernel, dim3(grid), dim3(256), 0, s, keys, n, world, counts);
    hipLaunchKernelGGL(part_scatter_kernel, dim3(grid), dim3(256), 0, s, keys, counts_in, first, n, world, counts,
                       cursor, rows);
    return hipGetLastError();
}
hipError_t launch_merge_rows(Table t, DevState* st, const u64* rows, u64 n, hipStream_t s) {
    if (!n) return hipSuccess;
    const int grid = (int)std::min<u64>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(merge_rows_kernel, dim3(grid), dim3(256), 0, s, t, st, rows, n);
    return hipGetLastError();
}

// per-file presence (R10) and the per-file distinct-code count (frender.py:175): after a
// file, exactly the slots whose last_tag is that file's tag hold a code seen in it.  Each pair keeps
// the code's running count (its per-file count is the difference to the code's previous pair).  A workgroup
// takes PS_K x 256 consecutive slots, one slot per lane per step with all the loads in flight
// together, reserves its output run with one atomic and writes its hits in slot order.
constexpr int PS_K = 16;
__global__ __launch_bounds__(CWG) void presence_scan_kernel(const GSlot* slots, u64 n, u32 tag, Presence* pres,
                                                            u64 cap, DevState* st) {
    __shared__ u32 wc[PS_K * (CWG / 64)];
    __shared__ u64 bbase;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const u64 b0 = (u64)blockIdx.x * (PS_K * CWG);
    u32 hits = 0;
#pragma unroll
    for (int k = 0; k < PS_K; ++k) {
        const u64 i = b0 + (u64)k * CWG + tid;
        if (i < n) {
            const uint2 key = *(const uint2*)&slots[i];
            const u32 lt = slots[i].last_tag;
            hits |= ((key.x | key.y) != 0u && lt == tag) ? (1u << k) : 0u;
        }
    }
    u64 m[PS_K];
#pragma unroll
    for (int k = 0; k < PS_K; ++k) {
        m[k] = __ballot((hits >> k) & 1u);
        if (lane == 0) wc[k * (CWG / 64) + wid] = (u32)__popcll(m[k]);
    }
    __syncthreads();
    if (tid == 0) {  // exclusive scan over (step, wave) = slot order, and the block's output run
        u32 run = 0;
        for (int j = 0; j < PS_K * (CWG / 64); ++j) {
            const u32 c = wc[j];
            wc[j] = run;
            run += c;
        }
        bbase = run ? atomicAdd((unsigned long long*)&st->n_presence, (unsigned long long)run) : 0ull;
    }
    __syncthreads();
    if (!hits) return;
    const u64 below = (1ull << lane) - 1ull;
#pragma unroll
    for (int k = 0; k < PS_K; ++k) {
        if ((hits >> k) & 1u) {
            const u64 kk = bbase + wc[k * (CWG / 64) + wid] + (u64)__popcll(m[k] & below);
            if (kk < cap) {
                const GSlot* sl = &slots[b0 + (u64)k * CWG + tid];
                pres[kk].key = sl->key;
                pres[kk].tc = (sl->count << PRES_TAG_BITS) | (u64)tag;  // count mod 2^44, file tag
            } else {
                atomicOr(&st->cap_flags, 1u);
            }
        }
    }
}

hipError_t launch_presence_scan(const GSlot* slots, u64 n, u32 tag, Presence* pres, u64 cap, DevState* st,
                                hipStream_t s) {
    const int grid = (int)std::max<u64>(1, (n + PS_K * CWG - 1) / (PS_K * CWG));
    hipLaunchKernelGGL(presence_scan_kernel, dim3(grid), dim3(CWG), 0, s, slots, n, tag, pres, cap, st);
    return hipGetLastError();
}

hipError_t launch_merge(Table t, DevState* st, const u64* keys, const u64* counts, const u64* first, u64 n,
                        hipStream_t s) {
    if (!n) return hipSuccess;
    const int grid = (int)std::min<u64>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(merge_kernel, dim3(grid), dim3(256), 0, s, t, st, keys, counts, first, n);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// classify: lane per unique code, the sheet broadcast from LDS
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int mism(u64 q, u64 s) {  // Hamming distance of two 3-bit packed strings
    const u64 x = q ^ s;
    return __popcll((x | (x >> 1) | (x >> 2)) & 0x1249249249249249ull);
}

constexpr int CLS_WG = 256;
#ifndef FR_CLS_SCALAR
#define FR_CLS_SCALAR 1  // sheet rows by scalar loads from HBM (class_pair_s), not broadcast from LDS
#endif
constexpr int CLS_LDS_BYTES = 48 * 1024;  // dynamic LDS cap: sheet images + per-name rc sums

__device__ __forceinline__ int mism32(u32 q, u32 s) {  // <= 10 symbols: 30 bits
    const u32 x = q ^ s;
    return __popc((x | (x >> 1) | (x >> 2)) & 0x09249249u);
}

template <typename W>
__device__ __forceinline__ int mism_w(W q, W s) {
    if constexpr (sizeof(W) == 4) return mism32(q, s);
    else return mism(q, s);
}

// R7/R8 for one unique over every sheet row, forward idx2 and (rc) rc(idx2) in the same pass
// (idx1's distances are shared): the first matching row of each list, |M1 ∩ M2| and its first row.
template <typename W>
__device__ __forceinline__ void class_pair(W q1, W q2, const W* s1, const W* s2, const W* s2rc, int S, int nsubs,
                                           bool rc, int& m1, int& m2, int& cls, int& row, int& rm2, int& rcls,
                                           int& rrow) {
    m1 = -1;
    m2 = -1;
    rm2 = -1;
    int both = 0, r = -1, rboth = 0, rr = -1;
    for (int i = 0; i < S; ++i) {
        const bool a = mism_w<W>(q1, s1[i]) <= nsubs;
        const bool b = mism_w<W>(q2, s2[i]) <= nsubs;
        m1 = (a && m1 < 0) ? i : m1;
        m2 = (b && m2 < 0) ? i : m2;
        r = (a && b && both == 0) ? i : r;
        both += (a && b) ? 1 : 0;
        if (rc) {
            const bool c = mism_w<W>(q2, s2rc[i]) <= nsubs;
            rm2 = (c && rm2 < 0) ? i : rm2;
            rr = (a && c && rboth == 0) ? i : rr;
            rboth += (a && c) ? 1 : 0;
        }
    }
    if (m1 >= 0 && m2 >= 0) {
        cls = both == 0 ? CLS_HOP : both == 1 ? CLS_DEMUX : CLS_AMBIG;
        row = both == 1 ? r : -1;
    } else {
        cls = CLS_UNDET;
        row = -1;
    }
    if (m1 >= 0 && rm2 >= 0) {
        rcls = rboth == 0 ? CLS_HOP : rboth == 1 ? CLS_DEMUX : CLS_AMBIG;
        rrow = rboth == 1 ? rr : -1;
    } else {
        rcls = CLS_UNDET;
        rm2 = -1;
        rrow = -1;
    }
    if (cls == CLS_UNDET) {  // pass A keeps matched_idx1 from the rc call (frender.py:319-323)
        if (rcls == CLS_UNDET) m1 = -1;
        m2 = -1;
    }
}

// class_pair with the rows read straight from the u64 sheet arrays in HBM:
// the row index is uniform, so every row arrives by scalar loads and the distance ops take it as a
// scalar operand (no LDS read per row), and the bookkeeping runs only on rows some lane matches
// (a code matches one or two rows of a well-separated sheet: the wave skips ~2/3 of the updates).
template <typename W, bool RC>
__device__ __forceinline__ void class_pair_s(W q1, W q2, const u64* __restrict__ s1, const u64* __restrict__ s2,
                                             const u64* __restrict__ s2rc, int S, int nsubs, int& m1, int& m2,
                                             int& cls, int& row, int& rm2, int& rcls, int& rrow) {
    m1 = -1;
    m2 = -1;
    rm2 = -1;
    int both = 0, r = -1, rboth = 0, rr = -1;
#pragma unroll 8
    for (int i = 0; i < S; ++i) {
        const bool a = mism_w<W>(q1, (W)s1[i]) <= nsubs;
        const bool b = mism_w<W>(q2, (W)s2[i]) <= nsubs;
        const bool c = RC && mism_w<W>(q2, (W)s2rc[i]) <= nsubs;
        if (a || b || c) {
            m1 = (a && m1 < 0) ? i : m1;
            m2 = (b && m2 < 0) ? i : m2;
            r = (a && b && both == 0) ? i : r;
            both += (a && b) ? 1 : 0;
            rm2 = (c && rm2 < 0) ? i : rm2;
            rr = (a && c && rboth == 0) ? i : rr;
            rboth += (a && c) ? 1 : 0;
        }
    }
    if (m1 >= 0 && m2 >= 0) {
        cls = both == 0 ? CLS_HOP : both == 1 ? CLS_DEMUX : CLS_AMBIG;
        row = both == 1 ? r : -1;
    } else {
        cls = CLS_UNDET;
        row = -1;
    }
    if (m1 >= 0 && rm2 >= 0) {
        rcls = rboth == 0 ? CLS_HOP : rboth == 1 ? CLS_DEMUX : CLS_AMBIG;
        rrow = rboth == 1 ? rr : -1;
    } else {
        rcls = CLS_UNDET;
        rm2 = -1;
        rrow = -1;
    }
    if (cls == CLS_UNDET) {  // pass A keeps matched_idx1 from the rc call (frender.py:319-323)
        if (rcls == CLS_UNDET) m1 = -1;
        m2 = -1;
    }
}

// ------------------------------------------------------------------------------------
// classify neighbourhood maps (fr_internal.h NbrMap): a code is classified by three map probes and
// two pair probes instead of a scan over every sheet row
// ------------------------------------------------------------------------------------
__host__ __device__ inline u64 nbr_binom(int n, int k) {
    if (k < 0 || k > n) return 0;
    u64 r = 1;
    for (int j = 1; j <= k; ++j) r = r * (u64)(n - k + j) / (u64)j;
    return r;
}

u64 nbr_codes_per_row(int L, int nsubs) {
    u64 t = 0, p5 = 1;
    for (int d = 0; d <= nsubs && d <= L; ++d, p5 *= 5) t += nbr_binom(L, d) * p5;
    return t;
}

template <class SL>
__device__ __forceinline__ SL* nbr_claim(SL* t, u32 mask, u64 key) {  // the table has >= 2x free slots
    u32 h = (u32)mix64(key) & mask;
    for (;;) {
        const u64 prev = atomicCAS((unsigned long long*)&t[h].key, 0ull, (unsigned long long)key);
        if (prev == 0 || prev == key) return &t[h];
        h = (h + 1) & mask;
    }
}

// thread per (row, neighbour index t): t ranks (d, combination of d positions, d symbols in 1..5);
// substitutions equal to the row's own symbol are left to the smaller d that produces the same code
__global__ void nbr_insert_kernel(const u64* __restrict__ vals, const int32_t* __restrict__ canon, int S, int L,
                                  int nsubs, u64 T, NSlot* m, u32 mask) {
    const u64 g = blockIdx.x * (u64)blockDim.x + threadIdx.x;
    if (g >= (u64)S * T) return;
    const int i = (int)(g / T);
    u64 t = g % T;
    if (canon[i] != i) return;  // one insertion per distinct value
    int d = 0;
    u64 p5 = 1;
    for (;; ++d, p5 *= 5) {
        const u64 nd = nbr_binom(L, d) * p5;
        if (t < nd) break;
        t -= nd;
    }
    u64 sub = t % p5, comb = t / p5;
    u64 v = vals[i];
    for (int k = d; k >= 1; --k) {  // colex unranking of the position set
        int c = k - 1;
        while (nbr_binom(c + 1, k) <= comb) ++c;
        comb -= nbr_binom(c, k);
        const u64 sy = sub % 5u + 1u;
        sub /= 5u;
        if (((v >> (3 * c)) & 7u) == sy) return;
        v = (v & ~(7ull << (3 * c))) | (sy << (3 * c));
    }
    NSlot* e = nbr_claim(m, mask, v | NBR_KEY);
    atomicMax(&e->vmin_c, ~(u32)i);
    atomicMax(&e->vmax1, (u32)i + 1u);
}

__global__ void nbr_pair_kernel(const int32_t* __restrict__ canon, int S, int rc, PSlot* p0, u32 m0, PSlot* p1,
                                u32 m1) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S) return;
    const u64 a = (u64)(u32)canon[i] << 32;
    PSlot* e = nbr_claim(p0, m0, a | (u32)canon[S + i] | NBR_KEY);
    atomicAdd(&e->cnt, 1u);
    atomicMax(&e->first_c, ~(u32)i);
    if (rc) {
        e = nbr_claim(p1, m1, a | (u32)canon[2 * S + i] | NBR_KEY);
        atomicAdd(&e->cnt, 1u);
        atomicMax(&e->first_c, ~(u32)i);
    }
}

hipError_t launch_nbr_build(const SheetArgs& sh, const int32_t* canon, int nsubs, int rc, const NbrMap& nm,
                            hipStream_t s) {
    const u64* vals[3] = {sh.i1, sh.i2, sh.i2rc};
    const int len[3] = {sh.L1u, sh.L2u, sh.L2u};
    for (int l = 0; l < (rc ? 3 : 2); ++l) {
        const u64 T = nbr_codes_per_row(len[l], nsubs);
        const u64 n = (u64)sh.S * T;
        hipLaunchKernelGGL(nbr_insert_kernel, dim3((u32)((n + 255) / 256)), dim3(256), 0, s, vals[l], canon + l * sh.S,
                           sh.S, len[l], nsubs, T, nm.m[l], nm.mmask[l]);
    }
    hipLaunchKernelGGL(nbr_pair_kernel, dim3((u32)((sh.S + 255) / 256)), dim3(256), 0, s, canon, sh.S, rc, nm.p[0],
                       nm.pmask[0], nm.p[1], nm.pmask[1]);
    return hipGetLastError();
}

// one map probe chain from a slot already loaded (the caller issues the first loads of several chains
// together, so a code waits for one round trip per stage, not one per map)
__device__ __forceinline__ int nbr_resolve(const NSlot* __restrict__ t, u32 mask, u64 key, u32 h, NSlot e) {
    for (;;) {
        if (e.key == key) return ~e.vmin_c == e.vmax1 - 1u ? (int)~e.vmin_c : -2;
        if (e.key == 0) return -1;
        h = (h + 1) & mask;
        e = t[h];
    }
}

// nbr_find on the idx1, idx2 and (rc) rc(idx2) maps with the three first probes in flight together
__device__ __forceinline__ void nbr_find3(const NbrMap& nm, u64 q1, u64 q2, bool rc, int& a1, int& a2, int& a3) {
    const u64 k1 = q1 | NBR_KEY, k2 = q2 | NBR_KEY;
    const u32 h1 = (u32)mix64(k1) & nm.mmask[0], h2 = (u32)mix64(k2) & nm.mmask[1], h3 = (u32)mix64(k2) & nm.mmask[2];
    const NSlot e1 = nm.m[0][h1], e2 = nm.m[1][h2];
    const NSlot e3 = rc ? nm.m[2][h3] : NSlot{0, 0, 0};
    a1 = nbr_resolve(nm.m[0], nm.mmask[0], k1, h1, e1);
    a2 = nbr_resolve(nm.m[1], nm.mmask[1], k2, h2, e2);
    a3 = rc ? nbr_resolve(nm.m[2], nm.mmask[2], k2, h3, e3) : -1;
}

__device__ __forceinline__ void pair_resolve(const PSlot* __restrict__ t, u32 mask, u64 key, u32 h, PSlot e, int& both,
                                             int& r) {
    for (;;) {
        if (e.key == key) {
            both = (int)e.cnt;
            r = (int)~e.first_c;
            return;
        }
        if (e.key == 0) return;
        h = (h + 1) & mask;
        e = t[h];
    }
}

// class_pair's result from the map probes: the rows near q1 are exactly the rows holding value a1 (a
// single distinct value), so its first row is a1 and |M1 ∩ M2| is the pair count of (a1, a2).  The two
// pair maps' first probes are in flight together.
__device__ __forceinline__ void class_pair_nbr(const NbrMap& nm, int a1, int a2, int a3, int& m1, int& m2, int& cls,
                                               int& row, int& rm2, int& rcls, int& rrow) {
    int both = 0, r = -1, rboth = 0, rr = -1;
    const bool f0 = a1 >= 0 && a2 >= 0, f1 = a1 >= 0 && a3 >= 0;
    const u64 pk0 = ((u64)(u32)a1 << 32) | (u32)a2 | NBR_KEY, pk1 = ((u64)(u32)a1 << 32) | (u32)a3 | NBR_KEY;
    const u32 ph0 = (u32)mix64(pk0) & nm.pmask[0], ph1 = (u32)mix64(pk1) & nm.pmask[1];
    const PSlot p0 = f0 ? nm.p[0][ph0] : PSlot{0, 0, 0};
    const PSlot p1 = f1 ? nm.p[1][ph1] : PSlot{0, 0, 0};
    if (f0) pair_resolve(nm.p[0], nm.pmask[0], pk0, ph0, p0, both, r);
    if (f1) pair_resolve(nm.p[1], nm.pmask[1], pk1, ph1, p1, rboth, rr);
    m1 = a1;
    m2 = a2;
    rm2 = a3;
    if (m1 >= 0 && m2 >= 0) {
        cls = both == 0 ? CLS_HOP : both == 1 ? CLS_DEMUX : CLS_AMBIG;
        row = both == 1 ? r : -1;
    } else {
        cls = CLS_UNDET;
        row = -1;
    }
    if (m1 >= 0 && rm2 >= 0) {
        rcls = rboth == 0 ? CLS_HOP : rboth == 1 ? CLS_DEMUX : CLS_AMBIG;
        rrow = rboth == 1 ? rr : -1;
    } else {
        rcls = CLS_UNDET;
        rm2 = -1;
        rrow = -1;
    }
    if (cls == CLS_UNDET) {  // pass A keeps matched_idx1 from the rc call (frender.py:319-323)
        if (rcls == CLS_UNDET) m1 = -1;
        m2 = -1;
    }
}

// One lane per unique code.  The sheet images (u32 when every entry has <= 10 symbols, else
// u64) and the per-name rc sums live in dynamic LDS sized to the sheet; sheets too large for it
// are read from HBM.
template <typename W>
__global__ __launch_bounds__(CLS_WG) void classify_kernel(const u64* keys, const u64* counts, u64 n, SheetArgs sh,
                                                          int nsubs, int rc, ClassOut o, NbrMap nm,
                                                          int sheet_in_lds, int names_in_lds) {
    extern __shared__ __attribute__((aligned(16))) u8 cls_lds[];
    unsigned long long* lf = (unsigned long long*)cls_lds;
    unsigned long long* lr = lf + (names_in_lds ? sh.n_names : 0);
    W* s1 = (W*)(lr + (names_in_lds ? sh.n_names : 0));
    W* s2 = s1 + sh.S;
    W* s2rc = s2 + sh.S;
    if (sheet_in_lds) {
        for (int i = threadIdx.x; i < sh.S; i += CLS_WG) {
            s1[i] = (W)sh.i1[i];
            s2[i] = (W)sh.i2[i];
            s2rc[i] = rc ? (W)sh.i2rc[i] : (W)0;
        }
    }
    if (rc && names_in_lds)
        for (int i = threadIdx.x; i < sh.n_names; i += CLS_WG) lf[i] = lr[i] = 0;
    __syncthreads();
    // sheets outside LDS: W is u64 then (the launcher guarantees it)
    const W* S1 = sheet_in_lds ? s1 : (const W*)sh.i1;
    const W* S2 = sheet_in_lds ? s2 : (const W*)sh.i2;
    const W* S2rc = sheet_in_lds ? s2rc : (const W*)sh.i2rc;

    // grid-stride: the per-name sums stay in LDS over many codes (one flush per workgroup: the
    // flush's atomics all land on the same 2 x names addresses)
    for (u64 u = blockIdx.x * (u64)CLS_WG + threadIdx.x; u < n; u += (u64)gridDim.x * CLS_WG) {
        const u64 key = keys[u];
        // split the code at '+': idx1, idx2 = code.split("+")[0:2]  (frender.py:306), both case-folded
        // and packed 3 bits per letter (a1 c2 g3 t4 n5) like the sheet
        int n1 = 0, n2 = 0;
        bool plus = false;
        u64 q1 = 0, q2 = 0;
        if (key & WIDE_BIT) {  // wide key (fr_internal.h): base-5 letters, '+' position in bits 57-61
            const u64 V = key & ((1ull << 57) - 1ull);
            const int pp = (int)((key >> 57) & 31u);
            int nl = 0;
            u64 off = 0, pw = 1;
            while (nl < WIDE_MAXN && off + pw <= V) {  // off = (5^nl - 1) / 4
                off += pw;
                pw *= 5;
                ++nl;
            }
            u64 D = V - off;
            plus = pp != WIDE_NOPLUS;
            n1 = plus ? pp : nl;
            n2 = plus ? nl - pp : 0;
            for (int i = 0; i < nl; ++i) {
                const u64 sy = D % 5u + 1u;
                D /= 5u;
                if (i < n1) q1 |= sy << (3 * i);
                else q2 |= sy << (3 * (i - n1));
            }
        } else {  // fast key: symbols A1 C2 G3 T4 N5 '+'6, folded they equal the sheet's a1..n5
            // SWAR over the 21 3-bit groups: len = symbols before the first empty group; the '+'
            // groups (== 6) among them give p1, p2 (no per-symbol loop)
            constexpr u64 G0 = 0x1249249249249249ull & ((1ull << 63) - 1ull);  // bit 0 of each group
            const u64 nz = (key | (key >> 1) | (key >> 2)) & G0;                // groups holding a symbol
            const u64 empty = ~nz & G0;
            const int len = empty ? (int)(__builtin_ctzll(empty) / 3) : MAXSYM;
            const u64 x = key ^ (G0 * 6ull);                                    // '+' groups become 0
            u64 pm = ~(x | (x >> 1) | (x >> 2)) & G0;
            pm &= len < MAXSYM ? (1ull << (3 * len)) - 1ull : ~0ull;
            const int p1 = pm ? (int)(__builtin_ctzll(pm) / 3) : -1;
            pm &= pm - 1ull;
            const int p2 = pm ? (int)(__builtin_ctzll(pm) / 3) : MAXSYM;
            plus = p1 >= 0;
            if (plus) {
                n1 = p1;
                const int e2 = p2 < len ? p2 : len;
                n2 = e2 - p1 - 1;
                q1 = n1 ? (key & ((1ull << (3 * n1)) - 1ull)) : 0ull;
                q2 = n2 ? ((key >> (3 * (p1 + 1))) & ((1ull << (3 * n2)) - 1ull)) : 0ull;
            }
        }
        int err = 0;
        int m1 = -1, m2 = -1, cls = CLS_UNDET, row = -1;
        int rm2 = -1, rcls = CLS_UNDET, rrow = -1;
        if (!plus) {
            err = 3;
        } else {
            // the length asserts (frender.py:227-229), idx1 list first
            if (sh.S > 0 && (sh.L1u == -2 || sh.L1u != n1)) err = 1;
            else if (sh.S > 0 && (sh.L2u == -2 || sh.L2u != n2)) err = 2;
            else {
                int a1 = -2, a2 = -2, a3 = -1;
                if (nm.on) nbr_find3(nm, q1, q2, rc != 0, a1, a2, a3);
                if (a1 != -2 && a2 != -2 && a3 != -2)
                    class_pair_nbr(nm, a1, a2, a3, m1, m2, cls, row, rm2, rcls, rrow);
                else if (FR_CLS_SCALAR && rc)
                    class_pair_s<W, true>((W)q1, (W)q2, sh.i1, sh.i2, sh.i2rc, sh.S, nsubs, m1, m2, cls, row, rm2,
                                          rcls, rrow);
                else if (FR_CLS_SCALAR)
                    class_pair_s<W, false>((W)q1, (W)q2, sh.i1, sh.i2, sh.i2rc, sh.S, nsubs, m1, m2, cls, row, rm2,
                                           rcls, rrow);
                else
                    class_pair<W>((W)q1, (W)q2, S1, S2, S2rc, sh.S, nsubs, rc != 0, m1, m2, cls, row, rm2, rcls, rrow);
                // both calls demuxable to different sample NAMES -> ambiguous (frender.py:336-349)
                if (rc && cls == CLS_DEMUX && rcls == CLS_DEMUX && sh.name[row] != sh.name[rrow]) {
                    cls = CLS_AMBIG;
                    row = -1;
                    rcls = CLS_AMBIG;
                    rrow = -1;
                }
            }
        }
        if (err) {
            atomicMax((unsigned long long*)o.err_first, (unsigned long long)~u);  // = min u
            if (o.err_which) o.err_which[u] = err;
        } else if (o.err_which) {
            o.err_which[u] = 0;
        }
        o.m1[u] = (int16_t)m1;
        o.m2[u] = (int16_t)m2;
        o.cls[u] = (u8)cls;
        o.row[u] = (int16_t)row;
        if (rc) {
            o.rc_m2[u] = (int16_t)rm2;
            o.rc_cls[u] = (u8)rcls;
            o.rc_row[u] = (int16_t)rrow;
            // the record count only where a sum takes it (most codes are hops or undetermined)
            const u64 cnt = (cls == CLS_DEMUX || rcls == CLS_DEMUX) ? counts[u] : 0ull;
            if (cls == CLS_DEMUX) {
                const int nm = sh.name[row];
                if (names_in_lds) atomicAdd(&lf[nm], (unsigned long long)cnt);
                else atomicAdd((unsigned long long*)&o.rc_f[nm], (unsigned long long)cnt);
            }
            if (rcls == CLS_DEMUX) {
                const int nm = sh.name[rrow];
                if (names_in_lds) atomicAdd(&lr[nm], (unsigned long long)cnt);
                else atomicAdd((unsigned long long*)&o.rc_r[nm], (unsigned long long)cnt);
            }
        }
    }
    if (rc && names_in_lds) {
        __syncthreads();
        for (int i = threadIdx.x; i < sh.n_names; i += CLS_WG) {
            if (lf[i]) atomicAdd((unsigned long long*)&o.rc_f[i], lf[i]);
            if (lr[i]) atomicAdd((unsigned long long*)&o.rc_r[i], lr[i]);
        }
    }
}

hipError_t launch_classify(const u64* keys, const u64* counts, u64 n, SheetArgs sh, int nsubs, int rc, ClassOut o,
                           const NbrMap& nm, hipStream_t s) {
    if (!n) return hipSuccess;
    // u32 images when every sheet entry (and so every matching query) has <= 10 symbols
    const bool narrow = sh.S > 0 && sh.L1u >= 0 && sh.L1u <= 10 && sh.L2u >= 0 && sh.L2u <= 10;
    const size_t wb = narrow ? 4 : 8;
    const size_t names_bytes = rc ? 2ull * 8 * sh.n_names : 0;
    const size_t sheet_bytes = 3 * wb * (size_t)std::max(sh.S, 0);
    const int names_in_lds = (rc && names_bytes <= CLS_LDS_BYTES / 2) ? 1 : 0;
    const size_t nb = names_in_lds ? names_bytes : 0;
    // the scalar-load path (FR_CLS_SCALAR) reads the rows from HBM; only the name sums use LDS then
    const int sheet_in_lds = (!FR_CLS_SCALAR && nb + sheet_bytes <= CLS_LDS_BYTES) ? 1 : 0;
    const size_t lds = nb + (sheet_in_lds ? sheet_bytes : 0) + 16;
    const u64 grid = std::min<u64>((n + CLS_WG - 1) / CLS_WG, 2048);
    const bool wide = !(narrow && (sheet_in_lds || FR_CLS_SCALAR));
    if (!wide)
        hipLaunchKernelGGL(classify_kernel<u32>, dim3((u32)grid), dim3(CLS_WG), lds, s, keys, counts, n, sh, nsubs, rc,
                           o, nm, sheet_in_lds, names_in_lds);
    else
        hipLaunchKernelGGL(classify_kernel<u64>, dim3((u32)grid), dim3(CLS_WG), lds, s, keys, counts, n, sh, nsubs, rc,
                           o, nm, sheet_in_lds, names_in_lds);
    return hipGetLastError();
}

// generic classifier over case-folded code points (codes outside the fast alphabet)
__device__ void class_of_cp(const u32* q1, int n1, const u32* q2, int n2, const u32* s1, const u32* s2, int stride,
                            int S, int nsubs, int& m1, int& m2, int& cls, int& row) {
    m1 = -1;
    m2 = -1;
    int both = 0, r = -1;
    for (int i = 0; i < S; ++i) {
        int d1 = 0, d2 = 0;
        for (int k = 0; k < n1; ++k) d1 += q1[k] != s1[(u64)i * stride + k];
        for (int k = 0; k < n2; ++k) d2 += q2[k] != s2[(u64)i * stride + k];
        const bool a = d1 <= nsubs, b = d2 <= nsubs;
        if (a && m1 < 0) m1 = i;
        if (b && m2 < 0) m2 = i;
        if (a && b) {
            if (!both) r = i;
            ++both;
        }
    }
    if (m1 >= 0 && m2 >= 0) {
        cls = both == 0 ? CLS_HOP : both == 1 ? CLS_DEMUX : CLS_AMBIG;
        row = both == 1 ? r : -1;
    } else {
        cls = CLS_UNDET;
        m1 = m2 = row = -1;
    }
}

__global__ void classify_cp_kernel(int n, const u32* q1, const int32_t* q1len, const u32* q2, const int32_t* q2len,
                                   int stride, int S, const u32* s1, const int32_t* s1len, const u32* s2,
                                   const int32_t* s2len, const u32* s2rc, const int32_t* name, int nsubs, int rc,
                                   ClassOut o) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= n) return;
    const int n1 = q1len[u], n2 = q2len[u];
    int err = 0;
    for (int i = 0; i < S && !err; ++i)
        if (s1len[i] != n1) err = 1;
    for (int i = 0; i < S && !err; ++i)
        if (s2len[i] != n2) err = 2;
    int m1 = -1, m2 = -1, cls = CLS_UNDET, row = -1, rm2 = -1, rcls = CLS_UNDET, rrow = -1;
    if (!err) {
        class_of_cp(q1 + (u64)u * stride, n1, q2 + (u64)u * stride, n2, s1, s2, stride, S, nsubs, m1, m2, cls, row);
        if (rc) {
            int rm1;
            class_of_cp(q1 + (u64)u * stride, n1, q2 + (u64)u * stride, n2, s1, s2rc, stride, S, nsubs, rm1, rm2,
                        rcls, rrow);
            if (cls == CLS_UNDET && rcls != CLS_UNDET) m1 = rm1;  // matched_idx1 of pass A (frender.py:319-323)
            if (cls == CLS_DEMUX && rcls == CLS_DEMUX && name[row] != name[rrow]) {
                cls = rcls = CLS_AMBIG;
                row = rrow = -1;
            }
        }
    }
    if (o.err_which) o.err_which[u] = err;
    o.m1[u] = (int16_t)m1;
    o.m2[u] = (int16_t)m2;
    o.cls[u] = (u8)cls;
    o.row[u] = (int16_t)row;
    if (rc) {
        o.rc_m2[u] = (int16_t)rm2;
        o.rc_cls[u] = (u8)rcls;
        o.rc_row[u] = (int16_t)rrow;
    }
}

hipError_t launch_classify_cp(int n, const u32* q1, const int32_t* q1len, const u32* q2, const int32_t* q2len,
                              int stride, int S, const u32* s1, const int32_t* s1len, const u32* s2,
                              const int32_t* s2len, const u32* s2rc, const int32_t* name, int nsubs, int rc,
                              ClassOut o, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(classify_cp_kernel, dim3((n + 127) / 128), dim3(128), 0, s, n, q1, q1len, q2, q2len, stride,
                       S, s1, s1len, s2, s2len, s2rc, name, nsubs, rc, o);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// SYN-v1 generator (byte-identical to frender_amd/synth.py generate_records)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ u64 syn_h(u64 base, u64 r, u32 k) { return mix64(((r << 8) | k) ^ base); }

__global__ void synth_kernel(u8* out, u64 r0, u64 n, int R, u64 base, const u8* idx1, const u8* idx2, int S, int L1,
                             int L2) {
    const u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u64 r = r0 + i;
    const int reclen = 36 + L1 + 1 + L2 + 1 + 2 * R + 4;
    u8* o = out + i * (u64)reclen;
    const char* ACGT = "ACGT";
    u8 idx[64];
    const u64 s = syn_h(base, r, 0) % (u64)S;
    for (int j = 0; j < L1; ++j) idx[j] = idx1[s * L1 + j];
    for (int j = 0; j < L2; ++j) idx[L1 + j] = idx2[s * L2 + j];
    if (syn_h(base, r, 1) % 10000ull < 200ull) {
        const u64 s2 = syn_h(base, r, 2) % (u64)S;
        for (int j = 0; j < L2; ++j) idx[L1 + j] = idx2[s2 * L2 + j];
    }
    if (syn_h(base, r, 3) % 10000ull < 100ull) {
        const u64 hj = syn_h(base, r, 4);
        for (int j = 0; j < L1 + L2; ++j) idx[j] = ACGT[(hj >> (2 * j)) & 3ull];
    }
    for (int j = 0; j < L1 + L2; ++j) {
        const u64 v = syn_h(base, r, 8 + j);
        const u64 p = v % 10000ull;
        if (p < 50ull) {
            const u8 c = idx[j];
            const u64 orig = c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : 0;
            idx[j] = ACGT[(orig + 1ull + (v >> 32) % 3ull) % 4ull];
        } else if (p < 70ull) {
            idx[j] = 'N';
        }
    }
    int pos = 0;
    const char* h0 = "@SYN:1:FCX:1:";
    for (int k = 0; k < 13; ++k) o[pos++] = h0[k];
    u64 v = (r / 10000000000ull) % 10000ull;
    for (int k = 3; k >= 0; --k) { o[pos + k] = '0' + (u8)(v % 10ull); v /= 10ull; }
    pos += 4;
    o[pos++] = ':';
    v = (r / 100000ull) % 100000ull;
    for (int k = 4; k >= 0; --k) { o[pos + k] = '0' + (u8)(v % 10ull); v /= 10ull; }
    pos += 5;
    o[pos++] = ':';
    v = r % 100000ull;
    for (int k = 4; k >= 0; --k) { o[pos + k] = '0' + (u8)(v % 10ull); v /= 10ull; }
    pos += 5;
    const char* h1 = " 1:N:0:";
    for (int k = 0; k < 7; ++k) o[pos++] = h1[k];
    for (int j = 0; j < L1; ++j) o[pos++] = idx[j];
    o[pos++] = '+';
    for (int j = 0; j < L2; ++j) o[pos++] = idx[L1 + j];
    o[pos++] = '\n';
    for (int w = 0; w < (R + 31) / 32; ++w) {
        const u64 hv = syn_h(base, r, 80 + w);
        for (int j = 32 * w; j < R && j < 32 * w + 32; ++j) o[pos + j] = ACGT[(hv >> (2 * (j - 32 * w))) & 3ull];
    }
    pos += R;
    o[pos++] = '\n';
    o[pos++] = '+';
    o[pos++] = '\n';
    for (int w = 0; w < (R + 7) / 8; ++w) {
        const u64 hv = syn_h(base, r, 100 + w);
        for (int j = 8 * w; j < R && j < 8 * w + 8; ++j) o[pos + j] = (u8)(((hv >> (8 * (j - 8 * w))) & 0xFFull) % 42ull) + 33;
    }
    pos += R;
    o[pos++] = '\n';
}

hipError_t launch_synth(u8* out, u64 r0, u64 n, int R, u64 seed, const u8* idx1, const u8* idx2, int S, int L1,
                        int L2, hipStream_t s) {
    if (!n) return hipSuccess;
    const u64 base = mix64(seed + 0x9E3779B97F4A7C15ull);
    const u64 grid = (n + 255) / 256;
    hipLaunchKernelGGL(synth_kernel, dim3((u32)grid), dim3(256), 0, s, out, r0, n, R, base, idx1, idx2, S, L1, L2);
    return hipGetLastError();
}

}  // namespace fr
