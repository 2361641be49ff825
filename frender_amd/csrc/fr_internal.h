// fr_internal.h — device data layout shared by the kernels (fr_kernels.hip) and the
// C-ABI context (fr_api.hip).  See DESIGN.md §3 for the HBM layout.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fr {

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;
typedef int64_t i64;

// ---- tally kernel geometry --------------------------------------------------------
constexpr int WG = 256;              // 4 waves of 64
constexpr int SEG = 64;              // contiguous bytes per lane
constexpr int TILE = 64 * SEG;       // bytes per wave-tile (one wave's step; chunks count these)
constexpr int TSTEP = TILE - SEG;    // tile stride: tiles overlap by one segment, so the bitmaps
                                     // of a tile's last own segment always have a successor
#ifndef FR_LOG_NS
#define FR_LOG_NS 10
#endif
constexpr int LOG_NS = FR_LOG_NS;
constexpr int NS = 1 << LOG_NS;      // LDS hash slots per workgroup
#ifndef FR_LPROBE
#define FR_LPROBE 2
#endif
constexpr int LPROBE = FR_LPROBE;          // LDS probe bound before going to HBM directly
constexpr int GPROBE = 256;          // HBM probe bound before the overflow list
constexpr int MAXSYM = 21;           // fast key: <= 21 symbols of 3 bits
// Wide keys: codes that are not fast keys but whose letters are all ACGTN or all
// acgtn, with at most one '+', each part <= 21 letters and <= 24 letters in total (12+12 dual
// indexes, lowercase files).  key = bit 63 | lowercase << 62 | plus position << 57 | V, with
// V = sum d_i 5^i + (5^n - 1) / 4 over the n letters (A0 C1 G2 T3 N4, case-folded): the length
// offset makes V unique across lengths, V < (5^25 - 1) / 4 < 2^57.  Plus position = letters before
// the '+', WIDE_NOPLUS without one.  Fast keys never set bit 63 (21 symbols x 3 bits).
constexpr u64 WIDE_BIT = 1ull << 63;
constexpr int WIDE_MAXN = 24;
constexpr int WIDE_NOPLUS = 31;
constexpr u64 RANGE_MAX = (16ull << 30) - (1ull << 20);  // bytes per tally launch (device feeds): positions
                                     // are u32 offsets inside a chunk (ScanShared::cbase), so a range is bounded
                                     // by the look-back arrays (tiles_cap) only
constexpr u64 RANGE_FIRST_MAX = (4ull << 30) - (1ull << 20);  // ranges of a device feed with no history (the
                                     // table grows between launches: a first feed of unknown cardinality is cut here)
constexpr u64 HOST_CHUNK_MAX = 1ull << 30;  // bytes per host-fed launch (pinned ring slot)
constexpr u64 RANGE_ROOM_MIN = 1ull << 20;  // smallest range of a device feed replayed for table room
constexpr u32 SPIN_MAX = 1u << 24;   // look-back spin bound (then FR_ERR_DEVICE)
constexpr int ORD_SHIFT = 44;        // ordinal = file_tag << 44 | file byte offset
constexpr int EXO_BUF = 32;          // chunk kernel: exotic records buffered while speculating
#ifndef FR_PHASE_LINES
#define FR_PHASE_LINES 16
#endif
constexpr int PHASE_LINES = FR_PHASE_LINES;  // lines the chunk phase guess looks at (>= 8)
constexpr u32 RARE_RING = 8192;      // chunk kernel: rare events queued per workgroup (a quarter per wave)
                                     // between drains (<= TILE/4 + 1 headers and 64 UTF-8 checks per wave-tile)

// ---- HBM structures ---------------------------------------------------------------
struct alignas(32) GSlot {           // open-addressing slot, one 32-B sector
    u64 key;                         // 0 = empty
    u64 count;
    u64 first;                       // min ordinal, ~0 = none
    u32 last_tag;                    // last file tag that inserted (presence detection)
    u32 uidx;                        // compact index (set by fr_finalize)
};

// One (code, file) presence pair, appended by presence_scan_kernel at the file's end (R10), with the
// code's running count at that moment: the per-file count (the reference's per-file dict,
// frender.py:171-177) is the difference to the code's previous pair (fr_get_presence_counts).  A file
// holds < 2^42 records (ordinal offsets are < 2^44 bytes and records >= 4 bytes), so the count kept
// modulo 2^44 gives exact differences.
constexpr int PRES_TAG_BITS = 20;    // file tags are < 2^20 (ordinal = tag << 44 | offset)
struct alignas(16) Presence {
    u64 key;
    u64 tc;                          // (running count mod 2^44) << 20 | file tag
};

struct alignas(32) Overflow {
    u64 key, count, first;
    u32 tag, pad;
};

// One tallied (code, count) pair on its way to the HBM table: a heavy chunk's LDS-table slots and
// cold-list misses go to the launch log at the chunk's commit, counted in LDS by the pairs' regions
// (log_region: the table home's top LOG_REGION_BITS bits) and appended as one run per region to that
// region's part of the log (one cursor atomic per region and commit: runs of tens of pairs).  After
// the launch a split pass counting-sorts every region's part by sub-region (the next LOG_SUB_BITS home
// bits) into the sub-region parts, and one workgroup per sub-region folds its part in LDS, so the HBM
// table sees one insert per distinct code per launch instead of one per commit and miss.
struct alignas(16) LogEntry {
    u64 key;
    u64 oc;              // min launch offset of the entry's records << LOG_CNT_BITS | records (log_pack): offsets of
                         // ranges up to RANGE_MAX (34 bits), so a logged launch may exceed 4 GiB
};
constexpr int LOG_CNT_BITS = 24;     // records of one key in one commit (a chunk): < 2^24 (else it inserts directly)
constexpr u64 LOG_CNT_MAX = (1ull << LOG_CNT_BITS) - 1ull;
__host__ __device__ inline u64 log_pack(u64 off, u64 cnt) { return (off << LOG_CNT_BITS) | cnt; }
__host__ __device__ inline u64 log_off(u64 oc) { return oc >> LOG_CNT_BITS; }
__host__ __device__ inline u32 log_cnt(u64 oc) { return (u32)(oc & LOG_CNT_MAX); }
#ifndef FR_LOG_REGION_BITS
#define FR_LOG_REGION_BITS 6
#endif
#ifndef FR_LOG_SUB_BITS
#define FR_LOG_SUB_BITS 3
#endif
constexpr int LOG_REGION_BITS = FR_LOG_REGION_BITS;
constexpr int LOG_NR = 1 << LOG_REGION_BITS;  // launch-log regions (parts of the log, one cursor each)
constexpr int LOG_SUB_BITS = FR_LOG_SUB_BITS;
constexpr int LOG_SUBS = 1 << LOG_SUB_BITS;   // sub-regions per region (aggregation workgroups)
constexpr int LOG_NSUB = LOG_NR * LOG_SUBS;    // sub-regions in all
#ifndef FR_LOG_DIRECT
#define FR_LOG_DIRECT 1
#endif
// round 6: commits append straight to the sub-region parts (LOG_NSUB runs per commit, no split pass);
// 0 = the region runs + split pass of rounds 4-5 (A/B builds)
constexpr bool LOG_DIRECT = FR_LOG_DIRECT != 0;
constexpr int LOG_NB = LOG_DIRECT ? LOG_NSUB : LOG_NR;  // a commit's log buckets
constexpr int AGG_LNS = 4096;  // LDS slots of one sub-region's fold in log_reduce_kernel (64 KB: 2 workgroups per CU)

struct DevState {
    // per-file block (contiguous: fr_begin_file resets it with one copy from the reset image)
    u64 lines[2];        // terminators before the current range (launch parity)
    u64 err_nospace;     // min file offset of a header without ' ' (~0 = none)
    u32 nonascii;        // a byte >= 0x80 was seen in the current file
    u32 utf8_bad;
    // per launch: the launch's last workgroup to exit zeroes them for the next launch
    u32 ticket;          // chunk ticket
    u32 chunks_done;     // chunks that published their line count
    u32 exits;           // workgroups that left the chunk loop
    u32 spin_fail;
    u32 spec_fail;       // a committed speculative chunk's guessed line phase was wrong (host redoes the feed)
    u64 n_keys;
    u64 n_overflow;
    u64 n_presence;
    u64 n_exotic;
    u64 exo_pool_used;
    u32 cap_flags;       // 1 presence, 2 overflow list, 4 exotic pool
    u32 spin_max;        // diagnostics: longest look-back wait (polls)
    u64 spin_total;      // diagnostics: total look-back polls that found a window not ready
    u64 log_n;           // entries appended to the launch log (may exceed its capacity: the rest went to HBM)
    u64 log_commits;     // commits that went to the launch log since the last reset (never emptied by the aggregation);
                         // a launch without a log counts the commits that would have logged
    u64 stamp[8];        // diagnostics (FR_STAMPS builds only): per-phase shader cycles, summed over workgroups
    // Heavy chunk geometry, decided on the device: the last workgroup to commit in a
    // launch sets heavy[par ^ 1] = (at least a quarter of the chunks since the reset logged their
    // commits); the next launch (parity par ^ 1) reads it at its start and never writes it, so every
    // workgroup of a launch walks the same geometry.  fr_reset zeroes all of it.
    u32 heavy[2];
    u32 commits_done;    // chunks of the current launch that finished their commit (back to 0 by the last)
    u32 heavy_launches;  // ramped launches since the reset that walked the heavy geometry (diagnostics)
    u64 chunks_total;    // chunks committed since the reset
    u32 log_rcur[LOG_NR];  // per launch-log region: entries claimed this launch (the aggregation zeroes them)
    u32 log_scur[LOG_NSUB];  // per sub-region: entries the split pass placed (the aggregation zeroes them)
    u32 log_red_done;    // aggregation workgroups finished (the last zeroes it)
    u32 log_fold_max;    // the fullest sub-region fold (distinct codes) of the current device feed's aggregations
    u32 log_fold_over;   // entries that found their sub-region's fold full (inserted on their own)
};

struct Table {
    GSlot* slots;
    u64 mask;
    Overflow* ovf;
    u64 ovf_cap;
    Presence* pres;
    u64 pres_cap;
    u64* exo_ord;
    u64* exo_off;
    u32* exo_len;
    u64 exo_cap;
    u8* exo_pool;
    u64 exo_pool_cap;
};

struct ScanArgs {
    const u8* buf;       // range base (16-B aligned); bytes [0, len) are scanned
    u64 len;
    u64 avail;           // readable bytes from buf (headers may extend up to here)
    u64 file_offset;     // file offset of buf[0]
    u32 file_tag;        // file index + 1
    u32 par;             // launch parity: read lines[par], write lines[par ^ 1]
    u32 epoch;           // look-back tag of this launch (>= 1)
    u32 num_tiles;
    int own_start;       // position 0 is a line start handled by this launch
    int own_end;         // a line start at position len is handled by this launch
    int pre_valid;       // buf[-16..-1] readable (device-split ranges)
    u32 flush_at;        // LDS table key cap: past it, new codes go to the HBM table directly
    i64 max_records;     // -s, <= 0: none
    u32 chunk_tiles;     // chunk kernel: tiles per chunk (a workgroup's contiguous unit)
    u32 num_chunks;
    u32 ramp_g;          // 0: uniform chunks of chunk_tiles.  Else the first ramp_g chunks grow and the
                         // last ramp_g shrink linearly (chunk_bounds), so workgroups finish their chunks
                         // (look-back, HBM commit) at staggered times and all run out of work together
    u32 mid_chunks;      // full chunks between the two ramps
    u32 ramp_up_s;       // the smallest chunk of the ramp-up / ramp-down (tiles, >= 1; FR_RAMP_UP_S,
    u32 ramp_down_s;     // FR_RAMP_DOWN_S)
    u32 ramp_down_g;     // chunks of the ramp-down (ramp_g of them grow; FR_RAMP_DOWN_PCT of ramp_g shrink),
    u32 ramp_down_g_h;   // and of the heavy geometry's (FR_RAMP_DOWN_PCT_H: its commits take longer)
    u32 chunk_tiles_h;   // the heavy geometry of the same ramped launch (num_chunks_h = 0: none; the
    u32 mid_chunks_h;    // kernel picks it when DevState::heavy[par] is set)
    u32 num_chunks_h;
    u32 cold_cap;        // chunk kernel: entries of each workgroup's cold list
    u64* cold;           // chunk kernel: cold lists, [grid][cold_cap] x {key, ordinal}
    uint4* rare;         // chunk kernel: rare-event rings, [grid][RARE_RING] (fr_kernels.hip)
    u64* chunk_info;     // chunk kernel: per chunk {line count, spec flag + guessed phase << 1 in the high word}
    LogEntry* log;       // the launch log (nullptr: commits insert into the HBM table directly)
    u64 log_cap;         // LOG_NB x log_rcap
    u32 log_rcap;        // entries per log bucket (a run past it inserts directly)
    u32 log_min;         // a commit of at least log_min pairs goes to the log, smaller ones straight into the table
    u32 log_hot;         // ... except its LDS entries of at least log_hot records, which insert directly
    u32 exo_only;        // replay of a launch whose exotic list overflowed: capture exotic records only (no
                         // table updates), every chunk with its exact line phase
    u32 spec_commit;     // commit speculative chunks without waiting for their exact prefix (checked at the
                         // launch end by verify_launch; a wrong guess sets spec_fail)
    DevState* st;
    u64* tiles;          // look-back descriptors
    const Table* tab;    // device copy (the exotic-only replay's table after the exotic list grew)
    Table tabv;          // the table by value: read from the kernarg segment where used (scalar loads,
                         // no dependent global load before a commit's first slot load)
};

// tiles before ramp chunk j of a ramp of G chunks growing from s to C tiles (chunk_bounds)
__host__ __device__ inline u64 ramp_tiles_before(u64 C, u64 G, u64 s, u64 j) {
    return s * j + ((C - s) * j * (j + 1)) / (2ull * G);
}

struct SheetArgs {
    int S;
    int n_names;
    int L1u;             // common case-folded idx1 length, -1 empty sheet, -2 mixed
    int L2u;
    const u64* i1;
    const u64* i2;
    const u64* i2rc;
    const int32_t* name;
};

struct ClassOut {
    int16_t* m1;
    int16_t* m2;
    u8* cls;
    int16_t* row;
    int16_t* rc_m2;
    u8* rc_cls;
    int16_t* rc_row;
    u64* rc_f;           // per name
    u64* rc_r;
    u64* err_first;      // ~(min unique index with an error), 0 none (zero-initialised with the rc sums)
    int32_t* err_which;  // per unique (optional): 1 idx1 len, 2 idx2 len, 3 no '+'
};

enum { CLS_UNDET = 0, CLS_HOP = 1, CLS_DEMUX = 2, CLS_AMBIG = 3 };

// Classify neighbourhood maps (fr_kernels.hip, nbr_*), built per (sheet, nsubs): for each sheet list
// (idx1, idx2, rc(idx2)) every packed code within nsubs substitutions of a distinct sheet value maps
// to that value's id = the first row holding it; a code near several distinct values is marked
// (vmin != vmax) and classified by the exact row scan.  The pair maps give, per (idx1 id, idx2 id),
// the rows holding both values: their count and first row.
constexpr u64 NBR_KEY = 1ull << 63;  // occupied-slot bit of a map key (packed codes use <= 63 bits)
struct NSlot {
    u64 key;     // packed code | NBR_KEY, 0 = empty
    u32 vmin_c;  // ~(smallest value id)   (atomicMax; 0 = none)
    u32 vmax1;   // largest value id + 1   (atomicMax)
};
struct PSlot {
    u64 key;      // (id1 << 32 | id2) | NBR_KEY
    u32 cnt;      // rows holding both values
    u32 first_c;  // ~(first such row)
};
struct NbrMap {
    NSlot* m[3];  // idx1, idx2, rc(idx2)
    u32 mmask[3];
    PSlot* p[2];  // (idx1, idx2), (idx1, rc(idx2))
    u32 pmask[2];
    int on;       // 0: every code takes the row scan
};

__host__ __device__ inline u64 mix64(u64 x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

// launch-log region of a code: the top bits of mix64, as the table's home slot, so a region's codes
// live in one contiguous part of a table of at least LOG_NR slots
__host__ __device__ inline u32 log_region(u64 key) { return (u32)(mix64(key) >> (64 - LOG_REGION_BITS)); }
// a commit's log bucket: the region, or with LOG_DIRECT the region and sub-region (region * LOG_SUBS + sub)
__host__ __device__ inline u32 log_bucket(u64 key) {
    return (u32)(mix64(key) >> (64 - LOG_REGION_BITS - (LOG_DIRECT ? LOG_SUB_BITS : 0)));
}
__host__ __device__ inline u32 log_subregion(u64 key) {
    return (u32)(mix64(key) >> (64 - LOG_REGION_BITS - LOG_SUB_BITS)) & (LOG_SUBS - 1);
}

// ---- launchers (fr_kernels.hip) --------------------------------------------------
hipError_t launch_table_init(GSlot* slots, u64 n, hipStream_t s);
hipError_t launch_chunk_scan(const ScanArgs& a, int grid, hipStream_t s);
int chunk_occupancy();  // tally workgroups per CU the kernel is built for
hipError_t launch_reinsert_overflow(Table t, DevState* st, const Overflow* src, u64 n, hipStream_t s);
hipError_t launch_rehash(Table dst, DevState* st, const GSlot* src, u64 nsrc, hipStream_t s);
hipError_t launch_compact(const GSlot* slots, u64 nslots, u64* keys, u64* counts, u64* first, u32* pos,
                          u64* counter, hipStream_t s);
hipError_t launch_set_uidx(GSlot* slots, u64 mask, const u64* keys, u64 n, const u32* rank_of_pos,
                           hipStream_t s);
hipError_t launch_order(const u64* first_in, const u32* pos_in, u64 n, u64* first_out, u32* perm_out,
                        void* temp, size_t* temp_bytes, int begin_bit, int end_bit, hipStream_t s);
hipError_t launch_gather(const u32* perm, u64 n, const u64* keys, const u64* counts, u64* keys_o,
                         u64* counts_o, u32* rank, hipStream_t s);
hipError_t launch_presence_one_file(const u64* counts, u64 n, u32 tag, u32* uidx, u32* file_idx, u64* snap,
                                    hipStream_t s);
hipError_t launch_presence_map(const GSlot* slots, u64 mask, const Presence* pres, u64 n, u32* uidx,
                               u32* file_idx, u64* snap, hipStream_t s);
// first-occurrence order by binning (fr_finalize without merged rows)
struct BinMap {
    u64 span;       // byte span given to each file tag (>= every ordinal offset)
    u32 first_tag;  // the context's first file tag
    u32 shift;      // bin = linear offset >> shift
    u64 nbins;      // bins (bin indices are clamped below it)
    u64 cap;        // rows of the scatter arrays
};
struct alignas(32) FinRow {  // one live slot on its way to its first-occurrence index
    u64 first, key, count;
    u32 slot, pad;
};
hipError_t launch_fin_hist(const GSlot* slots, u64 nslots, const BinMap& m, u32* cnt, u32* arr, hipStream_t s);
hipError_t launch_fin_scan(const u32* cnt, u32* base, u64 n, void* temp, size_t* temp_bytes, hipStream_t s);
hipError_t launch_fin_scatter(const GSlot* slots, u64 nslots, const BinMap& m, const u32* base, const u32* arr,
                              FinRow* rows, hipStream_t s);
hipError_t launch_fin_rank(GSlot* slots, u64 nk, const BinMap& m, const u32* base, const FinRow* rows, u64* keys_o,
                           u64* counts_o, u64* first_o, bool set_uidx, hipStream_t s);
hipError_t launch_classify(const u64* keys, const u64* counts, u64 n, SheetArgs sh, int nsubs, int rc,
                           ClassOut o, const NbrMap& nm, hipStream_t s);
// neighbourhood codes of one sheet row: sum over d <= nsubs of C(L, d) 5^d (every query symbol)
u64 nbr_codes_per_row(int L, int nsubs);
// (re)build the maps of nm (already allocated and zeroed) for the sheet sh; canon = 3 x S value ids
hipError_t launch_nbr_build(const SheetArgs& sh, const int32_t* canon, int nsubs, int rc, const NbrMap& nm,
                            hipStream_t s);
hipError_t launch_classify_cp(int n, const u32* q1, const int32_t* q1len, const u32* q2, const int32_t* q2len,
                              int stride, int S, const u32* s1, const int32_t* s1len, const u32* s2,
                              const int32_t* s2len, const u32* s2rc, const int32_t* name, int nsubs, int rc,
                              ClassOut o, hipStream_t s);
hipError_t launch_presence_scan(const GSlot* slots, u64 n, u32 tag, Presence* pres, u64 cap, DevState* st,
                                hipStream_t s);
hipError_t launch_merge(Table t, DevState* st, const u64* keys, const u64* counts, const u64* first, u64 n,
                        hipStream_t s);
// the multi-GPU merge's rows by owner rank (counts: world counters then world cursors, adjacent) and the
// row-major merge of received rows
hipError_t launch_partition_rows(const u64* keys, const u64* counts_in, const u64* first, u64 n, u32 world,
                                 u64* counts, u64* cursor, u64* rows, hipStream_t s);
hipError_t launch_merge_rows(Table t, DevState* st, const u64* rows, u64 n, hipStream_t s);
// aggregate the launch log into the table and empty it (stream-ordered; reads log_n and the region
// cursors on the device)
hipError_t launch_log_aggregate(Table t, DevState* st, const LogEntry* log, u32 rcap, LogEntry* sub, u32 scap,
                                u32 file_tag, u64 file_offset, hipStream_t s);
size_t log_aggregate_temp_bytes();
hipError_t launch_synth(u8* out, u64 r0, u64 n, int R, u64 seed, const u8* idx1, const u8* idx2, int S, int L1,
                        int L2, hipStream_t s);

}  // namespace fr
