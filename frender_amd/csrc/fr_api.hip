// fr_api.hip — the C ABI of libfrender_hip.so (declared in include/frender_amd.h).
//
// Host-side owner of one GPU's scan state: the pinned ring for host feeds, the HBM hash
// table (grown between launches, never during one: the overflow list absorbs in-flight
// growth), the look-back descriptors, the sheet image, and the finalized unique table.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/frender_amd.h"
#include "fr_internal.h"

using namespace fr;

// Host bytes into the pinned ring: one thread copies ~8-10 GB/s, so a scan's decoded files (GBs)
// would spend a fifth of a second per GB here alone; large copies split over up to 8 threads.
static void pinned_copy(u8* dst, const u8* src, u64 n) {
    constexpr u64 PART = 16ull << 20;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const u64 k = std::min<u64>({8, hw, n / PART});
    if (k < 2) {
        std::memcpy(dst, src, n);
        return;
    }
    std::vector<std::thread> t;
    const u64 per = (n + k - 1) / k;
    for (u64 i = 1; i < k; ++i) {
        const u64 b = i * per, e = std::min(n, b + per);
        if (b < e) t.emplace_back([=] { std::memcpy(dst + b, src + b, e - b); });
    }
    std::memcpy(dst, src, std::min(n, per));
    for (auto& x : t) x.join();
}

struct fr_ctx {
    int device = 0;
    GSlot* snap = nullptr;         // a speculative device feed's rollback copy of the table (kept between feeds)
    u64 snap_cap = 0;
    hipStream_t stream = nullptr;  // tally / classify / table kernels
    hipStream_t copy = nullptr;    // H2D of host feeds
    std::string err;
    int grid = 0;
    u32 flush_at = NS * 3 / 4;
    u64* cold = nullptr;
    u32 cold_cap = 8192;
    // launch log (fr_internal.h LogEntry): commits append, launch_log_aggregate folds it into the table
    LogEntry* log = nullptr;
    u64 log_cap = 0;
    u32 log_rcap = 0;              // entries per log region (LOG_NR regions)
    LogEntry* log_sub = nullptr;   // the split pass's sub-region parts (LOG_NSUB x log_scap)
    u32 log_scap = 0;
    void* log_temp = nullptr;
    size_t log_temp_bytes = 0;
    u32 log_min = 0;               // pairs from which a commit logs (round 6: every commit.  Direct commits are bound by
                                   // the memory-side atomics, ~23.7 G/s chip-wide whatever their scope or footprint:
                                   // scripts/ubench_l2atomic.hip; config 2's ~12M per 100M reads cost 0.4 ms)
    u32 log_hot = 0xFFFFFFFFu;     // a logged commit's LDS entries of >= log_hot records insert directly (round 6: none)
    uint4* rare = nullptr;

    DevState* st = nullptr;
    DevState* h_st = nullptr;      // pinned snapshot
    DevState* h_zero = nullptr;    // pinned reset image (zero counters, no error), never modified
    u8* h_byte = nullptr;          // pinned: a device feed's last byte (copied with the feed's state read), and at
                                   // bytes 8-15 fr_classify's error flag
    // fr_finalize returns without a host round trip; its live-count check and timing settle at the
    // next call that synchronises (settle_finalize)
    u64* h_fin = nullptr;          // pinned: the finalize's live-slot count
    hipEvent_t fin_e0 = nullptr, fin_e1 = nullptr;
    hipEvent_t cls_e0 = nullptr, cls_e1 = nullptr;  // fr_classify's timing (created once, not per call)
    bool fin_pending = false;
    u64 fin_expect = 0;
    bool st_fresh = false;         // h_st equals the device state (no device work on it since)
    Table* d_tab = nullptr;        // device copy of tab for the tally kernel
    Table* h_tab = nullptr;        // pinned staging of that copy (last uploaded value)
    hipEvent_t st_ev = nullptr;
    bool st_pending = false;
    u64* tiles = nullptr;
    u64* chunk_info = nullptr;  // per chunk: line count + speculation flags (verify_launch)
    u64 tiles_cap = 0;
    bool spec_ok = true;        // FR_SPEC_COMMIT=0: every chunk waits for its exact prefix
    u64 spec_replays = 0;       // feeds replayed after a wrong speculative guess (diagnostics)
    u64 big_rollbacks = 0;      // device feeds replayed in smaller ranges: the table ran out of room in a launch
    bool grow_sync = false;     // maybe_grow waits for the previous launch's state (room replays)
    u32 spec_commit = 0;        // the current feed commits speculative chunks at once
    u32 epoch = 0;
    u32 par = 0;

    Table tab{};
    u64 nslots = 0;

    // launch sizes: chunk_bytes bytes per tally launch of device feeds (<= RANGE_MAX; <= RANGE_FIRST_MAX until a
    // previous device feed's new codes are known to fit the table again: feed_keys); host feeds
    // go through a pinned ring of ring_bytes slots (<= HOST_CHUNK_MAX)
    u64 chunk_bytes = 0;
    u64 ring_bytes = 0;
    u64 feed_keys = ~0ull;    // codes the last device feed created (a range over RANGE_FIRST_MAX needs table room for them)
    bool feed_logged = true;  // the last device feed's commits went to the launch log: its ranges stay <= RANGE_FIRST_MAX
                              // unless its folds had room (one aggregation over a bigger range has more distinct codes
                              // per sub-region than log_reduce_kernel's LDS fold holds: measured 15 ms instead of 0.28
                              // per launch at the config-3 shape)
    u32 feed_fold_max = 0;    // the last device feed's fullest sub-region fold, its fold overflows and range size:
    u32 feed_fold_over = 0;   // a logged feed's next ranges may exceed RANGE_FIRST_MAX when the folds, scaled by the
    u64 feed_step = 0;        // range size, stay at most 0.85 full
    u32 chunk_tiles = 320;  // wave-tiles (4 KiB) per full chunk of a ramped launch (FR_CHUNK_TILES; round 2's
                            // 80 workgroup tiles of 16 KiB: 64-96 measured within 2 %, 80 best)
    // Ramped launches after one in which at least a quarter of the chunks since the reset logged their
    // commits (many distinct codes per chunk: the config-3 shape) walk larger chunks: fewer, bigger
    // commits, all logged (FR_CHUNK_TILES_HEAVY; the config-3 shape's tally 1.61 -> 1.53 ms per launch at
    // 112, config 2 never logs and keeps 80).  The device decides (DevState::heavy, note_commit in
    // fr_kernels.hip); fr_reset clears it.
    u32 chunk_tiles_heavy = 448;
    u32 ramp_up_s = 1, ramp_down_s = 1;  // the ramps' smallest chunks (tiles)
    u32 ramp_down_pct = 100;              // ramp-down chunks, % of the grid (FR_RAMP_DOWN_PCT; the heavy
    u32 ramp_down_pct_h = 70;             // geometry's: FR_RAMP_DOWN_PCT_H, config-3 shape 3.39 -> 3.29 ms)
    bool ramp = true;      // FR_RAMP=0: one uniform chunk per workgroup
    u8* pin[2] = {nullptr, nullptr};
    u8* dbuf[2] = {nullptr, nullptr};
    hipEvent_t copied[2] = {nullptr, nullptr};
    hipEvent_t consumed[2] = {nullptr, nullptr};
    bool used[2] = {false, false};
    int cur = 0;
    std::vector<u8> carry;

    // current file
    bool scanning = false;
    bool file_open = false;
    u32 file_tag = 0;         // current (last) file's tag = file index + 1; increases within a scan
    u32 first_tag = 0;        // the first file's tag since fr_reset (0: none yet)
    // the first file's presence scan, deferred by fr_end_file (0: none pending): its pairs are every live
    // key.  A second file runs the scan before it tallies (flush_presence); a scan of that one file ends
    // with fr_finalize writing its pairs straight from the finalized table (launch_presence_one_file)
    u32 pres_defer_tag = 0;
    u64 file_base = 0;        // file offset of the current file's first fed byte (fr_begin_file_at)
    bool merged = false;  // the table holds ordinals merged from other contexts (any file tag)
    u64 max_file_bytes = 0;  // bytes of the longest file tallied since fr_reset (ordinal offsets are below it)
    u64 file_offset = 0;
    i64 max_records = 0;
    int last_byte = -1;
    u64 pres_before = 0;
    // exotic codes (outside the fast and wide key forms): the device captures each record's bytes
    // into a list sized per launch; the host drains it after every launch that produced records
    // and aggregates by exact byte string here (count, first ordinal, per-file presence)
    struct ExoCode {
        u64 count, first;
        u32 last_tag;
        u32 last_pair;  // its presence pair of the last file that held it
    };
    std::unordered_map<std::string, u32> exo_index;
    std::vector<std::string> exo_str;     // first-appearance order of the drains
    std::vector<ExoCode> exo_codes;
    std::vector<u32> exo_pres_code, exo_pres_file;
    std::vector<u64> exo_pres_count;      // records of the code in the pair's file
    u64 exo_new_file = 0;                 // distinct exotic codes of the current file
    u64 exo_records_file = 0;             // exotic records of the current file
    bool host_feed = false;               // launches come from fr_feed (each checked before the next)
    ScanArgs last_args{};                 // the previous launch (exotic-only replay after an overflow)
    int last_grid = 0;
    bool last_valid = false;
    u64 exo_replays = 0;
    bool sample_done = false;

    // sheet
    int S = -1;
    int n_names = 0;
    int L1u = -1, L2u = -1;
    u64 *d_i1 = nullptr, *d_i2 = nullptr, *d_i2rc = nullptr;
    int32_t* d_name = nullptr;
    u32 *d_cp1 = nullptr, *d_cp2 = nullptr, *d_cp2rc = nullptr;
    int32_t *d_cpl1 = nullptr, *d_cpl2 = nullptr;
    u8* d_sheet = nullptr;  // one device blob holding every sheet array above
    u8* h_sheet = nullptr;  // its pinned staging copy
    u64 sheet_cap = 0;
    u64 sheet_bytes = 0;  // the blob last uploaded (h_sheet holds it)
    int cp_stride = 0;
    int32_t* d_canon = nullptr;  // per list (idx1, idx2, rc(idx2)): the first row holding the row's value
    u64 sheet_ver = 0;           // bumped on every upload of a different sheet

    // classify neighbourhood maps (fr_internal.h NbrMap) of sheet version nbr_ver and nbr_nsubs
    u8* d_nbr = nullptr;
    u64 nbr_cap = 0;
    u64 nbr_ver = ~0ull;
    int nbr_nsubs = -1, nbr_rc = 0;
    NbrMap nbr{};
    bool nbr_enabled = true;  // FR_NBR=0: every code takes the row scan (A/B and tests)

    // finalized table
    u64 U = 0;
    u64 ucap = 0;
    u64 *d_keys = nullptr, *d_counts = nullptr, *d_first = nullptr;
    u64 *d_keys_s = nullptr, *d_counts_s = nullptr, *d_first_s = nullptr;
    u32 *d_pos = nullptr, *d_perm = nullptr, *d_rank = nullptr;
    u64* d_counter = nullptr;
    void* d_temp = nullptr;
    size_t temp_bytes = 0;
    u32 *d_bins = nullptr, *d_binbase = nullptr;  // first-occurrence bins (fr_finalize)
    u64 bins_cap = 0;
    u32* d_arr = nullptr;  // per table slot: arrival index in its bin
    u64 arr_cap = 0;
    FinRow* d_rows = nullptr;  // live slots grouped by bin
    u64 rows_cap = 0;
    u64 n_pres = 0;
    u64 pmap_cap = 0;
    u32 *d_pres_u = nullptr, *d_pres_f = nullptr;
    u64* d_pres_c = nullptr;  // per pair: the code's running count at its file's end (mod 2^44)
    u64 n_exo = 0;  // exotic codes of the finalized scan

    // classify scratch
    u64 ccap = 0;
    int16_t *d_m1 = nullptr, *d_m2 = nullptr, *d_row = nullptr, *d_rm2 = nullptr, *d_rrow = nullptr;
    u8 *d_cls = nullptr, *d_rcls = nullptr;
    int32_t* d_errw = nullptr;
    u64* d_errf = nullptr;
    u64 *d_rcf = nullptr, *d_rcr = nullptr;
    int rc_names_cap = 0;

    // timing
    std::vector<hipEvent_t> ev_a, ev_b, ev_l;
    size_t ev_used = 0;
    u64 scan_launches = 0, scan_bytes = 0;
    double classify_ms = 0, finalize_ms = 0;
    bool timing = true;  // fr_set_timing: record the timing events
    bool fin_timed = false;  // the pending fr_finalize recorded fin_e0
};

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            ctx->err = std::string(#x) + ": " + hipGetErrorString(e_);                         \
            return FR_ERR_HIP;                                                                 \
        }                                                                                      \
    } while (0)

static int fail(fr_ctx* ctx, int code, const std::string& msg) {
    ctx->err = msg;
    return code;
}

template <class T>
static hipError_t dalloc(T** p, u64 n) {
    return hipMalloc((void**)p, std::max<u64>(n, 1) * sizeof(T));
}

static u64 pow2_at_least(u64 x) {
    u64 p = 1;
    while (p < x) p <<= 1;
    return p;
}

static int state_reset_counts(fr_ctx* ctx) {
    // the device copy comes from a pinned image that never changes, so nothing waits for it; the
    // host snapshot is overwritten only once no asynchronous snapshot can still land on it
    if (ctx->st_pending) CK(hipStreamSynchronize(ctx->stream));
    *ctx->h_st = *ctx->h_zero;
    CK(hipMemcpyAsync(ctx->st, ctx->h_zero, sizeof(DevState), hipMemcpyHostToDevice, ctx->stream));
    ctx->st_pending = false;
    ctx->st_fresh = true;
    return FR_OK;
}

static int read_state(fr_ctx* ctx) {  // exact snapshot (a host round trip only when stale)
    if (ctx->st_fresh && !ctx->st_pending) return FR_OK;
    CK(hipMemcpyAsync(ctx->h_st, ctx->st, sizeof(DevState), hipMemcpyDeviceToHost, ctx->stream));
    CK(hipStreamSynchronize(ctx->stream));
    ctx->st_pending = false;
    ctx->st_fresh = true;
    return FR_OK;
}

// grow the table (x4) and/or re-insert overflow entries; stream-ordered between launches
static int grow_table(fr_ctx* ctx, bool force_bigger) {
    int rc = read_state(ctx);
    if (rc) return rc;
    const u64 nkeys = ctx->h_st->n_keys;
    const u64 novf = std::min<u64>(ctx->h_st->n_overflow, ctx->tab.ovf_cap);
    if (force_bigger || (nkeys + novf) * 2 > ctx->nslots) {
        u64 ns = ctx->nslots;
        while ((nkeys + novf) * 4 > ns) ns <<= 1;
        if (ns == ctx->nslots) ns <<= 1;
        GSlot* ns_slots = nullptr;
        CK(dalloc(&ns_slots, ns));
        CK(launch_table_init(ns_slots, ns, ctx->stream));
        Table t = ctx->tab;
        t.slots = ns_slots;
        t.mask = ns - 1;
        CK(launch_rehash(t, ctx->st, ctx->tab.slots, ctx->nslots, ctx->stream));
        CK(hipStreamSynchronize(ctx->stream));
        CK(hipFree(ctx->tab.slots));
        ctx->tab = t;
        ctx->nslots = ns;
    }
    if (novf) {
        Overflow* old = ctx->tab.ovf;
        Overflow* fresh = nullptr;
        CK(dalloc(&fresh, ctx->tab.ovf_cap));
        ctx->tab.ovf = fresh;
        CK(hipMemsetAsync(&ctx->st->n_overflow, 0, sizeof(u64), ctx->stream));
        CK(launch_reinsert_overflow(ctx->tab, ctx->st, old, novf, ctx->stream));
        ctx->st_fresh = false;
        CK(hipStreamSynchronize(ctx->stream));
        CK(hipFree(old));
    }
    return FR_OK;
}

// the presence list must take one more entry per live key (appended by the per-file scan)
static int ensure_presence_cap(fr_ctx* ctx) {
    int rc = read_state(ctx);
    if (rc) return rc;
    const u64 need = ctx->h_st->n_presence + ctx->h_st->n_keys + 1024;
    if (need <= ctx->tab.pres_cap) return FR_OK;
    u64 ncap = ctx->tab.pres_cap;
    while (ncap < need * 2) ncap *= 2;
    Presence* np = nullptr;
    CK(dalloc(&np, ncap));
    CK(hipMemcpyAsync(np, ctx->tab.pres, std::min(ctx->h_st->n_presence, ctx->tab.pres_cap) * sizeof(Presence),
                      hipMemcpyDeviceToDevice, ctx->stream));
    CK(hipStreamSynchronize(ctx->stream));
    CK(hipFree(ctx->tab.pres));
    ctx->tab.pres = np;
    ctx->tab.pres_cap = ncap;
    return FR_OK;
}

// the deferred presence scan of the first file (see fr_ctx::pres_defer_tag), before anything else
// changes the table's last tags
static int flush_presence(fr_ctx* ctx) {
    if (!ctx->pres_defer_tag) return FR_OK;
    int rc = ensure_presence_cap(ctx);
    if (rc) return rc;
    ctx->st_fresh = false;
    CK(launch_presence_scan(ctx->tab.slots, ctx->nslots, ctx->pres_defer_tag, ctx->tab.pres, ctx->tab.pres_cap,
                            ctx->st, ctx->stream));
    ctx->pres_defer_tag = 0;
    return read_state(ctx);
}

// called before each tally launch: act on the latest asynchronous snapshot, if ready
static int maybe_grow(fr_ctx* ctx) {
    if (ctx->st_pending) {
        if (ctx->grow_sync) CK(hipEventSynchronize(ctx->st_ev));
        else if (hipEventQuery(ctx->st_ev) != hipSuccess) return FR_OK;
        ctx->st_pending = false;
    } else if (!ctx->st_fresh) {
        return FR_OK;  // nothing new since the last decision
    }
    const DevState& s = *ctx->h_st;
    if (s.n_overflow || s.n_keys * 2 > ctx->nslots) return grow_table(ctx, false);
    return FR_OK;
}

static int snapshot_async(fr_ctx* ctx) {
    CK(hipMemcpyAsync(ctx->h_st, ctx->st, sizeof(DevState), hipMemcpyDeviceToHost, ctx->stream));
    CK(hipEventRecord(ctx->st_ev, ctx->stream));
    ctx->st_pending = true;
    return FR_OK;
}

// the last fr_finalize's check: every live slot was counted once (its pinned count has landed once
// fin_e1 has: the copy is queued before the event), and its device time
static int settle_finalize(fr_ctx* ctx) {
    if (!ctx->fin_pending) return FR_OK;
    ctx->fin_pending = false;
    CK(hipEventSynchronize(ctx->fin_e1));
    float ms = 0;
    if (ctx->fin_timed) CK(hipEventElapsedTime(&ms, ctx->fin_e0, ctx->fin_e1));
    ctx->finalize_ms = ms;
    if (*ctx->h_fin != ctx->fin_expect) return fail(ctx, FR_ERR_DEVICE, "compaction count mismatch");
    return FR_OK;
}

static int upload_table(fr_ctx* ctx) {
    if (std::memcmp(&ctx->tab, ctx->h_tab, sizeof(Table)) != 0) {  // the table moved: refresh its device copy
        CK(hipStreamSynchronize(ctx->stream));  // the previous copy from h_tab has landed
        std::memcpy(ctx->h_tab, &ctx->tab, sizeof(Table));
        CK(hipMemcpyAsync(ctx->d_tab, ctx->h_tab, sizeof(Table), hipMemcpyHostToDevice, ctx->stream));
    }
    return FR_OK;
}

// exotic list capacity for `need` records and `need_bytes` code bytes (contents are dropped: the
// list is empty whenever it grows)
static int grow_exotic(fr_ctx* ctx, u64 need, u64 need_bytes) {
    if (need > ctx->tab.exo_cap) {
        CK(hipStreamSynchronize(ctx->stream));
        const u64 cap = std::max<u64>(need + need / 4, 2 * ctx->tab.exo_cap);
        CK(hipFree(ctx->tab.exo_ord));
        CK(hipFree(ctx->tab.exo_off));
        CK(hipFree(ctx->tab.exo_len));
        ctx->tab.exo_ord = nullptr;
        ctx->tab.exo_off = nullptr;
        ctx->tab.exo_len = nullptr;
        CK(dalloc(&ctx->tab.exo_ord, cap));
        CK(dalloc(&ctx->tab.exo_off, cap));
        CK(dalloc(&ctx->tab.exo_len, cap));
        ctx->tab.exo_cap = cap;
    }
    if (need_bytes > ctx->tab.exo_pool_cap) {
        CK(hipStreamSynchronize(ctx->stream));
        const u64 cap = std::max<u64>(need_bytes + need_bytes / 4, 2 * ctx->tab.exo_pool_cap);
        CK(hipFree(ctx->tab.exo_pool));
        ctx->tab.exo_pool = nullptr;
        CK(dalloc(&ctx->tab.exo_pool, cap));
        ctx->tab.exo_pool_cap = cap;
    }
    return upload_table(ctx);
}

// Move the device's exotic records into the host aggregate and empty the list (the state must be
// exact and hold no overflow).  Stream-ordered: later launches append to the emptied list.
static int drain_exotic(fr_ctx* ctx) {
    DevState& s = *ctx->h_st;
    const u64 n = s.n_exotic, used = s.exo_pool_used;
    if (!n) return FR_OK;
    if (n > ctx->tab.exo_cap || used > ctx->tab.exo_pool_cap)
        return fail(ctx, FR_ERR_DEVICE, "exotic list drained while overflowed");
    std::vector<u64> ord(n), off(n);
    std::vector<u32> len(n);
    std::vector<u8> pool(used);
    CK(hipMemcpyAsync(ord.data(), ctx->tab.exo_ord, n * 8, hipMemcpyDeviceToHost, ctx->stream));
    CK(hipMemcpyAsync(off.data(), ctx->tab.exo_off, n * 8, hipMemcpyDeviceToHost, ctx->stream));
    CK(hipMemcpyAsync(len.data(), ctx->tab.exo_len, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (used) CK(hipMemcpyAsync(pool.data(), ctx->tab.exo_pool, used, hipMemcpyDeviceToHost, ctx->stream));
    CK(hipMemsetAsync(&ctx->st->n_exotic, 0, 2 * sizeof(u64), ctx->stream));  // n_exotic, exo_pool_used
    CK(hipStreamSynchronize(ctx->stream));
    s.n_exotic = 0;
    s.exo_pool_used = 0;
    // records arrive in no particular order: the first ordinal is a min, presence a per-file flag
    for (u64 i = 0; i < n; ++i) {
        std::string code((const char*)pool.data() + off[i], len[i]);
        auto it = ctx->exo_index.find(code);
        u32 k;
        if (it == ctx->exo_index.end()) {
            k = (u32)ctx->exo_codes.size();
            ctx->exo_index.emplace(code, k);
            ctx->exo_str.push_back(std::move(code));
            ctx->exo_codes.push_back({0, ~0ull, 0, 0});
        } else {
            k = it->second;
        }
        auto& e = ctx->exo_codes[k];
        e.count += 1;
        e.first = std::min(e.first, ord[i]);
        const u32 tag = (u32)(ord[i] >> ORD_SHIFT);
        if (e.last_tag != tag) {  // a file's records all carry its tag; files are scanned in order
            e.last_tag = tag;
            e.last_pair = (u32)ctx->exo_pres_code.size();
            ctx->exo_pres_code.push_back(k);
            ctx->exo_pres_file.push_back(tag - 1u);
            ctx->exo_pres_count.push_back(0);
            ctx->exo_new_file++;
        }
        ctx->exo_pres_count[e.last_pair] += 1;
    }
    ctx->exo_records_file += n;
    return FR_OK;
}

static int launch_args(fr_ctx* ctx, const ScanArgs& a, int grid);

// After a launch whose exotic records overflowed the list: grow it to the counted totals and run
// the same launch again capturing exotic records only (no table updates; exact line phases).  The
// launch's input is still resident (host feeds check every launch before the next one's data
// overwrites its ring slot).
static int replay_exotic(fr_ctx* ctx) {
    if (!ctx->last_valid) return fail(ctx, FR_ERR_DEVICE, "exotic overflow without a launch to replay");
    DevState& s = *ctx->h_st;
    int rc = grow_exotic(ctx, s.n_exotic, s.exo_pool_used);
    if (rc) return rc;
    s.n_exotic = 0;
    s.exo_pool_used = 0;
    s.cap_flags &= ~4u;
    CK(hipMemsetAsync(&ctx->st->n_exotic, 0, 2 * sizeof(u64), ctx->stream));
    CK(hipMemcpyAsync(&ctx->st->cap_flags, &s.cap_flags, sizeof(u32), hipMemcpyHostToDevice, ctx->stream));
    ScanArgs a = ctx->last_args;
    a.exo_only = 1;
    a.spec_commit = 0;
    a.log = nullptr;
    a.epoch = ++ctx->epoch;
    a.tab = ctx->d_tab;
    a.tabv = ctx->tab;
    CK(hipMemsetAsync(&ctx->st->ticket, 0, 2 * sizeof(u32), ctx->stream));  // ticket, chunks_done
    rc = launch_args(ctx, a, ctx->last_grid);
    if (rc) return rc;
    ctx->exo_replays++;
    ctx->st_fresh = false;
    rc = read_state(ctx);
    if (rc) return rc;
    if (ctx->h_st->cap_flags & 4u) return fail(ctx, FR_ERR_DEVICE, "exotic replay overflowed");
    return FR_OK;
}

// the previous launch's exotic records: replay it on overflow, then drain (exact state needed)
static int settle_exotic(fr_ctx* ctx) {
    int rc = read_state(ctx);
    if (rc) return rc;
    if (ctx->h_st->cap_flags & 4u) {
        rc = replay_exotic(ctx);
        if (rc) return rc;
    }
    return drain_exotic(ctx);
}

static int launch_args(fr_ctx* ctx, const ScanArgs& a, int grid) {  // the caller zeroed the ticket
    if (a.num_tiles > ctx->tiles_cap) return fail(ctx, FR_ERR_INVALID, "range larger than the look-back array");
    ctx->st_fresh = false;
    CK(launch_chunk_scan(a, grid, ctx->stream));
    return FR_OK;
}

static int launch_range(fr_ctx* ctx, const u8* dptr, u64 len, u64 avail, int own_start, int own_end, int pre_valid,
                        int exo_only = 0) {
    if (len == 0) return FR_OK;
    int rc = FR_OK;
    if (ctx->host_feed && ctx->last_valid) {
        // host feeds: the previous launch's exotic records are settled before this one is queued (its
        // ring slot is still intact for a replay); the H2D copy of this launch is already in flight
        rc = settle_exotic(ctx);
        if (rc) return rc;
    }
    rc = maybe_grow(ctx);
    if (rc) return rc;
    ScanArgs a;
    std::memset(&a, 0, sizeof(a));
    a.buf = dptr;
    a.len = len;
    a.avail = avail;
    a.file_offset = ctx->file_offset;
    a.file_tag = ctx->file_tag;
    a.par = ctx->par;
    a.epoch = ++ctx->epoch;
    a.num_tiles = (u32)((len + TSTEP - 1) / TSTEP);
    a.own_start = own_start;
    a.own_end = own_end;
    a.pre_valid = pre_valid;
    a.flush_at = ctx->flush_at;
    a.max_records = ctx->max_records;
    a.st = ctx->st;
    a.tiles = ctx->tiles;
    a.chunk_info = ctx->chunk_info;
    a.spec_commit = exo_only ? 0u : ctx->spec_commit;
    a.exo_only = (u32)exo_only;
    rc = upload_table(ctx);
    if (rc) return rc;
    a.tab = ctx->d_tab;
    a.tabv = ctx->tab;
    if (ctx->epoch >= 0x7FFFFFFFu) {  // tag wrap: restart epochs on a cleared descriptor array
        CK(hipMemsetAsync(ctx->tiles, 0, ctx->tiles_cap * sizeof(u64), ctx->stream));
        ctx->epoch = 1;
        a.epoch = 1;
    }
    // ticket / chunks_done / exits are zero here: the reset image, or the previous launch's last workgroup
    ctx->st_fresh = false;
    const bool timed = ctx->timing;
    if (timed && ctx->ev_used == ctx->ev_a.size()) {
        hipEvent_t e1, e2, e3;
        CK(hipEventCreate(&e1));
        CK(hipEventCreate(&e2));
        CK(hipEventCreate(&e3));
        ctx->ev_a.push_back(e1);
        ctx->ev_b.push_back(e2);
        ctx->ev_l.push_back(e3);
    }
    if (timed) CK(hipEventRecord(ctx->ev_a[ctx->ev_used], ctx->stream));
    // chunking (chunk_bounds in fr_kernels.hip): ramped when the range holds both ramps and a full
    // chunk, else one uniform chunk per workgroup.  A ramped launch also carries the heavy geometry
    // when the range fits it; the kernel picks one (DevState::heavy)
    const u64 G = (u64)ctx->grid, C = ctx->chunk_tiles, Ch = ctx->chunk_tiles_heavy;
    // the ramp-down's chunk count: a workgroup's last chunk ends with a commit of roughly fixed length,
    // so the shrinking chunks are spread over fewer tickets than the grid where commits are long
    const u64 Gd = std::max<u64>(1, G * ctx->ramp_down_pct / 100), Gdh = std::max<u64>(1, G * ctx->ramp_down_pct_h / 100);
    a.ramp_up_s = ctx->ramp_up_s;
    a.ramp_down_s = ctx->ramp_down_s;
    a.ramp_down_g = (u32)Gd;
    a.ramp_down_g_h = (u32)Gdh;
    auto ramps = [&](u64 c, u64 gd) {  // R_up(G) + R_down(gd) at chunk size c (chunk_bounds)
        return ramp_tiles_before(c, G, std::min<u64>(ctx->ramp_up_s, c), G) +
               ramp_tiles_before(c, gd, std::min<u64>(ctx->ramp_down_s, c), gd);
    };
    const u64 rg = ramps(C, Gd), rgh = ramps(Ch, Gdh);
    if (ctx->ramp && (u64)a.num_tiles >= rg + C) {
        a.ramp_g = (u32)G;
        a.chunk_tiles = (u32)C;
        a.mid_chunks = (u32)(((u64)a.num_tiles - rg + C - 1) / C);
        a.num_chunks = (u32)(G + Gd) + a.mid_chunks;
        if (Ch != C && (u64)a.num_tiles >= rgh + Ch) {
            a.chunk_tiles_h = (u32)Ch;
            a.mid_chunks_h = (u32)(((u64)a.num_tiles - rgh + Ch - 1) / Ch);
            a.num_chunks_h = (u32)(G + Gdh) + a.mid_chunks_h;
        }
    } else {
        a.ramp_g = 0;
        a.mid_chunks = 0;
        a.chunk_tiles = (u32)std::max<u64>(1, (a.num_tiles + G - 1) / G);
        a.num_chunks = (a.num_tiles + a.chunk_tiles - 1) / a.chunk_tiles;
    }
    a.cold_cap = ctx->cold_cap;
    a.cold = ctx->cold;
    // launch-log first occurrences fold in 32 bits (4-B ordinals: ranges up to RANGE_MAX); one aggregation's
    // distinct codes must fit its LDS fold, which fr_feed_device's range size sees to
    // (direct logging: the commits append to the sub-region parts, log_scap entries each)
    a.log = exo_only ? nullptr : LOG_DIRECT ? ctx->log_sub : ctx->log;
    a.log_cap = LOG_DIRECT ? (u64)ctx->log_scap * LOG_NSUB : ctx->log_cap;
    a.log_rcap = LOG_DIRECT ? ctx->log_scap : ctx->log_rcap;
    a.log_min = ctx->log_min;
    a.log_hot = ctx->log_hot;
    a.rare = ctx->rare;
    // workgroups take chunks by ticket; never more than the resident grid (cold lists are per block)
    const int grid = (int)std::min<u64>(a.num_chunks, G);
    rc = launch_args(ctx, a, grid);
    if (rc) return rc;
    ctx->last_args = a;
    ctx->last_grid = grid;
    ctx->last_valid = true;
    if (timed) CK(hipEventRecord(ctx->ev_b[ctx->ev_used], ctx->stream));
    if (a.log)
        CK(launch_log_aggregate(ctx->tab, ctx->st, ctx->log, ctx->log_rcap, ctx->log_sub, ctx->log_scap, a.file_tag,
                                a.file_offset, ctx->stream));
    if (timed) {
        CK(hipEventRecord(ctx->ev_l[ctx->ev_used], ctx->stream));
        ctx->ev_used++;
    }
    ctx->scan_launches++;
    ctx->scan_bytes += len;
    ctx->par ^= 1u;
    ctx->file_offset += len;
    ctx->max_file_bytes = std::max(ctx->max_file_bytes, ctx->file_offset);  // bounds every ordinal's offset
    return snapshot_async(ctx);
}

extern "C" {

void fr_tuning_defaults(fr_tuning* t) {
    if (!t) return;
    const fr_ctx d{};  // the defaults live in fr_ctx's initialisers
    std::memset(t, 0, sizeof(*t));
    t->size = sizeof(fr_tuning);
    t->grid = 0;
    t->flush_at = d.flush_at;
    t->cold_cap = d.cold_cap;
    t->log = 1;
    t->log_min = d.log_min;
    t->log_hot = d.log_hot;
    t->chunk_tiles = d.chunk_tiles;
    t->chunk_tiles_heavy = d.chunk_tiles_heavy;
    t->ramp = d.ramp ? 1 : 0;
    t->ramp_up_s = d.ramp_up_s;
    t->ramp_down_s = d.ramp_down_s;
    t->ramp_down_pct = d.ramp_down_pct;
    t->ramp_down_pct_h = d.ramp_down_pct_h;
    t->spec_commit = d.spec_ok ? 1 : 0;
    t->nbr = d.nbr_enabled ? 1 : 0;
    t->ovf_cap = 0;
}

fr_ctx* fr_create(int device, uint64_t chunk_bytes, uint64_t table_slots) {
    return fr_create_tuned(device, chunk_bytes, table_slots, nullptr);
}

fr_ctx* fr_create_tuned(int device, uint64_t chunk_bytes, uint64_t table_slots, const fr_tuning* tuning) {
    fr_tuning t;
    fr_tuning_defaults(&t);
    if (tuning) {  // the caller's fields up to its size; the rest keep their defaults
        const size_t n = std::min<size_t>(std::max<uint32_t>(tuning->size, sizeof(uint32_t)), sizeof(fr_tuning));
        std::memcpy((char*)&t + sizeof(uint32_t), (const char*)tuning + sizeof(uint32_t), n - sizeof(uint32_t));
    }
    fr_ctx* ctx = new fr_ctx();
    ctx->device = device;
    auto bad = [&](const char* what, hipError_t e) {
        ctx->err = std::string(what) + ": " + hipGetErrorString(e);
        return ctx;  // caller inspects fr_last_error; the context is unusable
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return bad("hipSetDevice", e);
    if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess) return bad("stream", e);
    if ((e = hipStreamCreateWithFlags(&ctx->copy, hipStreamNonBlocking)) != hipSuccess) return bad("stream", e);
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return bad("props", e);
    const int per_cu = chunk_occupancy();  // ~40 KB LDS per workgroup; VGPRs sized by __launch_bounds__
    ctx->grid = t.grid > 0 ? t.grid : prop.multiProcessorCount * per_cu;
    ctx->flush_at = std::min<u32>(t.flush_at, NS);
    ctx->nbr_enabled = t.nbr != 0;
    ctx->cold_cap = std::max<u32>(1024, t.cold_cap);
    ctx->log_min = t.log_min;
    ctx->log_hot = std::max<u32>(1, t.log_hot);
    ctx->chunk_tiles = std::max<u32>(2, t.chunk_tiles);
    ctx->chunk_tiles_heavy = std::max<u32>(2, t.chunk_tiles_heavy);
    ctx->ramp = t.ramp != 0;
    ctx->ramp_up_s = std::max<u32>(1, t.ramp_up_s);
    ctx->ramp_down_s = std::max<u32>(1, t.ramp_down_s);
    ctx->ramp_down_pct = std::min<u32>(100, std::max<u32>(1, t.ramp_down_pct));
    ctx->ramp_down_pct_h = std::min<u32>(100, std::max<u32>(1, t.ramp_down_pct_h));
    ctx->spec_ok = t.spec_commit != 0;
    if ((e = dalloc(&ctx->cold, 2ull * ctx->cold_cap * (u64)ctx->grid)) != hipSuccess) return bad("cold lists", e);
    if ((e = dalloc(&ctx->rare, (u64)RARE_RING * (u64)ctx->grid)) != hipSuccess) return bad("rare rings", e);

    ctx->chunk_bytes = chunk_bytes ? ((chunk_bytes + TILE - 1) / TILE) * TILE : (256ull << 20);
    if (ctx->chunk_bytes > RANGE_MAX) ctx->chunk_bytes = RANGE_MAX;
    ctx->ring_bytes = std::min<u64>(ctx->chunk_bytes, HOST_CHUNK_MAX);
    // launch log: room for one pair per 256 B of a launch (SYN-v1 needs one per 350-500 B; a commit
    // that does not fit inserts into the table directly).  Only heavy commits log (ScanArgs::log_min);
    // fr_tuning::log = 0 turns the log off
    if (t.log) {
        // entries: 1 per 256 B of a launch (SYN-v1 config 3 logs ~1 per 700 B), in LOG_NR equal regions;
        // a run past its region's end inserts directly
        const u64 want = std::min<u64>(std::max<u64>(ctx->chunk_bytes / 256, 1ull << 16), 1ull << 26);
        ctx->log_rcap = (u32)(want / LOG_NR);
        ctx->log_cap = (u64)ctx->log_rcap * LOG_NR;
        ctx->log_scap = (u32)std::max<u64>(2ull * ctx->log_rcap / LOG_SUBS, 64);  // 2x the mean share
        // (direct logging: the commits fill the sub-region parts, no region parts)
        if (!LOG_DIRECT && (e = dalloc(&ctx->log, ctx->log_cap)) != hipSuccess) return bad("launch log", e);
        if ((e = dalloc(&ctx->log_sub, (u64)ctx->log_scap * LOG_NSUB)) != hipSuccess) return bad("launch log parts", e);
    }
    ctx->tiles_cap = RANGE_MAX / TSTEP + 2;
    ctx->nslots = pow2_at_least(std::max<u64>(table_slots, 1024));
    if ((e = hipMalloc((void**)&ctx->st, sizeof(DevState))) != hipSuccess) return bad("state", e);
    if ((e = hipMalloc((void**)&ctx->d_tab, sizeof(Table))) != hipSuccess) return bad("table copy", e);
    if ((e = hipHostMalloc((void**)&ctx->h_tab, sizeof(Table), hipHostMallocDefault)) != hipSuccess)
        return bad("table staging", e);
    std::memset(ctx->h_tab, 0, sizeof(Table));
    if ((e = hipHostMalloc((void**)&ctx->h_st, sizeof(DevState), hipHostMallocDefault)) != hipSuccess)
        return bad("pinned state", e);
    if ((e = hipHostMalloc((void**)&ctx->h_byte, 64, hipHostMallocDefault)) != hipSuccess) return bad("pinned byte", e);
    if ((e = hipHostMalloc((void**)&ctx->h_fin, 64, hipHostMallocDefault)) != hipSuccess) return bad("pinned count", e);
    if ((e = hipEventCreate(&ctx->fin_e0)) != hipSuccess) return bad("event", e);
    if ((e = hipEventCreate(&ctx->fin_e1)) != hipSuccess) return bad("event", e);
    if ((e = hipEventCreate(&ctx->cls_e0)) != hipSuccess) return bad("event", e);
    if ((e = hipEventCreate(&ctx->cls_e1)) != hipSuccess) return bad("event", e);
    if ((e = hipHostMalloc((void**)&ctx->h_zero, sizeof(DevState), hipHostMallocDefault)) != hipSuccess)
        return bad("pinned reset state", e);
    std::memset(ctx->h_zero, 0, sizeof(DevState));
    ctx->h_zero->err_nospace = ~0ull;
    if ((e = hipEventCreateWithFlags(&ctx->st_ev, hipEventDisableTiming)) != hipSuccess) return bad("event", e);
    if ((e = dalloc(&ctx->tiles, ctx->tiles_cap)) != hipSuccess) return bad("tiles", e);
    if ((e = dalloc(&ctx->chunk_info, ctx->tiles_cap)) != hipSuccess) return bad("chunk info", e);
    if ((e = hipMemset(ctx->tiles, 0, ctx->tiles_cap * sizeof(u64))) != hipSuccess) return bad("tiles", e);
    if ((e = dalloc(&ctx->tab.slots, ctx->nslots)) != hipSuccess) return bad("table", e);
    ctx->tab.mask = ctx->nslots - 1;
    ctx->tab.ovf_cap = t.ovf_cap ? std::max<u64>(t.ovf_cap, 1024) : (1ull << 22);
    ctx->tab.pres_cap = 1ull << 22;
    ctx->tab.exo_cap = 1ull << 20;
    ctx->tab.exo_pool_cap = 64ull << 20;
    if ((e = dalloc(&ctx->tab.ovf, ctx->tab.ovf_cap)) != hipSuccess) return bad("overflow", e);
    if ((e = dalloc(&ctx->tab.pres, ctx->tab.pres_cap)) != hipSuccess) return bad("presence", e);
    if ((e = dalloc(&ctx->tab.exo_ord, ctx->tab.exo_cap)) != hipSuccess) return bad("exotic", e);
    if ((e = dalloc(&ctx->tab.exo_off, ctx->tab.exo_cap)) != hipSuccess) return bad("exotic", e);
    if ((e = dalloc(&ctx->tab.exo_len, ctx->tab.exo_cap)) != hipSuccess) return bad("exotic", e);
    if ((e = dalloc(&ctx->tab.exo_pool, ctx->tab.exo_pool_cap)) != hipSuccess) return bad("exotic", e);
    for (int i = 0; i < 2; ++i) {
        if ((e = hipHostMalloc((void**)&ctx->pin[i], ctx->ring_bytes, hipHostMallocDefault)) != hipSuccess)
            return bad("pinned ring", e);
        if ((e = dalloc(&ctx->dbuf[i], ctx->ring_bytes + 64)) != hipSuccess) return bad("device ring", e);
        if ((e = hipEventCreateWithFlags(&ctx->copied[i], hipEventDisableTiming)) != hipSuccess) return bad("event", e);
        if ((e = hipEventCreateWithFlags(&ctx->consumed[i], hipEventDisableTiming)) != hipSuccess)
            return bad("event", e);
        if ((e = hipEventRecord(ctx->consumed[i], ctx->stream)) != hipSuccess) return bad("event", e);
    }
    if ((e = dalloc(&ctx->d_counter, 1)) != hipSuccess) return bad("counter", e);
    if (fr_reset(ctx) != FR_OK) return ctx;
    ctx->err.clear();
    return ctx;
}

void fr_destroy(fr_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->copy) (void)hipStreamSynchronize(ctx->copy);
    void* dev[] = {ctx->st, ctx->d_tab, ctx->tiles, ctx->tab.slots, ctx->tab.ovf, ctx->tab.pres, ctx->tab.exo_ord,
                   ctx->tab.exo_off, ctx->tab.exo_len, ctx->tab.exo_pool, ctx->dbuf[0], ctx->dbuf[1], ctx->d_sheet,
                   ctx->d_keys, ctx->d_counts, ctx->d_first, ctx->d_keys_s, ctx->d_counts_s,
                   ctx->d_first_s, ctx->d_pos, ctx->d_perm, ctx->d_rank, ctx->d_counter, ctx->d_temp, ctx->d_bins, ctx->d_binbase, ctx->d_arr, ctx->d_rows, ctx->d_pres_u,
                   ctx->d_pres_f, ctx->d_pres_c, ctx->d_m1, ctx->d_m2, ctx->d_row, ctx->d_rm2, ctx->d_rrow, ctx->d_cls, ctx->d_rcls,
                   ctx->d_errw, ctx->d_errf, ctx->d_nbr, ctx->cold, ctx->rare, ctx->chunk_info, ctx->log, ctx->log_sub, ctx->log_temp,
                   ctx->snap};
    for (void* p : dev)
        if (p) (void)hipFree(p);
    if (ctx->h_st) (void)hipHostFree(ctx->h_st);
    if (ctx->h_zero) (void)hipHostFree(ctx->h_zero);
    if (ctx->h_byte) (void)hipHostFree(ctx->h_byte);
    if (ctx->h_fin) (void)hipHostFree(ctx->h_fin);
    if (ctx->fin_e0) (void)hipEventDestroy(ctx->fin_e0);
    if (ctx->fin_e1) (void)hipEventDestroy(ctx->fin_e1);
    if (ctx->cls_e0) (void)hipEventDestroy(ctx->cls_e0);
    if (ctx->cls_e1) (void)hipEventDestroy(ctx->cls_e1);
    if (ctx->h_sheet) (void)hipHostFree(ctx->h_sheet);
    if (ctx->h_tab) (void)hipHostFree(ctx->h_tab);
    for (int i = 0; i < 2; ++i) {
        if (ctx->pin[i]) (void)hipHostFree(ctx->pin[i]);
        if (ctx->copied[i]) (void)hipEventDestroy(ctx->copied[i]);
        if (ctx->consumed[i]) (void)hipEventDestroy(ctx->consumed[i]);
    }
    for (auto e : ctx->ev_a) (void)hipEventDestroy(e);
    for (auto e : ctx->ev_b) (void)hipEventDestroy(e);
    for (auto e : ctx->ev_l) (void)hipEventDestroy(e);
    if (ctx->st_ev) (void)hipEventDestroy(ctx->st_ev);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->copy) (void)hipStreamDestroy(ctx->copy);
    delete ctx;
}

const char* fr_last_error(const fr_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int fr_get_diag(fr_ctx* ctx, uint64_t* out, int n) {
    if (int src = settle_finalize(ctx)) return src;
    int rc = read_state(ctx);
    if (rc) return rc;
    const DevState& s = *ctx->h_st;
    const uint64_t v[] = {s.spin_max,   s.spin_total, s.n_keys,   s.n_overflow, s.n_presence, s.n_exotic,
                          (uint64_t)ctx->grid, ctx->nslots, s.stamp[0], s.stamp[1], s.stamp[2], s.stamp[3],
                          s.stamp[4],  s.stamp[5],  s.stamp[6], s.stamp[7], ctx->spec_replays, ctx->exo_replays,
                          s.heavy[ctx->par] ? ctx->chunk_tiles_heavy : ctx->chunk_tiles,  // the next ramped launch's
                          s.heavy_launches, ctx->big_rollbacks, ctx->feed_fold_max, ctx->feed_fold_over, ctx->feed_step};
    for (int i = 0; i < n && i < (int)(sizeof(v) / sizeof(v[0])); ++i) out[i] = v[i];
    return FR_OK;
}

int fr_sync(fr_ctx* ctx) {
    CK(hipStreamSynchronize(ctx->stream));
    CK(hipStreamSynchronize(ctx->copy));
    return settle_finalize(ctx);
}

int fr_get_timing(fr_ctx* ctx, fr_timing* out) {
    CK(hipStreamSynchronize(ctx->stream));
    if (int src = settle_finalize(ctx)) return src;
    double tot = 0, last = 0, lg = 0;
    for (size_t i = 0; i < ctx->ev_used; ++i) {
        float ms = 0, ml = 0;
        CK(hipEventElapsedTime(&ms, ctx->ev_a[i], ctx->ev_b[i]));
        CK(hipEventElapsedTime(&ml, ctx->ev_b[i], ctx->ev_l[i]));
        tot += ms;
        last = ms;
        lg += ml;
    }
    out->log_ms = lg;
    out->scan_launches = ctx->scan_launches;
    out->scan_bytes = ctx->scan_bytes;
    out->scan_ms = tot;
    out->last_scan_ms = last;
    out->classify_ms = ctx->classify_ms;
    out->finalize_ms = ctx->finalize_ms;
    return FR_OK;
}

int fr_set_timing(fr_ctx* ctx, int on) {
    if (!ctx) return FR_ERR_INVALID;
    ctx->timing = on != 0;
    return FR_OK;
}

int fr_set_sheet(fr_ctx* ctx, int S, const uint64_t* idx1_packed, const int32_t* idx1_len,
                 const uint64_t* idx2_packed, const int32_t* idx2_len, const uint64_t* idx2rc_packed,
                 const int32_t* name_id, int n_names, const uint32_t* idx1_cp, const uint32_t* idx2_cp,
                 const uint32_t* idx2rc_cp, int cp_stride) {
    if (S < 0 || S > 32767) return fail(ctx, FR_ERR_INVALID, "sheet rows must be in [0, 32767]");
    const bool with_cp = idx1_cp && idx2_cp && idx2rc_cp && cp_stride > 0 && S > 0;
    const u64 ncp = with_cp ? (u64)S * cp_stride : 0;
    // blob layout (8-B aligned pieces): i1 i2 i2rc [S] u64 | name [S] i32 | cp1 cp2 cp2rc [S*stride] u32 |
    // cpl1 cpl2 [S] i32
    auto al = [](u64 b) { return (b + 7) & ~7ull; };
    const u64 o_i2 = al(S * 8ull), o_i2rc = o_i2 + al(S * 8ull), o_name = o_i2rc + al(S * 8ull);
    const u64 o_cp1 = o_name + al(S * 4ull), o_cp2 = o_cp1 + al(ncp * 4), o_cp2rc = o_cp2 + al(ncp * 4);
    const u64 o_l1 = o_cp2rc + al(ncp * 4), o_l2 = o_l1 + (with_cp ? al(S * 4ull) : 0);
    const u64 o_canon = o_l2 + (with_cp ? al(S * 4ull) : 0);
    const u64 total = o_canon + al(3 * S * 4ull) + 8;
    std::vector<u8> blob(total, 0);
    u8* h = blob.data();
    if (S) {
        std::memcpy(h, idx1_packed, S * 8ull);
        std::memcpy(h + o_i2, idx2_packed, S * 8ull);
        std::memcpy(h + o_i2rc, idx2rc_packed, S * 8ull);
        std::memcpy(h + o_name, name_id, S * 4ull);
    }
    if (with_cp) {
        std::memcpy(h + o_cp1, idx1_cp, ncp * 4);
        std::memcpy(h + o_cp2, idx2_cp, ncp * 4);
        std::memcpy(h + o_cp2rc, idx2rc_cp, ncp * 4);
        std::memcpy(h + o_l1, idx1_len, S * 4ull);
        std::memcpy(h + o_l2, idx2_len, S * 4ull);
    }
    // the same sheet again (pass B without rc rows, repeated scans): the device copy is current (the
    // canonical ids below derive from the lists, so the comparison stops before them)
    const bool same = ctx->h_sheet && total == ctx->sheet_bytes && std::memcmp(h, ctx->h_sheet, o_canon) == 0;
    if (!same && S) {
        // value ids of the neighbourhood maps: the first row with the same packed value
        const uint64_t* lists[3] = {idx1_packed, idx2_packed, idx2rc_packed};
        int32_t* canon = (int32_t*)(h + o_canon);
        for (int l = 0; l < 3; ++l) {
            std::unordered_map<u64, int32_t> first;
            first.reserve(S * 2);
            for (int i = 0; i < S; ++i) canon[l * S + i] = first.emplace(lists[l][i], i).first->second;
        }
    }
    if (!same) {
        CK(hipStreamSynchronize(ctx->stream));  // the previous sheet may still be in use / in flight
        if (total > ctx->sheet_cap) {
            if (ctx->d_sheet) CK(hipFree(ctx->d_sheet));
            if (ctx->h_sheet) CK(hipHostFree(ctx->h_sheet));
            ctx->d_sheet = nullptr;
            ctx->h_sheet = nullptr;
            const u64 cap = std::max<u64>(total * 2, 4096);
            CK(hipMalloc(&ctx->d_sheet, cap));
            CK(hipHostMalloc(&ctx->h_sheet, cap, hipHostMallocDefault));
            ctx->sheet_cap = cap;
        }
        std::memcpy(ctx->h_sheet, h, total);
        ctx->sheet_bytes = total;
        ++ctx->sheet_ver;
        CK(hipMemcpyAsync(ctx->d_sheet, ctx->h_sheet, total, hipMemcpyHostToDevice, ctx->stream));
    }
    u8* d = ctx->d_sheet;
    ctx->d_i1 = (u64*)d;
    ctx->d_i2 = (u64*)(d + o_i2);
    ctx->d_i2rc = (u64*)(d + o_i2rc);
    ctx->d_name = (int32_t*)(d + o_name);
    ctx->d_cp1 = with_cp ? (u32*)(d + o_cp1) : nullptr;
    ctx->d_cp2 = with_cp ? (u32*)(d + o_cp2) : nullptr;
    ctx->d_cp2rc = with_cp ? (u32*)(d + o_cp2rc) : nullptr;
    ctx->d_cpl1 = with_cp ? (int32_t*)(d + o_l1) : nullptr;
    ctx->d_cpl2 = with_cp ? (int32_t*)(d + o_l2) : nullptr;
    ctx->d_canon = (int32_t*)(d + o_canon);
    ctx->cp_stride = with_cp ? cp_stride : 0;
    ctx->S = S;
    ctx->n_names = n_names;
    auto common = [&](const int32_t* l) {
        if (S == 0) return -1;
        for (int i = 1; i < S; ++i)
            if (l[i] != l[0]) return -2;
        return (int)l[0];
    };
    ctx->L1u = common(idx1_len);
    ctx->L2u = common(idx2_len);
    return FR_OK;
}

int fr_reset(fr_ctx* ctx) {
    if (int src = settle_finalize(ctx)) return src;
    CK(hipSetDevice(ctx->device));
    CK(hipStreamSynchronize(ctx->copy));
    CK(launch_table_init(ctx->tab.slots, ctx->nslots, ctx->stream));
    int rc = state_reset_counts(ctx);
    if (rc) return rc;
    ctx->scanning = true;
    ctx->file_open = false;
    ctx->file_tag = 0;
    ctx->first_tag = 0;
    ctx->pres_defer_tag = 0;
    ctx->merged = false;
    ctx->max_file_bytes = 0;
    ctx->par = 0;
    ctx->U = 0;
    ctx->n_pres = 0;
    ctx->n_exo = 0;
    ctx->exo_index.clear();
    ctx->exo_str.clear();
    ctx->exo_codes.clear();
    ctx->exo_pres_code.clear();
    ctx->exo_pres_file.clear();
    ctx->exo_pres_count.clear();
    ctx->last_valid = false;
    ctx->ev_used = 0;
    ctx->scan_launches = ctx->scan_bytes = 0;
    ctx->classify_ms = ctx->finalize_ms = 0;
    ctx->st_pending = false;
    return FR_OK;
}

int fr_begin_file(fr_ctx* ctx, int64_t max_records) {
    return fr_begin_file_at(ctx, (int64_t)ctx->file_tag, 0, max_records);
}

int fr_begin_file_at(fr_ctx* ctx, int64_t file_index, uint64_t byte_base, int64_t max_records) {
    if (int src = settle_finalize(ctx)) return src;
    if (ctx->file_open) return fail(ctx, FR_ERR_INVALID, "fr_begin_file: a file is already open");
    if (file_index < 0 || file_index + 1 >= (1 << 19)) return fail(ctx, FR_ERR_INVALID, "too many files in one scan");
    if ((u32)file_index + 1u <= ctx->file_tag)
        return fail(ctx, FR_ERR_INVALID, "fr_begin_file_at: file indices must increase within a scan");
    if (byte_base >= (1ull << ORD_SHIFT)) return fail(ctx, FR_ERR_INVALID, "fr_begin_file_at: byte base too large");
    int rc = flush_presence(ctx);  // the first file's pairs, before this file changes any last tag
    if (rc) return rc;
    rc = read_state(ctx);
    if (rc) return rc;
    ctx->pres_before = ctx->h_st->n_presence;
    ctx->exo_new_file = 0;
    ctx->exo_records_file = 0;
    ctx->last_valid = false;
    // per-file device flags + line carry: DevState's per-file block, from the pinned reset image
    static_assert(offsetof(DevState, utf8_bad) + sizeof(u32) - offsetof(DevState, lines) == 32, "per-file block");
    CK(hipMemcpyAsync(&ctx->st->lines[0], &ctx->h_zero->lines[0], 32, hipMemcpyHostToDevice, ctx->stream));
    ctx->h_st->lines[0] = ctx->h_st->lines[1] = 0;  // the snapshot stays exact
    ctx->h_st->err_nospace = ~0ull;
    ctx->h_st->nonascii = ctx->h_st->utf8_bad = 0;
    ctx->file_tag = (u32)file_index + 1u;
    if (!ctx->first_tag) ctx->first_tag = ctx->file_tag;
    ctx->file_offset = byte_base;
    ctx->file_base = byte_base;
    ctx->max_records = max_records > 0 ? max_records : 0;
    ctx->last_byte = -1;
    ctx->carry.clear();
    ctx->sample_done = false;
    ctx->par = 0;
    ctx->file_open = true;
    return FR_OK;
}

static int check_sample(fr_ctx* ctx) {
    if (ctx->max_records <= 0) return FR_OK;
    int rc = read_state(ctx);
    if (rc) return rc;
    const u64 lines = ctx->h_st->lines[ctx->par];
    if (lines + 3 >= 4ull * (u64)ctx->max_records) ctx->sample_done = true;
    return FR_OK;
}

// launch [0, n) of ring slot `slot` (already filled in pin[slot])
static int ship_slot(fr_ctx* ctx, int slot, u64 n) {
    CK(hipStreamWaitEvent(ctx->copy, ctx->consumed[slot], 0));
    CK(hipMemcpyAsync(ctx->dbuf[slot], ctx->pin[slot], n, hipMemcpyHostToDevice, ctx->copy));
    CK(hipEventRecord(ctx->copied[slot], ctx->copy));
    CK(hipStreamWaitEvent(ctx->stream, ctx->copied[slot], 0));
    int rc = launch_range(ctx, ctx->dbuf[slot], n, n, 1, 0, 0);
    if (rc) return rc;
    CK(hipEventRecord(ctx->consumed[slot], ctx->stream));
    ctx->used[slot] = true;
    return FR_OK;
}

int fr_feed(fr_ctx* ctx, const uint8_t* data, uint64_t len) {
    if (!ctx->file_open) return fail(ctx, FR_ERR_INVALID, "fr_feed: no open file");
    ctx->host_feed = true;
    if (ctx->sample_done) return FR_SAMPLE_DONE;
    if (len) ctx->last_byte = data[len - 1];
    u64 done = 0;
    while (done < len) {
        const int slot = ctx->cur;
        if (ctx->used[slot]) CK(hipEventSynchronize(ctx->copied[slot]));  // pinned slot free again
        u8* pin = ctx->pin[slot];
        const u64 nc = ctx->carry.size();
        if (nc >= ctx->ring_bytes) return fail(ctx, FR_ERR_CAPACITY, "a line is longer than the chunk size");
        if (nc) std::memcpy(pin, ctx->carry.data(), nc);
        const u64 take = std::min<u64>(len - done, ctx->ring_bytes - nc);
        pinned_copy(pin + nc, data + done, take);
        done += take;
        const u64 n = nc + take;
        // cut after the last line terminator so no line crosses a launch (R1 universal newlines: the
        // line phase is carried on the device).  A '\r' ends a line only when the byte after it is
        // known and is not '\n', so a '\r' at the buffer's end waits in the carry (CR-only files
        // cut at their lone '\r's; a CRLF is never split)
        u64 cut = n;
        while (cut > 0 && !(pin[cut - 1] == '\n' || (pin[cut - 1] == '\r' && cut < n && pin[cut] != '\n'))) --cut;
        if (cut == 0) {
            ctx->carry.assign(pin, pin + n);
            continue;
        }
        ctx->carry.assign(pin + cut, pin + n);
        int rc = ship_slot(ctx, slot, cut);
        if (rc) return rc;
        ctx->cur ^= 1;
        rc = check_sample(ctx);
        if (rc) return rc;
        if (ctx->sample_done) return FR_SAMPLE_DONE;
    }
    return FR_OK;
}

int fr_feed_device(fr_ctx* ctx, const uint8_t* dev_data, uint64_t len) {
    if (!ctx->file_open) return fail(ctx, FR_ERR_INVALID, "fr_feed_device: no open file");
    if (ctx->file_offset != ctx->file_base || !ctx->carry.empty())
        return fail(ctx, FR_ERR_INVALID, "fr_feed_device takes a whole file (no prior fr_feed)");
    if (((uintptr_t)dev_data & 15u) != 0) return fail(ctx, FR_ERR_INVALID, "device data must be 16-byte aligned");
    // Speculative chunks commit without waiting for their exact line prefix; the launch's last
    // workgroup checks every guess (verify_launch).  A wrong guess -- possible only for inputs that
    // are not 4-line FASTQ -- rolls the table back to this feed's start and replays it with every
    // chunk waiting for its prefix.  The rollback point: the table slots (a device copy unless the
    // table is empty) and the device state.
    ctx->host_feed = false;
    int rc = settle_exotic(ctx);  // an empty exotic list at the feed's start
    if (rc) return rc;
    const DevState saved = *ctx->h_st;
    const u32 par0 = ctx->par;
    const u64 snap_slots = ctx->nslots;
    const bool empty = saved.n_keys == 0 && saved.n_overflow == 0;
    const bool spec = ctx->spec_ok && ctx->max_records == 0 && saved.n_overflow == 0;
    GSlot* snap = nullptr;
    if (spec && !empty) {  // the copy's buffer stays with the context: a feed per file would pay a synchronising free
        if (ctx->snap_cap < snap_slots) {
            if (ctx->snap) {
                CK(hipStreamSynchronize(ctx->stream));
                CK(hipFree(ctx->snap));
                ctx->snap = nullptr;
            }
            ctx->snap_cap = 0;
            CK(dalloc(&ctx->snap, snap_slots));
            ctx->snap_cap = snap_slots;
        }
        snap = ctx->snap;
        CK(hipMemcpyAsync(snap, ctx->tab.slots, snap_slots * sizeof(GSlot), hipMemcpyDeviceToDevice, ctx->stream));
    }
    // Equal ranges of at most chunk_bytes: one launch (one set of ramps and tail) for the bench's 7.4 GB,
    // DESIGN.md §4.1.  The table grows between launches, never inside one, so a range over RANGE_FIRST_MAX is
    // taken only for speculative feeds whose table holds the last feed's new codes again at load <= 1/2, and
    // whose last feed did not log (feed_logged).  The decision rests on the previous feed (fr_reset keeps it: a bench or a seam scanning the same
    // kind of data again).  A feed whose new codes outgrow the table inside one launch -- past the free
    // slots and the overflow list -- is rolled back like a wrong speculation and replayed in ranges of an
    // eighth of the size, with the table grown between them (each launch's state read before the next),
    // down to RANGE_ROOM_MIN (speculative feeds: the rollback needs the snapshot).
    // a logged feed's folds, scaled to this feed's big range, at most 0.85 full (distinct codes grow slower than the
    // bytes: config 2's 3.7-GB halves fill at most 1 626 of 4 096 slots, projected 3 252 for 7.4 GB; config 3's 3.9-GB
    // halves 2 424 (projected 4 848), scripts/fold_probe.py)
    const double big_range = (double)std::min<u64>(ctx->chunk_bytes, len);
    const bool fold_room = (u64)ctx->feed_fold_over * 64 <= ctx->feed_fold_max && ctx->feed_step > 0 &&  // (a few
                           // entries past a fold's probe bound insert on their own: harmless)
                           (double)ctx->feed_fold_max * big_range <= 0.85 * AGG_LNS * (double)ctx->feed_step;
    bool big = spec && (!ctx->feed_logged || fold_room) && ctx->feed_keys != ~0ull &&
               (saved.n_keys + ctx->feed_keys) * 2 <= ctx->nslots;
    bool spec_now = spec;
    u64 step = 0, lim_room = ~0ull;
    for (int attempt = 0; attempt < 12; ++attempt) {
        // the attempt's fold statistics start at zero (a rollback restores the state before the feed)
        CK(hipMemsetAsync(&ctx->st->log_fold_max, 0, 2 * sizeof(u32), ctx->stream));
        const u64 lim = std::min<u64>(big ? ctx->chunk_bytes : std::min<u64>(ctx->chunk_bytes, RANGE_FIRST_MAX),
                                      lim_room);
        const u64 nr = (len + lim - 1) / lim;
        step = nr ? (len + nr - 1) / nr : 0;
        ctx->spec_commit = spec_now ? 1u : 0u;
        for (u64 off = 0; off < len; off += step) {
            const u64 n = std::min<u64>(step, len - off);
            rc = launch_range(ctx, dev_data + off, n, len - off, off == 0 ? 1 : 0, 1, off ? 1 : 0);
            if (rc) break;
        }
        ctx->spec_commit = 0;
        // the feed's last byte lands with the state read below (one host round trip for both)
        if (!rc && len) CK(hipMemcpyAsync(ctx->h_byte, dev_data + len - 1, 1, hipMemcpyDeviceToHost, ctx->stream));
        if (!rc) rc = read_state(ctx);
        if (rc) break;
        const bool spec_bad = spec_now && ctx->h_st->spec_fail;
        // the overflow list ran out (fr_end_file would report FR_ERR_CAPACITY): smaller ranges, if any left
        const bool room_bad = spec && (ctx->h_st->cap_flags & 2u) && step > RANGE_ROOM_MIN;
        if (!spec_bad && !room_bad) break;
        if (room_bad) {
            big = false;
            lim_room = std::max<u64>(RANGE_ROOM_MIN, ((step / 8) + TILE - 1) / TILE * TILE);
            ctx->grow_sync = true;  // the replay's launches each see the table grown after the previous one
            ctx->big_rollbacks++;
        } else {
            spec_now = false;
        }
        // roll back: the table as it was (its size too), the device state, the launch parity
        if (ctx->nslots != snap_slots) {
            GSlot* fresh = nullptr;
            if ((rc = (dalloc(&fresh, snap_slots) == hipSuccess) ? FR_OK : fail(ctx, FR_ERR_DEVICE, "rollback alloc")))
                break;
            CK(hipStreamSynchronize(ctx->stream));
            CK(hipFree(ctx->tab.slots));
            ctx->tab.slots = fresh;
            ctx->tab.mask = snap_slots - 1;
            ctx->nslots = snap_slots;
        }
        if (empty) CK(launch_table_init(ctx->tab.slots, ctx->nslots, ctx->stream));
        else CK(hipMemcpyAsync(ctx->tab.slots, snap, snap_slots * sizeof(GSlot), hipMemcpyDeviceToDevice, ctx->stream));
        *ctx->h_st = saved;
        CK(hipMemcpyAsync(ctx->st, ctx->h_st, sizeof(DevState), hipMemcpyHostToDevice, ctx->stream));
        CK(hipStreamSynchronize(ctx->stream));
        ctx->st_pending = false;
        ctx->st_fresh = true;
        ctx->par = par0;
        ctx->file_offset = ctx->file_base;
        if (!room_bad) ctx->spec_replays++;
    }
    ctx->grow_sync = false;
    if (rc) return rc;
    ctx->feed_keys = ctx->h_st->n_keys - saved.n_keys;
    ctx->feed_logged = ctx->h_st->log_commits != saved.log_commits;  // read_state above: exact
    ctx->feed_fold_max = ctx->h_st->log_fold_max;
    ctx->feed_fold_over = ctx->h_st->log_fold_over;
    ctx->feed_step = step;
    // exotic records overflowed the list: grow it to the counted totals and run the feed's launches
    // again capturing exotic records only (the table is already complete), then drain
    rc = read_state(ctx);
    if (rc) return rc;
    if (ctx->h_st->cap_flags & 4u) {
        DevState& s = *ctx->h_st;
        rc = grow_exotic(ctx, s.n_exotic, s.exo_pool_used);
        if (rc) return rc;
        s.n_exotic = 0;
        s.exo_pool_used = 0;
        s.cap_flags &= ~4u;
        s.lines[par0] = saved.lines[par0];
        CK(hipMemcpyAsync(ctx->st, ctx->h_st, sizeof(DevState), hipMemcpyHostToDevice, ctx->stream));
        ctx->par = par0;
        ctx->file_offset = ctx->file_base;
        ctx->exo_replays++;
        for (u64 off = 0; off < len && !rc; off += step) {
            const u64 n = std::min<u64>(step, len - off);
            rc = launch_range(ctx, dev_data + off, n, len - off, off == 0 ? 1 : 0, 1, off ? 1 : 0, 1);
        }
        if (rc) return rc;
        ctx->st_fresh = false;
        rc = read_state(ctx);
        if (rc) return rc;
        if (ctx->h_st->cap_flags & 4u) return fail(ctx, FR_ERR_DEVICE, "exotic replay overflowed");
    }
    rc = drain_exotic(ctx);
    if (rc) return rc;
    if (len) ctx->last_byte = *ctx->h_byte;  // landed: read_state synchronised after the copy
    ctx->carry.clear();
    return FR_OK;
}

int fr_end_file(fr_ctx* ctx, fr_file_stats* out) {
    if (!ctx->file_open) return fail(ctx, FR_ERR_INVALID, "fr_end_file: no open file");
    if (!ctx->carry.empty() && !ctx->sample_done) {  // the last piece: no '\n' cut needed
        const int slot = ctx->cur;
        if (ctx->used[slot]) CK(hipEventSynchronize(ctx->copied[slot]));
        std::memcpy(ctx->pin[slot], ctx->carry.data(), ctx->carry.size());
        const u64 n = ctx->carry.size();
        ctx->carry.clear();
        int rc = ship_slot(ctx, slot, n);
        if (rc) return rc;
        ctx->cur ^= 1;
    }
    ctx->carry.clear();
    CK(hipStreamSynchronize(ctx->copy));
    int rc = ctx->host_feed ? settle_exotic(ctx) : FR_OK;  // device feeds settled at their end
    if (rc) return rc;
    ctx->last_valid = false;
    rc = grow_table(ctx, false);  // re-inserts any overflow; exact state afterwards
    if (rc) return rc;
    // the first file since the reset: every live key is its (it made them all), so its presence scan waits
    // until a second file begins (flush_presence) -- a one-file scan never runs it (fr_finalize)
    const bool defer = ctx->file_tag == ctx->first_tag && !ctx->merged && ctx->pres_before == 0 &&
                       ctx->h_st->n_presence == 0;
    if (!defer) {
        rc = ensure_presence_cap(ctx);
        if (rc) return rc;
        ctx->st_fresh = false;
        CK(launch_presence_scan(ctx->tab.slots, ctx->nslots, ctx->file_tag, ctx->tab.pres, ctx->tab.pres_cap,
                                ctx->st, ctx->stream));
    }
    rc = read_state(ctx);
    if (rc) return rc;
    const DevState& s = *ctx->h_st;
    if (s.spin_fail) return fail(ctx, FR_ERR_DEVICE, "tally look-back exceeded its spin bound");
    if (s.cap_flags) return fail(ctx, FR_ERR_CAPACITY, "a device list overflowed (flags " + std::to_string(s.cap_flags) + ")");
    u64 lines = s.lines[ctx->par];
    const bool ended = ctx->last_byte == '\n' || ctx->last_byte == '\r';
    if (ctx->last_byte >= 0 && !ended && !ctx->sample_done) lines += 1;  // trailing line without terminator
    u64 records = (lines + 3) / 4;
    if (ctx->max_records > 0 && records > (u64)ctx->max_records) records = (u64)ctx->max_records;
    std::memset(out, 0, sizeof(*out));
    out->records = records;
    out->lines = lines;
    out->new_keys = (defer ? s.n_keys : s.n_presence - ctx->pres_before) + ctx->exo_new_file;
    if (defer) ctx->pres_defer_tag = ctx->file_tag;
    out->exotic = ctx->exo_records_file;
    out->error = FR_SCAN_OK;
    if (s.utf8_bad) {
        out->error = FR_SCAN_UTF8;
        out->utf8_bad = 1;
    }
    if (s.err_nospace != ~0ull) {
        out->error = FR_SCAN_NO_SPACE;
        out->error_offset = s.err_nospace;
    }
    ctx->file_open = false;
    return FR_OK;
}

int fr_finalize(fr_ctx* ctx, uint64_t* n_unique, uint64_t* n_presence, uint64_t* n_exotic) {
    if (ctx->file_open) return fail(ctx, FR_ERR_INVALID, "fr_finalize: a file is still open");
    int rc = settle_finalize(ctx);
    if (rc) return rc;
    hipEvent_t e0 = ctx->fin_e0, e1 = ctx->fin_e1;
    rc = grow_table(ctx, false);
    if (rc) return rc;
    rc = read_state(ctx);
    if (rc) return rc;
    const u64 nk = ctx->h_st->n_keys;
    if (nk > 0xFFFFFFFFull) return fail(ctx, FR_ERR_CAPACITY, "more than 2^32 unique codes");
    if (nk > ctx->ucap) {
        void* old[] = {ctx->d_keys, ctx->d_counts, ctx->d_first, ctx->d_keys_s, ctx->d_counts_s, ctx->d_first_s,
                       ctx->d_pos, ctx->d_perm, ctx->d_rank, ctx->d_temp};
        for (void* p : old)
            if (p) CK(hipFree(p));
        ctx->d_temp = nullptr;
        ctx->temp_bytes = 0;
        const u64 cap = std::max<u64>(nk + nk / 4, 1024);
        CK(dalloc(&ctx->d_keys, cap));
        CK(dalloc(&ctx->d_counts, cap));
        CK(dalloc(&ctx->d_first, cap));
        CK(dalloc(&ctx->d_keys_s, cap));
        CK(dalloc(&ctx->d_counts_s, cap));
        CK(dalloc(&ctx->d_first_s, cap));
        CK(dalloc(&ctx->d_pos, cap));
        CK(dalloc(&ctx->d_perm, cap));
        CK(dalloc(&ctx->d_rank, cap));
        ctx->ucap = cap;
    }
    if (ctx->timing) CK(hipEventRecord(e0, ctx->stream));
    ctx->fin_timed = ctx->timing;
    // one context's own ordinals: bin them (fin_* kernels); merged rows (any file tag): radix sort
    BinMap bm{0, 0, 0, 0, 0};
    u64 nbins = 0;
    if (!ctx->merged && ctx->first_tag && ctx->file_tag >= ctx->first_tag) {
        const u64 ntags = (u64)(ctx->file_tag - ctx->first_tag) + 1u;
        bm.span = std::max<u64>(ctx->max_file_bytes, 1);
        bm.first_tag = ctx->first_tag;
        bm.shift = 13;
        const u64 range = ntags * bm.span;  // < 2^19 tags x 2^44 bytes: no overflow
        while (bm.shift < 20 && ((range >> bm.shift) + 1) > (1ull << 21)) ++bm.shift;
        nbins = (range >> bm.shift) + 1;
        if (nbins > (1ull << 21)) nbins = 0;  // more than 2^41 bytes of input: radix sort
    }
    if (nbins) {
        bm.nbins = nbins;
        bm.cap = ctx->ucap;
        if (ctx->nslots > ctx->arr_cap) {
            if (ctx->d_arr) CK(hipFree(ctx->d_arr));
            ctx->d_arr = nullptr;
            CK(hipMalloc(&ctx->d_arr, ctx->nslots * sizeof(u32)));
            ctx->arr_cap = ctx->nslots;
        }
        if (ctx->ucap > ctx->rows_cap) {
            if (ctx->d_rows) CK(hipFree(ctx->d_rows));
            ctx->d_rows = nullptr;
            CK(hipMalloc(&ctx->d_rows, ctx->ucap * sizeof(FinRow)));
            ctx->rows_cap = ctx->ucap;
        }
        if (nbins + 1 > ctx->bins_cap) {
            if (ctx->d_bins) CK(hipFree(ctx->d_bins));
            if (ctx->d_binbase) CK(hipFree(ctx->d_binbase));
            ctx->d_bins = ctx->d_binbase = nullptr;
            const u64 cap = std::max<u64>(nbins + 1, 1u << 16);
            CK(hipMalloc(&ctx->d_bins, cap * sizeof(u32)));
            CK(hipMalloc(&ctx->d_binbase, cap * sizeof(u32)));
            ctx->bins_cap = cap;
        }
        size_t need = 0;
        CK(launch_fin_scan(ctx->d_bins, ctx->d_binbase, nbins + 1, nullptr, &need, ctx->stream));
        if (need > ctx->temp_bytes) {
            if (ctx->d_temp) CK(hipFree(ctx->d_temp));
            CK(hipMalloc(&ctx->d_temp, need));
            ctx->temp_bytes = need;
        }
        size_t tb = ctx->temp_bytes;
        // the slots' uidx is read only by presence_map_kernel: a one-file scan (deferred presence) skips it
        const bool set_uidx = ctx->pres_defer_tag == 0;
        CK(hipMemsetAsync(ctx->d_bins, 0, (nbins + 1) * sizeof(u32), ctx->stream));
        CK(launch_fin_hist(ctx->tab.slots, ctx->nslots, bm, ctx->d_bins, ctx->d_arr, ctx->stream));
        CK(launch_fin_scan(ctx->d_bins, ctx->d_binbase, nbins + 1, ctx->d_temp, &tb, ctx->stream));
        CK(launch_fin_scatter(ctx->tab.slots, ctx->nslots, bm, ctx->d_binbase, ctx->d_arr, ctx->d_rows, ctx->stream));
        CK(launch_fin_rank(ctx->tab.slots, nk, bm, ctx->d_binbase, ctx->d_rows, ctx->d_keys_s, ctx->d_counts_s,
                           ctx->d_first_s, set_uidx, ctx->stream));
    } else {
        CK(hipMemsetAsync(ctx->d_counter, 0, sizeof(u64), ctx->stream));
        CK(launch_compact(ctx->tab.slots, ctx->nslots, ctx->d_keys, ctx->d_counts, ctx->d_first, ctx->d_pos,
                          ctx->d_counter, ctx->stream));
        // ordinals are < (file_tag + 1) << ORD_SHIFT: sort only the bits that can be set.  Without
        // merged rows every ordinal is a record start of this context's files, and records span at
        // least 4 bytes (four line terminators), so bits [0, 2) never decide the order; with one file
        // the ordinal is its byte offset (file tag 1 sits above every offset bit).  100M SYN-v1 reads
        // (7.4 GB): bits [2, 33), 4 radix passes instead of 6.
        int begin_bit = 0, end_bit = 64;
        if (!ctx->merged) {
            begin_bit = 2;
            end_bit = ORD_SHIFT;
            while (end_bit < 64 && ((u64)ctx->file_tag >> (end_bit - ORD_SHIFT)) != 0) ++end_bit;
            if (ctx->file_tag == ctx->first_tag) {  // one file: its tag is a constant above every offset bit
                end_bit = begin_bit + 1;
                while (end_bit < ORD_SHIFT && (ctx->max_file_bytes >> end_bit) != 0) ++end_bit;
            }
        }
        size_t need = 0;
        CK(launch_order(ctx->d_first, ctx->d_pos, nk, ctx->d_first_s, ctx->d_perm, nullptr, &need, begin_bit, end_bit,
                        ctx->stream));
        if (need > ctx->temp_bytes) {
            if (ctx->d_temp) CK(hipFree(ctx->d_temp));
            CK(hipMalloc(&ctx->d_temp, need));
            ctx->temp_bytes = need;
        }
        size_t tb = ctx->temp_bytes;
        if (nk)
            CK(launch_order(ctx->d_first, ctx->d_pos, nk, ctx->d_first_s, ctx->d_perm, ctx->d_temp, &tb, begin_bit,
                            end_bit, ctx->stream));
        CK(launch_gather(ctx->d_perm, nk, ctx->d_keys, ctx->d_counts, ctx->d_keys_s, ctx->d_counts_s, ctx->d_rank,
                         ctx->stream));
        CK(launch_set_uidx(ctx->tab.slots, ctx->tab.mask, ctx->d_keys_s, nk, ctx->d_rank, ctx->stream));
    }
    const u64 np = ctx->pres_defer_tag ? nk : std::min<u64>(ctx->h_st->n_presence, ctx->tab.pres_cap);
    if (np > ctx->pmap_cap) {
        if (ctx->d_pres_u) CK(hipFree(ctx->d_pres_u));
        if (ctx->d_pres_f) CK(hipFree(ctx->d_pres_f));
        if (ctx->d_pres_c) CK(hipFree(ctx->d_pres_c));
        CK(dalloc(&ctx->d_pres_u, np));
        CK(dalloc(&ctx->d_pres_f, np));
        CK(dalloc(&ctx->d_pres_c, np));
        ctx->pmap_cap = np;
    }
    if (ctx->pres_defer_tag)  // one file: its pairs are the finalized table itself
        CK(launch_presence_one_file(ctx->d_counts_s, np, ctx->pres_defer_tag, ctx->d_pres_u, ctx->d_pres_f,
                                    ctx->d_pres_c, ctx->stream));
    else
        CK(launch_presence_map(ctx->tab.slots, ctx->tab.mask, ctx->tab.pres, np, ctx->d_pres_u, ctx->d_pres_f,
                               ctx->d_pres_c, ctx->stream));
    *ctx->h_fin = 0;
    if (nbins)  // the scan's last entry: every live slot counted once
        CK(hipMemcpyAsync(ctx->h_fin, ctx->d_binbase + nbins, sizeof(u32), hipMemcpyDeviceToHost, ctx->stream));
    else
        CK(hipMemcpyAsync(ctx->h_fin, ctx->d_counter, sizeof(u64), hipMemcpyDeviceToHost, ctx->stream));
    CK(hipEventRecord(e1, ctx->stream));
    ctx->fin_pending = true;
    ctx->fin_expect = nk;
    ctx->U = nk;
    ctx->n_pres = np;
    ctx->n_exo = ctx->exo_codes.size();
    if (n_unique) *n_unique = ctx->U;
    if (n_presence) *n_presence = ctx->n_pres;
    if (n_exotic) *n_exotic = ctx->n_exo;
    return FR_OK;
}

int fr_get_unique(fr_ctx* ctx, uint64_t* keys, uint64_t* counts, uint64_t* first_ordinal) {
    if (int src = settle_finalize(ctx)) return src;
    const u64 n = ctx->U;
    if (!n) return FR_OK;
    if (keys) CK(hipMemcpy(keys, ctx->d_keys_s, n * 8, hipMemcpyDeviceToHost));
    if (counts) CK(hipMemcpy(counts, ctx->d_counts_s, n * 8, hipMemcpyDeviceToHost));
    if (first_ordinal) CK(hipMemcpy(first_ordinal, ctx->d_first_s, n * 8, hipMemcpyDeviceToHost));
    return FR_OK;
}

int fr_get_presence(fr_ctx* ctx, uint32_t* unique_idx, uint32_t* file_idx) {
    if (int src = settle_finalize(ctx)) return src;
    const u64 n = ctx->n_pres;
    if (!n) return FR_OK;
    CK(hipMemcpy(unique_idx, ctx->d_pres_u, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(file_idx, ctx->d_pres_f, n * 4, hipMemcpyDeviceToHost));
    return FR_OK;
}

int fr_get_presence_counts(fr_ctx* ctx, uint64_t* counts, uint64_t* exotic_counts) {
    if (int src = settle_finalize(ctx)) return src;
    const u64 n = ctx->n_pres;
    if (counts && n) {
        // pairs are appended file by file (fr_end_file), so a code's pairs come in file order and its
        // count in a file is its running count there minus the running count at its previous pair
        std::vector<u32> u(n);
        CK(hipMemcpy(u.data(), ctx->d_pres_u, n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(counts, ctx->d_pres_c, n * 8, hipMemcpyDeviceToHost));
        std::vector<u64> last(ctx->U, 0);
        const u64 m = (1ull << (64 - PRES_TAG_BITS)) - 1ull;
        for (u64 i = 0; i < n; ++i) {
            if (u[i] >= ctx->U) return fail(ctx, FR_ERR_DEVICE, "presence pair without a unique code");
            const u64 snap = counts[i];
            counts[i] = (snap - last[u[i]]) & m;
            last[u[i]] = snap;
        }
    }
    const u64 ne = ctx->exo_pres_count.size();
    if (exotic_counts && ne) std::memcpy(exotic_counts, ctx->exo_pres_count.data(), ne * 8);
    return FR_OK;
}

int fr_exotic_sizes(fr_ctx* ctx, uint64_t* n_codes, uint64_t* code_bytes, uint64_t* n_presence) {
    if (int src = settle_finalize(ctx)) return src;
    u64 b = 0;
    for (const auto& c : ctx->exo_str) b += c.size();
    if (n_codes) *n_codes = ctx->exo_str.size();
    if (code_bytes) *code_bytes = b;
    if (n_presence) *n_presence = ctx->exo_pres_code.size();
    return FR_OK;
}

int fr_get_exotic_table(fr_ctx* ctx, uint64_t* counts, uint64_t* first, uint64_t* offsets, uint8_t* bytes,
                        uint32_t* pres_code, uint32_t* pres_file) {
    if (int src = settle_finalize(ctx)) return src;
    const u64 n = ctx->exo_str.size();
    u64 b = 0;
    for (u64 i = 0; i < n; ++i) {
        if (counts) counts[i] = ctx->exo_codes[i].count;
        if (first) first[i] = ctx->exo_codes[i].first;
        if (offsets) offsets[i] = b;
        if (bytes) std::memcpy(bytes + b, ctx->exo_str[i].data(), ctx->exo_str[i].size());
        b += ctx->exo_str[i].size();
    }
    if (offsets) offsets[n] = b;
    const u64 np = ctx->exo_pres_code.size();
    if (pres_code && np) std::memcpy(pres_code, ctx->exo_pres_code.data(), np * 4);
    if (pres_file && np) std::memcpy(pres_file, ctx->exo_pres_file.data(), np * 4);
    return FR_OK;
}

static int ensure_class_scratch(fr_ctx* ctx, u64 n) {
    if (n <= ctx->ccap && ctx->n_names <= ctx->rc_names_cap && ctx->d_errf) return FR_OK;
    void* old[] = {ctx->d_m1, ctx->d_m2, ctx->d_row, ctx->d_rm2, ctx->d_rrow, ctx->d_cls, ctx->d_rcls, ctx->d_errw,
                   ctx->d_errf};  // d_rcf / d_rcr live inside d_errf's block
    for (void* p : old)
        if (p) CK(hipFree(p));
    const u64 cap = std::max<u64>(std::max(n, ctx->ccap), 1024);
    CK(dalloc(&ctx->d_m1, cap));
    CK(dalloc(&ctx->d_m2, cap));
    CK(dalloc(&ctx->d_row, cap));
    CK(dalloc(&ctx->d_rm2, cap));
    CK(dalloc(&ctx->d_rrow, cap));
    CK(dalloc(&ctx->d_cls, cap));
    CK(dalloc(&ctx->d_rcls, cap));
    CK(dalloc(&ctx->d_errw, cap));
    // one block zeroed by one memset per classify: ~(first error index) (0: none), then the rc sums
    const int names = std::max(ctx->n_names, 1);
    CK(dalloc(&ctx->d_errf, 1 + 2 * (u64)names));
    ctx->d_rcf = ctx->d_errf + 1;
    ctx->d_rcr = ctx->d_rcf + names;
    ctx->ccap = cap;
    ctx->rc_names_cap = names;
    return FR_OK;
}

// the classify neighbourhood maps of the current sheet and nsubs (stream-ordered, rebuilt only when
// the sheet, nsubs or the rc need changed); nbr.on = 0 when the sheet does not suit them (mixed or
// > 21-symbol lengths, or more than NBR_MAX codes per list) or FR_NBR=0
static int ensure_nbr(fr_ctx* ctx, const SheetArgs& sh, int nsubs, int rc) {
    constexpr u64 NBR_MAX = 1ull << 21;
    if (ctx->nbr_ver == ctx->sheet_ver && ctx->nbr_nsubs == nsubs && (ctx->nbr_rc || !rc)) return FR_OK;
    ctx->nbr.on = 0;
    ctx->nbr_ver = ctx->sheet_ver;
    ctx->nbr_nsubs = nsubs;
    ctx->nbr_rc = rc;
    if (!ctx->nbr_enabled || sh.S <= 0 || nsubs < 0 || sh.L1u < 0 || sh.L1u > 21 || sh.L2u < 0 || sh.L2u > 21)
        return FR_OK;
    const u64 c1 = (u64)sh.S * nbr_codes_per_row(sh.L1u, nsubs), c2 = (u64)sh.S * nbr_codes_per_row(sh.L2u, nsubs);
    if (c1 > NBR_MAX || c2 > NBR_MAX) return FR_OK;
    const u64 n1 = std::max<u64>(pow2_at_least(2 * c1), 1024), n2 = std::max<u64>(pow2_at_least(2 * c2), 1024);
    const u64 np = std::max<u64>(pow2_at_least(2 * (u64)sh.S), 64);
    const u64 bytes = (n1 + 2 * n2) * sizeof(NSlot) + 2 * np * sizeof(PSlot);
    if (bytes > ctx->nbr_cap) {
        CK(hipStreamSynchronize(ctx->stream));  // an earlier classify may still read the old maps
        if (ctx->d_nbr) CK(hipFree(ctx->d_nbr));
        ctx->d_nbr = nullptr;
        ctx->nbr_cap = 0;
        CK(hipMalloc(&ctx->d_nbr, bytes));
        ctx->nbr_cap = bytes;
    }
    NbrMap& m = ctx->nbr;
    m.m[0] = (NSlot*)ctx->d_nbr;
    m.m[1] = m.m[0] + n1;
    m.m[2] = m.m[1] + n2;
    m.p[0] = (PSlot*)(m.m[2] + n2);
    m.p[1] = m.p[0] + np;
    m.mmask[0] = (u32)(n1 - 1);
    m.mmask[1] = m.mmask[2] = (u32)(n2 - 1);
    m.pmask[0] = m.pmask[1] = (u32)(np - 1);
    CK(hipMemsetAsync(ctx->d_nbr, 0, bytes, ctx->stream));
    CK(launch_nbr_build(sh, ctx->d_canon, nsubs, rc, m, ctx->stream));
    m.on = 1;
    return FR_OK;
}

int fr_classify(fr_ctx* ctx, int num_subs, int rc_mode, int16_t* m1, int16_t* m2, uint8_t* cls, int16_t* row,
                int16_t* rc_m2, uint8_t* rc_cls, int16_t* rc_row, int64_t* err_unique, int32_t* err_which) {
    if (ctx->S < 0) return fail(ctx, FR_ERR_INVALID, "fr_classify: no sheet");
    const u64 n = ctx->U;
    int rc = ensure_class_scratch(ctx, n);
    if (rc) return rc;
    hipEvent_t e0 = ctx->cls_e0, e1 = ctx->cls_e1;
    // the whole block: d_rcr sits rc_names_cap entries after d_rcf, however many names this sheet has
    CK(hipMemsetAsync(ctx->d_errf, 0, (1 + 2 * (u64)ctx->rc_names_cap) * 8, ctx->stream));
    SheetArgs sh{ctx->S, ctx->n_names, ctx->L1u, ctx->L2u, ctx->d_i1, ctx->d_i2, ctx->d_i2rc, ctx->d_name};
    if ((rc = ensure_nbr(ctx, sh, num_subs, rc_mode ? 1 : 0))) return rc;
    ClassOut o{ctx->d_m1, ctx->d_m2, ctx->d_cls, ctx->d_row, ctx->d_rm2, ctx->d_rcls, ctx->d_rrow,
               ctx->d_rcf, ctx->d_rcr, ctx->d_errf, ctx->d_errw};
    const bool timed = ctx->timing;
    if (timed) CK(hipEventRecord(e0, ctx->stream));
    CK(launch_classify(ctx->d_keys_s, ctx->d_counts_s, n, sh, num_subs, rc_mode ? 1 : 0, o, ctx->nbr, ctx->stream));
    if (timed) CK(hipEventRecord(e1, ctx->stream));
    // (into pinned memory: a pageable destination makes the copy a staged, synchronous one)
    CK(hipMemcpyAsync(ctx->h_byte + 8, ctx->d_errf, 8, hipMemcpyDeviceToHost, ctx->stream));  // ~index, 0 none
    CK(hipStreamSynchronize(ctx->stream));
    u64 ef;
    std::memcpy(&ef, ctx->h_byte + 8, 8);
    ef = ~ef;  // the kernel kept ~(first error index): 0 -> ~0, none
    if (int src = settle_finalize(ctx)) return src;  // landed with the classify: no extra round trip
    float ms = 0;
    if (timed) CK(hipEventElapsedTime(&ms, e0, e1));
    ctx->classify_ms = ms;
    if (err_unique) *err_unique = ef == ~0ull ? -1 : (int64_t)ef;
    if (err_which) {
        *err_which = 0;
        if (ef != ~0ull) CK(hipMemcpy(err_which, ctx->d_errw + ef, 4, hipMemcpyDeviceToHost));
    }
    if (n) {
        if (m1) CK(hipMemcpy(m1, ctx->d_m1, n * 2, hipMemcpyDeviceToHost));
        if (m2) CK(hipMemcpy(m2, ctx->d_m2, n * 2, hipMemcpyDeviceToHost));
        if (cls) CK(hipMemcpy(cls, ctx->d_cls, n, hipMemcpyDeviceToHost));
        if (row) CK(hipMemcpy(row, ctx->d_row, n * 2, hipMemcpyDeviceToHost));
        if (rc_mode) {
            if (rc_m2) CK(hipMemcpy(rc_m2, ctx->d_rm2, n * 2, hipMemcpyDeviceToHost));
            if (rc_cls) CK(hipMemcpy(rc_cls, ctx->d_rcls, n, hipMemcpyDeviceToHost));
            if (rc_row) CK(hipMemcpy(rc_row, ctx->d_rrow, n * 2, hipMemcpyDeviceToHost));
        }
    }
    return FR_OK;
}

int fr_rc_counts(fr_ctx* ctx, uint64_t* reads_f, uint64_t* reads_rc) {
    if (int src = settle_finalize(ctx)) return src;
    if (!ctx->d_rcf) return fail(ctx, FR_ERR_INVALID, "fr_rc_counts: no rc classify yet");
    const int names = std::max(ctx->n_names, 1);
    std::vector<u64> f(names), r(names);
    CK(hipMemcpy(f.data(), ctx->d_rcf, names * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r.data(), ctx->d_rcr, names * 8, hipMemcpyDeviceToHost));
    for (int i = 0; i < ctx->n_names; ++i) {
        reads_f[i] = f[i];
        reads_rc[i] = r[i];
    }
    return FR_OK;
}

int fr_classify_cp(fr_ctx* ctx, int n, const uint32_t* q1, const int32_t* q1len, const uint32_t* q2,
                   const int32_t* q2len, int cp_stride, int num_subs, int rc_mode, int16_t* m1, int16_t* m2,
                   uint8_t* cls, int16_t* row, int16_t* rc_m2, uint8_t* rc_cls, int16_t* rc_row,
                   int32_t* err_which) {
    if (int src = settle_finalize(ctx)) return src;
    if (n <= 0) return FR_OK;
    if (ctx->S > 0 && (!ctx->d_cp1 || cp_stride != ctx->cp_stride))
        return fail(ctx, FR_ERR_INVALID, "fr_classify_cp: sheet code points missing or stride mismatch");
    u32 *dq1, *dq2;
    int32_t *dl1, *dl2;
    int16_t *o_m1, *o_m2, *o_row, *o_rm2, *o_rrow;
    u8 *o_cls, *o_rcls;
    int32_t* o_err;
    const u64 qn = (u64)n * cp_stride;
    CK(dalloc(&dq1, qn));
    CK(dalloc(&dq2, qn));
    CK(dalloc(&dl1, n));
    CK(dalloc(&dl2, n));
    CK(dalloc(&o_m1, n));
    CK(dalloc(&o_m2, n));
    CK(dalloc(&o_row, n));
    CK(dalloc(&o_rm2, n));
    CK(dalloc(&o_rrow, n));
    CK(dalloc(&o_cls, n));
    CK(dalloc(&o_rcls, n));
    CK(dalloc(&o_err, n));
    CK(hipMemcpy(dq1, q1, qn * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dq2, q2, qn * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dl1, q1len, n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dl2, q2len, n * 4, hipMemcpyHostToDevice));
    ClassOut o{o_m1, o_m2, o_cls, o_row, o_rm2, o_rcls, o_rrow, nullptr, nullptr, nullptr, o_err};
    CK(launch_classify_cp(n, dq1, dl1, dq2, dl2, cp_stride, ctx->S > 0 ? ctx->S : 0, ctx->d_cp1, ctx->d_cpl1,
                          ctx->d_cp2, ctx->d_cpl2, ctx->d_cp2rc, ctx->d_name, num_subs, rc_mode ? 1 : 0, o,
                          ctx->stream));
    CK(hipStreamSynchronize(ctx->stream));
    CK(hipMemcpy(m1, o_m1, n * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(m2, o_m2, n * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(cls, o_cls, n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(row, o_row, n * 2, hipMemcpyDeviceToHost));
    if (err_which) CK(hipMemcpy(err_which, o_err, n * 4, hipMemcpyDeviceToHost));
    if (rc_mode) {
        CK(hipMemcpy(rc_m2, o_rm2, n * 2, hipMemcpyDeviceToHost));
        CK(hipMemcpy(rc_cls, o_rcls, n, hipMemcpyDeviceToHost));
        CK(hipMemcpy(rc_row, o_rrow, n * 2, hipMemcpyDeviceToHost));
    }
    void* tmp[] = {dq1, dq2, dl1, dl2, o_m1, o_m2, o_row, o_rm2, o_rrow, o_cls, o_rcls, o_err};
    for (void* p : tmp) CK(hipFree(p));
    return FR_OK;
}

int fr_export_unique_device(fr_ctx* ctx, void* dev_keys, void* dev_counts, void* dev_first, uint64_t cap) {
    if (int src = settle_finalize(ctx)) return src;
    if (ctx->U > cap) return fail(ctx, FR_ERR_CAPACITY, "export buffer too small");
    if (ctx->U) {
        CK(hipMemcpyAsync(dev_keys, ctx->d_keys_s, ctx->U * 8, hipMemcpyDeviceToDevice, ctx->stream));
        CK(hipMemcpyAsync(dev_counts, ctx->d_counts_s, ctx->U * 8, hipMemcpyDeviceToDevice, ctx->stream));
        CK(hipMemcpyAsync(dev_first, ctx->d_first_s, ctx->U * 8, hipMemcpyDeviceToDevice, ctx->stream));
    }
    CK(hipStreamSynchronize(ctx->stream));
    return FR_OK;
}

int fr_export_partitioned_device(fr_ctx* ctx, int world, void* dev_rows, void* dev_counts, uint64_t cap) {
    if (int src = settle_finalize(ctx)) return src;
    if (world < 1 || world > 1024) return fail(ctx, FR_ERR_INVALID, "fr_export_partitioned_device: world out of range");
    if (ctx->U > cap) return fail(ctx, FR_ERR_CAPACITY, "export buffer too small");
    CK(launch_partition_rows(ctx->d_keys_s, ctx->d_counts_s, ctx->d_first_s, ctx->U, (u32)world, (u64*)dev_counts,
                             (u64*)dev_counts + world, (u64*)dev_rows, ctx->stream));
    CK(hipStreamSynchronize(ctx->stream));
    return FR_OK;
}

int fr_merge_rows_device(fr_ctx* ctx, const void* dev_rows, uint64_t n) {
    if (int src = settle_finalize(ctx)) return src;
    if (ctx->file_open) return fail(ctx, FR_ERR_INVALID, "fr_merge_rows_device: a file is open");
    int rc = flush_presence(ctx);
    if (rc) return rc;
    ctx->merged = true;
    rc = read_state(ctx);
    if (rc) return rc;
    if ((ctx->h_st->n_keys + n) * 2 > ctx->nslots) {
        rc = grow_table(ctx, true);
        if (rc) return rc;
    }
    ctx->st_fresh = false;
    CK(launch_merge_rows(ctx->tab, ctx->st, (const u64*)dev_rows, n, ctx->stream));
    return grow_table(ctx, false);
}

int fr_merge_unique_device(fr_ctx* ctx, const void* dev_keys, const void* dev_counts, const void* dev_first,
                           uint64_t n) {
    if (int src = settle_finalize(ctx)) return src;
    if (ctx->file_open) return fail(ctx, FR_ERR_INVALID, "fr_merge_unique_device: a file is open");
    int rc = flush_presence(ctx);  // this context's own file, before merged rows change the table
    if (rc) return rc;
    ctx->merged = true;
    rc = read_state(ctx);
    if (rc) return rc;
    if ((ctx->h_st->n_keys + n) * 2 > ctx->nslots) {
        rc = grow_table(ctx, true);
        if (rc) return rc;
    }
    ctx->st_fresh = false;
    CK(launch_merge(ctx->tab, ctx->st, (const u64*)dev_keys, (const u64*)dev_counts, (const u64*)dev_first, n,
                    ctx->stream));
    return grow_table(ctx, false);
}

void* fr_device_alloc(fr_ctx* ctx, uint64_t bytes) {
    void* p = nullptr;
    if (hipSetDevice(ctx->device) != hipSuccess || hipMalloc(&p, std::max<u64>(bytes, 1)) != hipSuccess) {
        ctx->err = "fr_device_alloc failed";
        return nullptr;
    }
    return p;
}

int fr_device_free(fr_ctx* ctx, void* ptr) {
    CK(hipFree(ptr));
    return FR_OK;
}

int fr_copy_to_host(fr_ctx* ctx, void* dst, const void* dev_src, uint64_t bytes) {
    CK(hipStreamSynchronize(ctx->stream));
    CK(hipMemcpy(dst, dev_src, bytes, hipMemcpyDeviceToHost));
    return FR_OK;
}

int fr_copy_to_device(fr_ctx* ctx, void* dev_dst, const void* src, uint64_t bytes) {
    CK(hipStreamSynchronize(ctx->stream));
    CK(hipMemcpy(dev_dst, src, bytes, hipMemcpyHostToDevice));
    return FR_OK;
}

int fr_synth_device(fr_ctx* ctx, uint8_t* dev_out, uint64_t r0, uint64_t n, int R, uint64_t seed,
                    const char* idx1_ascii, const char* idx2_ascii, int S, int L1, int L2) {
    if (S <= 0 || L1 <= 0 || L2 <= 0 || L1 + L2 > 32 || R < 0 || R > 256)
        return fail(ctx, FR_ERR_INVALID, "fr_synth_device: bad shape");
    u8 *d1, *d2;
    CK(dalloc(&d1, (u64)S * L1));
    CK(dalloc(&d2, (u64)S * L2));
    CK(hipMemcpy(d1, idx1_ascii, (u64)S * L1, hipMemcpyHostToDevice));
    CK(hipMemcpy(d2, idx2_ascii, (u64)S * L2, hipMemcpyHostToDevice));
    CK(launch_synth(dev_out, r0, n, R, seed, d1, d2, S, L1, L2, ctx->stream));
    CK(hipStreamSynchronize(ctx->stream));
    CK(hipFree(d1));
    CK(hipFree(d2));
    return FR_OK;
}

}  // extern "C"
