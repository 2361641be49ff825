/*
 * frender_amd.h — C ABI of libfrender_hip.so, the MI355X (gfx950) implementation of
 * frender's `scan` hot path: per-read header scan + barcode tally, Hamming
 * classification of the unique index combos, and the -rc per-sample call.
 *
 * The reference (njspix/frender, frender.py) has no FFI; its seam is three Python
 * calls inside frender_scan (frender.py:606, :610/:628, :614).  The entry points
 * below replace exactly those calls (each cites the reference function it
 * replaces); the host CLI (frender_amd/scan.py) keeps the reference's flags and
 * CSV formats and binds this header through ctypes (frender_amd/_lib.py).
 *
 * Conventions: every int-returning call returns FR_OK (0) or an FR_ERR_* code and
 * leaves a message in fr_last_error(ctx).  All pointers are plain host pointers
 * unless the name says _device.  Caller owns inputs; the library owns device
 * memory and the arrays it hands back until the next call that rebuilds them.
 * One context = one GPU = one host thread (not re-entrant).
 */
#ifndef FRENDER_AMD_H
#define FRENDER_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FR_OK 0
#define FR_ERR_INVALID 1   /* bad argument / call order */
#define FR_ERR_HIP 2       /* HIP runtime error */
#define FR_ERR_CAPACITY 3  /* a device table or pool is full */
#define FR_ERR_DEVICE 4    /* a kernel reported an internal failure (look-back spin bound) */
#define FR_ERR_IO 6        /* a .gz input could not be inflated (fr_gz_feed; message in fr_gz_error) */

/* scan-time data errors: reported in fr_file_stats.error, mirroring the reference's crash */
#define FR_SCAN_OK 0
#define FR_SCAN_NO_SPACE 1 /* header line without ' ': IndexError at frender.py:169 */
#define FR_SCAN_UTF8 2     /* invalid UTF-8: UnicodeDecodeError from gzip.open(...,"rt") at :159 */

/* classification classes (read_type, frender.py:266-284) */
#define FR_UNDETERMINED 0
#define FR_INDEX_HOP 1
#define FR_DEMUXABLE 2
#define FR_AMBIGUOUS 3

typedef struct fr_ctx fr_ctx;

typedef struct fr_file_stats {
    uint64_t records;        /* header lines counted (after -s), = `actual_reads` (frender.py:160-166) */
    uint64_t lines;          /* lines in the file (universal newlines) */
    uint64_t new_keys;       /* distinct codes in this file, exotic ones included (`new_barcodes`, :175) */
    uint64_t exotic;         /* records whose code is outside both key forms (see fr_get_exotic_table) */
    int32_t error;           /* FR_SCAN_* (FR_SCAN_NO_SPACE wins when both were seen) */
    int32_t utf8_bad;        /* 1: an invalid UTF-8 sequence lies in the bytes scanned (with -s possibly past the
                              * sample: the host decides whether the reference's reader would decode it) */
    uint64_t error_offset;   /* file byte offset of the first offending header (FR_SCAN_NO_SPACE) */
} fr_file_stats;

typedef struct fr_timing {
    uint64_t scan_launches;  /* tally kernel launches since fr_reset */
    uint64_t scan_bytes;     /* decoded bytes those launches scanned */
    double scan_ms;          /* summed HIP-event duration of those launches */
    double last_scan_ms;     /* duration of the most recent launch */
    double classify_ms;      /* last classify pass */
    double finalize_ms;      /* last compaction + ordering */
    double log_ms;           /* summed duration of the launch-log aggregations after those launches */
} fr_timing;

/* ---- lifecycle ------------------------------------------------------------------ */
/* chunk_bytes: bytes per tally launch of a device feed, at most 16 GiB - 1 MiB (device feeds are cut
 * into equal ranges of at most this size, and of at most 4 GiB - 1 MiB while their commits may go to
 * the launch log; host feeds use a pinned ring of min(chunk_bytes, 1 GiB) slots).
 * table_slots: initial HBM hash-table slots (grown between launches).  Nothing in the environment
 * changes a context's geometry: fr_create uses the library's defaults, fr_create_tuned the caller's
 * fr_tuning (tests, A/B runs). */
fr_ctx* fr_create(int device, uint64_t chunk_bytes, uint64_t table_slots);
/* The tally's launch geometry and thresholds.  Results never depend on them (every setting gives the
 * same table); only the speed does.  Fill with fr_tuning_defaults, change fields, pass to
 * fr_create_tuned.  `size` = sizeof(fr_tuning) of the caller (fields past it keep their defaults). */
typedef struct fr_tuning {
    uint32_t size;
    int32_t grid;               /* tally workgroups; 0 = CUs x the kernel's occupancy */
    uint32_t flush_at;          /* LDS-table keys per chunk before new codes go to the cold list */
    uint32_t cold_cap;          /* cold-list entries per workgroup (>= 1024) */
    int32_t log;                /* 1: heavy commits may go to the launch log; 0: every commit inserts directly */
    uint32_t log_min;           /* pairs from which a commit logs (0: every commit) */
    uint32_t log_hot;           /* a logged commit's LDS entries of >= log_hot records insert directly (>= 1) */
    uint32_t chunk_tiles;       /* 4-KiB wave-tiles per full chunk (>= 2) */
    uint32_t chunk_tiles_heavy; /* the same once commits log (>= 2) */
    int32_t ramp;               /* 1: ramped chunk sizes; 0: one uniform chunk per workgroup */
    uint32_t ramp_up_s;         /* the ramps' smallest chunks (tiles, >= 1) */
    uint32_t ramp_down_s;
    uint32_t ramp_down_pct;     /* ramp-down chunks, % of the grid (1..100), normal / heavy geometry */
    uint32_t ramp_down_pct_h;
    int32_t spec_commit;        /* 1: device feeds commit speculative chunks at once (checked at the launch end) */
    int32_t nbr;                /* 1: classify through the sheet's neighbourhood maps; 0: row scan only */
    uint64_t ovf_cap;           /* overflow-list entries (new codes a launch adds past the table's probe bound;
                                 * 0 = 4 Mi; a device feed that overflows it is replayed in smaller ranges) */
} fr_tuning;
void fr_tuning_defaults(fr_tuning* t);
fr_ctx* fr_create_tuned(int device, uint64_t chunk_bytes, uint64_t table_slots, const fr_tuning* t);
void fr_destroy(fr_ctx* ctx);
const char* fr_last_error(const fr_ctx* ctx);
int fr_get_timing(fr_ctx* ctx, fr_timing* out);
/* on != 0 (the default): HIP timing events around every tally launch, its launch-log aggregation,
 * fr_finalize and fr_classify (fr_get_timing's figures).  on = 0: none are recorded (each event
 * record is a bubble of a few microseconds on the stream); fr_get_timing then reports zeros for the
 * work done while off.  Results do not depend on it. */
int fr_set_timing(fr_ctx* ctx, int on);
int fr_sync(fr_ctx* ctx);
/* diagnostics: {look-back max polls, total polls, keys, overflow, presence, exotic, grid, slots,
 * 8 phase stamps, speculation replays, exotic-only replays, next full-chunk size, heavy launches,
 * big-feed rollbacks, the last device feed's fullest launch-log fold, its fold overflows, its range bytes} */
int fr_get_diag(fr_ctx* ctx, uint64_t* out, int n);

/* ---- sample sheet (the idx1/idx2/id lists of get_indexes, frender.py:90-116) -------
 * idx*_packed: each entry case-folded (str.lower(), :226) and packed 3 bits/char,
 * char i at bits [3i,3i+3): a=1 c=2 g=3 t=4 n=5, any other char=7; entries longer
 * than 21 chars pack as 0 (they can only fail the length assert).  idx2rc_packed is
 * the same for reverse_complement(idx2) (:210-211).  idx*_len are the case-folded
 * lengths.  name_id[i] = index of row i's id among the distinct ids in
 * first-appearance order (call_rc_mode_per_id's dict, :367).  The code-point
 * arrays (stride `cp_stride`, may be NULL) feed the generic classifier used for
 * codes outside the fast alphabet. */
int fr_set_sheet(fr_ctx* ctx, int S,
                 const uint64_t* idx1_packed, const int32_t* idx1_len,
                 const uint64_t* idx2_packed, const int32_t* idx2_len,
                 const uint64_t* idx2rc_packed, const int32_t* name_id, int n_names,
                 const uint32_t* idx1_cp, const uint32_t* idx2_cp, const uint32_t* idx2rc_cp,
                 int cp_stride);

/* ---- tally: replaces tally_barcodes (frender.py:183-207) / scan_file (:154-181) ----
 * Files are fed in parse_files order (:604); fr_reset starts a new scan. */
int fr_reset(fr_ctx* ctx);
int fr_begin_file(fr_ctx* ctx, int64_t max_records /* -s, <=0: no limit */);
/* fr_begin_file at a global position, for scans sharded over contexts / GPUs (SURVEY §8(e);
 * replaces the per-file work unit of the reference's Pool, frender.py:189-193): file_index is the
 * file's index in the whole scan's parse_files order and byte_base the file offset of the first
 * byte this context will be fed (a record-aligned shard of the file; 0 for a whole file).  The
 * ordinals ((file_index+1) << 44 | byte_base + offset), the presence pairs' file index and
 * therefore the merged first-occurrence order are the single-context ones.  file_index must
 * increase within a scan (fr_begin_file takes the next index). */
int fr_begin_file_at(fr_ctx* ctx, int64_t file_index, uint64_t byte_base, int64_t max_records);
/* Decoded (gunzipped) bytes of the current file, any split; the library cuts at
 * line ends, carries the remainder, copies through a pinned ring to HBM and
 * launches.  Returns FR_OK, or 5 (FR_SAMPLE_DONE) once -s records were seen. */
#define FR_SAMPLE_DONE 5
int fr_feed(fr_ctx* ctx, const uint8_t* data, uint64_t len);
/* ---- native inflate: replaces gzip.open(file, "rt") (frender.py:159) as
 * the source of the decoded bytes.  fr_gz_open starts `threads` host threads that inflate the
 * listed .gz files (zlib; multi-member, NUL padding between members as Python's gzip) up to
 * `threads` files ahead of the consumer, in list order, into 16 MiB blocks.  fr_gz_feed hands
 * file i's blocks to fr_feed (call it between fr_begin_file[_at] and fr_end_file; files in list
 * order) and returns FR_OK, FR_SAMPLE_DONE, or FR_ERR_IO when the stream is not valid gzip (the
 * caller re-reads the file with Python's gzip to raise the reference's exception). */
typedef struct fr_gz fr_gz;
fr_gz* fr_gz_open(const char* const* paths, int n_files, int threads);
/* the same with at most files_ahead files inflating at once: the other threads help split the big
 * single-member files among them (the demux reads a file pair at a time) */
fr_gz* fr_gz_open_ahead(const char* const* paths, int n_files, int threads, int files_ahead);
int fr_gz_feed(fr_gz* g, int i, fr_ctx* ctx);
/* The consumer-side alternative to fr_gz_feed (demux reads R1 and R2 in lockstep): the next decoded
 * block of file i.  *data / *len stay valid until the next fr_gz_next or fr_gz_close on the pool;
 * *len == 0 at the file's end.  FR_ERR_IO: not a valid gzip stream (fr_gz_error).  Replaces the
 * reference's gzip.open(read_file, "rt") iteration in frender_demux (frender.py:776-777). */
int fr_gz_next(fr_gz* g, int i, const uint8_t** data, uint64_t* len);
/* Record shards of one file (multi-GPU scans of fewer files than GPUs; SURVEY §8(e) "host cuts
 * record-aligned chunks and deals them to GPUs"): part `part` of `nparts` of file i's decoded
 * stream is [b_part, b_part+1), b_0 = 0, b_nparts = the end, and for 0 < j < nparts b_j = the first
 * record start (a line start whose index from the file start is 0 mod 4, universal newlines as
 * frender.py:159 reads them) at or after j * hint / nparts.  The function inflates the file from its
 * start, counts line ends on the host, calls fr_begin_file_at(ctx, file_index, b_part, 0) once the
 * part's start is known, feeds only the part's bytes, stops inflating at its end and stores b_part
 * in *byte_base; the caller then calls fr_end_file.  Every rank that passes the same `hint` cuts the
 * same way.  Not with -s (a sample is the head of each whole file). */
int fr_gz_feed_part(fr_gz* g, int i, fr_ctx* ctx, int64_t file_index, int part, int nparts, uint64_t hint,
                    uint64_t* byte_base);
/* The cuts fr_gz_feed_part makes: bounds[0..nparts] (b_0 = 0, b_nparts = the decoded size).  Host
 * only (no GPU context): FR_OK, or FR_ERR_IO when the file is not valid gzip. */
int fr_gz_part_bounds(const char* path, int nparts, uint64_t hint, uint64_t* bounds);
/* BGZF record parts without a prefix inflate (multi-GPU scans of fewer files than GPUs): a BGZF
 * file's members give every member's decoded offset from the headers alone, so part `part` of
 * `nparts` is decoded on its own.  Its member range is [M_part, M_part+1), M_j = the decoded offset of
 * the first member starting at or after j * total / nparts (M_0 = 0, M_nparts = the decoded size).
 * fr_gz_part_open decodes that range (threads: this thread plus helpers; libdeflate when present,
 * else zlib) and returns the line terminators whose terminating byte lies in it (universal newlines,
 * frender.py:159); *is_bgzf = 0 (and no handle) when the file is not BGZF: cut it with
 * fr_gz_feed_part instead.  FR_ERR_IO: a member does not decode (the host replays the file through
 * Python's gzip for the reference's exception).  With lines_before = the terminators before M_part
 * (the other parts' counts, exchanged by the caller), the part's records are [b_part, b_part+1), b_j =
 * the first record start at or after M_j: fr_gz_part_data hands them out (host bytes, valid until
 * fr_gz_part_close), fr_gz_part_feed calls fr_begin_file_at(ctx, file_index, b_part, 0) and fr_feed
 * with them (the caller then calls fr_end_file).  *inflated: decoded bytes produced for the part so far
 * (the part plus at most the members around its ends). */
typedef struct fr_gz_part fr_gz_part;
int fr_gz_part_open(const char* path, int part, int nparts, int threads, fr_gz_part** out, int* is_bgzf,
                    uint64_t* lines, uint64_t* inflated);
int fr_gz_part_data(fr_gz_part* p, uint64_t lines_before, const uint8_t** data, uint64_t* len, uint64_t* byte_base,
                    uint64_t* inflated);
int fr_gz_part_feed(fr_gz_part* p, fr_ctx* ctx, int64_t file_index, uint64_t lines_before, uint64_t* byte_base);
const char* fr_gz_part_error(const fr_gz_part* p);
void fr_gz_part_close(fr_gz_part* p);
/* The decoded size of a .gz file as far as its trailers tell (0 when unreadable): exact for BGZF (the
 * members' ISIZE fields) and for a single-member file of up to 4 GiB decoded; otherwise the last
 * member's ISIZE lifted toward 4x the compressed size.  A deterministic fr_gz_feed_part hint. */
uint64_t fr_gz_size_hint(const char* path);

/* ---- scan CSV (row a9; replaces report_analysis' csv.DictWriter, frender.py:482-501) ------------
 * Writes header, then one excel-dialect row per unique code: parts[0], parts[1] of code.split("+"),
 * matched_idx1, matched_idx2, read_type, sample_name, reads[, demux_ok].  keys[j] is row j's packed
 * key (fr_get_unique form, fast or wide); rows listed in exo_rows (increasing) take their first two
 * fields from exo_text[exo_off[e], exo_off[e+1]) instead ("p0,p1", already CSV-quoted).  dict holds
 * the CSV-quoted strings the other fields index: dict_n[0] idx1 entries (m1), dict_n[1] idx2
 * entries (m2), dict_n[2] sample names (row), dict_n[3] class names (cls); entry i is
 * dict[dict_off[i], dict_off[i+1]).  Negative m1/m2/row write an empty field; demux_ok NULL omits the
 * column.  FR_ERR_INVALID (nothing written) when a keyed code has no '+' or an index is out of
 * range; FR_ERR_IO when the file cannot be written. */
int fr_write_scan_csv(const char* path, const char* header, uint64_t n_rows, const uint64_t* keys,
                      const uint64_t* counts, const int16_t* m1, const int16_t* m2, const uint8_t* cls,
                      const int16_t* row, const uint8_t* demux_ok, const char* dict, const uint64_t* dict_off,
                      const uint32_t* dict_n, uint64_t n_exotic, const uint64_t* exo_rows, const char* exo_text,
                      const uint64_t* exo_off);
const char* fr_gz_error(const fr_gz* g);
void fr_gz_close(fr_gz* g);
/* Decode buffers outlive their pool: a process-wide cache keeps up to 4 GiB of them for the next scan
 * (no page faults per GB).  fr_gz_trim returns every cached buffer to the OS (long-lived processes that
 * scan once, e.g. the seam, call it after a scan). */
void fr_gz_trim(void);
/* Large single-member gzip files (the usual .fastq.gz of one lane) are not one thread's work: a member of
 * at least 16 MiB compressed is decoded by all of the pool's idle threads at once (chunks of the
 * compressed stream decoded from candidate block starts with their unknown 32 KiB windows as markers,
 * stitched and resolved in order, checked against the member's CRC-32 and ISIZE; any failure decodes the
 * file with one thread instead, whose decoders own the error behaviour).  The number of files decoded
 * that way in this process (diagnostics, tests). */
uint64_t fr_gz_parallel_members(void);

/* The whole current file is already resident in HBM (bench / device producers). */
int fr_feed_device(fr_ctx* ctx, const uint8_t* dev_data, uint64_t len);
int fr_end_file(fr_ctx* ctx, fr_file_stats* out);

/* ---- the merged unique table (barcode_counter["total"], :199-203) -----------------
 * fr_finalize compacts the device hash table and orders it by first occurrence
 * (file order, then byte offset) on the GPU.  Keys: fast keys are 3-bit packed codes over
 * {A=1,C=2,G=3,T=4,N=5,'+'=6}, char i at bits [3i,3i+3), at most 21 chars; wide keys (bit 63
 * set) hold codes whose letters are all ACGTN or all acgtn, at most one '+', each part <= 21 and
 * <= 24 letters in total: bit 62 lowercase, bits 57-61 the '+' position (letters before it; 31
 * none), bits 0-56 V = sum d_i 5^i + (5^n - 1)/4 over the n letters, d: A0 C1 G2 T3 N4. */
int fr_finalize(fr_ctx* ctx, uint64_t* n_unique, uint64_t* n_presence, uint64_t* n_exotic);
int fr_get_unique(fr_ctx* ctx, uint64_t* keys, uint64_t* counts, uint64_t* first_ordinal);
/* (unique index, file index) for every file a fast-path key occurs in (R10 demux_ok) */
int fr_get_presence(fr_ctx* ctx, uint32_t* unique_idx, uint32_t* file_idx);
/* The reads of each presence pair's code in the pair's file: the values of the reference's per-file
 * tables, barcode_counter[basename][code] (scan_file's file_barcodes, frender.py:171-177, kept by
 * tally_barcodes at :204-205).  counts[n_presence] aligns with fr_get_presence, exotic_counts with
 * fr_get_exotic_table's presence pairs; either may be NULL. */
int fr_get_presence_counts(fr_ctx* ctx, uint64_t* counts, uint64_t* exotic_counts);
/* Codes outside both key forms ("exotic": mixed case, other bytes, more than 24 letters, a part
 * longer than 21, two or more '+'), aggregated over the scan by exact byte string inside the
 * library: the device captures each such record's code bytes, the library drains them after the
 * launch that produced them (a launch that overflows the list is replayed capturing exotic codes
 * only, after the list grows) and merges them natively.  Order: first drained, not first
 * occurrence (use `first`).  fr_exotic_sizes gives the array sizes for fr_get_exotic_table:
 * counts/first per code, offsets[n+1] into the concatenated code bytes, and (code, file index)
 * presence pairs (R10). */
int fr_exotic_sizes(fr_ctx* ctx, uint64_t* n_codes, uint64_t* code_bytes, uint64_t* n_presence);
int fr_get_exotic_table(fr_ctx* ctx, uint64_t* counts, uint64_t* first, uint64_t* offsets, uint8_t* bytes,
                        uint32_t* pres_code, uint32_t* pres_file);

/* ---- classify: replaces process (:391-426) -> analyze_barcodes_with_rc (:294-351)
 *      -> analyze_barcode (:237-291) -> get_indexes_of_approx_matches (:214-234) ----
 * Runs over the finalized unique table with the current sheet and num_subs.
 * Per unique (host arrays of n_unique):  m1,m2 = first matching sheet row or -1
 * (matched_idx1/2, :261-262), cls = FR_* class, row = the demux row or -1.  With
 * rc_mode the rc_* arrays receive the rc(idx2) pass and the ambiguity override
 * (:336-349) is applied; may be NULL otherwise.  err_unique receives the first
 * unique index (in order) whose lengths fail the assert at :227 (or -1), and
 * err_which 1 = idx1, 2 = idx2, 3 = no '+' (ValueError at :306). */
int fr_classify(fr_ctx* ctx, int num_subs, int rc_mode,
                int16_t* m1, int16_t* m2, uint8_t* cls, int16_t* row,
                int16_t* rc_m2, uint8_t* rc_cls, int16_t* rc_row,
                int64_t* err_unique, int32_t* err_which);
/* per distinct name: reads demuxable with fwd idx2 / with rc idx2 (:367-373), from the
 * last rc_mode classify */
int fr_rc_counts(fr_ctx* ctx, uint64_t* reads_f, uint64_t* reads_rc);
/* generic classifier for codes outside the fast alphabet: queries as case-folded
 * code points (stride cp_stride), same outputs as fr_classify plus a per-query err_which */
int fr_classify_cp(fr_ctx* ctx, int n, const uint32_t* q1, const int32_t* q1len,
                   const uint32_t* q2, const int32_t* q2len, int cp_stride, int num_subs, int rc_mode,
                   int16_t* m1, int16_t* m2, uint8_t* cls, int16_t* row,
                   int16_t* rc_m2, uint8_t* rc_cls, int16_t* rc_row, int32_t* err_which);

/* ---- multi-GPU merge: export / import the compacted table ----------- */
int fr_export_unique_device(fr_ctx* ctx, void* dev_keys, void* dev_counts, void* dev_first, uint64_t cap);
/* The same rows as one int64 array [U][3] of (key, count, first), partitioned by owner rank: owner = the top 24
 * bits of key * 0x9E3779B97F4A7C15 (mod 2^64) mod world (frender_amd/dist.py owner_of), the blocks of owners
 * 0..world-1 contiguous in that order (order inside a block not fixed); dev_counts receives 2 x world int64:
 * the rows per owner, then scratch.  Synchronises the library's stream.  1 <= world <= 1024. */
int fr_export_partitioned_device(fr_ctx* ctx, int world, void* dev_rows, void* dev_counts, uint64_t cap);
/* Merge n int64 rows [n][3] (key, count, first) from device memory into the table (count = sum, first = min);
 * the row-major form of fr_merge_unique_device (the rows an all-to-all delivered). */
int fr_merge_rows_device(fr_ctx* ctx, const void* dev_rows, uint64_t n);
int fr_merge_unique_device(fr_ctx* ctx, const void* dev_keys, const void* dev_counts, const void* dev_first,
                           uint64_t n);

/* ---- device memory + SYN-v1 generator (bench and tests) --------------------------- */
void* fr_device_alloc(fr_ctx* ctx, uint64_t bytes);
int fr_device_free(fr_ctx* ctx, void* ptr);
int fr_copy_to_host(fr_ctx* ctx, void* dst, const void* dev_src, uint64_t bytes);
int fr_copy_to_device(fr_ctx* ctx, void* dev_dst, const void* src, uint64_t bytes);
/* records r0..r0+n-1 of SYN-v1 (frender_amd/synth.py) into dev_out; idx ascii S*L */
int fr_synth_device(fr_ctx* ctx, uint8_t* dev_out, uint64_t r0, uint64_t n, int R, uint64_t seed,
                    const char* idx1_ascii, const char* idx2_ascii, int S, int L1, int L2);

/* ---- demux: replaces the hot loop of frender_demux (frender.py:776-810)
 * One file pair at a time.  The caller hands over decoded text with universal newlines already
 * normalised to '\n' (the reference reads in text mode, :776).  Records are groups of 4 lines
 * (grouper, :719-723); the R2 record's code is the text after the last ':' of its first line
 * (:778).  Destinations are small non-negative ids chosen by the caller (one per writer pair). */
#define FR_DMX_MISSING (-1) /* code not in the results: SystemExit "Couldn't find barcode ..." (:807-810) */
#define FR_DMX_BADTYPE (-2) /* read type with no writers: SystemExit "Unrecognized read type ..." (:803-806) */
#define FR_DMX_EXOTIC (-3)  /* code outside the fast alphabet / > 21 chars: the host resolves it */

typedef struct fr_dmx fr_dmx;
fr_dmx* fr_dmx_create(int device);
void fr_dmx_destroy(fr_dmx* d);
const char* fr_dmx_last_error(const fr_dmx* d);
/* results table: fast-alphabet codes (3-bit packed like fr_get_unique keys) -> destination or
 * FR_DMX_BADTYPE; codes absent from the table resolve to FR_DMX_MISSING */
int fr_dmx_set_table(fr_dmx* d, const uint64_t* keys, const int32_t* vals, uint64_t n);
/* mate 0 = R1, 1 = R2 (R2 also resolves every record's destination); returns the record count */
int fr_dmx_load(fr_dmx* d, int mate, const uint8_t* data, uint64_t len, uint64_t* n_records);
/* the same over the concatenation of n_parts host buffers (a window without a host-side join) */
int fr_dmx_load_parts(fr_dmx* d, int mate, const uint8_t* const* parts, const uint64_t* lens, int n_parts,
                      uint64_t* n_records);
/* the same over bytes already resident in HBM (16-byte aligned; used in place until the next load) */
int fr_dmx_load_device(fr_dmx* d, int mate, const uint8_t* dev_data, uint64_t len, uint64_t* n_records);
/* byte span [start, end) of the given records of a mate (host error messages, exotic codes) */
int fr_dmx_records(fr_dmx* d, int mate, const uint64_t* recs, uint64_t n, uint64_t* starts, uint64_t* ends);
/* R2 records < n_pairs whose destination is FR_DMX_EXOTIC (first cap written; *n = total) */
int fr_dmx_exotic(fr_dmx* d, uint64_t n_pairs, uint64_t* recs, uint64_t cap, uint64_t* n);
/* set the destinations of the given R2 records (the host's resolution of exotic codes) */
int fr_dmx_patch(fr_dmx* d, const uint64_t* recs, const int32_t* dest, uint64_t n);
/* route the first n_pairs record pairs: if some pair has a negative destination, *first_error is
 * the first such pair and *error_val its value (nothing routed); otherwise both mates' records
 * are gathered destination-major (record order kept within a destination) and the byte count
 * of every destination is returned per mate */
int fr_dmx_route(fr_dmx* d, int n_dest, uint64_t n_pairs, int64_t* first_error, int32_t* error_val,
                 uint64_t* bytes_r1, uint64_t* bytes_r2);
/* the routed bytes of a mate (destination-major) */
int fr_dmx_fetch(fr_dmx* d, int mate, uint8_t* out, uint64_t len);
/* the demux writers' compression on the GPU (replaces the gzip.open(..., "wb") writer pairs of
 * frender.py:667-676 that frender.py:795-810 write every routed record to): the routed bytes of a mate
 * (the last fr_dmx_route) become one raw deflate stream (RFC 1951) per destination that has bytes;
 * comp_bytes[k] = its byte count (0: no bytes routed), crc32[k] = the CRC-32 of destination k's routed
 * bytes, so that a gzip member is header + stream + (crc32[k], bytes routed).  The streams stay on the
 * device, destination-major, until fr_dmx_fetch_deflated (the next fr_dmx_deflate of the mate replaces
 * them). */
int fr_dmx_deflate(fr_dmx* d, int mate, int n_dest, uint64_t* comp_bytes, uint32_t* crc32);
int fr_dmx_fetch_deflated(fr_dmx* d, int mate, uint8_t* out, uint64_t len);

/* ---- GPU deflate over any byte ranges (fr_deflate.hip; fr_dmx_deflate runs it on the routed bytes).
 * Stream s is bytes [offsets[s], offsets[s + 1]) of the device buffer dev_data (4-byte aligned, 16
 * readable bytes past offsets[n_streams]); every stream becomes one raw deflate stream, no larger than
 * zlib level 9 makes it on FASTQ-shaped text (64-KiB blocks, each with a dynamic Huffman code over a
 * cost-minimising parse; a block that would not shrink is stored). */
typedef struct fr_defl fr_defl;
fr_defl* fr_defl_create(int device);
void fr_defl_destroy(fr_defl* z);
const char* fr_defl_last_error(const fr_defl* z);
int fr_defl_run(fr_defl* z, const uint8_t* dev_data, const uint64_t* offsets, int n_streams, uint64_t* comp_bytes,
                uint32_t* crc32);
/* the same over a host buffer (copied to the device first) */
int fr_defl_run_host(fr_defl* z, const uint8_t* data, uint64_t len, const uint64_t* offsets, int n_streams,
                     uint64_t* comp_bytes, uint32_t* crc32);
/* the last run's streams, concatenated in stream order */
uint64_t fr_defl_out_bytes(const fr_defl* z);
/* blocks this context stored because their dynamic encoding's bit accounting did not add up (the stored
 * form is always a valid encoding of the block; a nonzero count is a diagnostic, not an error) */
uint64_t fr_defl_stored_fallbacks(const fr_defl* z);
int fr_defl_fetch(fr_defl* z, uint8_t* out, uint64_t len);

#ifdef __cplusplus
}
#endif
#endif
