// fr_gz.cpp — native inflate for the scan's input.
//
// The reference reads each file with gzip.open(file, "rt") (frender.py:159): one Python process
// per file (its Pool, :189-193).  Here a pool of host threads inflates the scan's .gz files with
// zlib, up to `threads` files at a time in scan order, into 16 MiB blocks queued per file; the
// consumer (the scan's host thread) hands each file's blocks to fr_feed in order, which copies them
// through the pinned ring to HBM while the next blocks inflate.  No GIL, no Python bytes objects.
//
// Stream rules follow Python's gzip module (3.10, _GzipReader): members are inflated one after
// another (multi-member files), NUL padding after a member is skipped, anything else after a
// member must start a new member, and an empty file is empty.  Any other deviation (bad magic,
// truncated member, CRC/length mismatch, deflate error) stops that file with FR_ERR_IO: the host
// then re-reads the file through Python's gzip to raise the reference's own exception.
//
// Fast path: when the image has libdeflate (whole-buffer DEFLATE, 2-3x zlib's inflate speed; loaded
// with dlopen, so the library is optional), a file of up to 256 MiB compressed whose last member's
// ISIZE trailer promises at most 1 GiB is decompressed whole, member by member, and queued in one
// piece; a BGZF file (every member carries its size) is decoded member-parallel in windows of
// BGZF_WINDOW output bytes.  Anything unusual -- bytes after a member that are neither NUL padding
// nor a new member, a member libdeflate rejects, more output than promised, a BGZF header field out
// of the format's bounds -- falls back to the zlib stream, which owns the exact rules and errors above.
//
// Memory and threads are bounded per pool: whole-file buffers (input + output) draw on a shared
// budget of WHOLE_BUDGET bytes (a file that does not fit streams through zlib instead), and the
// helper threads of a BGZF decode come out of the pool's own thread count (the workers that are
// idle), so at most `threads` threads inflate at once.
#include <dlfcn.h>
#include <sys/stat.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/frender_amd.h"
#include "fr_pinflate.h"

// Byte buffers whose resize() does not zero-fill: every byte of a decode buffer is written by the
// decoder before anything reads it, and zeroing 1-2 GB per scan cost as much as the copies.
template <class T>
struct DefaultInit : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = DefaultInit<U>;
    };
    DefaultInit() = default;
    template <class U>
    DefaultInit(const DefaultInit<U>&) {}
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        if constexpr (sizeof...(A) == 0) ::new ((void*)p) U;
        else ::new ((void*)p) U(std::forward<A>(a)...);
    }
};
using Bytes = std::vector<uint8_t, DefaultInit<uint8_t>>;

namespace {

// Decode buffers outlive the pool that used them.  A scan inflates GBs into buffers of hundreds of
// MB; giving them back to the OS at fr_gz_close (munmap) and faulting fresh pages in at the next
// scan's decode cost ~0.1 s per GB each way.  Released buffers of >= 1 MiB stay here (up to
// CACHE_MAX bytes of capacity, process-wide) and the next take() of at most their size reuses one.
class BufCache {
    static constexpr size_t CACHE_MAX = 4ull << 30;
    std::mutex m_;
    std::vector<Bytes> v_;
    size_t bytes_ = 0;

  public:
    Bytes take(size_t n) {
        Bytes b;
        {
            std::lock_guard<std::mutex> lk(m_);
            size_t best = v_.size();
            for (size_t i = 0; i < v_.size(); ++i)
                if (v_[i].capacity() >= n && (best == v_.size() || v_[i].capacity() < v_[best].capacity())) best = i;
            if (best < v_.size()) {
                b = std::move(v_[best]);
                v_[best] = std::move(v_.back());
                v_.pop_back();
                bytes_ -= b.capacity();
            }
        }
        b.resize(n);
        return b;
    }
    void trim() {  // every cached buffer back to the OS
        std::vector<Bytes> drop;
        {
            std::lock_guard<std::mutex> lk(m_);
            drop.swap(v_);
            bytes_ = 0;
        }
    }
    void give(Bytes&& b) {
        Bytes drop = std::move(b);  // freed outside the lock when it does not stay
        if (drop.capacity() < (1u << 20)) return;
        std::lock_guard<std::mutex> lk(m_);
        if (bytes_ + drop.capacity() > CACHE_MAX) return;
        bytes_ += drop.capacity();
        drop.clear();
        v_.push_back(std::move(drop));
    }
};

BufCache& buf_cache() {
    static BufCache* c = new BufCache();  // never destroyed: no teardown-order questions at exit
    return *c;
}

struct GzFile {
    std::string path;
    std::deque<Bytes> q;
    bool done = false;
    bool cancel = false;
    std::string err;
};

}  // namespace

struct fr_gz {
    std::vector<GzFile> files;
    int threads = 1;
    int ahead = 1;         // files inflating at once (fr_gz_open: threads; fr_gz_open_ahead: fewer)
    int busy = 0;          // threads inflating now (workers + BGZF helpers), <= threads
    size_t whole_used = 0; // bytes of whole-file buffers held now (<= WHOLE_BUDGET)
    size_t block = 16u << 20;
    size_t depth = 3;  // blocks queued per file (set by fr_gz_open)
    std::mutex m;
    std::condition_variable cv;
    std::vector<std::thread> workers;
    std::vector<Bytes> spare;  // consumed blocks for reuse (no page faults per block)
    Bytes held;                // the block fr_gz_next handed out last
    int next = 0;     // next file a worker starts
    int consume = 0;  // file the consumer reads (workers stay within [consume, consume + threads))
    bool stop = false;
    std::string err;
    ~fr_gz() {  // the buffers stay in the process-wide cache
        for (auto& f : files)
            for (auto& b : f.q) buf_cache().give(std::move(b));
        for (auto& b : spare) buf_cache().give(std::move(b));
        buf_cache().give(std::move(held));
    }
};

namespace {

// A consumed block back to the pool (g->m held): streaming blocks stay in its spare list; a parallel
// decode's pieces (bigger than a block) are left to the caller for the process-wide cache, where the
// next parallel decode takes them (kept in the spare list they were never reused, and a demux of
// 14 GB held them all until the pool closed: 1.1-1.4 s of munmap there)
bool keep_spare(fr_gz* g, Bytes& b) {
    if (b.capacity() > 2 * g->block || g->spare.size() >= (size_t)g->threads * g->depth) return false;
    g->spare.push_back(std::move(b));
    return true;
}

}  // namespace

namespace {

struct Libdeflate {
    void* (*alloc)();
    int (*gzip_ex)(void*, const void*, size_t, void*, size_t, size_t*, size_t*);
    void (*release)(void*);
};

const Libdeflate* libdeflate() {
    static const Libdeflate* ld = []() -> const Libdeflate* {
        if (const char* e = getenv("FR_GZ_ZLIB"))
            if (atoi(e) != 0) return nullptr;
        void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return nullptr;
        static Libdeflate l;
        l.alloc = (void* (*)())dlsym(h, "libdeflate_alloc_decompressor");
        l.gzip_ex = (int (*)(void*, const void*, size_t, void*, size_t, size_t*, size_t*))dlsym(
            h, "libdeflate_gzip_decompress_ex");
        l.release = (void (*)(void*))dlsym(h, "libdeflate_free_decompressor");
        return (l.alloc && l.gzip_ex && l.release) ? &l : nullptr;
    }();
    return ld;
}

constexpr size_t LD_MAX_IN = 256ull << 20;   // compressed bytes a file may have for the fast path
constexpr size_t LD_MAX_OUT = 1ull << 30;    // decoded bytes it may produce
constexpr size_t BGZF_MAX_IN = 1ull << 30;   // BGZF files: compressed bytes for the parallel path
constexpr size_t BGZF_MAX_BLOCK = 65536;     // the format's bound on a member's size and ISIZE
constexpr size_t BGZF_WINDOW = 64ull << 20;  // decoded bytes per parallel BGZF window
constexpr size_t WHOLE_BUDGET = 6ull << 30;  // whole-file buffers (input + output) held at once per pool
constexpr size_t PGZ_MIN_IN = 16ull << 20;   // single-member files from this compressed size decode in parallel
constexpr size_t PGZ_CHUNK_MIN = 2ull << 20;  // compressed bytes per parallel chunk (about 4 per thread)
constexpr size_t PGZ_CHUNK_MAX = 32ull << 20;

struct Member {
    size_t off, len, dst, isize;
};

inline uint32_t le16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
inline uint32_t le32(const uint8_t* p) { return le16(p) | (le16(p + 2) << 16); }

// BGZF: every member carries its own compressed length in a 'BC' extra subfield (BSIZE + 1 bytes)
// and its decoded length in the trailer, so the members of one file are found by walking headers
// alone and decode independently.  True with the member list when the whole file is such members
// (NUL padding at the end allowed); anything else is not BGZF.
bool bgzf_members(const Bytes& in, std::vector<Member>& ms) {
    const size_t n = in.size();
    size_t pos = 0, dst = 0;
    ms.clear();
    while (pos < n) {
        if (in[pos] == 0) {  // trailing NUL padding only
            while (pos < n && in[pos] == 0) ++pos;
            if (pos != n) return false;
            break;
        }
        if (n - pos < 18 || in[pos] != 0x1f || in[pos + 1] != 0x8b || in[pos + 2] != 8 || !(in[pos + 3] & 4))
            return false;
        const size_t xlen = le16(&in[pos + 10]);
        if (n - pos < 12 + xlen) return false;
        size_t bsize = 0;
        const size_t xend = pos + 12 + xlen;
        for (size_t q = pos + 12; q + 4 <= xend;) {
            const size_t slen = le16(&in[q + 2]);
            if (in[q] == 'B' && in[q + 1] == 'C' && slen == 2 && q + 6 <= xend) bsize = le16(&in[q + 4]) + 1;
            q += 4 + slen;
        }
        if (bsize < 12 + xlen + 8 || bsize > BGZF_MAX_BLOCK || n - pos < bsize) return false;
        const size_t isize = le32(&in[pos + bsize - 4]);
        if (isize > BGZF_MAX_BLOCK) return false;
        ms.push_back(Member{pos, bsize, dst, isize});
        dst += isize;
        pos += bsize;
    }
    return !ms.empty();
}

// Take up to `want` idle thread slots of the pool (BGZF helpers); returns how many were taken.
int take_threads(fr_gz* g, int want) {
    std::lock_guard<std::mutex> lk(g->m);
    const int k = std::max(0, std::min(want, g->threads - g->busy));
    g->busy += k;
    return k;
}
void give_threads(fr_gz* g, int k) {
    std::lock_guard<std::mutex> lk(g->m);
    g->busy -= k;
    g->cv.notify_all();
}

// decode BGZF members [k0, k1) in parallel into out (member m lands at m.dst - base): this thread
// plus the pool's idle threads, each with its own decompressor
bool bgzf_decode(fr_gz* g, const Libdeflate* ld, const Bytes& in, const std::vector<Member>& ms,
                 size_t k0, size_t k1, size_t base, uint8_t* out) {
    std::atomic<size_t> next{k0};
    std::atomic<bool> ok{true};
    auto run = [&]() {
        void* d = ld->alloc();
        if (!d) {
            ok = false;
            return;
        }
        for (size_t k; ok && (k = next.fetch_add(1)) < k1;) {
            const Member& m = ms[k];
            size_t used = 0, produced = 0;
            const int r = ld->gzip_ex(d, in.data() + m.off, m.len, out + (m.dst - base), m.isize, &used, &produced);
            if (r != 0 || used != m.len || produced != m.isize) ok = false;
        }
        ld->release(d);
    };
    const int nh = take_threads(g, (int)std::min<size_t>(k1 - k0, 64) - 1);
    std::vector<std::thread> helpers;
    for (int t = 0; t < nh; ++t) helpers.emplace_back(run);
    run();
    for (auto& h : helpers) h.join();
    give_threads(g, nh);
    return ok;
}

// a member's decoded size from its trailer's ISIZE (decoded length mod 2^32): lifted by whole 2^32 steps
// toward 4x the compressed size csize (exact for a single member of up to 4 GiB decoded)
inline uint64_t lift_isize(uint64_t isize, uint64_t csize) {
    const uint64_t want = 4 * csize;
    const uint64_t m = want > isize ? (want - isize + (1ull << 31)) >> 32 : 0;
    return isize + (m << 32);
}

// hold `bytes` of the pool's whole-file budget (false: it does not fit now; stream instead)
bool take_budget(fr_gz* g, size_t bytes) {
    std::lock_guard<std::mutex> lk(g->m);
    if (g->whole_used + bytes > WHOLE_BUDGET) return false;
    g->whole_used += bytes;
    return true;
}
void give_budget(fr_gz* g, size_t bytes) {
    std::lock_guard<std::mutex> lk(g->m);
    g->whole_used -= bytes;
}

// One big gzip member (plus NUL padding) decoded by every idle thread of the pool (fr_pinflate.h):
// true when the file's bytes were queued (or the scan cancelled it); false leaves nothing queued (not a
// single clean member, no budget, or any decode / CRC / ISIZE failure) and the caller decodes the file
// with one thread, whose decoders own the exact error behaviour.
std::atomic<uint64_t> g_parallel_members{0};  // files decoded by inflate_member_parallel (fr_gz_parallel_members)

bool inflate_member_parallel(fr_gz* g, GzFile& f, const Bytes& in) {
    const size_t n = in.size();
    if (n < 32 || in[0] != 0x1f || in[1] != 0x8b || in[2] != 8 || (in[3] & 0xE0)) return false;
    const uint8_t flg = in[3];
    size_t h = 10;
    if (flg & 4) {  // FEXTRA
        if (h + 2 > n) return false;
        h += 2 + le16(&in[h]);
    }
    for (int bit : {8, 16})  // FNAME, FCOMMENT: zero-terminated
        if (flg & bit) {
            while (h < n && in[h]) ++h;
            ++h;
        }
    if (flg & 2) h += 2;  // FHCRC
    if (h + 8 >= n) return false;
    // the trailer's ISIZE (decoded length mod 2^32) lifted by whole 2^32 steps toward 4x the input sizes
    // the output budget: exact for a member of up to 4 GiB decoded, and a 1-GiB member of FASTQ (4-6 GiB
    // decoded) is not sized by its wrapped ISIZE.  The decode stops once its chunks outgrow the budget.
    // (a trailer under n bytes is no trailer: NUL padding ends the file; then 4x the input)
    const size_t lifted = (size_t)lift_isize(le32(&in[n - 4]), n);
    const size_t est = lifted >= n ? lifted : 4 * n;
    if (!take_budget(g, est)) return false;
    struct Hold {
        fr_gz* g;
        size_t b;
        ~Hold() { give_budget(g, b); }
    } hold{g, est};
    // every idle thread (fr_gz_open), or the file's share threads / files_ahead (fr_gz_open_ahead)
    const int share = g->ahead >= g->threads ? g->threads : std::max(2, g->threads / g->ahead);
    const int nh = take_threads(g, share - 1);
    struct Threads {
        fr_gz* g;
        int k;
        ~Threads() { give_threads(g, k); }
    } held{g, nh};
    const int T = nh + 1;
    if (T < 2) return false;
    const size_t chunk = std::min<size_t>(PGZ_CHUNK_MAX, std::max<size_t>(PGZ_CHUNK_MIN, (n - h) / (4 * (size_t)T)));
    std::vector<Bytes> pieces;  // on the way in: buffers for the chunks' output, from the cache
    for (size_t k = 0, K = (n - h + chunk - 1) / chunk; k < K; ++k) pieces.push_back(buf_cache().take(est / K + 1));
    frpz::Result r;
    // the member's trailer (CRC-32, ISIZE), then nothing but NUL padding: one clean member.  The tail
    // test runs inside, right after the stitch (a concatenated multi-member file stops there, before the
    // window, resolve and CRC phases), and the decode gives up once its output passes est.
    bool ok = frpz::inflate_parallel<Bytes>(in.data() + h, n - h, T, chunk, pieces, r, est, true);
    // the decode is done: the helper threads go back to the pool before the queueing below, which
    // waits on the consumer
    give_threads(g, held.k);
    held.k = 0;
    if (ok) {
        const size_t t = h + r.dend;
        ok = t + 8 <= n && le32(&in[t]) == r.crc && le32(&in[t + 4]) == (uint32_t)r.total;
    }
    if (!ok) {
        for (auto& b : pieces) buf_cache().give(std::move(b));
        return false;
    }
    g_parallel_members.fetch_add(1);
    for (auto& b : pieces) {
        std::unique_lock<std::mutex> lk(g->m);
        g->cv.wait(lk, [&] { return f.q.size() < g->depth || f.cancel || g->stop; });
        if (f.cancel || g->stop) break;
        if (!b.empty()) f.q.push_back(std::move(b));
        g->cv.notify_all();
    }
    for (auto& b : pieces)
        if (b.capacity()) buf_cache().give(std::move(b));
    return true;
}

// the libdeflate fast path: true when the whole file was decoded and queued (or the scan cancelled
// it); false leaves nothing queued and the zlib stream takes the file from its start
bool inflate_whole(fr_gz* g, GzFile& f) {
    const Libdeflate* ld = libdeflate();
    if (!ld) return false;
    struct stat sb;
    if (stat(f.path.c_str(), &sb) != 0 || (size_t)sb.st_size > std::max(LD_MAX_IN, BGZF_MAX_IN)) return false;
    const size_t n = (size_t)sb.st_size;
    if (!take_budget(g, n)) return false;
    struct Hold {  // the input's share of the budget, returned on every path
        fr_gz* g;
        size_t b;
        ~Hold() { give_budget(g, b); }
    } hold{g, n};
    struct In {  // the compressed bytes, back to the cache on every path
        Bytes b;
        ~In() { buf_cache().give(std::move(b)); }
    } hin{buf_cache().take(n)};
    Bytes& in = hin.b;
    FILE* fp = fopen(f.path.c_str(), "rb");
    if (!fp) return false;
    const size_t got = n ? fread(in.data(), 1, n, fp) : 0;
    fclose(fp);
    if (got != n) return false;
    std::vector<Member> ms;
    if (bgzf_members(in, ms)) {  // member-parallel, one window of about BGZF_WINDOW output bytes at a time
        size_t k0 = 0;
        while (k0 < ms.size()) {
            size_t k1 = k0;
            while (k1 < ms.size() && ms[k1].dst + ms[k1].isize - ms[k0].dst <= BGZF_WINDOW) ++k1;
            if (k1 == k0) ++k1;
            const size_t base = ms[k0].dst, len = ms[k1 - 1].dst + ms[k1 - 1].isize - base;
            Bytes out;
            {  // wait for room in the file's queue (bounded memory), then decode the window
                std::unique_lock<std::mutex> lk(g->m);
                g->cv.wait(lk, [&] { return f.q.size() < g->depth || f.cancel || g->stop; });
                if (f.cancel || g->stop) return true;
                if (!g->spare.empty()) {
                    out = std::move(g->spare.back());
                    g->spare.pop_back();
                }
            }
            if (out.capacity() < len) out = buf_cache().take(len);
            out.resize(len);
            if (!bgzf_decode(g, ld, in, ms, k0, k1, base, out.data())) {
                if (k0 == 0) return false;  // nothing queued yet: the zlib stream redoes the file
                std::lock_guard<std::mutex> lk(g->m);  // windows already queued: the file is bad
                f.err = "bgzf member failed to decode";
                g->cv.notify_all();
                return true;
            }
            std::lock_guard<std::mutex> lk(g->m);
            if (f.cancel || g->stop) return true;
            if (len) f.q.push_back(std::move(out));
            g->cv.notify_all();
            k0 = k1;
        }
        return true;
    }
    if (n >= PGZ_MIN_IN && g->threads >= 2 && inflate_member_parallel(g, f, in)) return true;
    if (n > LD_MAX_IN || n < 18) return false;
    // the last member's ISIZE (decoded length mod 2^32): a file that will not fit LD_MAX_OUT streams
    const size_t hint = le32(&in[n - 4]);
    const size_t cap = std::min(LD_MAX_OUT, std::max<size_t>({hint + 4096, 4 * n, 1u << 20}));
    if (hint > LD_MAX_OUT || !take_budget(g, cap)) return false;
    Hold hold_out{g, cap};
    void* d = ld->alloc();
    if (!d) return false;
    struct Out {  // unless queued, back to the cache
        Bytes b;
        ~Out() { buf_cache().give(std::move(b)); }
    } hout{buf_cache().take(cap)};
    Bytes& out = hout.b;
    size_t len = 0, pos = 0;
    bool ok = true;
    while (ok) {
        while (pos < n && in[pos] == 0) ++pos;  // NUL padding between members
        if (pos == n) break;
        if (in[pos] != 0x1f) {
            ok = false;
            break;
        }
        for (;;) {
            size_t used = 0, produced = 0;
            const int r =
                ld->gzip_ex(d, in.data() + pos, n - pos, out.data() + len, out.size() - len, &used, &produced);
            if (r == 0) {  // LIBDEFLATE_SUCCESS
                len += produced;
                pos += used;
                break;
            }
            // LIBDEFLATE_INSUFFICIENT_SPACE (a multi-member file: ISIZE covered only its last member):
            // a bigger buffer within LD_MAX_OUT and the pool's budget, else the zlib stream
            const size_t more = std::min(LD_MAX_OUT, 2 * out.size()) - out.size();
            if (r != 3 || more == 0 || !take_budget(g, more)) {
                ok = false;
                break;
            }
            hold_out.b += more;
            out.resize(out.size() + more);
        }
    }
    ld->release(d);
    if (!ok) return false;
    out.resize(len);
    std::unique_lock<std::mutex> lk(g->m);
    if (f.cancel || g->stop) return true;
    if (len) f.q.push_back(std::move(out));
    g->cv.notify_all();
    return true;
}

// inflate one file into g->files[i].q (blocks of g->block bytes); returns "" or an error text
std::string inflate_stream(fr_gz* g, int i) {
    GzFile& f = g->files[i];
    if (inflate_whole(g, f)) {
        std::lock_guard<std::mutex> lk(g->m);
        return f.err;
    }
    FILE* fp = fopen(f.path.c_str(), "rb");
    if (!fp) return "cannot open " + f.path;
    Bytes in(4u << 20);
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) {
        fclose(fp);
        return "inflateInit2 failed";
    }
    auto fresh = [&]() {
        std::lock_guard<std::mutex> lk(g->m);
        if (g->spare.empty()) return buf_cache().take(g->block);
        Bytes v = std::move(g->spare.back());
        g->spare.pop_back();
        v.resize(g->block);
        return v;
    };
    Bytes out = fresh();
    size_t have = 0;  // bytes of `out` filled
    std::string err;
    bool in_member = false;  // a member has started and not ended
    bool eof = false;
    auto push = [&](bool last) -> bool {  // queue `out` (partial only at the end); false: cancelled
        if (!have && !last) return true;
        std::unique_lock<std::mutex> lk(g->m);
        g->cv.wait(lk, [&] { return f.q.size() < g->depth || f.cancel || g->stop; });
        if (f.cancel || g->stop) return false;
        if (have) {
            out.resize(have);
            f.q.push_back(std::move(out));
            have = 0;
            g->cv.notify_all();
            lk.unlock();
            if (!last) out = fresh();
            return true;
        }
        g->cv.notify_all();
        return true;
    };
    for (;;) {
        if (zs.avail_in == 0 && !eof) {
            const size_t n = fread(in.data(), 1, in.size(), fp);
            if (n == 0) eof = true;
            zs.next_in = in.data();
            zs.avail_in = (uInt)n;
        }
        if (!in_member) {  // between members: NUL padding, then a member or the end of the file
            while (zs.avail_in && *zs.next_in == 0) {
                ++zs.next_in;
                --zs.avail_in;
            }
            if (zs.avail_in == 0) {
                if (eof) break;
                continue;
            }
            if (*zs.next_in != 0x1f) {
                err = "not a gzip member";
                break;
            }
            in_member = true;
        }
        if (zs.avail_in == 0 && eof) {
            err = "compressed file ended before the end-of-stream marker was reached";
            break;
        }
        zs.next_out = out.data() + have;
        zs.avail_out = (uInt)(out.size() - have);
        const int rc = inflate(&zs, Z_NO_FLUSH);
        have = out.size() - zs.avail_out;
        if (rc == Z_STREAM_END) {
            in_member = false;
            if (inflateReset(&zs) != Z_OK) {
                err = "inflateReset failed";
                break;
            }
        } else if (rc == Z_BUF_ERROR) {
            if (zs.avail_in == 0 && eof) {
                err = "compressed file ended before the end-of-stream marker was reached";
                break;
            }
        } else if (rc != Z_OK) {
            err = std::string("inflate: ") + (zs.msg ? zs.msg : "error");
            break;
        }
        if (have == out.size() && !push(false)) break;
        {
            std::lock_guard<std::mutex> lk(g->m);
            if (f.cancel || g->stop) break;
        }
    }
    inflateEnd(&zs);
    fclose(fp);
    if (err.empty()) push(true);
    return err;
}

// a failed allocation (a huge or corrupt file) ends that file with an error, which the host replays
// through Python's gzip for the reference's exception, instead of terminating the process
std::string inflate_file(fr_gz* g, int i) {
    try {
        return inflate_stream(g, i);
    } catch (const std::bad_alloc&) {
        return "out of memory while inflating";
    } catch (const std::exception& e) {
        return std::string("inflate: ") + e.what();
    }
}

void worker(fr_gz* g) {
    for (;;) {
        int i;
        {
            std::unique_lock<std::mutex> lk(g->m);
            g->cv.wait(lk, [&] {
                return g->stop || (g->next < (int)g->files.size() && g->next < g->consume + g->ahead &&
                                   g->busy < g->threads);
            });
            if (g->stop) return;
            i = g->next++;
            g->busy++;
        }
        std::string err = inflate_file(g, i);
        std::lock_guard<std::mutex> lk(g->m);
        g->busy--;
        g->files[i].err = err;
        g->files[i].done = true;
        g->cv.notify_all();
    }
}

}  // namespace

extern "C" {

fr_gz* fr_gz_open_ahead(const char* const* paths, int n_files, int threads, int files_ahead) {
    fr_gz* g = new fr_gz();
    g->files.resize(n_files > 0 ? n_files : 0);
    for (int i = 0; i < n_files; ++i) g->files[i].path = paths[i];
    g->threads = threads < 1 ? 1 : threads;
    g->ahead = std::max(1, std::min(files_ahead, g->threads));
    // files inflating ahead of the consumer may buffer up to 2 GiB of decoded blocks in all, so a
    // worker is not parked behind a short queue while the consumer is still on an earlier file
    g->depth = std::max<size_t>(3, (2ull << 30) / ((size_t)g->ahead * g->block));
    const int nw = std::min(g->ahead, std::max(n_files, 1));
    for (int k = 0; k < nw; ++k) g->workers.emplace_back(worker, g);
    return g;
}

fr_gz* fr_gz_open(const char* const* paths, int n_files, int threads) {
    return fr_gz_open_ahead(paths, n_files, threads, threads);
}

const char* fr_gz_error(const fr_gz* g) { return g ? g->err.c_str() : "null inflate pool"; }

int fr_gz_feed(fr_gz* g, int i, fr_ctx* ctx) {
    if (i < 0 || i >= (int)g->files.size()) {
        g->err = "fr_gz_feed: no such file";
        return FR_ERR_INVALID;
    }
    GzFile& f = g->files[i];
    {
        std::lock_guard<std::mutex> lk(g->m);
        g->consume = i;
        g->cv.notify_all();
    }
    for (;;) {
        Bytes b;
        {
            std::unique_lock<std::mutex> lk(g->m);
            g->cv.wait(lk, [&] { return !f.q.empty() || f.done; });
            if (f.q.empty()) {  // done
                if (!f.err.empty()) {
                    g->err = f.path + ": " + f.err;
                    return FR_ERR_IO;
                }
                return FR_OK;
            }
            b = std::move(f.q.front());
            f.q.pop_front();
            g->cv.notify_all();
        }
        const int rc = fr_feed(ctx, b.data(), b.size());
        {
            std::lock_guard<std::mutex> lk(g->m);
            keep_spare(g, b);
        }
        if (b.capacity()) buf_cache().give(std::move(b));
        if (rc != FR_OK) {  // the -s sample is complete, or a feed error: this file is finished
            std::lock_guard<std::mutex> lk(g->m);
            f.cancel = true;
            f.q.clear();
            g->cv.notify_all();
            if (rc != FR_SAMPLE_DONE) g->err = fr_last_error(ctx);
            return rc;
        }
    }
}

int fr_gz_next(fr_gz* g, int i, const uint8_t** data, uint64_t* len) {
    *data = nullptr;
    *len = 0;
    if (i < 0 || i >= (int)g->files.size()) {
        g->err = "fr_gz_next: no such file";
        return FR_ERR_INVALID;
    }
    GzFile& f = g->files[i];
    std::unique_lock<std::mutex> lk(g->m);
    if (g->held.capacity()) {  // the block handed out last is the caller's no longer
        if (!keep_spare(g, g->held)) buf_cache().give(std::move(g->held));
        g->held = Bytes();
    }
    // readers of several files at once (demux: R1 and R2 in lockstep) keep the furthest one
    g->consume = std::max(g->consume, i);
    g->cv.notify_all();
    g->cv.wait(lk, [&] { return !f.q.empty() || f.done; });
    if (f.q.empty()) {  // done
        if (!f.err.empty()) {
            g->err = f.path + ": " + f.err;
            return FR_ERR_IO;
        }
        return FR_OK;
    }
    g->held = std::move(f.q.front());
    f.q.pop_front();
    g->cv.notify_all();
    *data = g->held.data();
    *len = g->held.size();
    return FR_OK;
}

// ---- record-aligned parts of one file (multi-GPU scans of fewer files than GPUs) ----------------
// Part j of k of a decoded stream covers [b_j, b_{j+1}): b_0 = 0, b_k = the end and, for 0 < j < k,
// b_j is the first record start at or after j * hint / k, a record start being a line start whose
// line index from the file start is 0 mod 4 under the reference's universal newlines (frender.py:159:
// '\n', '\r\n' and a lone '\r' each end a line).  `hint` (fr_gz_size_hint) depends on the file alone,
// so every rank that owns a part of the file cuts it the same way.

}  // extern "C"

namespace {

struct Cutter {
    uint64_t target[2];  // the part's two cut targets (b_part, b_part+1)
    uint64_t cut[2];
    int found = 0;       // cuts found so far (in order)
    uint64_t pos = 0;    // bytes consumed
    uint64_t lines = 0;  // terminators in [0, pos), except a '\r' at pos - 1 still pending
    bool pend_cr = false;

    // a line start at p with line index L
    void line_start(uint64_t p, uint64_t L) {
        while (found < 2 && p >= target[found] && (L & 3u) == 0) cut[found++] = p;
    }
    // consume [pos, pos + n) of the stream; returns when both cuts are found or the block is used up
    void consume(const uint8_t* b, size_t n) {
        size_t i = 0;
        while (i < n && found < 2) {
            if (!pend_cr) {  // fast part: '\n' only, no cut due before the block's byte t - 1
                const uint64_t t = target[found];
                const size_t fast_end = t > pos + 1 ? (size_t)std::min<uint64_t>(n, t - 1 - pos + i) : i;
                if (fast_end > i && !std::memchr(b + i, '\r', fast_end - i)) {
                    lines += (uint64_t)std::count(b + i, b + fast_end, (uint8_t)'\n');
                    pos += fast_end - i;
                    i = fast_end;
                    continue;
                }
            }
            const uint8_t c = b[i];
            if (pend_cr) {  // byte pos - 1 was '\r': a terminator unless this byte is '\n'
                pend_cr = false;
                if (c != '\n') {
                    ++lines;
                    line_start(pos, lines);
                }
            }
            if (c == '\n') {
                ++lines;
                line_start(pos + 1, lines);
            } else if (c == '\r') {
                pend_cr = true;
            }
            ++pos;
            ++i;
        }
    }
    void finish() {  // the end of the stream: a pending '\r' ends a line; cuts not found are the end
        if (pend_cr) {
            pend_cr = false;
            ++lines;
            line_start(pos, lines);
        }
        while (found < 2) cut[found++] = pos;
    }
};

}  // namespace

extern "C" {

uint64_t fr_gz_size_hint(const char* path) {
    FILE* fp = fopen(path, "rb");
    if (!fp) return 0;
    struct stat sb;
    if (fstat(fileno(fp), &sb) != 0 || sb.st_size < 18) {
        fclose(fp);
        return 0;
    }
    const uint64_t csize = (uint64_t)sb.st_size;
    // BGZF: the members' ISIZE trailers sum to the decoded size exactly (headers only are read)
    uint64_t pos = 0, sum = 0;
    bool bgzf = true;
    uint8_t h[18];
    while (bgzf && pos < csize) {
        if (fseek(fp, (long)pos, SEEK_SET) != 0 || fread(h, 1, 18, fp) != 18) {
            bgzf = false;
            break;
        }
        if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4) || le16(h + 10) != 6 || h[12] != 'B' ||
            h[13] != 'C' || le16(h + 14) != 2) {
            bgzf = false;
            break;
        }
        const uint64_t bsize = le16(h + 16) + 1u;
        uint8_t t[4];
        if (bsize < 26 || pos + bsize > csize || fseek(fp, (long)(pos + bsize - 4), SEEK_SET) != 0 ||
            fread(t, 1, 4, fp) != 4) {
            bgzf = false;
            break;
        }
        sum += le32(t);
        pos += bsize;
    }
    if (bgzf && pos == csize) {
        fclose(fp);
        return sum;
    }
    // otherwise the last member's ISIZE (decoded length mod 2^32), lifted by whole 2^32 steps toward
    // 4x the compressed size (exact for a single-member file of up to 4 GiB decoded)
    uint8_t t[4];
    const bool ok = fseek(fp, -4, SEEK_END) == 0 && fread(t, 1, 4, fp) == 4;
    fclose(fp);
    if (!ok) return 4 * csize;
    return lift_isize(le32(t), csize);
}

int fr_gz_part_bounds(const char* path, int nparts, uint64_t hint, uint64_t* bounds) {
    if (nparts < 1 || !bounds) return FR_ERR_INVALID;
    const char* paths[1] = {path};
    fr_gz* g = fr_gz_open(paths, 1, 1);
    bounds[0] = 0;
    int rc = FR_OK;
    // one pass per cut pair keeps the cutter identical to fr_gz_feed_part's (targets j and j + 1)
    std::vector<Cutter> cs(nparts);
    for (int j = 0; j < nparts; ++j) {
        Cutter& cu = cs[j];
        cu.target[0] = j == 0 ? 0 : (uint64_t)((unsigned __int128)hint * (unsigned)j / (unsigned)nparts);
        cu.target[1] = j + 1 == nparts ? ~0ull : (uint64_t)((unsigned __int128)hint * (unsigned)(j + 1) / (unsigned)nparts);
        if (cu.target[1] < cu.target[0]) cu.target[1] = cu.target[0];
        if (j == 0) cu.cut[cu.found++] = 0;
    }
    GzFile& f = g->files[0];
    {
        std::lock_guard<std::mutex> lk(g->m);
        g->consume = 0;
        g->cv.notify_all();
    }
    for (;;) {
        Bytes b;
        {
            std::unique_lock<std::mutex> lk(g->m);
            g->cv.wait(lk, [&] { return !f.q.empty() || f.done; });
            if (f.q.empty()) {
                if (!f.err.empty()) rc = FR_ERR_IO;
                break;
            }
            b = std::move(f.q.front());
            f.q.pop_front();
            g->cv.notify_all();
        }
        for (Cutter& cu : cs) cu.consume(b.data(), b.size());
    }
    for (int j = 0; j < nparts; ++j) {
        cs[j].finish();
        bounds[j] = cs[j].cut[0];
        if (j + 1 == nparts) bounds[nparts] = cs[j].cut[1];
    }
    fr_gz_close(g);
    return rc;
}

int fr_gz_feed_part(fr_gz* g, int i, fr_ctx* ctx, int64_t file_index, int part, int nparts, uint64_t hint,
                    uint64_t* byte_base) {
    if (i < 0 || i >= (int)g->files.size() || nparts < 1 || part < 0 || part >= nparts) {
        g->err = "fr_gz_feed_part: bad arguments";
        return FR_ERR_INVALID;
    }
    GzFile& f = g->files[i];
    {
        std::lock_guard<std::mutex> lk(g->m);
        g->consume = i;
        g->cv.notify_all();
    }
    Cutter cu;
    cu.target[0] = part == 0 ? 0 : (uint64_t)((unsigned __int128)hint * (unsigned)part / (unsigned)nparts);
    cu.target[1] = part + 1 == nparts ? ~0ull : (uint64_t)((unsigned __int128)hint * (unsigned)(part + 1) / (unsigned)nparts);
    if (cu.target[1] < cu.target[0]) cu.target[1] = cu.target[0];
    if (part == 0) cu.cut[cu.found++] = 0;  // b_0 = 0 (the file's first byte is a record start)
    bool begun = false;
    int rc = FR_OK;
    auto begin = [&]() -> int {
        begun = true;
        if (byte_base) *byte_base = cu.cut[0];
        const int r = fr_begin_file_at(ctx, file_index, cu.cut[0], 0);
        if (r != FR_OK) g->err = fr_last_error(ctx);
        return r;
    };
    auto finish_file = [&](bool cancel) {
        std::lock_guard<std::mutex> lk(g->m);
        if (cancel) {
            f.cancel = true;
            f.q.clear();
        }
        g->cv.notify_all();
    };
    for (;;) {
        Bytes b;
        bool end = false;
        {
            std::unique_lock<std::mutex> lk(g->m);
            g->cv.wait(lk, [&] { return !f.q.empty() || f.done; });
            if (f.q.empty()) {
                if (!f.err.empty()) {
                    g->err = f.path + ": " + f.err;
                    return FR_ERR_IO;
                }
                end = true;
            } else {
                b = std::move(f.q.front());
                f.q.pop_front();
                g->cv.notify_all();
            }
        }
        if (end) {
            cu.finish();
            if (!begun && (rc = begin()) != FR_OK) return rc;
            return FR_OK;
        }
        const uint64_t b0 = cu.pos;
        cu.consume(b.data(), b.size());
        const uint64_t e0 = cu.pos;  // bytes [b0, e0) of the block were scanned
        if (!begun && cu.found >= 1 && (rc = begin()) != FR_OK) {
            finish_file(true);
            return rc;
        }
        if (begun) {  // the part's bytes of this block: [max(b_part, b0), min(b_part+1, block end))
            const uint64_t lo = std::max(cu.cut[0], b0);
            const uint64_t hi = std::min(cu.found >= 2 ? cu.cut[1] : b0 + b.size(), b0 + b.size());
            if (hi > lo) rc = fr_feed(ctx, b.data() + (lo - b0), hi - lo);
            if (rc != FR_OK) {
                g->err = fr_last_error(ctx);
                finish_file(true);
                return rc;
            }
        }
        (void)e0;
        {
            std::lock_guard<std::mutex> lk(g->m);
            keep_spare(g, b);
        }
        if (b.capacity()) buf_cache().give(std::move(b));
        if (cu.found >= 2) {  // the part is complete: the rest of the file is another rank's
            finish_file(true);
            return FR_OK;
        }
    }
}

}  // extern "C"

// ---- BGZF record parts without a prefix inflate (multi-GPU scans of fewer files than GPUs) -----
// A BGZF file's members carry their compressed size (header) and decoded size (trailer), so the
// decoded offset of every member is known from the headers alone and a rank can decode its own part
// of the file without inflating what precedes it.  The part's targets are member starts: M_j = the
// decoded offset of the first member starting at or after j * total / k (M_0 = 0, M_k = total).
// Record cuts still need the exact line count before them, so the rank first decodes its members
// [M_j, M_j+1) (plus the member before, for the byte before M_j, and the members after M_j+1 up to the
// next record start), counts the line terminators whose terminating byte lies in [M_j, M_j+1) (host
// side), the ranks exchange those counts (frender_amd/dist.py: one all-reduce), and the part is
// [b_j, b_j+1): b_j = the first record start at or after M_j under the lines before M_j.  Each rank
// inflates its part plus at most a member or two on either side.  Single-member streams cannot be
// entered mid-stream (a deflate block's start is unknown without decoding what precedes it):
// fr_gz_feed_part keeps inflating those from their start.

namespace {

// the member table of a BGZF file from its headers and trailers alone; false when the file is not
// wholly BGZF members (NUL padding at the end allowed) or cannot be read
bool bgzf_table(FILE* fp, uint64_t csize, std::vector<Member>& ms) {
    ms.clear();
    uint64_t pos = 0, dst = 0;
    uint8_t h[18];
    while (pos < csize) {
        if (fseek(fp, (long)pos, SEEK_SET) != 0 || fread(h, 1, 1, fp) != 1) return false;
        if (h[0] == 0) {  // trailing NUL padding only
            Bytes rest(csize - pos - 1);
            if (!rest.empty() && fread(rest.data(), 1, rest.size(), fp) != rest.size()) return false;
            for (uint8_t c : rest)
                if (c) return false;
            break;
        }
        if (csize - pos < 26 || fseek(fp, (long)pos, SEEK_SET) != 0 || fread(h, 1, 18, fp) != 18) return false;
        if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4) || le16(h + 10) != 6 || h[12] != 'B' ||
            h[13] != 'C' || le16(h + 14) != 2)
            return false;
        const uint64_t bsize = le16(h + 16) + 1u;
        uint8_t t[4];
        if (bsize < 26 || pos + bsize > csize || fseek(fp, (long)(pos + bsize - 4), SEEK_SET) != 0 ||
            fread(t, 1, 4, fp) != 4)
            return false;
        const uint64_t isize = le32(t);
        if (isize > BGZF_MAX_BLOCK) return false;
        ms.push_back(Member{(size_t)pos, (size_t)bsize, (size_t)dst, (size_t)isize});
        dst += isize;
        pos += bsize;
    }
    return !ms.empty();
}

// decode members [k0, k1) of an open BGZF file into out (member m at m.dst - ms[k0].dst): the
// compressed bytes of the range are read once, then libdeflate (this thread plus up to threads - 1
// helpers) or zlib per member
bool bgzf_decode_range(FILE* fp, const std::vector<Member>& ms, size_t k0, size_t k1, int threads,
                       Bytes& out) {
    out.clear();
    if (k0 >= k1) return true;
    const size_t c0 = ms[k0].off, c1 = ms[k1 - 1].off + ms[k1 - 1].len;
    Bytes in(c1 - c0);
    if (fseek(fp, (long)c0, SEEK_SET) != 0 || fread(in.data(), 1, in.size(), fp) != in.size()) return false;
    const size_t base = ms[k0].dst;
    out.resize(ms[k1 - 1].dst + ms[k1 - 1].isize - base);
    const Libdeflate* ld = libdeflate();
    std::atomic<size_t> next{k0};
    std::atomic<bool> ok{true};
    auto run = [&]() {
        void* d = ld ? ld->alloc() : nullptr;
        if (ld && !d) {
            ok = false;
            return;
        }
        for (size_t k; ok && (k = next.fetch_add(1)) < k1;) {
            const Member& m = ms[k];
            const uint8_t* src = in.data() + (m.off - c0);
            uint8_t* dst = out.data() + (m.dst - base);
            if (ld) {
                size_t used = 0, produced = 0;
                const int r = ld->gzip_ex(d, src, m.len, dst, m.isize, &used, &produced);
                if (r != 0 || used != m.len || produced != m.isize) ok = false;
            } else {  // zlib, one gzip member (CRC and length checked by inflate)
                z_stream zs;
                std::memset(&zs, 0, sizeof(zs));
                if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) {
                    ok = false;
                    continue;
                }
                zs.next_in = const_cast<uint8_t*>(src);
                zs.avail_in = (uInt)m.len;
                zs.next_out = dst;
                zs.avail_out = (uInt)m.isize;
                const int r = inflate(&zs, Z_FINISH);
                if (r != Z_STREAM_END || zs.avail_in != 0 || zs.total_out != m.isize) ok = false;
                inflateEnd(&zs);
            }
        }
        if (d) ld->release(d);
    };
    const int nh = (int)std::min<size_t>(std::max(threads, 1) - 1, k1 - k0 - 1);
    std::vector<std::thread> helpers;
    for (int t = 0; t < nh; ++t) helpers.emplace_back(run);
    run();
    for (auto& h : helpers) h.join();
    return ok;
}

// first member whose decoded start is at or after x (ms.size() when none)
size_t member_at_or_after(const std::vector<Member>& ms, uint64_t x) {
    size_t lo = 0, hi = ms.size();
    while (lo < hi) {
        const size_t mid = (lo + hi) / 2;
        if (ms[mid].dst < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

}  // namespace

struct fr_gz_part {
    FILE* fp = nullptr;
    std::vector<Member> ms;
    uint64_t total = 0;         // decoded size of the file
    uint64_t M0 = 0, M1 = 0;    // the part's member range [M0, M1) (decoded offsets)
    size_t kn = 0;              // first member not decoded yet (past data's end)
    uint64_t dbase = 0;         // decoded offset of data[0]
    Bytes data;  // decoded bytes [dbase, dbase + data.size())
    uint64_t lines = 0;         // terminators whose terminating byte lies in [M0, M1)
    uint64_t inflated = 0;      // decoded bytes produced for this part
    int threads = 1;
    std::string err;
};

namespace {

// decode further members until data reaches at least decoded offset `want` (or the file's end)
bool part_extend(fr_gz_part* p, uint64_t want) {
    while (p->dbase + p->data.size() < std::min(want, p->total) && p->kn < p->ms.size()) {
        size_t k1 = p->kn + 1;
        while (k1 < p->ms.size() && k1 - p->kn < 16) ++k1;  // a few members at a time
        Bytes more;
        if (!bgzf_decode_range(p->fp, p->ms, p->kn, k1, p->threads, more)) return false;
        p->inflated += more.size();
        p->data.insert(p->data.end(), more.begin(), more.end());
        p->kn = k1;
    }
    return true;
}

// byte at decoded offset x (-1 past the file's end); data must cover it.  -2 when it does not (an
// internal error the caller reports as FR_ERR_IO: callers extend first, so it is never expected)
inline int part_byte(const fr_gz_part* p, uint64_t x) {
    if (x >= p->total) return -1;
    if (x < p->dbase || x - p->dbase >= p->data.size()) return -2;
    return p->data[x - p->dbase];
}

// the first record start at or after x, given L = terminators in [0, x) counted with x's own
// universal-newline convention (a '\r' at x - 1 counts when byte x is not '\n'); p->total when none
bool part_cut(fr_gz_part* p, uint64_t x, uint64_t L, uint64_t& cut) {
    if (x == 0) {
        cut = 0;
        return true;
    }
    if (!part_extend(p, x + 1)) return false;
    const int prev = part_byte(p, x - 1);
    const int cur = part_byte(p, x);
    if (prev == -2 || cur == -2) return false;
    bool start = prev == '\n' || (prev == '\r' && cur != '\n');
    uint64_t q = x, lines = L;
    for (;;) {
        if (start && (lines & 3u) == 0) {
            cut = q;
            return true;
        }
        if (q >= p->total) {
            cut = p->total;
            return true;
        }
        if (q + 2 > p->dbase + p->data.size() && !part_extend(p, q + 2 + (1u << 16))) return false;
        const int c = part_byte(p, q), nx = part_byte(p, q + 1);
        if (c == -2 || nx == -2) return false;
        start = false;
        if (c == '\n' || (c == '\r' && nx != '\n')) {
            ++lines;
            start = true;
        }
        ++q;
    }
}

}  // namespace

extern "C" {

int fr_gz_part_open(const char* path, int part, int nparts, int threads, fr_gz_part** out, int* is_bgzf,
                    uint64_t* lines, uint64_t* inflated) {
    *out = nullptr;
    *is_bgzf = 0;
    if (!path || nparts < 1 || part < 0 || part >= nparts) return FR_ERR_INVALID;
    FILE* fp = fopen(path, "rb");
    if (!fp) return FR_ERR_IO;
    struct stat sb;
    std::vector<Member> ms;
    if (fstat(fileno(fp), &sb) != 0 || !bgzf_table(fp, (uint64_t)sb.st_size, ms)) {
        fclose(fp);
        return FR_OK;  // not BGZF: the caller cuts with fr_gz_feed_part
    }
    fr_gz_part* p = nullptr;
    try {
        p = new fr_gz_part();
        p->fp = fp;
        p->ms = std::move(ms);
        p->threads = std::max(threads, 1);
        const Member& last = p->ms.back();
        p->total = last.dst + last.isize;
        auto target = [&](int j) -> uint64_t {
            if (j <= 0) return 0;
            if (j >= nparts) return p->total;
            const uint64_t t = (uint64_t)((unsigned __int128)p->total * (unsigned)j / (unsigned)nparts);
            const size_t k = member_at_or_after(p->ms, t);
            return k < p->ms.size() ? p->ms[k].dst : p->total;
        };
        p->M0 = target(part);
        p->M1 = std::max(target(part + 1), p->M0);
        // decode from the member before M0 (the byte before the range) through the member at M1
        size_t k0 = member_at_or_after(p->ms, p->M0);
        while (k0 > 0 && part > 0 && (k0 >= p->ms.size() || p->ms[k0].dst >= p->M0)) --k0;  // holds byte M0 - 1
        size_t k1 = member_at_or_after(p->ms, p->M1);
        k1 = std::min(k1 + 1, p->ms.size());
        if (k0 < p->ms.size()) {
            p->dbase = p->ms[k0].dst;
            if (!bgzf_decode_range(fp, p->ms, k0, std::max(k1, k0 + 1), p->threads, p->data)) {
                delete p;
                fclose(fp);
                return FR_ERR_IO;
            }
            p->kn = std::max(k1, k0 + 1);
        } else {
            p->dbase = p->total;
            p->kn = p->ms.size();
        }
        p->inflated = p->data.size();
        // the byte at M1 must be decoded too (a '\r' at M1 - 1 looks at it): the member found at M1 can
        // be empty (an EOF block left mid-file by `cat` of BGZF files), so extend past it when needed
        if (p->M1 < p->total && !part_extend(p, p->M1 + 1)) {
            delete p;
            fclose(fp);
            return FR_ERR_IO;
        }
        // terminators with their terminating byte in [M0, M1): every '\n', and every '\r' not followed
        // by '\n' (the byte after M1 - 1 is decoded above)
        uint64_t n = 0;
        if (p->M1 > p->M0) {
            const uint8_t* b = p->data.data() + (p->M0 - p->dbase);
            const size_t len = p->M1 - p->M0;
            n = (uint64_t)std::count(b, b + len, (uint8_t)'\n');
            for (const uint8_t* r = (const uint8_t*)std::memchr(b, '\r', len); r;
                 r = (const uint8_t*)std::memchr(r + 1, '\r', (size_t)(b + len - r - 1)))
                if (part_byte(p, p->M0 + (uint64_t)(r - b) + 1) != '\n') ++n;
        }
        p->lines = n;
    } catch (const std::bad_alloc&) {
        if (p) {
            p->fp = nullptr;
            delete p;
        }
        fclose(fp);
        return FR_ERR_IO;
    }
    *out = p;
    *is_bgzf = 1;
    if (lines) *lines = p->lines;
    if (inflated) *inflated = p->inflated;
    return FR_OK;
}

int fr_gz_part_data(fr_gz_part* p, uint64_t lines_before, const uint8_t** data, uint64_t* len, uint64_t* byte_base,
                    uint64_t* inflated) {
    *data = nullptr;
    *len = 0;
    uint64_t b0 = 0, b1 = 0;
    try {
        if (!part_cut(p, p->M0, lines_before, b0) || !part_cut(p, p->M1, lines_before + p->lines, b1)) {
            p->err = "bgzf member failed to decode";
            return FR_ERR_IO;
        }
        if (b1 < b0) b1 = b0;
        if (!part_extend(p, b1)) {
            p->err = "bgzf member failed to decode";
            return FR_ERR_IO;
        }
    } catch (const std::bad_alloc&) {
        p->err = "out of memory while inflating";
        return FR_ERR_IO;
    }
    if (b1 > b0) {
        *data = p->data.data() + (b0 - p->dbase);
        *len = b1 - b0;
    }
    if (byte_base) *byte_base = b0;
    if (inflated) *inflated = p->inflated;
    return FR_OK;
}

int fr_gz_part_feed(fr_gz_part* p, fr_ctx* ctx, int64_t file_index, uint64_t lines_before, uint64_t* byte_base) {
    const uint8_t* d = nullptr;
    uint64_t n = 0, b0 = 0;
    int rc = fr_gz_part_data(p, lines_before, &d, &n, &b0, nullptr);
    if (rc != FR_OK) return rc;
    if (byte_base) *byte_base = b0;
    rc = fr_begin_file_at(ctx, file_index, b0, 0);
    if (rc == FR_OK && n) rc = fr_feed(ctx, d, n);
    if (rc != FR_OK) p->err = fr_last_error(ctx);
    return rc;
}

const char* fr_gz_part_error(const fr_gz_part* p) { return p ? p->err.c_str() : "null part"; }

void fr_gz_part_close(fr_gz_part* p) {
    if (!p) return;
    if (p->fp) fclose(p->fp);
    delete p;
}

}  // extern "C"

extern "C" {

void fr_gz_trim(void) { buf_cache().trim(); }

uint64_t fr_gz_parallel_members(void) { return g_parallel_members.load(); }

void fr_gz_close(fr_gz* g) {
    if (!g) return;
    {
        std::lock_guard<std::mutex> lk(g->m);
        g->stop = true;
        g->cv.notify_all();
    }
    for (auto& t : g->workers) t.join();
    delete g;
}

}  // extern "C"
