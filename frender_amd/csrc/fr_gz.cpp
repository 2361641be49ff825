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
// with dlopen, so the library is optional), a file of up to 256 MiB compressed is decompressed
// whole, member by member, and queued in one piece.  Anything unusual -- bytes after a member that
// are neither NUL padding nor a new member, a member libdeflate rejects, more than 1 GiB of output --
// falls back to the zlib stream, which owns the exact rules and errors above.
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
#include <string>
#include <thread>
#include <vector>

#include "../../include/frender_amd.h"

namespace {

struct GzFile {
    std::string path;
    std::deque<std::vector<uint8_t>> q;
    bool done = false;
    bool cancel = false;
    std::string err;
};

}  // namespace

struct fr_gz {
    std::vector<GzFile> files;
    int threads = 1;
    size_t block = 16u << 20;
    size_t depth = 3;  // blocks queued per file (set by fr_gz_open)
    std::mutex m;
    std::condition_variable cv;
    std::vector<std::thread> workers;
    std::vector<std::vector<uint8_t>> spare;  // consumed blocks for reuse (no page faults per block)
    int next = 0;     // next file a worker starts
    int consume = 0;  // file the consumer reads (workers stay within [consume, consume + threads))
    bool stop = false;
    std::string err;
};

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

struct Member {
    size_t off, len, dst, isize;
};

inline uint32_t le16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
inline uint32_t le32(const uint8_t* p) { return le16(p) | (le16(p + 2) << 16); }

// BGZF: every member carries its own compressed length in a 'BC' extra subfield (BSIZE + 1 bytes)
// and its decoded length in the trailer, so the members of one file are found by walking headers
// alone and decode independently.  True with the member list when the whole file is such members
// (NUL padding at the end allowed); anything else is not BGZF.
bool bgzf_members(const std::vector<uint8_t>& in, std::vector<Member>& ms) {
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
        for (size_t q = pos + 12; q + 4 <= pos + 12 + xlen;) {
            const size_t slen = le16(&in[q + 2]);
            if (in[q] == 'B' && in[q + 1] == 'C' && slen == 2) bsize = le16(&in[q + 4]) + 1;
            q += 4 + slen;
        }
        if (bsize < 12 + xlen + 8 || n - pos < bsize) return false;
        const size_t isize = le32(&in[pos + bsize - 4]);
        ms.push_back(Member{pos, bsize, dst, isize});
        dst += isize;
        pos += bsize;
    }
    return !ms.empty();
}

// decode BGZF members in parallel (`threads` helpers, each with its own decompressor) into out
bool bgzf_decode(const Libdeflate* ld, const std::vector<uint8_t>& in, const std::vector<Member>& ms,
                 std::vector<uint8_t>& out, int threads) {
    std::atomic<size_t> next{0};
    std::atomic<bool> ok{true};
    auto run = [&]() {
        void* d = ld->alloc();
        if (!d) {
            ok = false;
            return;
        }
        for (size_t k; ok && (k = next.fetch_add(1)) < ms.size();) {
            const Member& m = ms[k];
            size_t used = 0, produced = 0;
            const int r = ld->gzip_ex(d, in.data() + m.off, m.len, out.data() + m.dst, m.isize, &used, &produced);
            if (r != 0 || used != m.len || produced != m.isize) ok = false;
        }
        ld->release(d);
    };
    std::vector<std::thread> helpers;
    for (int t = 1; t < threads; ++t) helpers.emplace_back(run);
    run();
    for (auto& h : helpers) h.join();
    return ok;
}

// the libdeflate fast path: true when the whole file was decoded and queued (or the scan cancelled
// it); false leaves nothing queued and the zlib stream takes the file from its start
bool inflate_whole(fr_gz* g, GzFile& f) {
    const Libdeflate* ld = libdeflate();
    if (!ld) return false;
    struct stat sb;
    if (stat(f.path.c_str(), &sb) != 0 || (size_t)sb.st_size > std::max(LD_MAX_IN, BGZF_MAX_IN)) return false;
    const size_t n = (size_t)sb.st_size;
    std::vector<uint8_t> in(n);
    FILE* fp = fopen(f.path.c_str(), "rb");
    if (!fp) return false;
    const size_t got = n ? fread(in.data(), 1, n, fp) : 0;
    fclose(fp);
    if (got != n) return false;
    std::vector<Member> ms;
    if (bgzf_members(in, ms)) {  // members split across the pool's thread count
        std::vector<uint8_t> out(ms.back().dst + ms.back().isize);
        if (!bgzf_decode(ld, in, ms, out, g->threads)) return false;
        std::unique_lock<std::mutex> lk(g->m);
        if (f.cancel || g->stop) return true;
        if (!out.empty()) f.q.push_back(std::move(out));
        g->cv.notify_all();
        return true;
    }
    if (n > LD_MAX_IN) return false;
    void* d = ld->alloc();
    if (!d) return false;
    std::vector<uint8_t> out(std::min(LD_MAX_OUT, std::max<size_t>(4 * n, 1u << 20)));
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
            const int r = ld->gzip_ex(d, in.data() + pos, n - pos, out.data() + len, out.size() - len, &used, &produced);
            if (r == 0) {  // LIBDEFLATE_SUCCESS
                len += produced;
                pos += used;
                break;
            }
            if (r == 3 && out.size() < LD_MAX_OUT) {  // LIBDEFLATE_INSUFFICIENT_SPACE: a bigger buffer, again
                out.resize(std::min(LD_MAX_OUT, 2 * out.size()));
                continue;
            }
            ok = false;
            break;
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
std::string inflate_file(fr_gz* g, int i) {
    GzFile& f = g->files[i];
    if (inflate_whole(g, f)) return "";
    FILE* fp = fopen(f.path.c_str(), "rb");
    if (!fp) return "cannot open " + f.path;
    std::vector<uint8_t> in(4u << 20);
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) {
        fclose(fp);
        return "inflateInit2 failed";
    }
    auto fresh = [&]() {
        std::lock_guard<std::mutex> lk(g->m);
        if (g->spare.empty()) return std::vector<uint8_t>(g->block);
        std::vector<uint8_t> v = std::move(g->spare.back());
        g->spare.pop_back();
        v.resize(g->block);
        return v;
    };
    std::vector<uint8_t> out = fresh();
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

void worker(fr_gz* g) {
    for (;;) {
        int i;
        {
            std::unique_lock<std::mutex> lk(g->m);
            g->cv.wait(lk, [&] {
                return g->stop || (g->next < (int)g->files.size() && g->next < g->consume + g->threads);
            });
            if (g->stop) return;
            i = g->next++;
        }
        std::string err = inflate_file(g, i);
        std::lock_guard<std::mutex> lk(g->m);
        g->files[i].err = err;
        g->files[i].done = true;
        g->cv.notify_all();
    }
}

}  // namespace

extern "C" {

fr_gz* fr_gz_open(const char* const* paths, int n_files, int threads) {
    fr_gz* g = new fr_gz();
    g->files.resize(n_files > 0 ? n_files : 0);
    for (int i = 0; i < n_files; ++i) g->files[i].path = paths[i];
    g->threads = threads < 1 ? 1 : threads;
    // files inflating ahead of the consumer may buffer up to 2 GiB of decoded blocks in all, so a
    // worker is not parked behind a short queue while the consumer is still on an earlier file
    g->depth = std::max<size_t>(3, (2ull << 30) / ((size_t)g->threads * g->block));
    const int nw = std::min(g->threads, std::max(n_files, 1));
    for (int k = 0; k < nw; ++k) g->workers.emplace_back(worker, g);
    return g;
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
        std::vector<uint8_t> b;
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
            if (g->spare.size() < (size_t)g->threads * g->depth) g->spare.push_back(std::move(b));
        }
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
