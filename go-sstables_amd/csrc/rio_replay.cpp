// rio_replay.cpp — ordered whole-file replay of a list of recordio files (the WAL replay adapter).
//
// wal.Replayer.Replay (wal/replayer.go:18-77) walks the WAL directory, sorts the *.wal paths and reads
// each file to its end through a ReaderI before opening the next one, calling `process` for every
// record in order. Here worker threads, each with its own rio_ctx (own stream, arenas and pinned
// staging; contexts pooled across replays, CtxPool below), read file k+1.. and run the device decode
// (framing + rio_decode) while the caller is still consuming file k. Decoded files are handed out
// strictly in list order, at most `depth` of them held ahead, and the H2D of one file overlaps the
// decode and D2H of another. Nothing decodes on the host: a file the device path does not handle shows
// up as RIO_ERR_UNSUPPORTED in its info and the Go adapter re-reads that file with the reference
// reader. Files are pread straight into the context's staging pieces (rio::frame_fill); records are
// returned in page-locked blocks from a process-wide cache (PinnedPool below). The second half of the
// file is the windowed decode of one large file (rio_stream_*).
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rio.h"
#include "rio_host.h"

using rio::HostPool;

namespace {

// Process-wide cache of page-locked host buffers. A replay streams gigabytes through host memory;
// fresh pageable buffers cost a zero-fill plus a page fault per 4 KiB (measured: more than the H2D,
// decode and D2H of the same file together), and pageable copies go through the staging pieces.
// Pinned buffers are reused across files and replays and DMA'd directly. Best fit within 1.25x
// (looser, a file's input block took a decoded-output block and forced a 15 ms hipHostMalloc),
// at most kMaxCached bytes kept; intentionally never destroyed (process lifetime, no
// static-destruction order against the HIP runtime).
class PinnedPool {
  public:
    static PinnedPool& get() {
        static PinnedPool* p = new PinnedPool();
        return *p;
    }
    void* take(size_t n, size_t& cap) {
        n = (std::max<size_t>(n, 1) + kGrain - 1) / kGrain * kGrain;
        {
            std::lock_guard<std::mutex> g(mu_);
            auto it = free_.lower_bound(n);
            if (it != free_.end() && it->first <= n + n / 4) {
                void* p = it->second;
                cap = it->first;
                cached_ -= cap;
                free_.erase(it);
                return p;
            }
        }
        void* p = nullptr;
        if (hipHostMalloc(&p, n, hipHostMallocPortable) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        rio::note_pinned(p, n);
        cap = n;
        return p;
    }
    void give(void* p, size_t cap) {
        if (!p) return;
        std::lock_guard<std::mutex> g(mu_);
        if (cached_ + cap > kMaxCached) {
            rio::forget_pinned(p);
            (void)hipHostFree(p);
            return;
        }
        free_.emplace(cap, p);
        cached_ += cap;
    }

  private:
    static constexpr size_t kGrain = 2u << 20;
    static constexpr size_t kMaxCached = 16ull << 30;
    std::mutex mu_;
    std::multimap<size_t, void*> free_;
    size_t cached_ = 0;
};

// Process-wide cache of idle decode contexts, per device. A rio_ctx's stream and device arenas
// grow to the largest file it has decoded; a replay that built fresh contexts paid that growth
// (hipMalloc of every arena, first-touch) on each of its first files again (measured: 12-16 ms
// decode+D2H of a 128 MiB file against 4.7 ms steady state; WAL bench 11.1 -> 16.7 GiB/s). rio_replay_free hands its contexts back here;
// at most kMaxIdle are kept per device, the rest are destroyed. Never destroyed itself (same
// reason as PinnedPool).
class CtxPool {
  public:
    static CtxPool& get() {
        static CtxPool* p = new CtxPool();
        return *p;
    }
    int take(int device, rio_ctx** out) {
        {
            std::lock_guard<std::mutex> g(mu_);
            auto& v = idle_[device];
            if (!v.empty()) {
                *out = v.back();
                v.pop_back();
                return RIO_OK;
            }
        }
        return rio_ctx_create(device, out);
    }
    void give(int device, rio_ctx* c) {
        {
            std::lock_guard<std::mutex> g(mu_);
            auto& v = idle_[device];
            if (v.size() < kMaxIdle) {
                v.push_back(c);
                return;
            }
        }
        rio_ctx_destroy(c);
    }

  private:
    static constexpr size_t kMaxIdle = 4;
    std::mutex mu_;
    std::map<int, std::vector<rio_ctx*>> idle_;
};

struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool alloc(size_t n) {
        p = PinnedPool::get().take(n, cap);
        return p != nullptr;
    }
    ~PinnedBuf() { PinnedPool::get().give(p, cap); }
    uint8_t* bytes() const { return static_cast<uint8_t*>(p); }
};

constexpr uint64_t align64(uint64_t x) { return (x + 63) & ~63ull; }

// one decoded file: out | out_off[n+1] | rec_off[n+1] | flags[n+1] in one pinned block
struct Decoded {
    uint64_t index = 0;
    int rc = RIO_OK;  // RIO_OK (see info.status), RIO_ERR_IO (open/read), RIO_ERR_HIP
    rio_file_info info{};
    PinnedBuf buf;
    uint8_t* out = nullptr;
    uint64_t* out_off = nullptr;
    uint64_t* rec_off = nullptr;
    uint8_t* flags = nullptr;
};

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

const bool kTrace = getenv("RIO_REPLAY_TRACE") != nullptr;

// Bytes [off, off + n) of a file descriptor or of host memory into `dst`, split over the host
// pool for large ranges (one thread's pread, a kernel copy out of the page cache, ran at 11-20 GB/s).
// pread: no mapping, so no page faults and no mm-lock contention between the workers.
struct Source {
    int fd = -1;
    const uint8_t* mem = nullptr;
    int read(uint8_t* dst, uint64_t off, uint64_t n) const {
        std::atomic<int> err{RIO_OK};
        auto part_copy = [&](uint64_t o, uint64_t end) {
            if (mem) {
                memcpy(dst + (o - off), mem + o, end - o);
                return;
            }
            while (o < end && err.load(std::memory_order_relaxed) == RIO_OK) {
                const ssize_t k = pread(fd, dst + (o - off), std::min<uint64_t>(end - o, 64ull << 20), (off_t)o);
                if (k < 0 && errno == EINTR) continue;
                if (k <= 0) err = RIO_ERR_IO;  // error, or the file shrank under us
                else o += (uint64_t)k;
            }
        };
        if (n < (8u << 20)) {
            part_copy(off, off + n);
        } else {
            HostPool::get().run([&](size_t part, size_t parts) {
                const uint64_t step = ((n + parts - 1) / parts + 4095) & ~4095ull, o = part * step;
                if (o < n) part_copy(off + o, off + std::min<uint64_t>(n, o + step));
            });
        }
        return err.load();
    }
};

// phase B of a framed ctx into one pinned block: out | out_off[n+1] | rec_off[n+1] | flags[n+1]
int decode_into(rio_ctx* ctx, Decoded& d) {
    const uint64_t n = d.info.n_records, nb = d.info.total_out_bytes;
    const uint64_t o_off = align64(nb + 1), o_rec = o_off + align64((n + 1) * 8), o_fl = o_rec + align64((n + 1) * 8);
    if (!d.buf.alloc(o_fl + n + 1)) return RIO_ERR_HIP;
    d.out = d.buf.bytes();
    d.out_off = reinterpret_cast<uint64_t*>(d.buf.bytes() + o_off);
    d.rec_off = reinterpret_cast<uint64_t*>(d.buf.bytes() + o_rec);
    d.flags = d.buf.bytes() + o_fl;
    d.out_off[0] = 0;
    return rio_decode(ctx, d.out, nb, d.out_off, d.rec_off, d.flags, n, &d.info);
}

// Source bytes [base + off, base + off + n) behind an optional synthetic prefix (a window's file
// header): the rio::frame_fill producer
struct Fill {
    const Source* src;
    uint64_t base = 0;
    const uint8_t* prefix = nullptr;
    uint64_t prefix_len = 0;
    static int fn(void* user, uint8_t* dst, uint64_t off, uint64_t n) {
        const Fill& f = *static_cast<const Fill*>(user);
        if (off < f.prefix_len) {
            const uint64_t k = std::min(n, f.prefix_len - off);
            memcpy(dst, f.prefix + off, k);
            dst += k;
            off += k;
            n -= k;
        }
        return n ? f.src->read(dst, f.base + (off - f.prefix_len), n) : RIO_OK;
    }
};

int decode_file(rio_ctx* ctx, const std::string& path, Decoded& d) {
    const double t0 = now_ms();
    const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) return RIO_ERR_IO;
    struct stat st;
    if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode)) {
        ::close(fd);
        return RIO_ERR_IO;
    }
    posix_fadvise(fd, 0, 0, POSIX_FADV_SEQUENTIAL);
    // pread straight into the context's staging pieces, overlapping the H2D of the previous piece
    const Source src{fd, nullptr};
    Fill f{&src};
    int rc = rio::frame_fill(ctx, (uint64_t)st.st_size, &Fill::fn, &f, &d.info);
    ::close(fd);
    if (rc) return rc;
    const double t1 = now_ms();
    rc = decode_into(ctx, d);
    if (rc) return rc;
    if (kTrace)
        fprintf(stderr, "replay %s: read+H2D+frame %.1f decode(B+D2H) %.1f ms\n", path.c_str(), t1 - t0, now_ms() - t1);
    return RIO_OK;
}

}  // namespace

struct rio_replay {
    std::vector<std::string> paths;
    uint32_t depth = 2;
    std::vector<int> devs;       // worker w's device
    std::vector<rio_ctx*> ctxs;  // one per worker (from CtxPool): own stream, arenas and pinned staging
    std::vector<std::thread> workers;
    std::mutex mu;
    std::condition_variable cv;
    std::map<uint64_t, std::unique_ptr<Decoded>> ready;
    std::unique_ptr<Decoded> current;  // handed out by the last rio_replay_next
    uint64_t next_out = 0;             // index the caller gets next
    bool stop = false;

    // worker w of W takes files w, w + W, ...; file i starts only once i < next_out + depth, so at
    // most `depth` files are decoded or in flight beyond the one the caller holds
    void run(uint32_t w, uint32_t W) {
        for (uint64_t i = w; i < paths.size(); i += W) {
            {
                std::unique_lock<std::mutex> g(mu);
                cv.wait(g, [&] { return stop || i < next_out + depth; });
                if (stop) return;
            }
            auto d = std::make_unique<Decoded>();
            d->index = i;
            d->rc = decode_file(ctxs[w], paths[i], *d);
            std::lock_guard<std::mutex> g(mu);
            ready.emplace(i, std::move(d));
            cv.notify_all();
        }
    }
};

extern "C" int rio_replay_open(int device, const char* const* paths, uint64_t n_paths, uint32_t depth,
                               uint32_t workers, rio_replay** out) {
    // rio.h's single-device contract: workers (0 = 2) at most depth (0 = 2), so at most `depth`
    // decoded files are held (the device-list form raises depth to its worker count instead)
    const uint32_t d = depth ? depth : 2u;
    const uint32_t w = std::min<uint32_t>(workers ? workers : 2u, d);
    return rio_replay_open_devices(&device, 1, paths, n_paths, d, w, out);
}

// Workers are dealt to the devices round-robin (worker w on devices[w % n_devices]), each with a
// pooled context of its device; file i goes to worker i % W as before, so consecutive files decode
// on different GPUs and the ordered hand-out interleaves them (one host thread and
// context per GPU, no communication between them).
extern "C" int rio_replay_open_devices(const int* devices, uint32_t n_devices, const char* const* paths,
                                       uint64_t n_paths, uint32_t depth, uint32_t workers_per_device,
                                       rio_replay** out) {
    if (!out || !devices || !n_devices || (n_paths && !paths)) return RIO_ERR_ARG;
    *out = nullptr;
    for (uint64_t i = 0; i < n_paths; i++)
        if (!paths[i]) return RIO_ERR_ARG;
    auto* r = new rio_replay();
    r->paths.assign(paths, paths + n_paths);
    const uint32_t per = workers_per_device ? workers_per_device : 2;
    uint32_t W = per * n_devices;
    // at least one file in flight per worker, never fewer than the caller's depth
    r->depth = std::max<uint32_t>(depth ? depth : 2, W);
    W = (uint32_t)std::min<uint64_t>(W, std::max<uint64_t>(n_paths, 1));
    for (uint32_t w = 0; w < W; w++) {
        const int dev = devices[w % n_devices];
        rio_ctx* c = nullptr;
        int rc = CtxPool::get().take(dev, &c);
        if (rc) {
            for (size_t x = 0; x < r->ctxs.size(); x++) CtxPool::get().give(r->devs[x], r->ctxs[x]);
            delete r;
            return rc;
        }
        r->ctxs.push_back(c);
        r->devs.push_back(dev);
    }
    for (uint32_t w = 0; w < W; w++) r->workers.emplace_back([r, w, W] { r->run(w, W); });
    *out = r;
    return RIO_OK;
}

extern "C" int rio_replay_next(rio_replay* r, uint64_t* index, const uint8_t** out, const uint64_t** out_off,
                               const uint8_t** flags, rio_file_info* info) {
    if (!r) return RIO_ERR_ARG;
    std::unique_lock<std::mutex> g(r->mu);
    r->current.reset();  // the previous file's arrays are released here
    if (r->next_out >= r->paths.size()) return RIO_EOF;
    const uint64_t want = r->next_out;
    r->cv.wait(g, [&] { return r->ready.count(want) != 0; });
    auto it = r->ready.find(want);
    r->current = std::move(it->second);
    r->ready.erase(it);
    r->next_out++;
    r->cv.notify_all();
    Decoded& d = *r->current;
    if (index) *index = d.index;
    if (info) *info = d.info;
    if (out) *out = d.out;
    if (out_off) *out_off = d.out_off;
    if (flags) *flags = d.flags;
    return d.rc;
}

extern "C" void rio_replay_free(rio_replay* r) {
    if (!r) return;
    {
        std::lock_guard<std::mutex> g(r->mu);
        r->stop = true;
        r->cv.notify_all();
    }
    for (auto& t : r->workers)
        if (t.joinable()) t.join();
    for (size_t x = 0; x < r->ctxs.size(); x++) CtxPool::get().give(r->devs[x], r->ctxs[x]);
    delete r;
}

// ---- pooled contexts for per-file readers (the Go adapter's Open / Close) ---------------------
extern "C" int rio_ctx_acquire(int device, rio_ctx** out) {
    if (!out) return RIO_ERR_ARG;
    *out = nullptr;
    return CtxPool::get().take(device, out);
}

extern "C" void rio_ctx_release(rio_ctx* ctx) {
    if (ctx) CtxPool::get().give(rio_ctx_device(ctx), ctx);
}

// ---- a file set decoded over several devices (rio_fileset_*) ----------------------------------
// One host thread per device, each with a pooled context of its device; files are assigned by
// longest-processing-time first on their sizes (LPT over GPUs, round-robin for equal
// sizes), and a thread decodes its files in that order into page-locked blocks. No communication
// between the threads: the files are independent (a WAL directory, the tables of an SSTable set).
struct rio_fileset {
    std::vector<std::unique_ptr<Decoded>> files;
    std::vector<int> device;  // device that decoded file i
};

extern "C" int rio_fileset_decode(const int* devices, uint32_t n_devices, const char* const* paths, uint64_t n_paths,
                                  rio_fileset** out) {
    if (!out || !devices || !n_devices || (n_paths && !paths)) return RIO_ERR_ARG;
    *out = nullptr;
    std::vector<uint64_t> size(n_paths, 0);
    for (uint64_t i = 0; i < n_paths; i++) {
        if (!paths[i]) return RIO_ERR_ARG;
        struct stat st;
        if (stat(paths[i], &st) == 0 && S_ISREG(st.st_mode)) size[i] = (uint64_t)st.st_size;
    }
    // LPT: largest file first, each to the device with the least assigned bytes (ties: lowest index)
    std::vector<uint64_t> order(n_paths);
    for (uint64_t i = 0; i < n_paths; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return size[a] > size[b]; });
    std::vector<std::vector<uint64_t>> mine(n_devices);
    std::vector<uint64_t> load(n_devices, 0);
    auto* fs = new rio_fileset();
    fs->files.resize(n_paths);
    fs->device.assign(n_paths, -1);
    for (uint64_t i : order) {
        uint32_t best = 0;
        for (uint32_t d = 1; d < n_devices; d++)
            if (load[d] < load[best]) best = d;
        load[best] += size[i] + 1;
        mine[best].push_back(i);
        fs->device[i] = devices[best];
    }
    std::atomic<int> fail{RIO_OK};
    std::vector<std::thread> th;
    for (uint32_t d = 0; d < n_devices; d++) {
        if (mine[d].empty()) continue;
        th.emplace_back([&, d] {
            rio_ctx* c = nullptr;
            if (int rc = CtxPool::get().take(devices[d], &c)) {
                fail = rc;
                return;
            }
            for (uint64_t i : mine[d]) {
                auto f = std::make_unique<Decoded>();
                f->index = i;
                f->rc = decode_file(c, paths[i], *f);
                fs->files[i] = std::move(f);
            }
            CtxPool::get().give(devices[d], c);
        });
    }
    for (auto& t : th) t.join();
    if (fail.load() != RIO_OK) {
        delete fs;
        return fail.load();
    }
    *out = fs;
    return RIO_OK;
}

extern "C" int rio_fileset_get(const rio_fileset* s, uint64_t i, const uint8_t** out, const uint64_t** out_off,
                               const uint64_t** rec_off, const uint8_t** flags, rio_file_info* info, int* device) {
    if (!s || i >= s->files.size() || !s->files[i]) return RIO_ERR_ARG;
    const Decoded& d = *s->files[i];
    if (out) *out = d.out;
    if (out_off) *out_off = d.out_off;
    if (rec_off) *rec_off = d.rec_off;
    if (flags) *flags = d.flags;
    if (info) *info = d.info;
    if (device) *device = s->device[i];
    return d.rc;
}

extern "C" void rio_fileset_free(rio_fileset* s) { delete s; }

// ---- windowed sequential decode of one file (rio_stream_*) ------------------------------------
//
// FileReader.ReadNext over a file larger than the staging it should take (SURVEY §8b "per window
// for files larger than staging"; the Go adapter's cgo call per window). Window k is the file's
// 8-byte header followed by the bytes [s_k, e_k): a recordio file of its own, framed and decoded by
// the whole-file path. Its terminal status decides the next window:
//   * e_k = file end: the window's status is the file's;
//   * raised at p > s_k: records before p are complete; the next window starts at p (a status at p
//     may be an artifact of the cut, so p is framed again as the first record of the next window);
//   * raised at p = s_k (no record completed): a truncation-type status (the EOF family,
//     io.ErrUnexpectedEOF; the zero-tail test reads to the end of the file) doubles the window;
//     any other status depends only on bytes inside the window and is the file's.
// A record that fails to decompress is flagged in whichever window holds it (its bytes are inside
// the window, so the cut cannot change the codec's verdict); first_bad is a file record index. The driver
// thread reads and frames window k+1 on one context while a worker runs window k's decode and D2H
// on the other, so the file's H2D overlaps its D2H. Records, offsets and statuses are those of the
// whole-file decode: rec_off and status_offset are file offsets, out_off is window-relative.
namespace {

bool cut_type(int st) {
    return st == RIO_EOF || st == RIO_EOF_ZERO_TAIL || st == RIO_EOF_HEADER || st == RIO_EOF_PAYLOAD || st == RIO_EOF_CODEC ||
           st == RIO_ERR_UNEXPECTED_EOF;
}

struct Window {
    Decoded d;
    uint64_t k = 0;
    uint64_t first_record = 0;
    bool terminal = false;
};

}  // namespace

struct rio_stream {
    Source src;
    int fd = -1;
    uint64_t len = 0;
    uint64_t window = 0;
    uint32_t depth = 4;
    int device = 0;
    bool pinned = false;  // a host image the caller page-locked (rio_host_register): windows go by DMA in place
    // three contexts: window k+2 reads and frames while k and k+1 decode and copy out (VERDICT r3 #5:
    // the D2H of consecutive windows runs back to back)
    static constexpr int kCtx = 3;
    rio_ctx* ctx[kCtx] = {nullptr, nullptr, nullptr};
    std::thread driver, worker[kCtx];
    std::mutex mu;
    std::condition_variable cv;
    struct Job {
        bool has = false, terminal = false;
        uint64_t k = 0, s = 0, first_record = 0;
        rio_file_info fi{};
    } job[kCtx];
    bool busy[kCtx] = {false, false, false};
    std::map<uint64_t, std::unique_ptr<Window>> ready;
    std::unique_ptr<Window> current;
    uint64_t next_out = 0;
    uint64_t end_k = ~0ull;  // index of the terminal window once known
    bool stop = false;
    double t_origin = now_ms();  // RIO_REPLAY_TRACE timestamps are relative to the open

    void post_fatal(uint64_t k, int rc) {
        auto w = std::make_unique<Window>();
        w->k = k;
        w->d.rc = rc;
        w->terminal = true;
        std::lock_guard<std::mutex> g(mu);
        end_k = std::min(end_k, k);
        ready.emplace(k, std::move(w));
        cv.notify_all();
    }

    void run_driver() {
        uint8_t hdr[RIO_FILE_HEADER_BYTES] = {0};
        // (saturating: a window near 2^64 is a whole-file window, not a wrapped sum)
        const bool whole = len <= RIO_FILE_HEADER_BYTES || window >= len - RIO_FILE_HEADER_BYTES;
        if (!whole && src.read(hdr, 0, RIO_FILE_HEADER_BYTES)) return post_fatal(0, RIO_ERR_IO);
        uint64_t s = whole ? 0 : RIO_FILE_HEADER_BYTES, first = 0;
        for (uint64_t k = 0;; k++) {
            const int c = (int)(k % kCtx);
            {
                std::unique_lock<std::mutex> g(mu);
                cv.wait(g, [&] { return stop || k > end_k || (!busy[c] && k < next_out + depth); });
                if (stop || k > end_k) return;
            }
            // ramp: the first windows are smaller, so the first D2H starts after a short H2D instead
            // of a whole window's (windows of >= 8 MiB only; the ramp never changes what is decoded)
            uint64_t w = window, next_s = 0;
            if (window >= (8ull << 20)) w = k == 0 ? window / 8 : (k == 1 ? window / 2 : window);
            rio_file_info fi{};
            bool terminal = false;
            for (;;) {
                const uint64_t e = whole ? len : s + std::min(w, len - s);
                const uint64_t hl = whole ? 0 : RIO_FILE_HEADER_BYTES, n = hl + (e - s);
                Fill f{&src, s, hdr, hl};
                const double tf0 = kTrace ? now_ms() : 0.0;
                if (int rc = pinned ? rio::frame_direct(ctx[c], hdr, hl, src.mem + s, e - s, &fi)
                                    : rio::frame_fill(ctx[c], n, &Fill::fn, &f, &fi))
                    return post_fatal(k, rc);
                if (kTrace)
                    fprintf(stderr, "stream w%llu ctx%d: read+H2D+frame %llu B %.3f-%.3f ms\n", (unsigned long long)k, c,
                            (unsigned long long)n, tf0 - t_origin, now_ms() - t_origin);
                const uint64_t p = fi.status_offset + s - hl;  // file offset of the status
                if (e == len) {
                    terminal = true;
                } else if (p > s) {
                    next_s = p;
                } else if (cut_type(fi.status)) {
                    w = w > (len - s) / 2 ? len - s : 2 * w;  // (reaches the file end, never wraps)
                    continue;
                } else {
                    terminal = true;
                }
                break;
            }
            {
                std::lock_guard<std::mutex> g(mu);
                job[c] = Job{true, terminal, k, whole ? RIO_FILE_HEADER_BYTES : s, first, fi};
                busy[c] = true;
                if (terminal) end_k = std::min(end_k, k);
                cv.notify_all();
            }
            if (terminal) return;
            first += fi.n_records;
            s = next_s;
        }
    }

    void run_worker(int c) {
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> g(mu);
                cv.wait(g, [&] { return stop || job[c].has; });
                if (stop) return;
                j = job[c];
            }
            auto w = std::make_unique<Window>();
            w->k = j.k;
            w->first_record = j.first_record;
            w->d.info = j.fi;
            const double td0 = kTrace ? now_ms() : 0.0;
            w->d.rc = decode_into(ctx[c], w->d);
            if (kTrace)
                fprintf(stderr, "stream w%llu ctx%d: decode+D2H %llu B out %.3f-%.3f ms\n", (unsigned long long)j.k, c,
                        (unsigned long long)w->d.info.total_out_bytes, td0 - t_origin, now_ms() - t_origin);
            rio_file_info& fi = w->d.info;
            const uint64_t shift = j.s - RIO_FILE_HEADER_BYTES;  // window offset -> file offset
            for (uint64_t i = 0; !w->d.rc && shift && i < fi.n_records; i++) w->d.rec_off[i] += shift;
            if (fi.n_bad) fi.first_bad += j.first_record;  // a file record index, like first_record
            // a record the decode hands back (RIO_ERR_UNSUPPORTED truncates the window) ends the
            // file here, whatever the cut; one that does not decompress is only flagged
            w->terminal = j.terminal || w->d.rc || fi.n_records < j.fi.n_records || fi.status != j.fi.status;
            if (w->terminal) {
                fi.status_offset += shift;
            } else {
                fi.status = RIO_OK;
                fi.status_offset = 0;
                fi.detail0 = fi.detail1 = 0;
            }
            std::lock_guard<std::mutex> g(mu);
            if (w->terminal) end_k = std::min(end_k, j.k);
            ready.emplace(j.k, std::move(w));
            job[c].has = false;
            busy[c] = false;
            cv.notify_all();
        }
    }
};

static int stream_start(rio_stream* r, int device, uint64_t window, uint32_t depth, rio_stream** out) {
    r->device = device;
    r->window = window ? window : (128ull << 20);
    r->depth = depth ? depth : 4;
    for (int c = 0; c < rio_stream::kCtx; c++) {
        if (int rc = CtxPool::get().take(device, &r->ctx[c])) {
            for (int x = 0; x < c; x++) CtxPool::get().give(device, r->ctx[x]);
            if (r->fd >= 0) ::close(r->fd);
            delete r;
            return rc;
        }
    }
    for (int c = 0; c < rio_stream::kCtx; c++) r->worker[c] = std::thread([r, c] { r->run_worker(c); });
    r->driver = std::thread([r] { r->run_driver(); });
    *out = r;
    return RIO_OK;
}

extern "C" int rio_stream_open(int device, const char* path, uint64_t window_bytes, uint32_t depth, rio_stream** out) {
    if (!out || !path) return RIO_ERR_ARG;
    *out = nullptr;
    const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return RIO_ERR_IO;
    struct stat st;
    if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode)) {
        ::close(fd);
        return RIO_ERR_IO;
    }
    posix_fadvise(fd, 0, 0, POSIX_FADV_SEQUENTIAL);
    auto* r = new rio_stream();
    r->fd = fd;
    r->src = Source{fd, nullptr};
    r->len = (uint64_t)st.st_size;
    return stream_start(r, device, window_bytes, depth, out);
}

extern "C" int rio_stream_open_host(int device, const uint8_t* data, uint64_t len, uint64_t window_bytes, uint32_t depth,
                                    rio_stream** out) {
    if (!out || (len && !data)) return RIO_ERR_ARG;
    *out = nullptr;
    auto* r = new rio_stream();
    r->src = Source{-1, data};
    r->len = len;
    r->pinned = len && rio::is_host_pinned(data, len);
    return stream_start(r, device, window_bytes, depth, out);
}

extern "C" int rio_stream_next(rio_stream* r, uint64_t* first_record, const uint8_t** out, const uint64_t** out_off,
                               const uint64_t** rec_off, const uint8_t** flags, rio_file_info* info) {
    if (!r) return RIO_ERR_ARG;
    std::unique_lock<std::mutex> g(r->mu);
    r->current.reset();  // the previous window's arrays are released here
    const uint64_t want = r->next_out;
    r->cv.wait(g, [&] { return want > r->end_k || r->ready.count(want) != 0; });
    if (want > r->end_k) return RIO_EOF;
    auto it = r->ready.find(want);
    r->current = std::move(it->second);
    r->ready.erase(it);
    r->next_out++;
    r->cv.notify_all();
    const Window& w = *r->current;
    if (first_record) *first_record = w.first_record;
    if (info) *info = w.d.info;
    if (out) *out = w.d.out;
    if (out_off) *out_off = w.d.out_off;
    if (rec_off) *rec_off = w.d.rec_off;
    if (flags) *flags = w.d.flags;
    return w.d.rc;
}

extern "C" void rio_stream_free(rio_stream* r) {
    if (!r) return;
    {
        std::lock_guard<std::mutex> g(r->mu);
        r->stop = true;
        r->cv.notify_all();
    }
    if (r->driver.joinable()) r->driver.join();
    for (auto& t : r->worker)
        if (t.joinable()) t.join();
    for (rio_ctx* c : r->ctx) CtxPool::get().give(r->device, c);
    if (r->fd >= 0) ::close(r->fd);
    delete r;
}
