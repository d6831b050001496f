// rio_replay.cpp — ordered whole-file replay of a list of recordio files (the WAL replay adapter).
//
// wal.Replayer.Replay (wal/replayer.go:18-77) walks the WAL directory, sorts the *.wal paths and reads
// each file to its end through a ReaderI before opening the next one, calling `process` for every
// record in order. Here worker threads, each with its own rio_ctx (own stream, arenas and pinned
// staging), map file k+1.. and run the device decode (rio_frame + rio_decode) while the caller is
// still consuming file k. Decoded files are handed out strictly in list order, at most `depth` of them
// held ahead, and the staged H2D of one file overlaps the decode and D2H of another. Nothing decodes
// on the host: a file the device path does not handle shows up as RIO_ERR_UNSUPPORTED in its info and
// the Go adapter re-reads that file with the reference reader. Files are read into, and records
// returned in, page-locked host buffers from a process-wide cache (PinnedPool below).
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
        cap = n;
        return p;
    }
    void give(void* p, size_t cap) {
        if (!p) return;
        std::lock_guard<std::mutex> g(mu_);
        if (cached_ + cap > kMaxCached) {
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

// whole file into a pinned buffer (pread: no mapping, so no page faults and no mm-lock contention
// between the workers)
int read_file(const std::string& path, PinnedBuf& in, uint64_t& len) {
    const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) return RIO_ERR_IO;
    struct stat st;
    int rc = RIO_OK;
    if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode)) rc = RIO_ERR_IO;
    len = rc ? 0 : (uint64_t)st.st_size;
    if (!rc && len) {
        if (!in.alloc(len)) rc = RIO_ERR_HIP;
        posix_fadvise(fd, 0, 0, POSIX_FADV_SEQUENTIAL);
        // the file's byte ranges read in parallel on the host pool (one thread's pread, a kernel
        // copy out of the page cache, ran at 11-20 GB/s)
        std::atomic<int> err{RIO_OK};
        auto read_range = [&](uint64_t o, uint64_t end) {
            while (o < end && err.load(std::memory_order_relaxed) == RIO_OK) {
                const ssize_t k = pread(fd, in.bytes() + o, std::min<uint64_t>(end - o, 64ull << 20), (off_t)o);
                if (k < 0 && errno == EINTR) continue;
                if (k <= 0) err = RIO_ERR_IO;  // error, or the file shrank under us
                else o += (uint64_t)k;
            }
        };
        if (!rc) {
            if (len < (8u << 20)) {
                read_range(0, len);
            } else {
                HostPool::get().run([&](size_t part, size_t parts) {
                    const uint64_t step = ((len + parts - 1) / parts + 4095) & ~4095ull, o = part * step;
                    if (o < len) read_range(o, std::min<uint64_t>(len, o + step));
                });
            }
            rc = err.load();
        }
    }
    ::close(fd);
    return rc;
}

int decode_file(rio_ctx* ctx, const std::string& path, Decoded& d) {
    const double t0 = now_ms();
    uint64_t len = 0;
    double t1, t2;
    {
        PinnedBuf in;
        int rc = read_file(path, in, len);
        if (rc) return rc;
        t1 = now_ms();
        rc = rio_frame(ctx, in.bytes(), len, &d.info);  // synchronises: `in` can go back to the pool
        if (rc) return rc;
        t2 = now_ms();
    }
    const uint64_t n = d.info.n_records, nb = d.info.total_out_bytes;
    const uint64_t o_off = align64(nb + 1), o_rec = o_off + align64((n + 1) * 8), o_fl = o_rec + align64((n + 1) * 8);
    if (!d.buf.alloc(o_fl + n + 1)) return RIO_ERR_HIP;
    d.out = d.buf.bytes();
    d.out_off = reinterpret_cast<uint64_t*>(d.buf.bytes() + o_off);
    d.rec_off = reinterpret_cast<uint64_t*>(d.buf.bytes() + o_rec);
    d.flags = d.buf.bytes() + o_fl;
    d.out_off[0] = 0;
    const double t3 = now_ms();
    const int rc = rio_decode(ctx, d.out, nb, d.out_off, d.rec_off, d.flags, n, &d.info);
    if (rc) return rc;
    if (kTrace)
        fprintf(stderr, "replay %s: read %.1f frame(H2D+A) %.1f alloc %.1f decode(B+D2H) %.1f ms\n", path.c_str(),
                t1 - t0, t2 - t1, t3 - t2, now_ms() - t3);
    return RIO_OK;
}

}  // namespace

struct rio_replay {
    std::vector<std::string> paths;
    uint32_t depth = 2;
    int device = 0;
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
    if (!out || (n_paths && !paths)) return RIO_ERR_ARG;
    *out = nullptr;
    for (uint64_t i = 0; i < n_paths; i++)
        if (!paths[i]) return RIO_ERR_ARG;
    auto* r = new rio_replay();
    r->device = device;
    r->paths.assign(paths, paths + n_paths);
    r->depth = depth ? depth : 2;
    uint32_t W = workers ? workers : 2;
    W = std::min<uint32_t>(W, r->depth);
    W = (uint32_t)std::min<uint64_t>(W, std::max<uint64_t>(n_paths, 1));
    for (uint32_t w = 0; w < W; w++) {
        rio_ctx* c = nullptr;
        int rc = CtxPool::get().take(device, &c);
        if (rc) {
            for (rio_ctx* x : r->ctxs) CtxPool::get().give(device, x);
            delete r;
            return rc;
        }
        r->ctxs.push_back(c);
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
    for (rio_ctx* c : r->ctxs) CtxPool::get().give(r->device, c);
    delete r;
}
