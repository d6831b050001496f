// rio_host.h — host-side helpers shared by the runtime files (rio_capi.cpp, rio_replay.cpp).
#pragma once
#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "rio.h"

namespace rio {

// A small persistent pool for host-side byte moving: copies into / out of the pinned staging pieces,
// and the WAL replay's file reads. One core's memcpy (~10 GB/s) or pread otherwise bounds the PCIe
// paths well below the link. One job at a time (callers on other contexts or workers wait their
// turn); workers live for the process. RIO_COPY_THREADS sets the worker count (default 4; measured
// on C2 end-to-end: 0 -> 8.0, 4 -> 14.7, 6 -> 14.3, 12 -> 14.1 GiB/s).
class HostPool {
  public:
    static HostPool& get() {
        static HostPool* p = new HostPool();
        return *p;
    }
    size_t parts() const { return workers_.size() + 1; }
    // fn(part, parts) for part in [0, parts): part 0 on the caller, the rest on the workers
    void run(const std::function<void(size_t, size_t)>& fn) {
        const size_t W = workers_.size();
        if (W == 0) {
            fn(0, 1);
            return;
        }
        std::lock_guard<std::mutex> one(submit_);
        {
            std::lock_guard<std::mutex> g(mu_);
            fn_ = &fn;
            remaining_ = W;
            gen_++;
        }
        cv_.notify_all();
        fn(0, W + 1);
        std::unique_lock<std::mutex> g(mu_);
        done_.wait(g, [&] { return remaining_ == 0; });
    }
    void copy(void* dst, const void* src, size_t n) {
        if (workers_.empty() || n < (4u << 20)) {
            memcpy(dst, src, n);
            return;
        }
        run([&](size_t part, size_t parts) {
            const size_t step = ((n + parts - 1) / parts + 63) & ~size_t(63), o = part * step;
            if (o < n) memcpy(static_cast<uint8_t*>(dst) + o, static_cast<const uint8_t*>(src) + o, std::min(step, n - o));
        });
    }

  private:
    HostPool() {
        const char* v = getenv("RIO_COPY_THREADS");
        // 8 copy threads (+ the caller): the staged H2D of a host image (rio_stream_open_host, rio_frame)
        // ran at ~32 GB/s with 4, under PCIe's 57 GB/s (round 4); the GPU box gives a job 16 cores
        const long t = v ? strtol(v, nullptr, 0) : 8;
        for (long i = 0; i < std::min(t, 32L); i++) workers_.emplace_back([this, i] { loop((size_t)i + 1); });
        for (auto& w : workers_) w.detach();
    }
    void loop(size_t part) {
        uint64_t seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> g(mu_);
            cv_.wait(g, [&] { return gen_ != seen; });
            seen = gen_;
            const std::function<void(size_t, size_t)>* fn = fn_;
            g.unlock();
            (*fn)(part, workers_.size() + 1);
            g.lock();
            if (--remaining_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex submit_, mu_;
    std::condition_variable cv_, done_;
    const std::function<void(size_t, size_t)>* fn_ = nullptr;
    size_t remaining_ = 0;
    uint64_t gen_ = 0;
};

// Framing of a file whose bytes a host producer writes piece by piece into the context's pinned
// staging (rio_capi.cpp): fill(user, dst, off, n) writes file bytes [off, off + n) to dst and
// returns RIO_OK or an error, which aborts the frame. Producing piece k+1 overlaps the DMA of
// piece k; then rio_frame's device work. Used by rio_replay.cpp (pread straight into staging, and
// the windows of rio_stream: a synthetic file header followed by a byte range of the file).
typedef int (*FillFn)(void* user, uint8_t* dst, uint64_t off, uint64_t n);
int frame_fill(rio_ctx* ctx, uint64_t len, FillFn fill, void* user, rio_file_info* info);
// rio_frame of prefix[0, prefix_len) + src[0, n): src page-locked (rio_host_register) is copied by DMA in place
int frame_direct(rio_ctx* ctx, const uint8_t* prefix, uint64_t prefix_len, const uint8_t* src, uint64_t n,
                 rio_file_info* info);
bool is_host_pinned(const void* p, uint64_t n);
// page-locked host ranges the library itself knows (rio_host_register, PinnedPool blocks)
void note_pinned(const void* p, uint64_t n);
void forget_pinned(const void* p);

}  // namespace rio
