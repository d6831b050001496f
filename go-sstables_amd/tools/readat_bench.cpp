// readat_bench — ReadAtI lookup latency of the device-backed MMapReader (rio_reader_read_next_at /
// rio_reader_seek_next, include/rio.h) from T host threads sharing one reader, as a Go service's
// goroutines would call MMapReader.ReadNextAt (recordio/mmap_reader.go:130-203) through cgo.
//
//   rio_readat_bench <file> <record-offsets.u64> <threads> <lookups-per-thread> <at|seek>
//
// record-offsets.u64: the file's record start offsets (little-endian u64), e.g. from the writer.
// at:   ReadNextAt at uniformly random record starts;  seek: SeekNext from uniformly random byte
// offsets. The first call (which decodes the file into the reader's view) is timed on its own.
// Prints one JSON line.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "rio.h"

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    if (argc != 6) {
        fprintf(stderr, "usage: %s <file> <offsets.u64> <threads> <lookups-per-thread> <at|seek>\n", argv[0]);
        return 2;
    }
    const char* path = argv[1];
    FILE* fo = fopen(argv[2], "rb");
    if (!fo) return 3;
    std::vector<uint64_t> offs;
    uint64_t v;
    while (fread(&v, 8, 1, fo) == 1) offs.push_back(v);
    fclose(fo);
    const int T = atoi(argv[3]);
    const uint64_t K = strtoull(argv[4], nullptr, 10);
    const bool seek = strcmp(argv[5], "seek") == 0;
    if (offs.empty() || T <= 0) return 3;

    rio_ctx* ctx = nullptr;
    if (rio_ctx_create(0, &ctx)) return 4;
    rio_reader* r = nullptr;
    if (rio_reader_new_mmap(ctx, path, &r) || rio_reader_open(r)) return 5;
    const uint64_t size = rio_reader_size(r);

    const uint8_t* d = nullptr;
    uint64_t n = 0, ro = 0;
    int nil = 0;
    double t0 = now_s();
    int rc = rio_reader_read_next_at(r, offs[0], &d, &n, &nil);
    const double build_s = now_s() - t0;
    if (rc) {
        fprintf(stderr, "first ReadNextAt: %s\n", rio_strerror(rc));
        return 6;
    }

    std::vector<uint64_t> bytes(T, 0), fails(T, 0);
    std::vector<std::thread> th;
    t0 = now_s();
    for (int t = 0; t < T; t++) {
        th.emplace_back([&, t] {
            uint64_t x = 0x9E3779B97F4A7C15ull * (t + 1), sum = 0, bad = 0;
            for (uint64_t k = 0; k < K; k++) {
                x ^= x << 13;
                x ^= x >> 7;
                x ^= x << 17;
                const uint8_t* p = nullptr;
                uint64_t len = 0, at = 0;
                int isnil = 0;
                const int e = seek ? rio_reader_seek_next(r, x % (size + 1), &at, &p, &len, &isnil)
                                   : rio_reader_read_next_at(r, offs[x % offs.size()], &p, &len, &isnil);
                if (e && !(seek && rio_status_is_eof(e))) bad++;
                sum += len + (p && len ? p[0] : 0);
            }
            bytes[t] = sum;
            fails[t] = bad;
        });
    }
    for (auto& x : th) x.join();
    const double dt = now_s() - t0;
    uint64_t sum = 0, bad = 0;
    for (int t = 0; t < T; t++) {
        sum += bytes[t];
        bad += fails[t];
    }
    const double total = (double)K * T;
    printf("{\"mode\": \"%s\", \"threads\": %d, \"lookups\": %.0f, \"seconds\": %.6f, \"lookups_per_s\": %.1f, "
           "\"us_per_lookup_per_thread\": %.4f, \"first_call_ms\": %.3f, \"records\": %zu, \"failures\": %llu, "
           "\"checksum\": %llu}\n",
           seek ? "seek" : "at", T, total, dt, total / dt, dt * 1e6 * T / total, build_s * 1e3, offs.size(),
           (unsigned long long)bad, (unsigned long long)sum);
    (void)ro;
    rio_reader_free(r);
    rio_ctx_destroy(ctx);
    return bad ? 7 : 0;
}
