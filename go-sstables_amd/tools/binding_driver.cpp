// binding_driver — the Go adapter's exact call sequence (rocmFileReader) in C++,
// so the binding can be tested without a Go toolchain: a context from the pool (rio_ctx_acquire),
// the file read into memory, rio_frame (open-time errors), caller-sized arrays, rio_decode, then
// ReadNext / SkipNext served from the arrays with the flag-to-error mapping the Go code applies:
//
//   ReadNext  (recordio/file_reader.go:61-131): record i, nil for RIO_FLAG_NIL, the codec's error
//             returned as is for RIO_FLAG_CORRUPT, a bare io.EOF for RIO_FLAG_EOF; after the last
//             record the terminal status with the reference's wrapping (terminal()).
//   SkipNext  (recordio/file_reader.go:133-172): never decompresses, so record i (flagged or not) is
//             passed over with nil; at the end it reports what readRecordHeaderV4 would: a zero tail
//             is a magic mismatch (SkipNext does not test for zeros), a payload cut short or a
//             truncated-payload status is skipped once (the seek succeeds) and io.EOF follows.
//
//   rio_binding_driver <file> <ops> [<file> <ops> ...]
//       ops: a string of R (ReadNext) / S (SkipNext); a trailing '*' repeats the last op until it
//       returns an error. Each pair opens its own reader (Open, the ops, Close) in one process.
// Prints "== <k>" before pair k, then one line per op: "R rec <len> <fnv1a64>", "R nil", "S nil", or
// "<op> err <class>" where class is eof_wrapped | eof | unexpected_eof | magic |
// header_crc:<exp>:<got> | corrupt:<codec> | version:<n> | comptype:<n> | rio:<status>. Open errors
// print "O err <class>".
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rio.h"

namespace {

const char* codec_name(uint32_t c) {
    switch (c) {
    case RIO_COMP_SNAPPY: return "snappy";  // snappy.ErrCorrupt (snappy_compression.go:22-24)
    case RIO_COMP_GZIP: return "gzip";      // the compress/gzip reader's error
    case RIO_COMP_LZW: return "lzw";        // the compress/lzw reader's error
    default: return "none";
    }
}

// terminal(): the device status -> the reference's error and wrap depth
std::string terminal(const rio_file_info& fi, int st) {
    char b[96];
    switch (st) {
    case RIO_EOF:
    case RIO_EOF_HEADER:
    case RIO_EOF_PAYLOAD: return "eof_wrapped";  // fmt.Errorf("...: %w", io.EOF)
    case RIO_EOF_ZERO_TAIL: return "eof";         // bare io.EOF (file_reader.go:90)
    case RIO_ERR_UNEXPECTED_EOF: return "unexpected_eof";
    case RIO_ERR_MAGIC: return "magic";
    case RIO_ERR_HEADER_CRC:
        snprintf(b, sizeof b, "header_crc:%llx:%llx", (unsigned long long)fi.detail0, (unsigned long long)fi.detail1);
        return b;
    default: snprintf(b, sizeof b, "rio:%d", st); return b;
    }
}

uint64_t fnv1a(const uint8_t* p, uint64_t n) {
    uint64_t h = 1469598103934665603ull;
    for (uint64_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}

// rocmFileReader
struct Reader {
    rio_ctx* ctx = nullptr;
    rio_file_info info{};
    std::vector<uint8_t> out, flags;
    std::vector<uint64_t> out_off, rec_off;
    uint64_t next = 0;
    bool past_end = false;  // SkipNext passed a record whose payload is cut short

    // Open: returns "" or the open error's class
    std::string open(const std::vector<uint8_t>& data) {
        if (int rc = rio_ctx_acquire(0, &ctx)) return "rio:" + std::to_string(rc);
        if (int rc = rio_frame(ctx, data.data(), data.size(), &info)) return "rio:" + std::to_string(rc);
        switch (info.status) {  // open-time errors keep the reference's messages (file_reader.go:36-48)
        case RIO_ERR_VERSION: return "version:" + std::to_string(info.detail0);
        case RIO_ERR_COMPRESSION_TYPE: return "comptype:" + std::to_string(info.detail0);
        case RIO_ERR_SHORT_FILE_HEADER:  // io.ReadFull of the 8-byte header (file_reader.go:37-40)
            return data.empty() ? "eof_wrapped" : "unexpected_eof";
        case RIO_ERR_UNSUPPORTED: return "rio:" + std::to_string(RIO_ERR_UNSUPPORTED);  // pure-Go reader
        }
        const uint64_t n = info.n_records;
        out.assign(info.total_out_bytes + 1, 0);
        out_off.assign(n + 1, 0);
        rec_off.assign(n + 1, 0);
        flags.assign(n + 1, 0);
        if (int rc = rio_decode(ctx, out.data(), info.total_out_bytes, out_off.data(), rec_off.data(), flags.data(), n,
                                &info))
            return "rio:" + std::to_string(rc);
        return "";
    }

    std::string read_next() {
        char b[96];
        if (past_end) return "err eof_wrapped";  // after SkipNext passed a cut payload
        if (next < info.n_records) {
            const uint64_t i = next++;
            if (flags[i] & RIO_FLAG_NIL) return "nil";
            if (flags[i] & RIO_FLAG_CORRUPT) return std::string("err corrupt:") + codec_name(info.compression);
            if (flags[i] & RIO_FLAG_EOF) return "err eof";
            const uint64_t a = out_off[i], e = out_off[i + 1];
            snprintf(b, sizeof b, "rec %llu %016llx", (unsigned long long)(e - a),
                     (unsigned long long)fnv1a(out.data() + a, e - a));
            return b;
        }
        return "err " + terminal(info, info.status);
    }

    std::string skip_next() {
        if (past_end) return "err eof_wrapped";
        if (next < info.n_records) {
            next++;
            return "nil";
        }
        switch (info.status) {
        case RIO_EOF_ZERO_TAIL: return "err magic";  // SkipNext does not test for a zero tail
        case RIO_ERR_UNEXPECTED_EOF:  // detail0 == 1: raised by the payload read, not a header varint
            if (info.detail0 != 1) return "err " + terminal(info, info.status);
            [[fallthrough]];
        case RIO_EOF_PAYLOAD:
            // the header parsed: SkipNext seeks past the payload without reading it
            past_end = true;
            return "nil";
        default: return "err " + terminal(info, info.status);
        }
    }

    ~Reader() {
        if (ctx) rio_ctx_release(ctx);
    }
};

}  // namespace

// one reader over one file: Open, the ops, Close (the context goes back to the pool)
static int run_pair(const char* path, std::string ops) {
    FILE* f = fopen(path, "rb");
    if (!f) return 3;
    std::vector<uint8_t> data;
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) data.insert(data.end(), buf, buf + k);
    fclose(f);
    Reader r;
    const std::string oerr = r.open(data);
    if (!oerr.empty()) {
        printf("O err %s\n", oerr.c_str());
        return 0;
    }
    const bool repeat = !ops.empty() && ops.back() == '*';
    if (repeat) ops.pop_back();
    auto run = [&](char op) {
        const std::string res = op == 'S' ? r.skip_next() : r.read_next();
        printf("%c %s\n", op, res.c_str());
        return res.rfind("err", 0) != 0;
    };
    for (char op : ops) run(op);
    if (repeat && !ops.empty())
        for (uint64_t guard = 0; guard < (1ull << 32) && run(ops.back()); guard++) {
        }
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 3 || (argc - 1) % 2) {
        fprintf(stderr, "usage: %s <file> <ops> [<file> <ops> ...]\n", argv[0]);
        return 2;
    }
    for (int i = 1; i + 1 < argc; i += 2) {
        printf("== %d\n", (i - 1) / 2);
        if (int rc = run_pair(argv[i], argv[i + 1])) return rc;
    }
    return 0;
}
