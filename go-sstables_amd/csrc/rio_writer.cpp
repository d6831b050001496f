// rio_writer.cpp — recordio v4 input generator (host C++). NOT on the decode path.
//
// Byte-identical to the reference FileWriter for v4 files:
//   fileHeaderAsByteSlice   recordio/file_writer.go:93-99
//   fillRecordHeaderV4      recordio/file_writer.go:160-176
//   FileWriter.Write        recordio/file_writer.go:189-233 (nil record => header only, c of the
//                           compressed nil payload still written into the header)
// Snappy payloads use a block encoder that follows golang/snappy v1.0.0 (encode.go,
// encode_other.go: emitLiteral / emitCopy / encodeBlock with the 1<<14 hash table and the
// skip heuristic), so files match the Go writer byte for byte (checked against the reference
// fixtures recordio_SnappyWriterMultiRecord_asc and _comp2 in tests/test_writer.py).
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "rio.h"

namespace {

// ------------------------------------------------------------------------------------------
// golang/snappy v1.0.0 encoder
// ------------------------------------------------------------------------------------------
constexpr int kMaxBlockSize = 65536;
constexpr int kInputMargin = 16 - 1;
constexpr int kMinNonLiteralBlockSize = 1 + 1 + kInputMargin;

inline uint32_t load32(const uint8_t* b, int i) {
    uint32_t v;
    memcpy(&v, b + i, 4);
    return v;
}
inline uint64_t load64(const uint8_t* b, int i) {
    uint64_t v;
    memcpy(&v, b + i, 8);
    return v;
}
inline uint32_t shash(uint32_t u, uint32_t shift) { return (u * 0x1e35a7bdu) >> shift; }

int emit_literal(uint8_t* dst, const uint8_t* lit, int n) {
    int i = 0;
    unsigned m = (unsigned)(n - 1);
    if (m < 60) {
        dst[0] = (uint8_t)(m << 2);
        i = 1;
    } else if (m < (1u << 8)) {
        dst[0] = 60 << 2;
        dst[1] = (uint8_t)m;
        i = 2;
    } else {
        dst[0] = 61 << 2;
        dst[1] = (uint8_t)m;
        dst[2] = (uint8_t)(m >> 8);
        i = 3;
    }
    memcpy(dst + i, lit, (size_t)n);
    return i + n;
}

int emit_copy(uint8_t* dst, int offset, int length) {
    int i = 0;
    while (length >= 68) {
        dst[i + 0] = 63 << 2 | 2;
        dst[i + 1] = (uint8_t)offset;
        dst[i + 2] = (uint8_t)(offset >> 8);
        i += 3;
        length -= 64;
    }
    if (length > 64) {
        dst[i + 0] = 59 << 2 | 2;
        dst[i + 1] = (uint8_t)offset;
        dst[i + 2] = (uint8_t)(offset >> 8);
        i += 3;
        length -= 60;
    }
    if (length >= 12 || offset >= 2048) {
        dst[i + 0] = (uint8_t)((length - 1) << 2 | 2);
        dst[i + 1] = (uint8_t)offset;
        dst[i + 2] = (uint8_t)(offset >> 8);
        return i + 3;
    }
    dst[i + 0] = (uint8_t)((offset >> 8) << 5 | (length - 4) << 2 | 1);
    dst[i + 1] = (uint8_t)offset;
    return i + 2;
}

int encode_block(uint8_t* dst, const uint8_t* src, int n) {
    constexpr int kMaxTable = 1 << 14;
    constexpr int kMask = kMaxTable - 1;
    uint32_t shift = 32 - 8;
    for (int ts = 1 << 8; ts < kMaxTable && ts < n; ts *= 2) shift--;
    static thread_local uint16_t table[kMaxTable];
    memset(table, 0, sizeof table);
    int d = 0;
    const int s_limit = n - kInputMargin;
    int next_emit = 0;
    int s = 1;
    uint32_t next_hash = shash(load32(src, s), shift);
    for (;;) {
        int skip = 32;
        int next_s = s;
        int candidate = 0;
        for (;;) {
            s = next_s;
            int between = skip >> 5;
            next_s = s + between;
            skip += between;
            if (next_s > s_limit) goto emit_remainder;
            candidate = table[next_hash & kMask];
            table[next_hash & kMask] = (uint16_t)s;
            next_hash = shash(load32(src, next_s), shift);
            if (load32(src, s) == load32(src, candidate)) break;
        }
        d += emit_literal(dst + d, src + next_emit, s - next_emit);
        for (;;) {
            int base = s;
            s += 4;
            for (int i = candidate + 4; s < n && src[i] == src[s]; i++, s++) {
            }
            d += emit_copy(dst + d, base - candidate, s - base);
            next_emit = s;
            if (s >= s_limit) goto emit_remainder;
            uint64_t x = load64(src, s - 1);
            uint32_t prev_hash = shash((uint32_t)(x >> 0), shift);
            table[prev_hash & kMask] = (uint16_t)(s - 1);
            uint32_t curr_hash = shash((uint32_t)(x >> 8), shift);
            candidate = table[curr_hash & kMask];
            table[curr_hash & kMask] = (uint16_t)s;
            if ((uint32_t)(x >> 8) != load32(src, candidate)) {
                next_hash = shash((uint32_t)(x >> 16), shift);
                s++;
                break;
            }
        }
    }
emit_remainder:
    if (next_emit < n) d += emit_literal(dst + d, src + next_emit, n - next_emit);
    return d;
}

int put_uvarint(uint8_t* b, uint64_t v) {
    int i = 0;
    while (v >= 0x80) {
        b[i++] = (uint8_t)(v | 0x80);
        v >>= 7;
    }
    b[i++] = (uint8_t)v;
    return i;
}

// CRC-32C (host copy for header emission; the decode-side CRC runs on the device)
struct CrcTab {
    uint32_t t[256];
    CrcTab() {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
            t[i] = c;
        }
    }
};
const CrcTab kCrc;
uint32_t crc32c(const uint8_t* p, size_t n) {
    uint32_t c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; i++) c = kCrc.t[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return c ^ 0xFFFFFFFFu;
}

// gzip payloads (GzipCompressor.Compress, gzip_compression.go:13-41) via zlib; the byte stream
// differs from Go's compress/gzip but decodes to the same record.
uint64_t gzip_encode(std::vector<uint8_t>& out, const uint8_t* src, uint64_t n) {
    z_stream z;
    memset(&z, 0, sizeof z);
    deflateInit2(&z, Z_DEFAULT_COMPRESSION, Z_DEFLATED, 16 + 15, 8, Z_DEFAULT_STRATEGY);
    out.resize(deflateBound(&z, (uLong)n) + 32);
    z.next_in = (Bytef*)src;
    z.avail_in = (uInt)n;
    z.next_out = out.data();
    z.avail_out = (uInt)out.size();
    deflate(&z, Z_FINISH);
    uint64_t len = out.size() - z.avail_out;
    deflateEnd(&z);
    out.resize(len);
    return len;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// C-ABI: encoder primitives
// ------------------------------------------------------------------------------------------
extern "C" uint64_t rio_snappy_max_encoded_len(uint64_t n) { return 32 + n + n / 6; }

extern "C" uint64_t rio_snappy_encode(uint8_t* dst, uint64_t dst_cap, const uint8_t* src, uint64_t n) {
    if (dst_cap < rio_snappy_max_encoded_len(n)) return 0;
    uint64_t d = (uint64_t)put_uvarint(dst, n);
    while (n > 0) {
        int blk = (int)std::min<uint64_t>(n, kMaxBlockSize);
        if (blk < kMinNonLiteralBlockSize)
            d += (uint64_t)emit_literal(dst + d, src, blk);
        else
            d += (uint64_t)encode_block(dst + d, src, blk);
        src += blk;
        n -= (uint64_t)blk;
    }
    return d;
}

extern "C" void rio_encode_file_header(uint8_t* buf8, uint32_t version, uint32_t compression) {
    for (int i = 0; i < 4; i++) buf8[i] = (uint8_t)(version >> (8 * i));
    for (int i = 0; i < 4; i++) buf8[4 + i] = (uint8_t)(compression >> (8 * i));
}

// LzwCompressor.Compress (lzw_compressor.go:12-26): Go compress/lzw Writer, LSB bit order, litWidth 8,
// one Write + Close. A leading clear code, codes of 9..12 bits (the width grows when the next code
// reaches 512 / 1024 / 2048), a clear code and a reset when the next code would be 4095, then the
// pending code and the eof code. The dictionary (prefix code, byte) -> code is an open-addressed
// table whose entries carry a generation, so a reset or a new record costs no clearing.
namespace {
struct LzwDict {
    static constexpr uint32_t kSize = 1u << 14, kMask = kSize - 1;
    std::vector<uint32_t> key = std::vector<uint32_t>(kSize), gen = std::vector<uint32_t>(kSize, 0);
    std::vector<uint16_t> code = std::vector<uint16_t>(kSize);
    uint32_t cur = 0;
    void reset() { cur++; }
    int find(uint32_t k) const {
        for (uint32_t h = (k >> 12 ^ k) & kMask;; h = (h + 1) & kMask) {
            if (gen[h] != cur) return -1;
            if (key[h] == k) return code[h];
        }
    }
    void put(uint32_t k, uint32_t c) {
        uint32_t h = (k >> 12 ^ k) & kMask;
        while (gen[h] == cur) h = (h + 1) & kMask;
        gen[h] = cur;
        key[h] = k;
        code[h] = (uint16_t)c;
    }
};
}  // namespace

static uint64_t lzw_encode(std::vector<uint8_t>& out, const uint8_t* src, uint64_t n) {
    thread_local LzwDict D;
    constexpr uint32_t kClear = 256, kEof = 257, kMaxCode = 4095;
    out.clear();
    out.reserve(2 * n + 16);
    uint32_t bits = 0, nbits = 0, width = 9, hi = kEof, overflow = 512;
    auto put = [&](uint32_t c) {
        bits |= c << nbits;
        nbits += width;
        for (; nbits >= 8; nbits -= 8, bits >>= 8) out.push_back((uint8_t)bits);
    };
    auto inc_hi = [&]() {  // true: out of codes, the dictionary was reset
        if (++hi == overflow) {
            width++;
            overflow <<= 1;
        }
        if (hi != kMaxCode) return false;
        put(kClear);
        width = 9;
        hi = kEof;
        overflow = 512;
        D.reset();
        return true;
    };
    D.reset();
    if (n == 0) {
        put(kClear);
    } else {
        put(kClear);
        uint32_t cur = src[0];
        for (uint64_t i = 1; i < n; i++) {
            const uint32_t k = cur << 8 | src[i];
            const int hit = D.find(k);
            if (hit >= 0) {
                cur = (uint32_t)hit;
                continue;
            }
            put(cur);
            cur = src[i];
            if (!inc_hi()) D.put(k, hi);
        }
        put(cur);
        inc_hi();
    }
    put(kEof);
    if (nbits) out.push_back((uint8_t)bits);
    return out.size();
}

extern "C" uint64_t rio_encode_record_v4(uint8_t* buf, uint64_t cap, uint32_t compression,
                                         const uint8_t* record, uint64_t len) {
    const bool nil = (record == nullptr);
    uint64_t u = nil ? 0 : len;
    uint64_t c = 0;
    std::vector<uint8_t> comp;
    const uint8_t* payload = record;
    uint64_t plen = u;
    if (compression == RIO_COMP_SNAPPY) {
        comp.resize(rio_snappy_max_encoded_len(u));
        c = rio_snappy_encode(comp.data(), comp.size(), record ? record : (const uint8_t*)"", u);
        payload = comp.data();
        plen = c;
    } else if (compression == RIO_COMP_GZIP) {
        c = gzip_encode(comp, record ? record : (const uint8_t*)"", u);
        payload = comp.data();
        plen = c;
    } else if (compression == RIO_COMP_LZW) {
        c = lzw_encode(comp, record ? record : (const uint8_t*)"", u);
        payload = comp.data();
        plen = c;
    } else if (compression != RIO_COMP_NONE) {
        return 0;
    }
    uint8_t hdr[RIO_RECORD_HEADER_V4_MAX];
    int off = put_uvarint(hdr, RIO_MAGIC);
    hdr[off++] = nil ? 1 : 0;
    off += put_uvarint(hdr + off, u);
    off += put_uvarint(hdr + off, c);
    off += put_uvarint(hdr + off, crc32c(hdr, (size_t)off));
    uint64_t total = (uint64_t)off + (nil ? 0 : plen);
    if (total > cap) return 0;
    memcpy(buf, hdr, (size_t)off);
    if (!nil && plen) memcpy(buf + off, payload, (size_t)plen);
    return total;
}

// ------------------------------------------------------------------------------------------
// C-ABI: FileWriter-like streaming writer
// ------------------------------------------------------------------------------------------
struct rio_writer {
    FILE* f = nullptr;
    uint32_t compression = 0;
    uint64_t offset = 0;
    std::vector<uint8_t> buf;
};

extern "C" int rio_writer_new(const char* path, uint32_t compression, rio_writer** out) {
    if (!path || !out || compression > RIO_COMP_LZW) return RIO_ERR_ARG;
    FILE* f = fopen(path, "wb");
    if (!f) return RIO_ERR_IO;
    auto* w = new rio_writer();
    w->f = f;
    w->compression = compression;
    uint8_t h[8];
    rio_encode_file_header(h, RIO_VERSION4, compression);
    fwrite(h, 1, 8, f);
    w->offset = 8;
    *out = w;
    return RIO_OK;
}

extern "C" int rio_writer_write(rio_writer* w, const uint8_t* record, uint64_t len, uint64_t* offset) {
    if (!w || !w->f) return RIO_ERR_STATE;
    uint64_t bound = RIO_RECORD_HEADER_V4_MAX + rio_snappy_max_encoded_len(len) + len + 128;  // (lzw: <= 1.5 len)
    if (w->buf.size() < bound) w->buf.resize(bound);
    uint64_t n = rio_encode_record_v4(w->buf.data(), w->buf.size(), w->compression, record, len);
    if (n == 0) return RIO_ERR_CAPACITY;
    if (fwrite(w->buf.data(), 1, n, w->f) != n) return RIO_ERR_IO;
    if (offset) *offset = w->offset;
    w->offset += n;
    return RIO_OK;
}

extern "C" uint64_t rio_writer_size(rio_writer* w) { return w ? w->offset : 0; }

extern "C" int rio_writer_close(rio_writer* w) {
    if (!w) return RIO_ERR_ARG;
    int rc = RIO_OK;
    if (w->f && fclose(w->f) != 0) rc = RIO_ERR_IO;
    delete w;
    return rc;
}

// ------------------------------------------------------------------------------------------
// Synthetic workloads (BASELINE.json configs)
// ------------------------------------------------------------------------------------------
namespace {

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x2545F4914F6CDD1Dull) {
        if (!s) s = 1;
    }
    uint64_t next() {  // xorshift64*
        s ^= s >> 12;
        s ^= s << 25;
        s ^= s >> 27;
        return s * 0x2545F4914F6CDD1Dull;
    }
    uint32_t below(uint32_t n) { return (uint32_t)((next() >> 32) * (uint64_t)n >> 32); }
};

// text-like: 4096-word seeded vocabulary (3..10 lowercase letters), Zipf(1.4) word choice (snappy ratio ~0.55 at 1 KiB)
struct Vocab {
    std::vector<std::string> words;
    std::vector<double> cdf;
    Vocab(uint64_t seed) {
        Rng r(seed ^ 0xC0FFEEull);
        words.resize(4096);
        for (auto& w : words) {
            int l = 3 + (int)r.below(8);
            w.resize((size_t)l);
            for (auto& ch : w) ch = (char)('a' + r.below(26));
        }
        cdf.resize(words.size());
        double acc = 0;
        for (size_t i = 0; i < words.size(); i++) {
            acc += 1.0 / std::pow((double)(i + 1), 1.4);
            cdf[i] = acc;
        }
        for (auto& c : cdf) c /= acc;
    }
    const std::string& pick(Rng& r) const {
        double u = (double)(r.next() >> 11) * (1.0 / 9007199254740992.0);
        size_t i = (size_t)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
        return words[std::min(i, words.size() - 1)];
    }
};

void make_record(std::vector<uint8_t>& rec, uint64_t len, int kind, uint64_t seed, uint64_t idx,
                 const Vocab* vocab, const std::vector<uint8_t>& shared) {
    rec.resize(len);
    if (kind == 0) {
        memcpy(rec.data(), shared.data(), len);
        return;
    }
    Rng r(seed * 1000003ull + idx * 0x9E3779B97F4A7C15ull + 17);
    if (kind == 2) {
        for (uint64_t i = 0; i < len; i++) rec[i] = (uint8_t)r.below(255);
        return;
    }
    uint64_t o = 0;
    while (o < len) {
        const std::string& w = vocab->pick(r);
        for (size_t k = 0; k < w.size() && o < len; k++) rec[o++] = (uint8_t)w[k];
        if (o < len) rec[o++] = ' ';
    }
}

}  // namespace

extern "C" uint64_t rio_generate_bound(uint32_t compression, uint64_t n_records, uint64_t record_len) {
    uint64_t per = RIO_RECORD_HEADER_V4_MAX + record_len;
    if (compression == RIO_COMP_SNAPPY) per = RIO_RECORD_HEADER_V4_MAX + rio_snappy_max_encoded_len(record_len);
    if (compression == RIO_COMP_GZIP) per = RIO_RECORD_HEADER_V4_MAX + record_len + record_len / 100 + 64;
    if (compression == RIO_COMP_LZW) per = RIO_RECORD_HEADER_V4_MAX + 2 * record_len + 16;
    return 8 + n_records * per;
}

extern "C" uint64_t rio_generate(uint8_t* buf, uint64_t cap, uint32_t compression, uint64_t n_records,
                                 uint64_t record_len, int kind, uint64_t seed, int threads) {
    if (cap < 8 || kind < 0 || kind > 2) return 0;
    rio_encode_file_header(buf, RIO_VERSION4, compression);
    std::vector<uint8_t> shared;
    if (kind == 0) {  // one record of rand.Intn(255) bytes, reused (benchmark/recordio_read_test.go:32)
        Rng r(seed);
        shared.resize(record_len);
        for (auto& b : shared) b = (uint8_t)r.below(255);
    }
    Vocab vocab(seed);
    if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    threads = (int)std::min<uint64_t>((uint64_t)threads, std::max<uint64_t>(1, n_records / 64));
    std::vector<std::vector<uint8_t>> parts((size_t)threads);
    std::vector<int> fail((size_t)threads, 0);
    auto work = [&](int t) {
        uint64_t lo = n_records * (uint64_t)t / (uint64_t)threads;
        uint64_t hi = n_records * (uint64_t)(t + 1) / (uint64_t)threads;
        auto& out = parts[(size_t)t];
        uint64_t per = rio_generate_bound(compression, 1, record_len) - 8;
        out.resize(per * (hi - lo));
        uint64_t o = 0;
        std::vector<uint8_t> rec;
        for (uint64_t i = lo; i < hi; i++) {
            make_record(rec, record_len, kind, seed, i, &vocab, shared);
            uint64_t n = rio_encode_record_v4(out.data() + o, out.size() - o, compression, rec.data(), record_len);
            if (!n) { fail[(size_t)t] = 1; return; }
            o += n;
        }
        out.resize(o);
    };
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) th.emplace_back(work, t);
    for (auto& x : th) x.join();
    uint64_t o = 8;
    for (int t = 0; t < threads; t++) {
        if (fail[(size_t)t] || o + parts[(size_t)t].size() > cap) return 0;
        memcpy(buf + o, parts[(size_t)t].data(), parts[(size_t)t].size());
        o += parts[(size_t)t].size();
    }
    return o;
}
