// rio_encode.hip — recordio v4 file encoding on the device (the write side):
// FileWriter.Write (recordio/file_writer.go:189-233) for a batch of records, byte-identical to the
// reference writer: per record the Snappy block encoding of golang/snappy v1.0.0 (encode.go,
// encode_other.go: emitLiteral, emitCopy, encodeBlock with its table size, hash and skip rule;
// 64 KiB blocks after a uvarint length), then the v4 header (fillRecordHeaderV4, :160-176: magic,
// nil byte, uvarint u, uvarint c, uvarint CRC-32C of the preceding header bytes) and the payload at
// the record's file offset (the running sum of the record sizes, which Write returns).
//
// k_snappy_encode_lds    one lane per record of at most 1 KiB: the hash table (<= 1024 uint16
//                        entries) sits in LDS laid out [hash][64 virtual lanes], which spreads the
//                        lanes over the 64 banks whatever hashes they hold; 32 KiB per group of 16
//                        records, run as 4 waves of 4 active lanes (more instruction streams).
// k_snappy_encode_global one lane per larger record: table in a per-lane slot of global scratch
//                        (16384 entries, reset per 64 KiB block).
// k_enc_sizes             per record: header bytes (into a 64-B slot) and the record's file size.
// k_enc_emit              16 lanes per record copy header + payload to the file offset from the
//                         exclusive scan (hipCUB) of the sizes; lane 0 writes the 8-byte file header.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "rio_device.h"
#include "rio_dev_util.h"

namespace rio {

namespace {
constexpr uint32_t kMaxBlock = 65536;
constexpr int kInputMargin = 16 - 1;
constexpr int kMinNonLiteralBlock = 1 + 1 + kInputMargin;
constexpr uint32_t kMaxTable = 1u << 14;
constexpr uint32_t kLdsTable = 1024;  // records up to 1 KiB use the LDS table
constexpr uint32_t kHdrSlot = 64;
// global table slot: kMaxTable entries + 64 (128 B) so that the slots of a group do not all start
// on the same L2 set
constexpr uint32_t kTabSlot = kMaxTable + 64;

typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint64_t __attribute__((aligned(1))) u64u;
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const u32u*>(p); }
__device__ __forceinline__ uint64_t ld64(const uint8_t* p) { return *reinterpret_cast<const u64u*>(p); }
__device__ __forceinline__ uint32_t shash(uint32_t u, uint32_t shift) { return (u * 0x1e35a7bdu) >> shift; }

// golang/snappy's bound (encode.go MaxEncodedLen) plus 16 bytes of slack for the 16-byte literal copies
__host__ __device__ __forceinline__ uint64_t enc_bound(uint64_t n) { return 32 + n + n / 6 + 16; }

__device__ __forceinline__ uint32_t put_uvarint(uint8_t* b, uint64_t v) {
    uint32_t i = 0;
    while (v >= 0x80) {
        b[i++] = (uint8_t)(v | 0x80);
        v >>= 7;
    }
    b[i++] = (uint8_t)v;
    return i;
}

// literal bytes in 16-byte pieces; may write up to 15 bytes past the literal (scratch slack) and
// read up to 15 past the source (RIO_DEVICE_PAD past the records arena)
__device__ __forceinline__ uint32_t emit_literal(uint8_t* dst, const uint8_t* lit, uint32_t n) {
    uint32_t i;
    const uint32_t m = n - 1;
    if (m < 60) {
        dst[0] = (uint8_t)(m << 2);
        i = 1;
    } else if (m < 256) {
        dst[0] = 60 << 2;
        dst[1] = (uint8_t)m;
        i = 2;
    } else {
        dst[0] = 61 << 2;
        dst[1] = (uint8_t)m;
        dst[2] = (uint8_t)(m >> 8);
        i = 3;
    }
    for (uint32_t k = 0; k < n; k += 16) stu16(dst + i + k, ldu16(lit + k));
    return i + n;
}

__device__ __forceinline__ uint32_t emit_copy(uint8_t* dst, uint32_t offset, uint32_t length) {
    uint32_t i = 0;
    while (length >= 68) {
        dst[i] = 63 << 2 | 2;
        dst[i + 1] = (uint8_t)offset;
        dst[i + 2] = (uint8_t)(offset >> 8);
        i += 3;
        length -= 64;
    }
    if (length > 64) {
        dst[i] = 59 << 2 | 2;
        dst[i + 1] = (uint8_t)offset;
        dst[i + 2] = (uint8_t)(offset >> 8);
        i += 3;
        length -= 60;
    }
    if (length >= 12 || offset >= 2048) {
        dst[i] = (uint8_t)((length - 1) << 2 | 2);
        dst[i + 1] = (uint8_t)offset;
        dst[i + 2] = (uint8_t)(offset >> 8);
        return i + 3;
    }
    dst[i] = (uint8_t)((offset >> 8) << 5 | (length - 4) << 2 | 1);
    dst[i + 1] = (uint8_t)offset;
    return i + 2;
}

// hash table views: LDS [hash][lane] or a global per-lane slot
template <int kRecs>
struct LdsTable {
    uint16_t* t;
    uint32_t lane;
    __device__ __forceinline__ uint32_t get(uint32_t h) const { return t[h * kRecs + lane]; }
    __device__ __forceinline__ void put(uint32_t h, uint32_t v) const { t[h * kRecs + lane] = (uint16_t)v; }
};
struct GlobalTable {
    uint16_t* t;
    __device__ __forceinline__ uint32_t get(uint32_t h) const { return t[h]; }
    __device__ __forceinline__ void put(uint32_t h, uint32_t v) const { t[h] = (uint16_t)v; }
};

// encodeBlock (encode_other.go) of src[0, n), 17 <= n <= 65536; returns the bytes written
template <class Table>
__device__ uint32_t encode_block(uint8_t* dst, const uint8_t* src, int n, const Table& tab) {
    uint32_t shift = 32 - 8, ts = 1u << 8;
    for (; ts < kMaxTable && (int)ts < n; ts *= 2) shift--;
    for (uint32_t h = 0; h < ts; h++) tab.put(h, 0);
    uint32_t d = 0;
    const int s_limit = n - kInputMargin;
    int next_emit = 0, s = 1;
    uint32_t next_hash = shash(ld32(src + s), shift);
    for (;;) {
        int skip = 32, next_s = s, candidate = 0;
        for (;;) {
            s = next_s;
            const int between = skip >> 5;
            next_s = s + between;
            skip += between;
            if (next_s > s_limit) goto emit_remainder;
            candidate = (int)tab.get(next_hash);
            tab.put(next_hash, (uint32_t)s);
            next_hash = shash(ld32(src + next_s), shift);
            if (ld32(src + s) == ld32(src + candidate)) break;
        }
        d += emit_literal(dst + d, src + next_emit, (uint32_t)(s - next_emit));
        for (;;) {
            const int base = s;
            // extend the 4-byte match: first differing byte, 8 bytes per compare
            int i = candidate + 4;
            s += 4;
            while (s + 8 <= n) {
                const uint64_t x = ld64(src + i) ^ ld64(src + s);
                if (x) {
                    s += __builtin_ctzll(x) >> 3;
                    goto extended;
                }
                i += 8;
                s += 8;
            }
            while (s < n && src[i] == src[s]) {
                i++;
                s++;
            }
        extended:
            d += emit_copy(dst + d, (uint32_t)(base - candidate), (uint32_t)(s - base));
            next_emit = s;
            if (s >= s_limit) goto emit_remainder;
            const uint64_t x = ld64(src + s - 1);
            const uint32_t prev_hash = shash((uint32_t)x, shift);
            tab.put(prev_hash, (uint32_t)(s - 1));
            const uint32_t curr_hash = shash((uint32_t)(x >> 8), shift);
            candidate = (int)tab.get(curr_hash);
            tab.put(curr_hash, (uint32_t)s);
            if ((uint32_t)(x >> 8) != ld32(src + candidate)) {
                next_hash = shash((uint32_t)(x >> 16), shift);
                s++;
                break;
            }
        }
    }
emit_remainder:
    if (next_emit < n) d += emit_literal(dst + d, src + next_emit, (uint32_t)(n - next_emit));
    return d;
}

// snappy.Encode (encode.go:18-41): uvarint length, then 64 KiB blocks
template <class Table>
__device__ uint64_t snappy_encode(uint8_t* dst, const uint8_t* src, uint64_t n, const Table& tab) {
    uint64_t d = put_uvarint(dst, n);
    while (n > 0) {
        const uint32_t blk = n < kMaxBlock ? (uint32_t)n : kMaxBlock;
        if ((int)blk < kMinNonLiteralBlock)
            d += emit_literal(dst + d, src, blk);
        else
            d += encode_block(dst + d, src, (int)blk, tab);
        src += blk;
        n -= blk;
    }
    return d;
}

__device__ uint32_t crc32c_bytes(const uint8_t* p, uint32_t n) {
    uint32_t c = ~0u;
    for (uint32_t k = 0; k < n; k++) {
        c ^= p[k];
        for (int b = 0; b < 8; b++) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    }
    return ~c;
}
}  // namespace



__global__ void __launch_bounds__(256) k_enc_bounds(EncParams P) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= P.n; i += stride) {
        const uint64_t u = i < P.n ? P.rec_off[i + 1] - P.rec_off[i] : 0;
        P.tmp[i] = (i < P.n && P.compression == RIO_COMP_SNAPPY) ? enc_bound(u) : 0;
    }
}

// kRecs records per group share one LDS table image [hash][kRecs] (virtual lane = wave * kLanes +
// lane; bank-conflict-free for kRecs / 2 dividing the 64 banks); kLanes active lanes per wave, so
// fewer lanes per wave give the CU more independent instruction streams over the same table bytes.
template <int kRecs, int kLanes>
__global__ void __launch_bounds__(64 * (kRecs / kLanes)) k_snappy_encode_lds(EncParams P) {
    __shared__ uint16_t lds_tab[kLdsTable * kRecs];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane >= (uint32_t)kLanes) return;
    const uint32_t vlane = wave * kLanes + lane;
    const uint64_t stride = (uint64_t)gridDim.x * kRecs;
    for (uint64_t i = (uint64_t)blockIdx.x * kRecs + vlane; i < P.n; i += stride) {
        const uint64_t u = P.rec_off[i + 1] - P.rec_off[i];
        if (u > kLdsTable) continue;
        const bool nil = P.flags && (P.flags[i] & RIO_FLAG_NIL);
        const LdsTable<kRecs> t{lds_tab, vlane};
        P.clen[i] = snappy_encode(P.scratch + P.scr_off[i], P.rec + P.rec_off[i], nil ? 0 : u, t);
    }
}

// records the LDS kernel does not take (larger than 1 KiB, or all of them when lds_small == 0)
__global__ void __launch_bounds__(64) k_snappy_encode_global(EncParams P) {
    const uint64_t slot = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * 64;
    for (uint64_t i = slot; i < P.n; i += stride) {
        const uint64_t u = P.rec_off[i + 1] - P.rec_off[i];
        if (P.lds_small && u <= kLdsTable) continue;
        const bool nil = P.flags && (P.flags[i] & RIO_FLAG_NIL);
        const GlobalTable t{P.gtab + slot * kTabSlot};
        P.clen[i] = snappy_encode(P.scratch + P.scr_off[i], P.rec + P.rec_off[i], nil ? 0 : u, t);
    }
}

__global__ void __launch_bounds__(256) k_enc_sizes(EncParams P) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= P.n; i += stride) {
        if (i == P.n) {
            P.tmp[i] = 0;
            continue;
        }
        const bool nil = P.flags && (P.flags[i] & RIO_FLAG_NIL);
        const uint64_t u = nil ? 0 : P.rec_off[i + 1] - P.rec_off[i];
        const uint64_t c = P.compression == RIO_COMP_SNAPPY ? P.clen[i] : 0;
        uint8_t* h = P.hdr + i * kHdrSlot;
        uint32_t k = put_uvarint(h, RIO_MAGIC);
        h[k++] = nil ? 1 : 0;
        k += put_uvarint(h + k, u);
        k += put_uvarint(h + k, c);
        k += put_uvarint(h + k, crc32c_bytes(h, k));
        h[kHdrSlot - 1] = (uint8_t)k;
        const uint64_t plen = nil ? 0 : (P.compression == RIO_COMP_SNAPPY ? c : u);
        P.tmp[i] = k + plen;
    }
}

__global__ void __launch_bounds__(256) k_enc_emit(EncParams P) {
    const uint64_t total = 8 + P.size[P.n];  // size[] now holds the exclusive scan, size[n] = sum
    if (blockIdx.x == 0 && threadIdx.x == 0) *P.out_len = total;
    if (total > P.out_cap) return;  // the host reports RIO_ERR_CAPACITY from out_len
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const uint8_t fh[8] = {RIO_VERSION4, 0, 0, 0, (uint8_t)P.compression, 0, 0, 0};
        for (int b = 0; b < 8; b++) P.out[b] = fh[b];
    }
    const uint32_t lane = threadIdx.x & 15;
    const uint64_t grp = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const uint64_t ngrp = ((uint64_t)gridDim.x * blockDim.x) >> 4;
    for (uint64_t i = grp; i < P.n; i += ngrp) {
        const uint64_t o = 8 + P.size[i];
        const uint8_t* hs = P.hdr + i * kHdrSlot;
        const uint32_t hl = hs[kHdrSlot - 1];
        if (lane == 0) P.out_rec_off[i] = o;
        for (uint32_t b = lane; b < hl; b += 16) P.out[o + b] = hs[b];
        const uint64_t plen = P.size[i + 1] - P.size[i] - hl;
        if (!plen) continue;
        const uint8_t* src = P.compression == RIO_COMP_SNAPPY ? P.scratch + P.scr_off[i] : P.rec + P.rec_off[i];
        uint8_t* dst = P.out + o + hl;
        for (uint64_t k = 16 * lane; k < plen; k += 256) {
            const uint4 v = ldu16(src + k);
            if (k + 16 <= plen)
                stu16(dst + k, v);
            else
                st_partial(dst + k, v, (uint32_t)(plen - k));
        }
    }
}

// scratch sizes for n records of `bytes` total (host side, before any launch)
uint64_t enc_scratch_bytes(uint64_t n, uint64_t bytes, uint32_t compression) {
    return compression == RIO_COMP_SNAPPY ? 48 * n + bytes + bytes / 6 + 64 : 64;
}

// k_snappy_encode<false>: groups x 64 lanes, a 32 KiB table slot each. RIO_ENC_GROUPS / RIO_ENC_LDS
// (0 = every record on the global-table kernel) are tuning knobs read once.
static uint32_t enc_groups() {
    static const uint32_t g = [] {
        const char* v = getenv("RIO_ENC_GROUPS");
        const long x = v ? strtol(v, nullptr, 0) : 0;
        return x > 0 && x <= 16384 ? (uint32_t)x : 128u;
    }();
    return g;
}
static bool enc_lds() {
    static const bool b = [] {
        const char* v = getenv("RIO_ENC_LDS");
        return !(v && v[0] == '0');
    }();
    return b;
}

static int enc_lanes() {
    static const int l = [] {
        const char* v = getenv("RIO_ENC_LANES");
        return v ? atoi(v) : 16;
    }();
    return l;
}

uint64_t enc_table_bytes() { return (uint64_t)enc_groups() * 64 * kTabSlot * 2; }

hipError_t launch_encode(const EncParams& P0, void* cub_tmp, size_t cub_bytes, hipStream_t s) {
    EncParams P = P0;
    const uint64_t n = P.n;
    const unsigned g = (unsigned)std::min<uint64_t>((n + 256) / 256 + 1, 4096);
    if (P.compression == RIO_COMP_SNAPPY) {
        hipLaunchKernelGGL(k_enc_bounds, dim3(g), dim3(256), 0, s, P);
        size_t tb = cub_bytes;
        hipError_t e = hipcub::DeviceScan::ExclusiveSum(cub_tmp, tb, P.tmp, P.scr_off, n + 1, s);
        if (e != hipSuccess) return e;
        P.lds_small = enc_lds() ? 1 : 0;
        if (n) {
            if (P.lds_small) {
                auto grid = [&](uint64_t recs) { return dim3((unsigned)std::min<uint64_t>((n + recs - 1) / recs, 16384)); };
                // 16 records per group (32 KiB of tables, five groups = 80 records per CU) as 4 waves
                // of 4 lanes. Measured on C2-shaped input: one 64-lane wave per 64 records 20.7 GiB/s,
                // 32 records as 8 waves x 4 lanes 35.5, 16 records as 4 x 4 36.4, 16 as 8 x 2 34.1
                switch (enc_lanes()) {
                case 64: hipLaunchKernelGGL((k_snappy_encode_lds<64, 4>), grid(64), dim3(1024), 0, s, P); break;
                case 32: hipLaunchKernelGGL((k_snappy_encode_lds<32, 4>), grid(32), dim3(512), 0, s, P); break;
                case 8: hipLaunchKernelGGL((k_snappy_encode_lds<16, 2>), grid(16), dim3(512), 0, s, P); break;
                default: hipLaunchKernelGGL((k_snappy_encode_lds<16, 4>), grid(16), dim3(256), 0, s, P); break;
                }
            }
            hipLaunchKernelGGL(k_snappy_encode_global, dim3(enc_groups()), dim3(64), 0, s, P);
        }
    }
    hipLaunchKernelGGL(k_enc_sizes, dim3(g), dim3(256), 0, s, P);
    size_t tb = cub_bytes;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(cub_tmp, tb, P.tmp, P.size, n + 1, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_enc_emit, dim3((unsigned)std::min<uint64_t>((n + 15) / 16 + 1, 4096)), dim3(256), 0, s, P);
    return hipGetLastError();
}

size_t enc_cub_bytes(uint64_t n) {
    size_t b = 0;
    if (hipcub::DeviceScan::ExclusiveSum(nullptr, b, (uint64_t*)nullptr, (uint64_t*)nullptr, n + 1) != hipSuccess)
        return 0;
    return b;
}

}  // namespace rio
