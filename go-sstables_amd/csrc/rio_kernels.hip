// rio_kernels.hip — CDNA4 (gfx950) kernels of the recordio v3/v4 decode path.
//
// Pipeline for one file already in HBM: six launches for a Snappy file when the
// host passes the codec (rio_device_decode_ex), follow-up steps run by the last block to arrive.
//   k_walk          one wave per 32 KiB chunk: speculative entries at every 91 8d 4c candidate,
//                   framed in parallel (readRecordHeaderV4/V3, common_reader.go:83-151; payload
//                   sizing common_reader.go:162-169; snappy preamble = decoded size), chain picked
//                   by a lane vote; records to per-chunk scratch. Block 0 also reads the file
//                   header (readFileHeaderFromBuffer, common_reader.go:22-44) and resets ScanState.
//   k_scan_blocks   256-chunk blocks: inclusive scan of key-point chunk summaries (stitches each
//                   chunk's speculative entry to its predecessor's exit; a mismatch => sequential
//                   repair walk); the last block runs the top level: record/byte prefix sums,
//                   terminal status (FileReader.ReadNext loop, file_reader.go:61-131).
//   k_place         prologue: arena capacity, zero-tail check behind a magic mismatch
//                   (file_reader.go:76-91); scratch -> rec_off / out_off / flags at their global index.
//   k_copy_records  uncompressed payloads and single-literal Snappy records (16-lane copies).
//   k_snappy_pipe   golang/snappy v1.0.0 block decode (rio_snappy.hip); k_gzip_* (rio_gzip.hip).
//   k_finish        re-check of records handed over by decoder lanes; last block: rio_file_info.
// Host-API phase A (rio_frame) adds k_zero + k_finalize after the scan. Seek map (k_count91 ..
// k_seek_jump) and single-record k_read_at / k_seek_next serve the ReadAtI handle.
// Byte/integer work only: no MFMA. All offsets 64-bit.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <vector>

#include "rio_device.h"
#include "rio_dev_util.h"
#include "rio_pb.h"

namespace rio {

// RIO_SCAN_PROBE=1 (diagnostic builds only): 100 MHz wall-clock stamps of the framing kernels' phases in a
// device array, printed after each decode by k_probe_dump (where a small file's framing time goes)
#ifndef RIO_SCAN_PROBE
#define RIO_SCAN_PROBE 0
#endif
#if RIO_SCAN_PROBE
__device__ unsigned long long g_probe[32];
#define PROBE_MIN(i) atomicMin(&g_probe[i], (unsigned long long)wall_clock64())
#define PROBE_MAX(i) atomicMax(&g_probe[i], (unsigned long long)wall_clock64())
#else
#define PROBE_MIN(i) ((void)0)
#define PROBE_MAX(i) ((void)0)
#endif

// Code prefetch: after a MALL flush a launch's instruction fetches come from HBM one
// 64-byte line at a time, a dependent miss chain through the kernel's straight-line code (round 6 probe: the
// scan's cold chain 36 -> 31 us with the next 4 KiB of its code read as data at entry, profiles/r6/
// r6k_small_file_framing.txt). Lane t < lines of the calling wave loads the dword at pc + 64 t into L2 (one line
// each; the SQC's misses then hit L2); code_pf_done consumes the value where the wave waits anyway. `lines` stays
// within the kernel's own code: tests/test_kernel_lint.py checks every prefetching kernel against the code object.
__device__ __forceinline__ uint32_t code_pf(uint32_t lines) {
    uint32_t v = 0;
    if (threadIdx.x < lines)
        v = *reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(__builtin_amdgcn_s_getpc() +
                                                                                  64u * threadIdx.x);
    return v;
}
__device__ __forceinline__ void code_pf_done(uint32_t v) {
    asm volatile("" ::"v"(v));
}
// lines per kernel (tests/test_kernel_lint.py: within each kernel's own code); the wide grids prefetch from their first
// 16 blocks only (two per XCD: each XCD's L2 then holds the code)
constexpr uint32_t kPfScan = 64, kPfPlace = 48, kPfCopy = 64, kPfFinish = 64, kPfWalk = 64, kPfBlocks = 16;

// ------------------------------------------------------------------------------------------
// Byte-level primitives
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t crc32c_byte(uint32_t c, uint32_t b) {
    c ^= b;
#pragma unroll
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    return c;
}

// Byte sources for the header / scan code: RawBytes reads the file directly; WinBytes (rio_pb.h)
// serves a lane's bytes from a 16-byte window and reloads it only when a position leaves it.
// io.ByteReader over file bytes [base, base+avail); `cap` = checksumByteReader cache (36 for v4
// FileReader, checksum_byte_reader.go:25-27), ~0 when no cache applies.
template <class B>
struct SrcT {
    B& get;
    uint64_t base, avail, pos, cap;
};

template <class B>
__device__ __forceinline__ int src_byte(SrcT<B>& s, uint32_t& b) {
    if (s.pos >= s.avail) return RIO_EOF;
    if (s.pos >= s.cap) {
        s.pos++;
        return RIO_ERR_HEADER_TOO_LONG;
    }
    b = s.get(s.base + s.pos++);
    return RIO_OK;
}

// encoding/binary.ReadUvarint semantics
template <class B>
__device__ __forceinline__ int read_uvarint(SrcT<B>& s, uint64_t& x) {
    uint64_t v = 0;
    uint32_t sh = 0;
    for (int i = 0; i < 10; i++) {
        uint32_t b;
        int e = src_byte(s, b);
        if (e) return (e == RIO_EOF && i > 0) ? RIO_ERR_UNEXPECTED_EOF : e;
        if (b < 0x80) {
            if (i == 9 && b > 1) return RIO_ERR_VARINT_OVERFLOW;
            x = v | ((uint64_t)b << sh);
            return RIO_OK;
        }
        v |= (uint64_t)(b & 0x7F) << sh;
        sh += 7;
    }
    return RIO_ERR_VARINT_OVERFLOW;
}

struct Hdr {
    uint64_t u, c, exp_crc, act_crc;
    uint32_t hdr_len, magic_len;
    int nil;
};

__device__ __forceinline__ int later_field(int e) { return e == RIO_EOF ? RIO_EOF_HEADER : e; }

// readRecordHeaderV4 (common_reader.go:110-151) / readRecordHeaderV3 (:83-108) / readRecordHeaderV2
// (:61-81: no nil byte, no CRC)
template <class B>
__device__ __forceinline__ int parse_header_t(B& get, uint64_t p, uint64_t avail, uint64_t cap, uint32_t ver, Hdr& h,
                                              const uint32_t* crc_tab = nullptr) {
    h.nil = 0;
    h.hdr_len = 0;
    if (ver == RIO_VERSION1) {
        // readRecordHeaderV1 (common_reader.go:46-59) after io.ReadFull of 20 bytes (file_reader.go:282-293):
        // nothing left -> io.EOF, a partial header -> io.ErrUnexpectedEOF; no zero-tail rule
        h.magic_len = 0;
        if (avail == 0) return RIO_EOF;
        if (avail < RIO_RECORD_HEADER_V1_BYTES) return RIO_ERR_UNEXPECTED_EOF;
        uint32_t m = 0;
        uint64_t u = 0, c = 0;
        for (uint32_t i = 0; i < 4; i++) m |= (uint32_t)get(p + i) << (8 * i);
        if (m != RIO_MAGIC) return RIO_ERR_MAGIC;
        for (uint32_t i = 0; i < 8; i++) {
            u |= (uint64_t)get(p + 4 + i) << (8 * i);
            c |= (uint64_t)get(p + 12 + i) << (8 * i);
        }
        h.u = u;
        h.c = c;
        h.hdr_len = RIO_RECORD_HEADER_V1_BYTES;
        return RIO_OK;
    }
    SrcT<B> s{get, p, avail, 0, cap};
    uint64_t m = 0;
    int e = read_uvarint(s, m);
    h.magic_len = (uint32_t)s.pos;
    if (e) return e;
    if (m != RIO_MAGIC) return RIO_ERR_MAGIC;
    uint32_t nb = 0;
    if (ver >= RIO_VERSION3) {
        e = src_byte(s, nb);
        if (e) return later_field(e);
    }
    e = read_uvarint(s, h.u);
    if (e) return later_field(e);
    e = read_uvarint(s, h.c);
    if (e) return later_field(e);
    if (ver == RIO_VERSION4) {
        uint32_t crc = 0xFFFFFFFFu;
        // byte table in LDS when the kernel has one (T[0..255] of crc32c_tab_init), else bitwise
        if (crc_tab)
            for (uint64_t i = 0; i < s.pos; i++) crc = crc_tab[(crc ^ get(p + i)) & 0xFFu] ^ (crc >> 8);
        else
            for (uint64_t i = 0; i < s.pos; i++) crc = crc32c_byte(crc, get(p + i));
        h.act_crc = crc ^ 0xFFFFFFFFu;
        e = read_uvarint(s, h.exp_crc);
        if (e) return later_field(e);
        if (h.act_crc != h.exp_crc) return RIO_ERR_HEADER_CRC;
    }
    h.nil = (nb == 1);
    h.hdr_len = (uint32_t)s.pos;
    return RIO_OK;
}

__device__ __forceinline__ int parse_header(const uint8_t* f, uint64_t p, uint64_t avail, uint64_t cap, uint32_t ver,
                                            Hdr& h) {
    RawBytes raw{f};
    return parse_header_t(raw, p, avail, cap, ver, h);
}

// ---- register-window header parse (fast path) --------------------------------------------
// 8 bytes starting at byte k (0..23: dwords j .. j + 2 with j <= 5) of a 32-byte window held in 8 dwords
__device__ __forceinline__ uint64_t win8(const uint32_t (&w)[8], uint32_t k) {
    const uint32_t j = k >> 2, r = 8 * (k & 3);
    uint32_t d0 = w[0], d1 = w[1], d2 = w[2];
#pragma unroll
    for (uint32_t t = 1; t < 6; t++) {
        d0 = j == t ? w[t] : d0;
        d1 = j == t ? w[t + 1] : d1;
        d2 = j == t ? w[t + 2] : d2;
    }
    const uint64_t a = ((uint64_t)d1 << 32) | d0, b = d2;
    return r ? (a >> r) | (b << (64 - r)) : a;
}

// 7-bit groups of the four bytes of x packed (LEB128 payload bits of bytes 0..3)
__device__ __forceinline__ uint32_t leb_pack4(uint32_t x) {
    return (x & 0x7Fu) | ((x >> 1) & 0x3F80u) | ((x >> 2) & 0x1FC000u) | ((x >> 3) & 0x0FE00000u);
}

// LEB128 of at most 8 bytes at the bottom of x: returns the byte count (0 if longer than 8)
__device__ __forceinline__ uint32_t varint8(uint64_t x, uint64_t& v) {
    const uint64_t stop = ~x & 0x8080808080808080ull;
    const uint32_t nb = stop ? (__builtin_ctzll(stop) >> 3) + 1 : 0u;
    const uint64_t y = x & (nb >= 8 || nb == 0 ? ~0ull : ((1ull << (8 * nb)) - 1));
    // two 32-bit halves of 28 payload bits each (the 64-bit group loop cost ~45 VALU per call)
    const uint32_t lo = leb_pack4((uint32_t)y), hi = leb_pack4((uint32_t)(y >> 32));
    v = ((uint64_t)hi << 28) | lo;
    return nb;
}

__device__ __forceinline__ uint32_t crc32c_bytes(uint32_t c, uint64_t x, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) c = crc32c_byte(c, (uint32_t)(x >> (8 * i)) & 0xFF);
    return c;
}

// CRC-32C register state after the canonical magic bytes 91 8d 4c (before the final xor)
__device__ __forceinline__ uint32_t crc_after_magic() {
    uint32_t c = 0xFFFFFFFFu;
    c = crc32c_byte(c, 0x91);
    c = crc32c_byte(c, 0x8D);
    return crc32c_byte(c, 0x4C);
}

// CRC-32C slice-by-4 over LDS tables T[0..1023] (T0..T3, reflected polynomial 0x82F63B78):
// n <= 16 bytes given little-endian in x0 (bytes 0..7) and x1 (bytes 8..15). Register state in/out.
__device__ __forceinline__ uint32_t crc32c_tab(uint32_t c, uint64_t x0, uint64_t x1, uint32_t n, const uint32_t* T) {
    uint32_t i = 0;
    for (; i + 4 <= n; i += 4) {
        const uint32_t w = c ^ (uint32_t)((i < 8 ? x0 >> (8 * i) : x1 >> (8 * (i - 8))));
        c = T[768 + (w & 0xFF)] ^ T[512 + ((w >> 8) & 0xFF)] ^ T[256 + ((w >> 16) & 0xFF)] ^ T[w >> 24];
    }
    for (; i < n; i++) {
        const uint32_t b = (uint32_t)((i < 8 ? x0 >> (8 * i) : x1 >> (8 * (i - 8)))) & 0xFF;
        c = T[(c ^ b) & 0xFF] ^ (c >> 8);
    }
    return c;
}

// The slice-by-4 tables, computed at compile time (CRC-32C, reflected polynomial 0x82F63B78)
struct Crc32cTables {
    uint32_t t[1024];
    constexpr Crc32cTables() : t() {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
            t[i] = c;
        }
        for (uint32_t i = 0; i < 256; i++)
            for (uint32_t k = 1; k < 4; k++) t[256 * k + i] = (t[256 * (k - 1) + i] >> 8) ^ t[t[256 * (k - 1) + i] & 0xFF];
    }
};
__device__ const Crc32cTables kCrc32c{};

// Copy the slice-by-4 tables into LDS (blockDim.x >= 256: one 16-byte piece per thread; round 4:
// a load instead of ~45 VALU per thread of bitwise table building); ends with a workgroup barrier.
__device__ void crc32c_tab_init(uint32_t* T) {
    const uint32_t i = threadIdx.x;
    if (i < 256) reinterpret_cast<uint4*>(T)[i] = reinterpret_cast<const uint4*>(kCrc32c.t)[i];
    __syncthreads();
}

// lzw records are sized by the header's u (the reference's buffer size, the decoded length for every
// file its writer produces) while an lzw stream of `plen` bytes can reach it: a 9-bit code expands to
// at most 4096 bytes (oracle ORC_LZW_MAX_RATIO). k_lzw_decode counts and re-places any other size.
__device__ __forceinline__ uint64_t lzw_size(uint64_t u, uint64_t plen) { return u <= 4096ull * plen ? u : 0; }

// The fast path of frame_record on the 32 bytes at p already in registers (w; p + 32 <= len): RIO_OK
// with the record framed (lflags 0), or kFrameSlow when the record needs the byte-wise path below.
constexpr int kFrameSlow = -1000;
__device__ __forceinline__ int frame_fast(const uint32_t (&w)[8], uint64_t len, uint64_t p, uint32_t ver, uint32_t comp,
                                          Hdr& h, uint64_t& next, uint64_t& out_len, uint64_t& pay,
                                          const uint32_t* crct) {
    const uint4 a = make_uint4(w[0], w[1], w[2], w[3]), b = make_uint4(w[4], w[5], w[6], w[7]);
    {
        if (ver == RIO_VERSION1 ? a.x == RIO_MAGIC : (a.x & 0xFFFFFFu) == 0x4C8D91u) {
            // v3 / v4: the nil byte at 3, the sizes from 4; v2: no nil byte (readRecordHeaderV2)
            // v1: fixed 20 bytes, LE u64 sizes at 4 and 12 (readRecordHeaderV1)
            const uint32_t hb = ver >= RIO_VERSION3 ? 4u : 3u;
            uint64_t u = 0, c = 0, crc = 0;
            uint32_t nu, nc;
            if (ver == RIO_VERSION1) {
                u = ((uint64_t)a.z << 32) | a.y;
                c = ((uint64_t)b.x << 32) | a.w;
                nu = 8;
                nc = 9;  // hb (3) + 8 + 9 = 20
            } else {
                nu = varint8(win8(w, hb), u);
                nc = nu ? varint8(win8(w, hb + nu), c) : 0;
            }
            uint32_t hl = hb + nu + nc;
            bool ok = nu && nc;
            uint32_t act = 0;
            if (ok && ver == RIO_VERSION4) {
                const uint32_t ncrc = varint8(win8(w, hl), crc);
                uint32_t cs;
                if (crct && nu + nc <= 15) {  // nil byte + both varints: bytes [3, 4 + nu + nc)
                    cs = crc32c_tab(crc_after_magic(), win8(w, 3), win8(w, 11), 1 + nu + nc, crct);
                } else {
                    cs = crc32c_byte(crc_after_magic(), (a.x >> 24) & 0xFF);
                    cs = crc32c_bytes(cs, win8(w, 4), nu);
                    cs = crc32c_bytes(cs, win8(w, 4 + nu), nc);
                }
                act = cs ^ 0xFFFFFFFFu;
                ok = ncrc && act == crc;
                hl += ncrc;
            }
            if (ok) {
                const bool nil = ver >= RIO_VERSION3 && ((a.x >> 24) & 0xFF) == 1;
                const uint64_t plen = comp != RIO_COMP_NONE ? c : u;
                const uint64_t avail = len - p - hl;
                uint64_t dl = plen;
                uint32_t k = 0;
                if (!nil && comp == RIO_COMP_SNAPPY && hl <= 20) {  // win8 covers k <= 20 with 8 bytes inside the window
                    k = varint8(win8(w, hl), dl);
                    ok = k && k <= plen && dl <= 0xFFFFFFFFull && dl <= 22ull * (plen - k) + 64;
                } else if (!nil && comp == RIO_COMP_LZW) {
                    dl = lzw_size(u, plen);
                } else if (!nil && comp != RIO_COMP_NONE) {
                    ok = false;  // snappy preamble outside the window; gzip: sized by its trailer
                }
                if (ok && (nil || plen <= avail)) {
                    h.u = u;
                    h.c = c;
                    h.exp_crc = crc;
                    h.act_crc = act;
                    h.hdr_len = hl;
                    h.magic_len = ver == RIO_VERSION1 ? 0 : 3;
                    h.nil = nil;
                    if (nil) {  // file_reader.go:96-99: nil => no payload bytes
                        next = p + hl;
                        out_len = 0;
                        pay = hl;
                    } else {
                        next = p + hl + plen;
                        out_len = dl;
                        pay = ((plen - k) << 8) | (hl + k);
                    }
                    return RIO_OK;
                }
            }
        }
    }
    return kFrameSlow;
}

// The byte-wise path of frame_record (ReadUvarint restatement): every record the fast path does not take,
// and every failure's exact classification.
__device__ int frame_slow(const uint8_t* f, uint64_t len, uint64_t p, uint32_t ver, uint32_t comp, Hdr& h,
                          uint64_t& next, uint64_t& out_len, uint64_t& pay, uint64_t& lflags) {
    lflags = 0;
    uint64_t cap = ver == RIO_VERSION4 ? RIO_RECORD_HEADER_V4_MAX : ~0ull;
    int e = parse_header(f, p, len - p, cap, ver, h);
    if (e) return e;
    if (h.nil) {  // file_reader.go:96-99: nil => no payload bytes
        next = p + h.hdr_len;
        out_len = 0;
        pay = h.hdr_len;
        return RIO_OK;
    }
    uint64_t plen = comp != RIO_COMP_NONE ? h.c : h.u;
    uint64_t avail = len - p - h.hdr_len;
    if (plen > avail) return avail == 0 ? RIO_EOF_PAYLOAD : RIO_ERR_UNEXPECTED_EOF;
    uint64_t k = 0;
    next = p + h.hdr_len + plen;
    if (comp == RIO_COMP_SNAPPY) {
        uint64_t d = 0;
        const int kk = uvarint_buf(f + p + h.hdr_len, plen, d);
        // snappy decodedLen: n<=0 or > 0xffffffff => ErrCorrupt; a preamble above 22x the element
        // bytes cannot be produced (max 64 output bytes per 3-byte tagCopy2) => ErrCorrupt later.
        if (kk <= 0 || d > 0xFFFFFFFFull || d > 22ull * (plen - (uint64_t)kk) + 64) {
            out_len = 0;
            pay = h.hdr_len;
            lflags = kBadBit;
            return RIO_OK;
        }
        out_len = d;
        k = (uint64_t)kk;
    } else if (comp == RIO_COMP_GZIP) {
        // gzip.NewReader on an empty payload returns a bare io.EOF, which ReadNext passes through
        // unwrapped (file_reader.go:118-121, gzip_compression.go:56-59)
        // decoded size = ISIZE, the payload's last four bytes (trailer of its only member; more
        // members -> RIO_ERR_UNSUPPORTED at decode). A member is at least 18 bytes, and above
        // DEFLATE's maximum ratio (258 bytes per 2 bits) no valid stream ends this way: the reader
        // fails on either.
        uint64_t isz = 0;
        if (plen >= 18) {
            const uint8_t* t = f + p + h.hdr_len + plen - 4;
            isz = t[0] | (uint64_t)t[1] << 8 | (uint64_t)t[2] << 16 | (uint64_t)t[3] << 24;
        }
        if (plen == 0 || plen < 18 || isz > 1032ull * plen + 64) {
            out_len = 0;
            pay = h.hdr_len;
            lflags = plen == 0 ? kEofBit : kBadBit;
            return RIO_OK;
        }
        out_len = isz;
    } else if (comp == RIO_COMP_LZW) {
        out_len = lzw_size(h.u, plen);
    } else {
        out_len = plen;
    }
    pay = ((plen - k) << 8) | (h.hdr_len + k);
    return RIO_OK;
}

// FileReader sequential semantics at record start p: header + payload availability + decoded
// size. next = start of the following record; pay = rec_pay descriptor (rio_device.h).
// Common records (canonical magic, header + preamble inside 32 bytes, valid) are parsed from two
// 16-byte loads; everything else (and every failure, for its exact classification) takes the
// byte-wise ReadUvarint restatement.
// A payload whose codec preamble / size already fails (snappy: unusable preamble; gzip: empty, too
// short, or an ISIZE no DEFLATE stream reaches) frames normally: FileReader consumed it, and its
// ReadNext fails without ending the file. `lflags` then carries kBadBit / kEofBit and out_len 0.
__device__ int frame_record(const uint8_t* f, uint64_t len, uint64_t p, uint32_t ver, uint32_t comp,
                            Hdr& h, uint64_t& next, uint64_t& out_len, uint64_t& pay, uint64_t& lflags,
                            const uint32_t* crct = nullptr) {
    lflags = 0;
    if (p + 32 <= len) {
        const uint4 a = ldu16(f + p), b = ldu16(f + p + 16);
        const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        if (frame_fast(w, len, p, ver, comp, h, next, out_len, pay, crct) == RIO_OK) return RIO_OK;
    }
    return frame_slow(f, len, p, ver, comp, h, next, out_len, pay, lflags);
}

// ------------------------------------------------------------------------------------------
// File header (readFileHeaderFromBuffer, common_reader.go:22-44) and the per-call state reset; run
// by k_walk: every wave reads the 8 header bytes itself, block 0's first thread resets the state
// the later kernels accumulate into (no separate launch)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int file_header_status(const FrameParams& P, uint32_t& v, uint32_t& c) {
    v = c = 0;
    if (P.len < RIO_FILE_HEADER_BYTES) return RIO_ERR_SHORT_FILE_HEADER;
    const uint8_t* f = P.file;
    v = f[0] | (uint32_t)f[1] << 8 | (uint32_t)f[2] << 16 | (uint32_t)f[3] << 24;
    c = f[4] | (uint32_t)f[5] << 8 | (uint32_t)f[6] << 16 | (uint32_t)f[7] << 24;
    if (v > RIO_VERSION4 || v < RIO_VERSION1) return RIO_ERR_VERSION;
    if (c > RIO_COMP_LZW) return RIO_ERR_COMPRESSION_TYPE;
    return RIO_OK;
}

__device__ __forceinline__ void init_state(const FrameParams& P) {
    ScanState* st = P.state;
    const uint8_t* f = P.file;
    st->n_records = 0;
    st->total_bytes = 0;
    st->status = RIO_OK;
    st->status_offset = RIO_FILE_HEADER_BYTES;
    st->det0 = st->det1 = 0;
    st->zero_from = kNone;
    st->zero_nonzero = 0;
    st->n_repairs = 0;
    st->first_bad = kNone;
    st->n_bad = 0;
    st->unsupported_rec = kNone;
    st->n_fail_lanes = 0;
    st->capacity_fail = 0;
    st->huge_streams = 0;
    st->any_mixed = 0;
    st->slow = 0;
    st->scan_ticket = 0;
    st->finish_ticket = 0;
    st->pipe_next = 0;
    st->gz_resize = 0;
    st->gz_redo = 0;
    if (P.len < RIO_FILE_HEADER_BYTES) {
        st->hdr_status = RIO_ERR_SHORT_FILE_HEADER;
        st->version = st->compression = 0;
        return;
    }
    uint32_t v = f[0] | (uint32_t)f[1] << 8 | (uint32_t)f[2] << 16 | (uint32_t)f[3] << 24;
    uint32_t c = f[4] | (uint32_t)f[5] << 8 | (uint32_t)f[6] << 16 | (uint32_t)f[7] << 24;
    st->version = v;
    st->compression = c;
    int hs = RIO_OK;
    if (v > RIO_VERSION4 || v < RIO_VERSION1) {
        hs = RIO_ERR_VERSION;
        st->det0 = v;
    } else if (c > RIO_COMP_LZW) {
        hs = RIO_ERR_COMPRESSION_TYPE;
        st->det0 = c;
    }
    st->hdr_status = hs;
}

// ------------------------------------------------------------------------------------------
// Chunk walk
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t chunk_start(const FrameParams& P, uint64_t c) {
    return RIO_FILE_HEADER_BYTES + c * P.chunk_bytes;
}
__device__ __forceinline__ uint64_t chunk_end(const FrameParams& P, uint64_t c) {
    uint64_t e = chunk_start(P, c) + P.chunk_bytes;
    return e < P.len ? e : P.len;
}

// bytes 1 and 2 of a record's magic: 8d 4c (uvarint 0x130691, v2..v4), 06 13 (LE u32, v1)
__device__ __forceinline__ uint32_t magic3(uint32_t ver) { return ver == RIO_VERSION1 ? 0x130691u : 0x4C8D91u; }

// First position in [cs, ce) holding the canonical magic bytes 91 8d 4c (v1: 91 06 13) whose header
// and payload validate under FileReader semantics (CRC for v4). Speculative; stitched by the scan.
__device__ uint64_t find_entry(const FrameParams& P, uint64_t cs, uint64_t ce, uint32_t ver, uint32_t comp) {
    const uint8_t* f = P.file;
    const uint32_t m3 = magic3(ver);
    for (uint64_t q = cs & ~15ull; q < ce; q += 16) {
        const uint4 w = *reinterpret_cast<const uint4*>(f + q);
        uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint32_t x = ws[k] ^ 0x91919191u;
            uint32_t hit = (x - 0x01010101u) & ~x & 0x80808080u;
            while (hit) {
                int b = __builtin_ctz(hit) >> 3;
                hit &= hit - 1;
                uint64_t p = q + 4 * k + b;
                if (p < cs || p >= ce || p + 2 >= P.len) continue;
                if (f[p + 1] != ((m3 >> 8) & 0xFF) || f[p + 2] != (m3 >> 16)) continue;
                Hdr h;
                uint64_t nx, ol, pd, lf;
                if (frame_record(f, P.len, p, ver, comp, h, nx, ol, pd, lf) == RIO_OK) return p;
            }
        }
    }
    return kNone;
}

// Continue walking chunk c from record start p (count/bytes already in s), filling its scratch
// slots; sets s.exit / s.status. Serial header-to-header hops (FileReader order).
__device__ void walk_from(const FrameParams& P, uint64_t c, uint64_t p, uint32_t ver, uint32_t comp, ChunkSum& s,
                          const uint32_t* crct = nullptr) {
    const uint64_t ce = chunk_end(P, c);
    uint64_t* so = P.scratch_off + c * P.slots;
    uint64_t* sl = P.scratch_len + c * P.slots;
    uint64_t* sp = P.scratch_pay + c * P.slots;
    while (p < ce) {
        Hdr h;
        uint64_t next = 0, olen = 0, pd = 0, lf = 0;
        int e = frame_record(P.file, P.len, p, ver, comp, h, next, olen, pd, lf, crct);
        if (e) {
            s.status = e;
            s.err_off = p;
            if (e == RIO_ERR_HEADER_CRC) {
                s.det0 = h.exp_crc;
                s.det1 = h.act_crc;
            } else if (e == RIO_ERR_MAGIC) {
                s.det0 = h.magic_len;
            } else if (e == RIO_ERR_UNEXPECTED_EOF && h.hdr_len != 0) {
                s.det0 = 1;  // raised by the payload read, not by a header varint
            }
            break;
        }
        if (s.count < P.slots) {
            so[s.count] = p;
            sl[s.count] = olen | lf | (h.nil ? kNilBit : 0);
            sp[s.count] = pd;
        }
        s.count++;
        s.bytes += olen;
        p = next;
    }
    s.exit = s.status ? s.err_off : p;
}

__device__ __forceinline__ ChunkSum chunk_sum_empty(uint64_t entry) {
    ChunkSum s;
    s.entry = entry;
    s.exit = kNone;
    s.bytes = 0;
    s.err_off = 0;
    s.det0 = s.det1 = 0;
    s.count = 0;
    s.status = RIO_OK;
    return s;
}

// Walk chunk c from record start `from` (kNone => nothing to walk), filling its scratch slots.
__device__ void walk_chunk(const FrameParams& P, uint64_t c, uint64_t from, uint32_t ver, uint32_t comp) {
    ChunkSum s = chunk_sum_empty(from);
    if (from != kNone) walk_from(P, c, from, ver, comp, s);
    P.chunks[c] = s;
}

// Wave-wide exclusive prefix sum (64 lanes).
template <typename T>
__device__ __forceinline__ T wave_excl_scan(T v, uint32_t lane) {
    T x = v;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const T y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    return x - v;
}

// Wave-wide inclusive sum on DPP (row shifts within 16-lane rows, then row broadcasts 15 / 31):
// VALU latency instead of the LDS round trips of __shfl_up
__device__ __forceinline__ uint32_t wave_incl_sum32(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}
__device__ __forceinline__ uint32_t lane63(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, 63); }

// exclusive prefix of 64-bit values and the wave total: 32-bit DPP when every value is below 2^26
// (64 of them sum below 2^32), else the shuffle scan
__device__ __forceinline__ uint64_t wave_excl_scan64(uint64_t v, uint32_t lane, uint64_t& total) {
    if (__all(v < (1ull << 26))) {
        const uint32_t x = wave_incl_sum32((uint32_t)v);
        total = lane63(x);
        return x - (uint32_t)v;
    }
    const uint64_t e = wave_excl_scan(v, lane);
    total = __shfl(e + v, 63);
    return e;
}

// The same within 16-lane groups (a wave's four DPP rows; lane = the lane within its group): exclusive prefix
// and the group's total
__device__ __forceinline__ uint64_t group16_excl_scan64(uint64_t v, uint32_t lane, uint64_t& total) {
    if (__all(v < (1ull << 26))) {
        uint32_t x = (uint32_t)v;
        x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
        x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
        x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
        x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
        total = (uint32_t)__shfl((int)x, 15, 16);
        return x - (uint32_t)v;
    }
    uint64_t x = v;
#pragma unroll
    for (uint32_t d = 1; d < 16; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 16);
        if (lane >= d) x += y;
    }
    total = __shfl(x, 15, 16);
    return x - v;
}

// a predicate's lanes within the caller's group of G lanes (G = 16 or 64), bit 0 = the group's lane 0
template <uint32_t G>
__device__ __forceinline__ uint64_t group_ballot(bool b) {
    const uint64_t m = __ballot(b);
    return G == 64 ? m : (m >> (threadIdx.x & 48u)) & 0xFFFFull;
}

// Cooperative chunk walk: one wave per chunk, processed in windows of up to 64 candidates.
//   1. fill: the wave reads 4 KiB at a time (four 1 KiB coalesced blocks, loads in flight
//      together) and compacts the positions of the canonical magic bytes 91 8d 4c (find_entry's
//      candidates) into LDS in file order, until ~48 are listed or 16 KiB were read; a 65th
//      candidate ends the window exactly at its position (the next window starts there);
//   2. every listed candidate is framed at once (frame_record, one lane each, result in registers);
//   3. the chain is followed with wave votes: the entry is the first candidate that frames
//      (find_entry); a run of candidates chains while each record's successor is the next
//      candidate; a record whose successor skips candidates (magic bytes inside its payload)
//      restarts the vote at its successor. Windows the chain jumps over (long records) are not
//      read. Wherever the chain leaves the candidates (a header that fails, a non-canonical magic
//      encoding) lane 0 takes over with the serial walk (walk_from) for the rest of the chunk.
// Result and slots are identical to find_entry + walk_chunk (the serial thread-per-chunk walk,
// which paid ~50 dependent global round trips per 4 KiB chunk).
constexpr uint32_t kWalkWaves = 4;      // chunks per workgroup
#ifndef RIO_WALK_FILL
#define RIO_WALK_FILL 56
#endif
#ifndef RIO_WALK_FILL_MAX
#define RIO_WALK_FILL_MAX 8
#endif
constexpr uint32_t kWalkFill = RIO_WALK_FILL;         // stop filling a window at this many candidates
constexpr uint32_t kWalkFillMax = RIO_WALK_FILL_MAX;  // ... or after this many 4 KiB fill rounds

struct WalkLds {
    uint64_t pos[64];
    uint64_t overflow;  // first candidate beyond the 64 listed (kNone if none)
};

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t lane_ffs(uint64_t m) { return m ? (uint32_t)__builtin_ctzll(m) : 64u; }

// lane k's value for a wave-uniform k < 64: v_readlane into scalars (no LDS round trip of __shfl)
__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t k) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)k);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)k);
    return ((uint64_t)hi << 32) | lo;
}

// exact per-byte equality with a byte value: bit 7 of every byte of the result = (byte == v)
__device__ __forceinline__ uint32_t bytes_eq(uint32_t d, uint32_t v4) {
    const uint32_t x = d ^ v4;
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}

// candidate bits of the 16 positions q .. q+15 in [lo, hi) (91 8d 4c at the position, the magic
// inside the file); d = the 16 bytes at q plus the next 4
__device__ __forceinline__ uint32_t magic_mask(const uint32_t (&d)[5], uint64_t q, uint64_t lo, uint64_t hi,
                                               uint64_t len, uint32_t m3) {
    // bytes equal to 0x91, gathered without a multiply: bit 8j + k of c = byte j of dword k (position
    // 4k + j); only those (~1 in 256 bytes) get the full 3-byte test and the bounds, in the loop
    // (round 4: the gather was a v_mul_lo_u32 per dword and the bounds a mask per block)
    uint32_t c = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) c |= bytes_eq(d[k], 0x91919191u) >> (7 - k);
    uint32_t mask = 0;
    if (c) {
        // positions [a, b) of the 16 are inside [lo, hi): lo and hi lie within 2^31 bytes of q (one
        // chunk's window, lo < hi), so 32-bit differences clamped to [0, 16] give a <= b; the three
        // magic bytes must lie in the file: i + 2 < len - q (64-bit: the file may extend far past q);
        // rio_ctx_create caps chunks at 1 GiB, which keeps lo and hi that close
        auto clamp16 = [](int32_t x) { return (uint32_t)(x < 0 ? 0 : (x > 16 ? 16 : x)); };
        const uint32_t a = clamp16((int32_t)((uint32_t)lo - (uint32_t)q));
        const uint32_t b = clamp16((int32_t)((uint32_t)hi - (uint32_t)q));
        const uint32_t lim = (uint32_t)umin(len - q, (uint64_t)18);
        do {
            const uint32_t bit = __ffs(c) - 1;
            c &= c - 1;
            const uint32_t k = bit & 7u, j = bit >> 3, i = 4 * k + j;
            const uint32_t d0 = k == 0 ? d[0] : (k == 1 ? d[1] : (k == 2 ? d[2] : d[3]));  // select, not index
            const uint32_t d1 = k == 0 ? d[1] : (k == 1 ? d[2] : (k == 2 ? d[3] : d[4]));
            const uint32_t x = __builtin_amdgcn_alignbyte(d1, d0, j) & 0xFFFFFFu;
            if (x == m3 && i >= a && i < b && i + 2 < lim) mask |= 1u << i;
        } while (c);
    }
    return mask;
}

// minimum waves per SIMD for k_walk (0 = the compiler's choice, 4 waves). Round 1: 6 waves with 60 B
// spilled to scratch beat 5 (walk 0.210 -> 0.185 ms on C2). With the packed DPP fill scans and the
// 32-bit LEB128 packing the spills landed in the fill loop: 6 waves 0.413 ms on C3, 5 waves (96
// VGPRs, no scratch) 0.300 ms, against 0.363 before (C2 0.183 -> 0.164 ms)
// k_copy_records (round 5): the next record's sizes prefetched and 1 KiB in flight per 16-lane group, non-temporal loads
// and stores (C2-ref-random copy 0.423 -> 0.370 ms, 5.8 TB/s; C1 +7 %, C5 +4 % against plain ones and the round-4 loop:
// profiles/r5/r5aa_copy_ab.txt)
// k_copy_records' grid (4096 x 256: C1's 100 k records over twice the groups, copy 0.067 -> 0.057 ms; C2-ref-random
// -2 %; 1024: C1 +45 %; two records in flight per group: +10 %, r5ab)
#ifndef RIO_COPY_GRID
#define RIO_COPY_GRID 4096
#endif
// files whose records average fewer bytes than this copy with 4 lanes per record instead of 16
#ifndef RIO_COPY_SMALL
#define RIO_COPY_SMALL 128
#endif
constexpr uint64_t kCopySmall = RIO_COPY_SMALL;
#ifndef RIO_WALK_OCC
#define RIO_WALK_OCC 5
#endif
#if RIO_SCAN_PROBE
// per wave of k_walk: start, end, and the time in fill / frame / the rest, windows and fill rounds (probe build)
__device__ unsigned long long g_wave[1 << 18][6];
#endif
#if RIO_WALK_OCC
__global__ void __launch_bounds__(64 * kWalkWaves, RIO_WALK_OCC) k_walk(FrameParams P) {
#else
__global__ void __launch_bounds__(64 * kWalkWaves) k_walk(FrameParams P) {
#endif
    __shared__ WalkLds W[kWalkWaves];
    __shared__ uint32_t crct[1024];
    const uint32_t pf = code_pf(blockIdx.x < kPfBlocks ? kPfWalk : 0);
    if (threadIdx.x == 0) PROBE_MIN(0);
    if (blockIdx.x == 0 && threadIdx.x == 0) init_state(P);
    crc32c_tab_init(crct);
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t c = (uint64_t)blockIdx.x * kWalkWaves + wv;
    uint32_t ver, comp;
    if (c >= P.n_chunks || file_header_status(P, ver, comp) != RIO_OK) return;  // wave-uniform
    WalkLds& L = W[wv];
    const uint64_t cs = chunk_start(P, c), ce = chunk_end(P, c);
    const uint8_t* f = P.file;
    uint64_t* so = P.scratch_off + c * P.slots;
    uint64_t* sl = P.scratch_len + c * P.slots;
    uint64_t* sp = P.scratch_pay + c * P.slots;
    // wave-uniform chain state
    uint64_t p = (c == 0) ? (uint64_t)RIO_FILE_HEADER_BYTES : kNone;  // next record start to chain
    uint32_t mode = (c == 0) ? 1u : 0u;  // 0 entry search, 1 chaining, 2 serial takeover at p
    uint64_t count = 0, bytes = 0, entry = p;
    uint64_t ws = cs;  // window start: candidates are positions >= ws
#if RIO_SCAN_PROBE
    const unsigned long long tw0 = wall_clock64();
    unsigned long long tfill = 0, tframe = 0, nwin = 0, nround = 0, tq = 0;
#endif
    while (ws < ce && mode < 2) {
        if (mode == 1) {
            if (p >= ce) break;
            ws = umax(ws, p);  // skip what the chain jumped over
        }
#if RIO_SCAN_PROBE
        tq = wall_clock64();
        nwin++;
#endif
        // 1. fill the window [ws, we)
        if (lane == 0) L.overflow = kNone;
        uint32_t total = 0;
        uint64_t rd = ws & ~15ull;  // next 16-B aligned read position
        // a round that lists no new candidate after some were found ends the fill (long records: the
        // rest of the window would be payload the chain jumps over)
        uint32_t added = 1;
        for (uint32_t r = 0; r < kWalkFillMax && rd < ce && total < kWalkFill && total <= 64 && (total == 0 || added);
             r++) {
            uint4 blk[4];
            uint32_t tail[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) {
                const uint64_t q = rd + 1024 * j + 16 * lane;
                if (q < ce) {  // 16-B aligned; q + 20 <= len + RIO_DEVICE_PAD
                    blk[j] = *reinterpret_cast<const uint4*>(f + q);
                    tail[j] = *reinterpret_cast<const uint32_t*>(f + q + 16);
                }
            }
            uint32_t masks[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) {
                const uint64_t q = rd + 1024 * j + 16 * lane;
                masks[j] = 0;
                if (q < ce) {
                    const uint32_t d[5] = {blk[j].x, blk[j].y, blk[j].z, blk[j].w, tail[j]};
                    masks[j] = magic_mask(d, q, ws, ce, P.len, magic3(ver));
                }
            }
            // list slots of the four blocks' candidates (file order: block j, then lane) from two
            // packed DPP scans (16-bit fields: a block holds at most 1024 candidates)
            const uint32_t c01 = __popc(masks[0]) | (__popc(masks[1]) << 16);
            const uint32_t c23 = __popc(masks[2]) | (__popc(masks[3]) << 16);
            const uint32_t i01 = wave_incl_sum32(c01), i23 = wave_incl_sum32(c23);
            const uint32_t t01 = lane63(i01), t23 = lane63(i23);
            const uint32_t e01 = i01 - c01, e23 = i23 - c23;
            const uint32_t T0 = t01 & 0xFFFFu, T1 = t01 >> 16, T2 = t23 & 0xFFFFu;
            const uint32_t kb[4] = {total + (e01 & 0xFFFFu), total + T0 + (e01 >> 16), total + T0 + T1 + (e23 & 0xFFFFu),
                                    total + T0 + T1 + T2 + (e23 >> 16)};
            added = T0 + T1 + T2 + (t23 >> 16);
            total += added;
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) {
                const uint64_t q = rd + 1024 * j + 16 * lane;
                uint32_t mask = masks[j];
                uint32_t k = kb[j];
                while (mask) {
                    const uint32_t i = __ffs(mask) - 1;
                    mask &= mask - 1;
                    if (k < 64)
                        L.pos[k] = q + i;
                    else if (k == 64)
                        L.overflow = q + i;
                    k++;
                }
            }
            rd += 4096;
#if RIO_SCAN_PROBE
            nround++;
#endif
        }
        wave_sync_lds();
#if RIO_SCAN_PROBE
        {
            const unsigned long long t = wall_clock64();
            tfill += t - tq;
            tq = t;
        }
#endif
        const uint64_t overflow = L.overflow;
        const uint64_t we = overflow != kNone ? overflow : umin(rd, ce);  // window end
        // 2. frame one candidate per lane
        const uint32_t nst = umin(total, 64u);
        const bool have = lane < nst;
        const uint64_t cpos = have ? L.pos[lane] : kNone;
        Hdr h;
        h.nil = false;
        uint64_t nx = 0, ol = 0, pd = 0, lf = 0;
        int e = RIO_ERR_MAGIC;
        if (have) e = frame_record(f, P.len, cpos, ver, comp, h, nx, ol, pd, lf, crct);
        const bool ok = have && e == RIO_OK;
        const uint64_t ok_mask = __ballot(ok);
#if RIO_SCAN_PROBE
        {
            const unsigned long long t = wall_clock64();
            tframe += t - tq;
            tq = t;
        }
#endif
        const uint64_t succ_pos = __shfl_down(cpos, 1);  // next candidate's position
        // 3. entry and chain by votes
        if (mode == 0) {
            const uint32_t k = lane_ffs(ok_mask);
            if (k < 64) {
                p = readlane64(cpos, k);
                mode = 1;
            }
            entry = p;
        }
        uint32_t slot = ~0u;
        while (mode == 1 && p < we) {
            // the candidate at p, if listed and framed
            const uint32_t e0 = lane_ffs(__ballot(have && cpos >= p));
            if (e0 >= nst || readlane64(cpos, e0) != p || !((ok_mask >> e0) & 1)) {
                mode = 2;  // serial takeover at p
                break;
            }
            // maximal run e0..b where each record's successor is the next candidate
            const bool link = ok && lane + 1 < nst && nx == succ_pos;
            const uint64_t brk = ~__ballot(link) & (~0ull << e0);
            const uint32_t b = lane_ffs(brk);  // first non-linking candidate (< nst: lane nst-1 never links)
            // b is reached by the chain; if its header fails, the chain stops AT it (serial takeover
            // classifies the error), else b is the run's last record
            const bool bok = (ok_mask >> b) & 1;
            const uint32_t last = bok ? b : b - 1;  // b > e0 when !bok (e0 frames)
            if (lane >= e0 && lane <= last) slot = (uint32_t)count + (lane - e0);
            count += last - e0 + 1;
            p = bok ? readlane64(nx, b) : readlane64(cpos, b);
        }
        // 4. scratch slots of the chained candidates + their decoded bytes
        const uint64_t mylen = slot != ~0u ? ol : 0;
        if (slot != ~0u && slot < P.slots) {
            so[slot] = cpos;
            sl[slot] = ol | lf | (h.nil ? kNilBit : 0);
            sp[slot] = pd;
        }
        uint64_t wsum;
        wave_excl_scan64(mylen, lane, wsum);
        bytes += wsum;
        wave_sync_lds();
        ws = we;
    }
    // 5. serial takeover where the chain left the candidates; the chunk summary
    if (lane == 0) {
        ChunkSum s = chunk_sum_empty(entry);
        s.count = (uint32_t)count;
        s.bytes = bytes;
        if (mode == 2)
            walk_from(P, c, p, ver, comp, s);
        else if (entry != kNone)
            s.exit = p;  // the chain left the chunk (or ended at the file end) cleanly
        P.chunks[c] = s;
        PROBE_MAX(1);
#if RIO_SCAN_PROBE
        if (c < (1u << 18)) {
            const unsigned long long te = wall_clock64();
            g_wave[c][0] = tw0;
            g_wave[c][1] = te;
            g_wave[c][2] = tfill;
            g_wave[c][3] = tframe;
            g_wave[c][4] = nwin;
            g_wave[c][5] = nround;
        }
#endif
    }
    code_pf_done(pf);
}

// ------------------------------------------------------------------------------------------
// Lane walk (round 5, RIO_WALK_LANE): one LANE per chunk (small chunks, 16 KiB by default, RIO_LANE_CHUNK_BYTES), the serial
// FileReader walk of find_entry + walk_chunk with the memory access shaped for a lane:
//   * entry search: 64 bytes per step as four aligned 16-byte loads issued together (plus the next
//     dword), candidates from magic_mask (0x91 bytes, then the 3-byte test), each framed by
//     frame_record; the first that frames is the chunk's speculative entry (as find_entry);
//   * then header to header: each hop is ONE round trip (frame_record's two 16-byte loads, header
//     parsed in registers, CRC-32C from the LDS slice-by-4 table) and the payload is never read.
// Slots and ChunkSum are the serial walk's, so the scan, the repair and the placement are unchanged.
// Against the wave-per-chunk walk (k_walk) it reads ~64 bytes per record instead of every byte, and
// its framing work is per record, not per candidate window; its cost is one dependent round trip per
// record per lane, covered by the lanes of ~2 waves per SIMD.
// ------------------------------------------------------------------------------------------
__device__ uint64_t find_entry_lane(const FrameParams& P, uint64_t cs, uint64_t ce, uint32_t ver, uint32_t comp,
                                    const uint32_t* crct) {
    const uint8_t* f = P.file;
    const uint32_t m3 = magic3(ver);
    // a whole 128-byte line per step (8 loads, the next dword too), the next line loaded before this one's candidates are
    // tested: two steps in flight. Round 6: the entry search was a chain of dependent 64-byte steps, ~3.5 us each under
    // the walk's load (probe build), C2-ref-random walk 0.129 -> 0.117 ms (profiles/r6/r6r_lane_walk_entry.txt). 16-byte
    // loads at or past the file end read nothing (the device pad covers 64 bytes only).
    auto fetch = [&](uint64_t q, uint4 (&v)[8], uint32_t& t) __attribute__((always_inline)) {
#pragma unroll
        for (uint32_t j = 0; j < 8; j++)
            v[j] = q + 16 * j < P.len ? *reinterpret_cast<const uint4*>(f + q + 16 * j) : zero4();
        t = q + 128 < P.len ? *reinterpret_cast<const uint32_t*>(f + q + 128) : 0u;
    };
    uint64_t q0 = cs & ~127ull;
    uint4 a[8];
    uint32_t t;
    fetch(q0, a, t);
    for (;;) {
        const uint64_t q1 = q0 + 128;
        uint4 na[8];
        uint32_t nt = 0;
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) na[j] = zero4();
        if (q1 < ce) fetch(q1, na, nt);
        // candidate bits of the line's 128 positions (static indices only: the blocks stay in registers)
        uint64_t mlo = 0, mhi = 0;
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const uint32_t nx = j < 7 ? a[j + 1].x : t;
            const uint32_t d[5] = {a[j].x, a[j].y, a[j].z, a[j].w, nx};
            const uint64_t m = (uint64_t)magic_mask(d, q0 + 16 * j, cs, ce, P.len, m3) << (16 * (j & 3));
            if (j < 4)
                mlo |= m;
            else
                mhi |= m;
        }
        while (mlo | mhi) {
            const bool lo = mlo != 0;
            const uint64_t mm = lo ? mlo : mhi;
            const uint64_t p = q0 + (lo ? 0u : 64u) + (uint64_t)__builtin_ctzll(mm);
            if (lo)
                mlo &= mlo - 1;
            else
                mhi &= mhi - 1;
            Hdr hd;
            uint64_t nxp, ol, pd, lf;
            if (frame_record(f, P.len, p, ver, comp, hd, nxp, ol, pd, lf, crct) == RIO_OK) return p;
        }
        if (q1 >= ce) return kNone;
        q0 = q1;
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) a[j] = na[j];
        t = nt;
    }
}

// walk_from for one lane: the same records, slots and summary, with the next record's header loads
// issued before this record's slot stores (on CDNA vmcnt retires loads and stores in issue order: a
// load issued after the stores would wait for them too), so each hop costs one load round trip.
__device__ void walk_from_lane(const FrameParams& P, uint64_t c, uint64_t p, uint32_t ver, uint32_t comp, ChunkSum& s,
                               const uint32_t* crct) {
    const uint8_t* f = P.file;
    const uint64_t ce = chunk_end(P, c);
    uint64_t* so = P.scratch_off + c * P.slots;
    uint64_t* sl = P.scratch_len + c * P.slots;
    uint64_t* sp = P.scratch_pay + c * P.slots;
    bool have = p < ce && p + 32 <= P.len;
    uint4 a = zero4(), b = zero4();
    if (have) {
        a = ldu16(f + p);
        b = ldu16(f + p + 16);
    }
    while (p < ce) {
        Hdr h;
        uint64_t next = 0, olen = 0, pd = 0, lf = 0;
        int e = kFrameSlow;
        if (have) {
            const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            e = frame_fast(w, P.len, p, ver, comp, h, next, olen, pd, crct);
        }
        if (e != RIO_OK) e = frame_slow(f, P.len, p, ver, comp, h, next, olen, pd, lf);
        if (e) {
            s.status = e;
            s.err_off = p;
            if (e == RIO_ERR_HEADER_CRC) {
                s.det0 = h.exp_crc;
                s.det1 = h.act_crc;
            } else if (e == RIO_ERR_MAGIC) {
                s.det0 = h.magic_len;
            } else if (e == RIO_ERR_UNEXPECTED_EOF && h.hdr_len != 0) {
                s.det0 = 1;  // raised by the payload read, not by a header varint
            }
            break;
        }
        have = next < ce && next + 32 <= P.len;
        if (have) {
            a = ldu16(f + next);
            b = ldu16(f + next + 16);
        }
        if (s.count < P.slots) {
            so[s.count] = p;
            sl[s.count] = olen | lf | (h.nil ? kNilBit : 0);
            sp[s.count] = pd;
        }
        s.count++;
        s.bytes += olen;
        p = next;
    }
    s.exit = s.status ? s.err_off : p;
}

constexpr uint32_t kWalkLaneBlock = 256;
#if RIO_SCAN_PROBE
__device__ unsigned long long g_lane[1 << 18][4];
#endif
__global__ void __launch_bounds__(kWalkLaneBlock) k_walk_lane(FrameParams P) {
    __shared__ uint32_t crct[1024];
#if RIO_SCAN_PROBE
    const unsigned long long ta = wall_clock64();
#endif
    if (blockIdx.x == 0 && threadIdx.x == 0) init_state(P);
    crc32c_tab_init(crct);
    const uint64_t c = (uint64_t)blockIdx.x * kWalkLaneBlock + threadIdx.x;
    uint32_t ver, comp;
    if (c >= P.n_chunks || file_header_status(P, ver, comp) != RIO_OK) return;
    const uint64_t cs = chunk_start(P, c), ce = chunk_end(P, c);
#if RIO_SCAN_PROBE
    const unsigned long long tb = wall_clock64();
#endif
    const uint64_t from = c == 0 ? (uint64_t)RIO_FILE_HEADER_BYTES : find_entry_lane(P, cs, ce, ver, comp, crct);
#if RIO_SCAN_PROBE
    const unsigned long long tc = wall_clock64();
#endif
    ChunkSum s = chunk_sum_empty(from);
    if (from != kNone) walk_from_lane(P, c, from, ver, comp, s, crct);
    P.chunks[c] = s;
#if RIO_SCAN_PROBE
    if (c < (1u << 18)) {
        g_lane[c][0] = ta;
        g_lane[c][1] = tb;
        g_lane[c][2] = tc;
        g_lane[c][3] = ((unsigned long long)s.count << 40) | (wall_clock64() & 0xFFFFFFFFFFull);
    }
#endif
}

// ------------------------------------------------------------------------------------------
// Key-point run composition. combine(A, B): A's byte range precedes B's.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ RunSum run_identity() {
    RunSum r;
    r.key = kNone;
    r.out = 0;
    r.cnt = 0;
    r.bytes = 0;
    r.ce = 0;
    r.term = 0;
    r.broken = 0;
    r.term_chunk = 0;
    return r;
}

__device__ __forceinline__ RunSum combine(const RunSum& A, const RunSum& B) {
    if (B.ce == 0) return A;
    if (A.ce == 0) return B;
    if (A.key == kNone) {  // A owns nothing for the inputs the composite can represent
        RunSum r = B;
        return r;
    }
    RunSum r = A;
    r.ce = B.ce;
    if (A.broken || A.term) return r;
    const uint64_t y = A.out;
    if (y >= B.ce) return r;  // B passed through
    if (B.key != kNone && y == B.key) {
        r.out = B.out;
        r.cnt = A.cnt + B.cnt;
        r.bytes = A.bytes + B.bytes;
        r.term = B.term;
        r.broken = B.broken;
        r.term_chunk = B.term_chunk;
        return r;
    }
    r.broken = 1;
    return r;
}

__device__ __forceinline__ RunSum chunk_run(const FrameParams& P, uint64_t c) {
    const ChunkSum s = P.chunks[c];
    RunSum r;
    r.key = s.entry;
    r.out = s.exit;
    r.cnt = s.count;
    r.bytes = s.bytes;
    r.ce = chunk_end(P, c);
    r.term = s.status != RIO_OK;
    r.broken = 0;
    r.term_chunk = c;
    return r;
}

constexpr int kScanBlock = 256;

__device__ void scan_top(const FrameParams& P, RunSum (*buf)[kScanBlock]);
__device__ void scan_finish(const FrameParams& P, const RunSum& total);

// Level 1: inclusive scan of 256 chunk runs per block in LDS (Hillis-Steele, 8 steps). The last
// block to finish (arrival ticket) runs level 2 over the block runs: one launch for the scan.
__global__ void __launch_bounds__(kScanBlock) k_scan_blocks(FrameParams P) {
    __shared__ RunSum buf[2][kScanBlock];
    __shared__ uint32_t last;
    const int t = threadIdx.x;
    const uint64_t c = (uint64_t)blockIdx.x * kScanBlock + t;
    const uint32_t pf = code_pf(kPfScan);
#if RIO_SCAN_PROBE
    uint64_t pt[7];
    pt[0] = wall_clock64();
    if (t == 0) {
        PROBE_MIN(2);
        PROBE_MAX(3);
    }
#endif
    if (P.state->hdr_status != RIO_OK) return;  // block-uniform
    if (P.redo && (!P.state->gz_redo || P.state->compression != P.redo)) return;  // another codec's redo round
    RunSum v = c < P.n_chunks ? chunk_run(P, c) : run_identity();
    int cur = 0;
    buf[cur][t] = v;
    __syncthreads();
#if RIO_SCAN_PROBE
    pt[1] = wall_clock64();
#endif
#pragma unroll 1
    for (int d = 1; d < kScanBlock; d <<= 1) {
        RunSum x = buf[cur][t];
        if (t >= d) x = combine(buf[cur][t - d], x);
        buf[cur ^ 1][t] = x;
        cur ^= 1;
        __syncthreads();
    }
#if RIO_SCAN_PROBE
    pt[2] = wall_clock64();
#endif
    if (c < P.n_chunks) P.chunk_excl[c] = t > 0 ? buf[cur][t - 1] : run_identity();
    if (t == kScanBlock - 1) P.block_runs[blockIdx.x] = buf[cur][t];
    // release this block's run, take a ticket; the last arriver acquires every block's run
    __syncthreads();
#if RIO_SCAN_PROBE
    pt[3] = wall_clock64();
#endif
    if (t == 0) {
        __threadfence();
#if RIO_SCAN_PROBE
        pt[4] = wall_clock64();
#endif
        last = atomicAdd(&P.state->scan_ticket, 1u) == gridDim.x - 1;
#if RIO_SCAN_PROBE
        pt[5] = wall_clock64();
#endif
    }
    code_pf_done(pf);
    __syncthreads();
    if (!last) return;
    __threadfence();
#if RIO_SCAN_PROBE
    pt[6] = wall_clock64();
    if (t == 0)
        for (int k = 0; k < 7; k++) g_probe[4 + k] = pt[k];
#endif
    scan_top(P, buf);
}

// Sequential repair (slow path): walks the true chain chunk by chunk, re-walking any chunk whose
// speculative entry does not match. Runs on one thread; only for files whose speculation broke.
__device__ void slow_path(const FrameParams& P, uint32_t ver, uint32_t comp) {
    ScanState* st = P.state;
    uint64_t cur = RIO_FILE_HEADER_BYTES, base_idx = 0, base_bytes = 0, repairs = 0;
    bool term = false;
    uint64_t term_chunk = 0;
    for (uint64_t c = 0; c < P.n_chunks; c++) {
        ChunkPlace pl{base_idx, base_bytes, 0};
        if (!term && cur < chunk_end(P, c)) {
            if (P.chunks[c].entry != cur) {
                walk_chunk(P, c, cur, ver, comp);
                repairs++;
            }
            const ChunkSum s = P.chunks[c];
            pl.owned = s.count;
            base_idx += s.count;
            base_bytes += s.bytes;
            if (s.status != RIO_OK) {
                term = true;
                term_chunk = c;
            } else {
                cur = s.exit;
            }
        }
        P.place[c] = pl;
    }
    st->slow = 1;
    st->n_repairs = repairs;
    st->n_records = base_idx;
    st->total_bytes = base_bytes;
    if (term) {
        const ChunkSum s = P.chunks[term_chunk];
        st->status = s.status;
        st->status_offset = s.err_off;
        st->det0 = s.det0;
        st->det1 = s.det1;
    } else {
        st->status = RIO_EOF;
        st->status_offset = cur;
    }
}

// Level 2 (k_scan_blocks' last block): scans the block runs in tiles of kScanBlock with a carry,
// decides fast/slow path and the terminal status.
__device__ void scan_top(const FrameParams& P, RunSum (*buf)[kScanBlock]) {
    __shared__ RunSum carry_s;
    ScanState* st = P.state;
    const int t = threadIdx.x;
    if (P.n_chunks == 0) {
        if (t == 0) {
            st->status = RIO_EOF;
            st->status_offset = P.len;
        }
        return;  // (len == 8: the first ReadNext hits EOF)
    }
    if (P.n_blocks <= 64) {
        // one wave, no block barriers: entries 0..63 of the 256-wide Hillis-Steele below are exactly this 64-lane
        // one (its steps d >= 64 leave them alone), and its total is entry 63 (combine returns the other operand
        // of an identity unchanged): the same association, so the same RunSums (files up to 16384 chunks)
        if (t >= 64) return;
        buf[0][t] = t < P.n_blocks ? P.block_runs[t] : run_identity();
        wave_sync_lds();
        int cur = 0;
#pragma unroll 1
        for (int d = 1; d < 64; d <<= 1) {
            RunSum x = buf[cur][t];
            if (t >= d) x = combine(buf[cur][t - d], x);
            buf[cur ^ 1][t] = x;
            cur ^= 1;
            wave_sync_lds();
        }
        if ((uint64_t)t < P.n_blocks) P.block_excl[t] = combine(run_identity(), t > 0 ? buf[cur][t - 1] : run_identity());
        if (t != 0) return;
        const RunSum total = combine(run_identity(), buf[cur][63]);
#if RIO_SCAN_PROBE
        g_probe[19] = wall_clock64();
#endif
        scan_finish(P, total);
#if RIO_SCAN_PROBE
        g_probe[20] = wall_clock64();
#endif
        return;
    }
    if (t == 0) carry_s = run_identity();
    __syncthreads();
    for (uint64_t base = 0; base < P.n_blocks; base += kScanBlock) {
        const uint64_t b = base + t;
        RunSum v = b < P.n_blocks ? P.block_runs[b] : run_identity();
        int cur = 0;
        buf[cur][t] = v;
        __syncthreads();
#if RIO_SCAN_PROBE
        if (t == 0 && base == 0) g_probe[18] = wall_clock64();
#endif
#pragma unroll 1
        for (int d = 1; d < kScanBlock; d <<= 1) {
            RunSum x = buf[cur][t];
            if (t >= d) x = combine(buf[cur][t - d], x);
            buf[cur ^ 1][t] = x;
            cur ^= 1;
            __syncthreads();
        }
        const RunSum carry = carry_s;
        RunSum excl = combine(carry, t > 0 ? buf[cur][t - 1] : run_identity());
        if (b < P.n_blocks) P.block_excl[b] = excl;
        __syncthreads();
        if (t == kScanBlock - 1) carry_s = combine(carry, buf[cur][t]);
        __syncthreads();
    }
    const RunSum total = carry_s;
    if (t != 0) return;
#if RIO_SCAN_PROBE
    g_probe[19] = wall_clock64();
#endif
    scan_finish(P, total);
#if RIO_SCAN_PROBE
    g_probe[20] = wall_clock64();
#endif
}

// The file's state from the composed run of all chunks (one thread): the terminal status, the counts, or the
// sequential repair when a speculative entry did not chain.
__device__ void scan_finish(const FrameParams& P, const RunSum& total) {
    ScanState* st = P.state;
    const uint32_t ver = st->version, comp = st->compression;
    // total.key is chunk 0's forced entry (8): total describes the true chain unless broken.
    if (total.broken) {
        slow_path(P, ver, comp);
        if (st->status == RIO_ERR_MAGIC && st->version != RIO_VERSION1) st->zero_from = st->status_offset + st->det0;
        return;
    }
    st->n_records = total.cnt;
    st->total_bytes = total.bytes;
    if (total.term) {
        const ChunkSum s = P.chunks[total.term_chunk];
        st->status = s.status;
        st->status_offset = s.err_off;
        st->det0 = s.det0;
        st->det1 = s.det1;
    } else {
        st->status = RIO_EOF;  // chain ended exactly at the file end
        st->status_offset = total.out;
    }
    if (st->status == RIO_ERR_MAGIC && st->version != RIO_VERSION1) st->zero_from = st->status_offset + st->det0;
}

// Header length of a snappy stream that is one literal element producing exactly `len` bytes with
// nothing after it, or 0 (an empty stream for an empty record counts as such, header length 0 is
// then harmless). Tag 00: literal, length - 1 = tag >> 2, or 60..63 => 1..4 little-endian bytes.
__device__ __forceinline__ uint32_t snappy_literal_hdr(const uint8_t* p, uint64_t slen, uint64_t len) {
    if (slen == 0) return len == 0 ? 1u : 0u;
    // one literal = 1..5 header bytes + exactly len data bytes: decided from the sizes alone for
    // every compressible record, so only candidates cost a load
    if (slen <= len || slen > len + 5) return 0;
    const uint32_t tag = p[0];
    if (tag & 3u) return 0;
    const uint32_t x = tag >> 2;
    uint64_t L;
    uint32_t h;
    if (x < 60) {
        L = (uint64_t)x + 1;
        h = 1;
    } else {
        const uint32_t nb = x - 59;
        if (slen < 1 + nb) return 0;
        uint64_t v = 0;
        for (uint32_t b = 0; b < nb; b++) v |= (uint64_t)p[1 + b] << (8 * b);
        L = v + 1;
        h = 1 + nb;
    }
    return (L == len && h + L == slen) ? h : 0u;
}
__device__ __forceinline__ bool snappy_single_literal(const uint8_t* p, uint64_t slen, uint64_t len) {
    return snappy_literal_hdr(p, slen, len) != 0;
}

// A chunk's records, placed: file records [base_idx, base_idx + owned) are chunk c's scratch slots
// [0, owned); rec_off / rec_pay / out_off / flags / rec_desc at their global index, 64 records per wave
// step, out_off by a wave prefix sum (coalesced stores instead of one thread's serial record loop).
// `snappy`: look for a record that is not one literal element of its whole length (the probe stops at
// the first). What the chunk found goes back to the caller, which merges it into ScanState.
struct PlaceFlags {
    uint64_t first_bad;  // first record flagged at framing (kNone: none)
    uint64_t n_bad;
    bool mixed;          // a Snappy record that is not one literal (or the probe was off)
    bool huge;           // a stream or record past 32-bit sizes
};

template <uint32_t G>
__device__ PlaceFlags place_chunk(const FrameParams& P, uint64_t c, uint64_t base_idx, uint64_t base_bytes,
                                  uint64_t owned, bool snappy, bool pay_all, uint32_t lane) {
    PlaceFlags fl{kNone, 0, false, false};
    const uint64_t* so = P.scratch_off + c * P.slots;
    const uint64_t* sl = P.scratch_len + c * P.slots;
    const uint64_t* sp = P.scratch_pay + c * P.slots;
    bool mixed = false, huge = false;
    uint64_t carry = base_bytes;
    // scratch of the next 64 records loaded before this step's stores: on CDNA vmcnt retires loads
    // and stores in issue order, so a load issued after the stores would wait for them
    uint64_t l_n = 0, ro_n = 0, pay_n = 0;
    if (lane < owned) {
        l_n = sl[lane];
        ro_n = so[lane];
        pay_n = sp[lane];
    }
    for (uint64_t k0 = 0; k0 < owned; k0 += G) {
        const uint64_t k = k0 + lane;
        const bool v = k < owned;
        const uint64_t l = l_n, ro = ro_n, pay = pay_n, len = v ? l & kLenMask : 0;
        if (k + G < owned) {
            l_n = sl[k + G];
            ro_n = so[k + G];
            pay_n = sp[k + G];
        }
        uint64_t wsum;
        const uint64_t excl = G == 64 ? wave_excl_scan64(len, lane, wsum) : group16_excl_scan64(len, lane, wsum);
        bool bad = false;
        if (v) {
            const uint64_t i = base_idx + k;
            const uint64_t start = ro + (pay & 0xFF), slen = pay >> 8;
            // rec_pay only where a consumer needs it (rec_stream): the stream position and length of a
            // snappy / uncompressed record travel in rec_desc
            const bool wide = slen >= kDescWide || len >= kDescWide;
            P.rec_off[i] = ro;
            if (pay_all || wide) P.rec_pay[i] = pay;
            P.out_off[i] = carry + excl;
            const uint8_t fg = ((l & kNilBit) ? RIO_FLAG_NIL : 0) | ((l & kBadBit) ? RIO_FLAG_CORRUPT : 0) |
                               ((l & kEofBit) ? RIO_FLAG_EOF : 0);
            P.flags[i] = fg;
            bad = (fg & (RIO_FLAG_CORRUPT | RIO_FLAG_EOF)) != 0;  // failed at framing (stream length 0)
            P.rec_desc[i] = make_uint4((uint32_t)start, (uint32_t)(start >> 32), wide ? kDescWide : (uint32_t)slen,
                                       wide ? kDescWide : (uint32_t)len);
            huge = huge || wide;  // (also a size of exactly 2^32 - 1: rec_desc holds the sentinel)
            // a snappy stream that is exactly one literal element of the record's whole length
            // (what golang/snappy emits for incompressible input) decodes as a copy
            if (snappy && fg == 0) mixed |= !snappy_single_literal(P.file + start, slen, len);
        }
        const uint64_t bm = group_ballot<G>(bad);
        if (bm) {
            fl.n_bad += (uint64_t)__popcll(bm);
            if (fl.first_bad == kNone) fl.first_bad = base_idx + k0 + (uint64_t)__builtin_ctzll(bm);
        }
        carry += wsum;
        snappy = snappy && !group_ballot<G>(mixed);
        mixed = mixed || !snappy;  // keep the group's verdict
    }
    fl.mixed = group_ballot<G>(mixed) != 0;
    fl.huge = group_ballot<G>(huge) != 0;
    return fl;
}

// a chunk's flags into the file's state (one lane)
__device__ __forceinline__ void merge_place_flags(const FrameParams& P, const PlaceFlags& f) {
    ScanState* st = P.state;
    if (f.first_bad != kNone) atomicMin((unsigned long long*)&st->first_bad, (unsigned long long)f.first_bad);
    if (f.n_bad) atomicAdd((unsigned long long*)&st->n_bad, (unsigned long long)f.n_bad);
    if (f.huge) atomicOr(&st->huge_streams, 1u);
    // every writer stores the same 1: a plain store, not an atomic (17 k same-address atomics from
    // the chunk waves of a 1 M-record file serialized at L2 and cost 0.35 ms)
    if (f.mixed && st->compression == RIO_COMP_SNAPPY) st->any_mixed = 1u;
}

// Placement: one wave per chunk (place_chunk). Its prologue also does what used to be two launches:
// the capacity check + sentinel out_off[n] (block 0) and, on the device-resident path, the zero-tail
// test of a magic mismatch (grid-stride).
// G lanes per chunk: 64 (a wave) for the wave walk's 32 KiB chunks, 16 for the lane walk's small ones (2..21
// records of 768 B .. 8 KiB: a wave per chunk left most lanes idle, C2-ref-random place 0.058 -> 0.080 ms)
template <uint32_t G>
__global__ void __launch_bounds__(256) k_place(FrameParams P) {
    const uint32_t lane = threadIdx.x & (G - 1);
    const uint64_t c = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    ScanState* st = P.state;
    const uint32_t pf = code_pf(blockIdx.x < kPfBlocks ? kPfPlace : 0);
    if (threadIdx.x == 0) {
        PROBE_MIN(11);
        PROBE_MAX(12);
    }
    if (st->hdr_status != RIO_OK) return;
    if (P.redo && (!st->gz_redo || st->compression != P.redo)) return;  // another codec's redo round
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (st->n_records > P.rec_cap || st->total_bytes > P.out_cap)
            st->capacity_fail = 1;
        else
            P.out_off[st->n_records] = st->total_bytes;
    }
    if (!P.zero_done && st->zero_from != kNone) {
        const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
        uint32_t nz = 0;
        for (uint64_t q = st->zero_from + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < P.len; q += stride)
            nz |= P.file[q];
        if (__any(nz != 0) && lane == 0) atomicOr(&st->zero_nonzero, 1u);
    }
    if (c >= P.n_chunks) return;  // wave-uniform
    ChunkPlace pl;
    if (st->slow) {
        pl = P.place[c];
    } else {
        const uint64_t b = c / kScanBlock;
        const RunSum B = P.block_excl[b];
        const RunSum E = P.chunk_excl[c];
        // chain position entering block b (block 0 is entered at 8 = its forced key). A block
        // owns records only if the chain enters it exactly at its key; otherwise it was passed
        // through (a record spans it) or the chain terminated before it.
        const uint64_t xb = (b == 0) ? (uint64_t)RIO_FILE_HEADER_BYTES : B.out;
        const bool entered = (b == 0) || (!B.term && !B.broken && xb == P.block_runs[b].key);
        pl.owned = 0;
        pl.base_idx = B.cnt + E.cnt;
        pl.base_bytes = B.bytes + E.bytes;
        if (entered && !E.term && !E.broken) {
            const uint64_t y = (E.key == kNone) ? xb : E.out;
            const ChunkSum s = P.chunks[c];
            if (s.entry != kNone && y == s.entry) pl.owned = s.count;
        }
        if (lane == 0) P.place[c] = pl;
    }
    if (pl.owned == 0) return;
    if (pl.base_idx + pl.owned > P.rec_cap || st->n_records > P.rec_cap) return;
    // once any wave has found a mixed record the file takes k_snappy_pipe: later waves skip the probe
    const bool snappy = st->compression == RIO_COMP_SNAPPY && !*(volatile const uint32_t*)&st->any_mixed;
    const bool pay_all = st->compression == RIO_COMP_GZIP || st->compression == RIO_COMP_LZW;
    const PlaceFlags f = place_chunk<G>(P, c, pl.base_idx, pl.base_bytes, pl.owned, snappy, pay_all, lane);
    if (lane == 0) merge_place_flags(P, f);
    if (lane == 0) PROBE_MAX(13);
    code_pf_done(pf);
}

__global__ void __launch_bounds__(256) k_zero(FrameParams P) {
    ScanState* st = P.state;
    const uint64_t from = st->zero_from;
    if (from == kNone || st->hdr_status != RIO_OK) return;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t nz = 0;
    for (uint64_t q = from + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < P.len; q += stride)
        nz |= P.file[q];
    if (nz) atomicOr(&st->zero_nonzero, 1u);
}

// ------------------------------------------------------------------------------------------
// Decode
// ------------------------------------------------------------------------------------------
// dst[d, d+len) = src[0, len), 16 bytes at a time; whole 16-byte stores may overrun the element
// (later elements overwrite those bytes) but never the record end `dlen`.
__device__ __forceinline__ void copy_fwd(uint8_t* dst, uint64_t d, const uint8_t* src, uint64_t len, uint64_t dlen) {
    for (uint64_t k = 0; k < len; k += 16) {
        const uint4 v = ldu16(src + k);
        if (d + k + 16 <= dlen)
            stu16(dst + d + k, v);
        else
            st_partial(dst + d + k, v, (uint32_t)(dlen - d - k));
    }
}

// Uncompressed files, and Snappy files whose every record is one literal (incompressible values:
// the reference benchmark's random records; k_snappy_pipe exits at once for those): 16-lane groups,
// one record per group; each lane moves 16 bytes per step (unaligned load and store; the record's
// last piece is stored exactly).
// kG lanes per record (16, or 4 for files of small records: their 16-lane groups left 12 lanes idle and took a
// dependent round trip per 50-byte record, C5's index copy 0.12 ms for 61 MB); each group's next record's sizes
// are loaded while the current one is copied, and a record moves in rounds of 64 kG bytes (four 16-byte loads per
// lane in flight, then the four stores): the copy was a chain of dependent round trips (sizes, literal header
// byte, then 256 bytes at a time)
template <uint32_t kG>
__device__ __forceinline__ void copy_groups(const FrameParams& P, uint64_t n, bool none) {
    const uint32_t lane = threadIdx.x & (kG - 1);
    const uint64_t grp = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / kG;
    const uint64_t ngrp = ((uint64_t)gridDim.x * blockDim.x) / kG;
    auto meta = [&](uint64_t i, uint64_t& o0, uint64_t& len, const uint8_t*& src) __attribute__((always_inline)) {
        o0 = P.out_off[i];
        len = P.out_off[i + 1] - o0;
        uint64_t start, slen;
        rec_stream(P, i, start, slen);
        // a Snappy record here is one literal of its whole length (k_place checked every record with
        // bytes): its header is the slen - len bytes in front of them, no byte to read
        src = P.file + start + (none ? 0 : slen - len);
    };
    uint64_t o0 = 0, len = 0;
    const uint8_t* src = P.file;
    if (grp < n) meta(grp, o0, len, src);
    for (uint64_t i = grp; i < n; i += ngrp) {
        uint64_t no0 = 0, nlen = 0;
        const uint8_t* nsrc = P.file;
        if (i + ngrp < n) meta(i + ngrp, no0, nlen, nsrc);
        uint8_t* dst = P.out + o0;
        for (uint64_t k0 = 0; k0 < len; k0 += 64 * kG) {
            uint4 v[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) {
                const uint64_t k = k0 + 16 * kG * j + 16 * lane;
                v[j] = k < len ? ldu16_nt(src + k) : zero4();
            }
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) {
                const uint64_t k = k0 + 16 * kG * j + 16 * lane;
                if (k + 16 <= len) {
                    stu16_nt(dst + k, v[j]);
                } else if (k < len) {
                    st_partial(dst + k, v[j], (uint32_t)(len - k));
                }
            }
        }
        o0 = no0;
        len = nlen;
        src = nsrc;
    }
}

__global__ void __launch_bounds__(256) k_copy_records(FrameParams P) {
    const ScanState* st = P.state;
    const uint32_t pf = code_pf(blockIdx.x < kPfBlocks ? kPfCopy : 0);
    if (threadIdx.x == 0 && (blockIdx.x & 63) == 0) PROBE_MIN(14);
    if (st->hdr_status != RIO_OK || st->capacity_fail) return;
    const bool none = st->compression == RIO_COMP_NONE;
    if (!none && !(st->compression == RIO_COMP_SNAPPY && !st->any_mixed)) return;
    const uint64_t n = st->n_records;
    // wave-uniform: the file's mean record size picks the group width
    if (st->total_bytes < kCopySmall * n)
        copy_groups<4>(P, n, none);
    else
        copy_groups<16>(P, n, none);
    if (threadIdx.x == 0 && (blockIdx.x & 63) == 63) PROBE_MAX(15);
    code_pf_done(pf);
}

__device__ void finalize_info(const FrameParams& P) {
    // the file's mean bytes per record, for the context's choice of walk on its next decode (ctx_frame_params)
    if (P.walk_hint && P.state->n_records && P.len > RIO_FILE_HEADER_BYTES)
        *reinterpret_cast<volatile uint64_t*>(P.walk_hint) = (P.len - RIO_FILE_HEADER_BYTES) / P.state->n_records;
    ScanState* st = P.state;
    rio_file_info info;
    info.version = st->version;
    info.compression = st->compression;
    info.reserved0 = 0;
    info.n_chunks = P.n_chunks;
    info.n_repairs = st->n_repairs;
    info.detail0 = 0;
    info.detail1 = 0;
    info.first_bad = kNone;
    info.n_bad = 0;
    if (st->hdr_status != RIO_OK) {
        info.n_records = 0;
        info.total_out_bytes = 0;
        info.status = st->hdr_status;
        info.status_offset = 0;
        info.detail0 = st->det0;
        *P.info = info;
        return;
    }
    info.n_records = st->n_records;
    info.total_out_bytes = st->total_bytes;
    info.status = st->status;
    info.status_offset = st->status_offset;
    info.detail0 = st->det0;
    info.detail1 = st->det1;
    if (st->status == RIO_ERR_MAGIC && st->zero_from != kNone && !st->zero_nonzero) {
        info.status = RIO_EOF_ZERO_TAIL;
        info.detail0 = 0;
    }
    info.first_bad = kNone;
    info.n_bad = 0;
    if (st->capacity_fail) {
        info.status = RIO_ERR_CAPACITY;
    } else {
        // a record the device path hands back ends the sequence there (the adapter re-reads the file)
        const uint64_t u = st->unsupported_rec;
        if (u != kNone && u < st->n_records) {
            info.n_records = u;
            info.total_out_bytes = P.out_off[u];
            info.status = RIO_ERR_UNSUPPORTED;
            info.status_offset = P.rec_off[u];
            info.detail0 = info.detail1 = 0;
        }
        if (st->first_bad < info.n_records) {
            info.first_bad = st->first_bad;
            info.n_bad = st->n_bad;  // (records past a hand-back point never reach this kernel's view)
        }
    }
    if (P.comp_hint != RIO_COMP_UNKNOWN && st->hdr_status == RIO_OK && st->compression != P.comp_hint) {
        info.status = RIO_ERR_ARG;  // the caller's hint launched another codec's kernels: nothing decoded
        info.n_records = 0;
        info.total_out_bytes = 0;
    }
    *P.info = info;
}

// The framing result (host API phase A: the sizes the caller allocates for)
__global__ void k_finalize(FrameParams P) {
    if (threadIdx.x == 0 && blockIdx.x == 0) finalize_info(P);
}

// Last decode step: records of Snappy lanes that met a corrupt record are decoded again one thread
// each (k_snappy_pipe lists the lanes; every record when more than kFailLanes did) in place (a record
// that decoded is rewritten with the same bytes) and flagged where golang/snappy's Decode returns
// ErrCorrupt; then the last block to finish publishes the result (k_finalize's work). One launch.
__device__ __forceinline__ void finish_file(const FrameParams& P) {
    __shared__ uint32_t last;
    ScanState* st = P.state;
    const uint32_t pf = code_pf(kPfFinish);
    if (threadIdx.x == 0) PROBE_MIN(16);
    if (st->hdr_status == RIO_OK && !st->capacity_fail && st->compression == RIO_COMP_SNAPPY && st->n_fail_lanes) {
        auto verify = [&](uint64_t i) {
            if (P.flags[i] & (RIO_FLAG_NIL | RIO_FLAG_CORRUPT | RIO_FLAG_EOF)) return;
            const uint64_t o0 = P.out_off[i], o1 = P.out_off[i + 1];
            uint64_t start, slen;
            rec_stream(P, i, start, slen);
            if (!snappy_decode_thread(P.file + start, slen, P.out + o0, o1 - o0))
                mark_bad(P, i);
        };
        if (st->n_fail_lanes > kFailLanes) {  // the list overflowed: every record
            const uint64_t n = st->n_records, stride = (uint64_t)gridDim.x * blockDim.x;
            for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) verify(i);
        } else {
            for (uint64_t l = blockIdx.x; l < st->n_fail_lanes; l += gridDim.x)
                for (uint64_t i = P.fail_lanes[2 * l] + threadIdx.x; i < P.fail_lanes[2 * l + 1]; i += blockDim.x)
                    verify(i);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd(&st->finish_ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (last && threadIdx.x == 0) {
        __threadfence();
        finalize_info(P);
        PROBE_MAX(17);
    }
    code_pf_done(pf);
}

#if RIO_SCAN_PROBE
// the stamps of the decode that just ran, in us from the walk's first wave; then reset for the next one
__global__ void k_probe_dump(uint64_t n_lane, uint64_t n_wave) {
    if (n_wave) {  // the wave walk's per-wave phases (us): span, fill, frame, rest; windows and fill rounds per wave
        const uint64_t m = n_wave < (1u << 18) ? n_wave : (1u << 18);
        unsigned long long t0 = ~0ull, tend = 0;
        double dur = 0, fl = 0, fr = 0, nw = 0, nr = 0, durmax = 0, sk = 0;
        for (uint64_t c = 0; c < m; c++) t0 = g_wave[c][0] < t0 ? g_wave[c][0] : t0;
        for (uint64_t c = 0; c < m; c++) {
            const double d = (double)(g_wave[c][1] - g_wave[c][0]);
            dur += d;
            durmax = d > durmax ? d : durmax;
            sk += (double)(g_wave[c][0] - t0);
            fl += (double)g_wave[c][2];
            fr += (double)g_wave[c][3];
            nw += (double)g_wave[c][4];
            nr += (double)g_wave[c][5];
            tend = g_wave[c][1] > tend ? g_wave[c][1] : tend;
        }
        printf("WAVE n %llu span %.2f | start mean %.2f | wave mean %.2f max %.2f | fill %.2f frame %.2f rest %.2f | "
               "windows %.2f rounds %.2f\n", (unsigned long long)m, (double)(tend - t0) * 0.01, sk / m * 0.01,
               dur / m * 0.01, durmax * 0.01, fl / m * 0.01, fr / m * 0.01, (dur - fl - fr) / m * 0.01, nw / m, nr / m);
    }
    if (n_lane) {  // the lane walk's per-lane stamps (us): start skew, table + header, entry search, hops, records per lane
        const uint64_t m = n_lane < (1u << 18) ? n_lane : (1u << 18);
        unsigned long long t0 = ~0ull, tend = 0;
        double sk = 0, s1 = 0, s2 = 0, s3 = 0, cnt = 0, skmax = 0, s2max = 0, s3max = 0;
        for (uint64_t c = 0; c < m; c++) t0 = g_lane[c][0] < t0 ? g_lane[c][0] : t0;
        for (uint64_t c = 0; c < m; c++) {
            const unsigned long long a = g_lane[c][0], b = g_lane[c][1], d = g_lane[c][2];
            const unsigned long long e = (d & ~0xFFFFFFFFFFull) | (g_lane[c][3] & 0xFFFFFFFFFFull);
            const unsigned long long e2 = e < d ? e + (1ull << 40) : e;
            const double k = (double)(a - t0), x = (double)(b - a), y = (double)(d - b), z = (double)(e2 - d);
            sk += k; s1 += x; s2 += y; s3 += z; cnt += (double)(g_lane[c][3] >> 40);
            skmax = k > skmax ? k : skmax; s2max = y > s2max ? y : s2max; s3max = z > s3max ? z : s3max;
            tend = e2 > tend ? e2 : tend;
        }
        printf("LANE n %llu span %.2f | start skew mean %.2f max %.2f | table+hdr %.2f | entry mean %.2f max %.2f | hops mean %.2f "
               "max %.2f | records/lane %.2f\n", (unsigned long long)m, (double)(tend - t0) * 0.01, sk / m * 0.01,
               skmax * 0.01, s1 / m * 0.01, s2 / m * 0.01, s2max * 0.01, s3 / m * 0.01, s3max * 0.01, cnt / m);
    }
    const unsigned long long t0 = g_probe[0];
    auto us = [&](int i) { return g_probe[i] >= t0 && g_probe[i] != ~0ull ? (double)(g_probe[i] - t0) * 0.01 : -1.0; };
    printf("PROBE walk_end %.2f scan_first %.2f scan_lastin %.2f | last blk in %.2f ld %.2f hs %.2f st %.2f fence %.2f "
           "atomic %.2f acq %.2f top_ld %.2f top %.2f fin %.2f | place_first %.2f place_lastin %.2f place_end %.2f | "
           "copy_first %.2f copy_end %.2f | finish_first %.2f finish_end %.2f\n",
           us(1), us(2), us(3), us(4), us(5), us(6), us(7), us(8), us(9), us(10), us(18), us(19), us(20), us(11),
           us(12), us(13), us(14), us(15), us(16), us(17));
    for (int i = 0; i < 32; i++) g_probe[i] = (i == 0 || i == 2 || i == 11 || i == 14 || i == 16) ? ~0ull : 0ull;
}
#endif
__global__ void __launch_bounds__(256) k_finish(FrameParams P) { finish_file(P); }
// the files of a batch in one launch: blockIdx.y is the file (each file's 64 blocks take its own ticket)
__global__ void __launch_bounds__(256) k_finish_batch(FrameBatch B) { finish_file(B.f[blockIdx.y]); }

// ------------------------------------------------------------------------------------------
// Single record at an arbitrary offset: MMapReader.ReadNextAt (mmap_reader.go:130-203, 298-356)
// ------------------------------------------------------------------------------------------
// ReadNextAt up to the payload: bounds, header, nil, payload extent. RIO_OK with r.nil, or with
// r.payload_off / r.len (= the payload length in the file) set.
template <class B>
__device__ __forceinline__ int read_at_locate(B& get, uint64_t len, uint32_t ver, uint32_t comp, uint64_t off,
                                              ReadAtResult& r, Hdr& h, const uint32_t* crc_tab = nullptr) {
    r.nil = 0;
    r.len = 0;
    r.det0 = r.det1 = 0;
    if (off > len) return RIO_ERR_INVALID_OFFSET;  // x/exp/mmap ReadAt bounds
    // readNextAtV1 (mmap_reader.go:205-221): a 20-byte ReadAt short of its buffer fails wrapping io.EOF
    if (ver == RIO_VERSION1 && len - off < RIO_RECORD_HEADER_V1_BYTES) return RIO_EOF_HEADER;
    const uint64_t wmax = ver == RIO_VERSION4 ? RIO_RECORD_HEADER_V4_MAX : RIO_RECORD_HEADER_V3_MAX;
    const uint64_t w = len - off < wmax ? len - off : wmax;
    if (w == 0) return RIO_EOF;  // bare io.EOF
    int e = parse_header_t(get, off, w, ver == RIO_VERSION4 ? RIO_RECORD_HEADER_V4_MAX : ~0ull, ver, h, crc_tab);
    if (e == RIO_EOF) e = RIO_EOF_HEADER;
    if (e == RIO_ERR_HEADER_CRC) {
        r.det0 = h.exp_crc;
        r.det1 = h.act_crc;
    }
    if (e) return e;
    r.hdr_len = h.hdr_len;
    if (h.nil) {
        r.nil = 1;
        return RIO_OK;
    }
    const uint64_t plen = comp != RIO_COMP_NONE ? h.c : h.u;
    if (plen > len - off - h.hdr_len) return RIO_EOF_PAYLOAD;
    r.payload_off = off + h.hdr_len;
    r.len = plen;
    return RIO_OK;
}

__device__ int read_at_dev(const uint8_t* f, uint64_t len, uint32_t ver, uint32_t comp, uint64_t off,
                           uint8_t* out, uint64_t out_cap, ReadAtResult& r, bool write) {
    Hdr h;
    RawBytes raw{f};
    const int e0 = read_at_locate(raw, len, ver, comp, off, r, h);
    if (e0 || r.nil) return e0;
    const uint64_t plen = r.len;
    const uint8_t* pay = f + off + h.hdr_len;
    if (comp == RIO_COMP_NONE) {
        if (!write) return RIO_OK;
        if (plen > out_cap) return RIO_ERR_CAPACITY;
        for (uint64_t k = 0; k < plen; k++) out[k] = pay[k];
        return RIO_OK;
    }
    if (comp == RIO_COMP_GZIP || comp == RIO_COMP_LZW) {
        // gzip.NewReader on an empty payload: io.EOF (mmap_reader.go:189-191 wraps it); lzw: an empty
        // payload is io.ErrUnexpectedEOF. A payload to inflate / expand is the host's: it serves record
        // starts from the reader's decoded index and hands anything else back (r.payload_off / r.len
        // locate it)
        if (plen == 0) return comp == RIO_COMP_GZIP ? RIO_EOF_CODEC : RIO_ERR_DECOMPRESS;
        return RIO_ERR_UNSUPPORTED;
    }
    uint64_t dl = 0;
    const int k = uvarint_buf(pay, plen, dl);
    if (k <= 0 || dl > 0xFFFFFFFFull || dl > 22ull * (plen - (uint64_t)k) + 64) return RIO_ERR_DECOMPRESS;
    r.len = dl;
    if (dl > out_cap) return RIO_ERR_CAPACITY;
    if (!snappy_decode_thread(pay + k, plen - (uint64_t)k, out, dl)) return RIO_ERR_DECOMPRESS;
    return RIO_OK;
}

__global__ void k_read_at(const uint8_t* f, uint64_t len, uint64_t off, uint8_t* out, uint64_t out_cap,
                          ReadAtResult* res) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    ReadAtResult r{};
    uint32_t ver = 0, comp = 0;
    int e = RIO_OK;
    if (len < RIO_FILE_HEADER_BYTES) {
        e = RIO_ERR_SHORT_FILE_HEADER;
    } else {
        ver = f[0] | (uint32_t)f[1] << 8 | (uint32_t)f[2] << 16 | (uint32_t)f[3] << 24;
        comp = f[4] | (uint32_t)f[5] << 8 | (uint32_t)f[6] << 16 | (uint32_t)f[7] << 24;
        if (ver > RIO_VERSION4 || ver < RIO_VERSION1) e = RIO_ERR_VERSION;
        else if (comp > RIO_COMP_LZW) e = RIO_ERR_COMPRESSION_TYPE;
    }
    if (e == RIO_OK) e = read_at_dev(f, len, ver, comp, off, out, out_cap, r, true);
    r.status = e;
    *res = r;
}

// MMapReader.SeekNext (mmap_reader.go:58-128): windowed scan for 91 8d 4c with its skip rule,
// trial ReadNextAt per hit; CRC / magic / io.EOF-class failures continue the scan. Returns the
// status; on RIO_OK r describes the record at rec_off (payload_off / len when !write).
template <class B, class Trial>
__device__ __forceinline__ int seek_next_t(B& get, uint64_t len, uint64_t off, uint64_t seek_len, Trial&& trial, uint64_t& rec_off) {
    const uint8_t M[3] = {0x91, 0x8D, 0x4C};
    rec_off = 0;
    uint64_t next = off;
    for (;;) {
        if (next > len) return RIO_ERR_INVALID_OFFSET;
        const uint64_t num = len - next < seek_len ? len - next : seek_len;
        if (num == 0) return RIO_EOF;
        uint64_t i = 0;
        bool boundary = false;
        while (i < num) {
            uint64_t ix = i;
            for (int j = 0; j < 3; j++) {
                if (get(next + ix) != M[j]) break;
                ix++;
                if (ix >= num) {
                    boundary = true;
                    break;
                }
            }
            if (boundary) break;
            if (ix - i < 3) {
                i = ix + 1;
                continue;
            }
            const uint64_t at = next + i;
            const int te = trial(at);
            if (te != RIO_OK && (te == RIO_ERR_HEADER_CRC || te == RIO_ERR_MAGIC || te == RIO_EOF ||
                                 te == RIO_EOF_HEADER || te == RIO_EOF_PAYLOAD || te == RIO_EOF_CODEC)) {
                i = ix;
                continue;
            }
            rec_off = at;
            return te;
        }
        if (i == 0) return RIO_EOF;
        next += i;
    }
}

__device__ int seek_next_dev(const uint8_t* f, uint64_t len, uint32_t ver, uint32_t comp, uint64_t off,
                             uint64_t seek_len, uint8_t* out, uint64_t out_cap, bool write, ReadAtResult& r,
                             uint64_t& rec_off) {
    RawBytes raw{f};
    return seek_next_t(raw, len, off, seek_len,
                       [&](uint64_t at) { return read_at_dev(f, len, ver, comp, at, out, out_cap, r, write); }, rec_off);
}

__device__ __forceinline__ int file_header_dev(const uint8_t* f, uint64_t len, uint32_t& ver, uint32_t& comp) {
    ver = comp = 0;
    if (len < RIO_FILE_HEADER_BYTES) return RIO_ERR_SHORT_FILE_HEADER;
    ver = f[0] | (uint32_t)f[1] << 8 | (uint32_t)f[2] << 16 | (uint32_t)f[3] << 24;
    comp = f[4] | (uint32_t)f[5] << 8 | (uint32_t)f[6] << 16 | (uint32_t)f[7] << 24;
    if (ver > RIO_VERSION4 || ver < RIO_VERSION1) return RIO_ERR_VERSION;
    if (comp > RIO_COMP_LZW) return RIO_ERR_COMPRESSION_TYPE;
    if (ver < RIO_VERSION2) return RIO_ERR_UNSUPPORTED;  // SeekNext: mmap_reader.go:62-64
    return RIO_OK;
}

__global__ void k_seek_next(const uint8_t* f, uint64_t len, uint64_t off, uint64_t seek_len, uint8_t* out,
                            uint64_t out_cap, ReadAtResult* res, uint64_t* rec_off) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    ReadAtResult r{};
    uint64_t ro = 0;
    uint32_t ver, comp;
    int e = file_header_dev(f, len, ver, comp);
    if (e == RIO_OK) e = seek_next_dev(f, len, ver, comp, off, seek_len, out, out_cap, true, r, ro);
    r.status = e;
    *rec_off = ro;
    *res = r;
}

// ------------------------------------------------------------------------------------------
// SeekNext map of a decoded file (rio_reader_seek_next). MMapReader.SeekNext (mmap_reader.go:58-128)
// visits positions from its offset one by one; only a 0x91 byte changes the walk: 91 X (X != 8d)
// jumps to p+2, 91 8d Y (Y != 4c) to p+3, and a marker 91 8d 4c runs a trial ReadNextAt whose
// io.EOF / magic / header-CRC class continues at p+3 while anything else ends the call. With windows
// of >= 4 bytes the walk does not depend on where windows start (a marker cut by a window end is
// re-read from its start). So the answer from offset s is fixed by the first 0x91 at or after s:
// P = every 0x91 position in file order, R[k] = the walk's end from P[k] — a record j of the decoded
// sequence (its trial is record j, answered from the decoded arena), kSeekEof (the walk passes the
// last 0x91 and the scan reads to the file end: io.EOF) or kSeekOther (a trial outside the sequence
// that ends the walk: the single-record kernel answers those; a partial marker at the file end is
// kSeekEof, as the reference's rewind there returns io.EOF). Built once per reader:
//   k_count91 / k_scan_segs / k_list91: P (a wave per 4 KiB segment, ballot-free lane prefix);
//   k_seek_step: each position's own step (terminal, or the index of the next 0x91 visited);
//   k_seek_jump: pointer jumping to each walk's end (log2 of the longest walk rounds).
// ------------------------------------------------------------------------------------------
constexpr uint64_t kSeekOther = ~0ull >> 1;
constexpr uint64_t kSeekEof = kSeekOther - 1;  // the walk passed the last 0x91 without a trial ending it: io.EOF
constexpr uint64_t kSeekTerm = 1ull << 63;
constexpr uint32_t kSegBytes = 4096;

__device__ __forceinline__ uint32_t count91(const uint8_t* f, uint64_t at, uint64_t len, uint32_t* mask4) {
    // bytes [at, at + 64) equal to 0x91 (bounded by len); mask4[q]: bit j = byte 16q + j. Loads stay
    // below len + RIO_DEVICE_PAD: a lane starting at or past len reads nothing
    uint32_t c = 0;
    if (at >= len) {
        mask4[0] = mask4[1] = mask4[2] = mask4[3] = 0;
        return 0;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint4 v = *reinterpret_cast<const uint4*>(f + at + 16 * q);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t m = 0;
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int j = 0; j < 4; j++)
                m |= (((w[t] >> (8 * j)) & 0xFFu) == 0x91u ? 1u : 0u) << (4 * t + j);
        const uint64_t base = at + 16 * q;
        if (base + 16 > len) m &= base >= len ? 0u : ((1u << (len - base)) - 1u);
        mask4[q] = m;
        c += __builtin_popcount(m);
    }
    return c;
}

__device__ __forceinline__ uint32_t wave_excl_sum(uint32_t v, uint32_t lane, uint32_t& total) {
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        x += lane >= (uint32_t)d ? y : 0u;
    }
    total = __shfl(x, 63, 64);
    return x - v;
}

__global__ void __launch_bounds__(256) k_count91(const uint8_t* f, uint64_t len, uint64_t nseg, uint64_t* cnt) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t seg = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (seg >= nseg) return;
    uint32_t m[4];
    const uint32_t c = count91(f, seg * kSegBytes + lane * 64, len, m);
    uint32_t total;
    (void)wave_excl_sum(c, lane, total);
    if (lane == 0) cnt[seg] = total;
}

// exclusive prefix sum of cnt[0, n) in place, one block; cnt[n] = the total
__global__ void __launch_bounds__(1024) k_scan_segs(uint64_t* cnt, uint64_t n) {
    __shared__ uint64_t part[1024];
    const uint64_t per = (n + 1023) / 1024, a = threadIdx.x * per, b = a + per < n ? a + per : n;
    uint64_t sum = 0;
    for (uint64_t i = a; i < b; i++) sum += cnt[i];
    part[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint64_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint64_t run = part[threadIdx.x] - sum;
    for (uint64_t i = a; i < b; i++) {
        const uint64_t c = cnt[i];
        cnt[i] = run;
        run += c;
    }
    if (threadIdx.x == 1023) cnt[n] = part[1023];
}

__global__ void __launch_bounds__(256) k_list91(const uint8_t* f, uint64_t len, uint64_t nseg, const uint64_t* base,
                                                uint64_t* P) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t seg = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (seg >= nseg) return;
    const uint64_t at = seg * kSegBytes + lane * 64;
    uint32_t m[4];
    const uint32_t c = count91(f, at, len, m);
    uint32_t total;
    uint64_t o = base[seg] + wave_excl_sum(c, lane, total);
    for (int q = 0; q < 4; q++)
        for (uint32_t x = m[q]; x; x &= x - 1) P[o++] = at + 16 * q + __builtin_ctz(x);
}

__device__ __forceinline__ uint64_t lower_u64(const uint64_t* a, uint64_t n, uint64_t key) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(256) k_seek_step(const uint8_t* f, uint64_t len, const uint64_t* P, uint64_t K,
                                                   const uint64_t* rec_off, const uint8_t* flags, uint64_t n,
                                                   uint64_t* step) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t ver = 0, comp = 0;
    const int he = file_header_dev(f, len, ver, comp);
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < K; k += stride) {
        const uint64_t p = P[k];
        uint64_t out = kSeekTerm | kSeekOther, c = 0;
        if (he == RIO_OK && (p + 1 >= len || (f[p + 1] == 0x8D && p + 2 >= len))) {
            // a partial marker at the file end: SeekNext re-reads from it, its window ends inside the
            // marker with i == 0, and the call returns io.EOF (mmap_reader.go:88-124)
            out = kSeekTerm | kSeekEof;
        } else if (he == RIO_OK) {
            if (f[p + 1] != 0x8D) {
                c = p + 2;
            } else {
                if (f[p + 2] != 0x4C) {
                    c = p + 3;
                } else {
                    const uint64_t j = lower_u64(rec_off, n, p);
                    if (j < n && rec_off[j] == p) {
                        if (flags[j] & RIO_FLAG_EOF) c = p + 3;  // its trial is io.EOF class: the walk goes on
                        else out = kSeekTerm | j;
                    } else {  // a marker outside the decoded sequence: its own trial, as the reference runs it
                        ReadAtResult r{};
                        Hdr h;
                        RawBytes raw{f};
                        const int te = read_at_locate(raw, len, ver, comp, p, r, h);
                        const bool benign = te == RIO_ERR_HEADER_CRC || te == RIO_ERR_MAGIC || te == RIO_EOF ||
                                            te == RIO_EOF_HEADER || te == RIO_EOF_PAYLOAD ||
                                            (te == RIO_OK && !r.nil && comp == RIO_COMP_GZIP && r.len == 0);
                        if (benign) c = p + 3;
                    }
                }
            }
        }
        if (c) {
            const uint64_t nk = lower_u64(P, K, c);
            out = nk < K ? nk : (kSeekTerm | kSeekEof);  // no 0x91 left: the scan reads to the file end
        }
        step[k] = out;
    }
}

__global__ void __launch_bounds__(256) k_seek_jump(const uint64_t* in, uint64_t* out, uint64_t K) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < K; k += stride) {
        const uint64_t v = in[k];
        out[k] = (v & kSeekTerm) ? v : in[v];
    }
}

// P and R (host vectors) of a device-resident file and its decoded record offsets / flags
int build_seek_map(const uint8_t* f, uint64_t len, const uint64_t* rec_off, const uint8_t* flags, uint64_t n,
                   std::vector<uint64_t>& P, std::vector<uint64_t>& R, hipStream_t s) {
    P.clear();
    R.clear();
    const uint64_t nseg = (len + kSegBytes - 1) / kSegBytes;
    if (nseg == 0) return 0;
    uint64_t *cnt = nullptr, *dP = nullptr, *a = nullptr, *b = nullptr;
    auto done = [&](int rc) {
        if (cnt) (void)hipFree(cnt);
        if (dP) (void)hipFree(dP);
        if (a) (void)hipFree(a);
        if (b) (void)hipFree(b);
        return rc;
    };
    if (hipMalloc(&cnt, (nseg + 1) * 8) != hipSuccess) return done(-1);
    const unsigned gs = (unsigned)((nseg + 3) / 4);
    hipLaunchKernelGGL(k_count91, dim3(gs), dim3(256), 0, s, f, len, nseg, cnt);
    hipLaunchKernelGGL(k_scan_segs, dim3(1), dim3(1024), 0, s, cnt, nseg);
    uint64_t K = 0;
    if (hipMemcpyAsync(&K, cnt + nseg, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        return done(-1);
    if (K == 0) return done(0);
    if (hipMalloc(&dP, K * 8) != hipSuccess || hipMalloc(&a, K * 8) != hipSuccess || hipMalloc(&b, K * 8) != hipSuccess)
        return done(-1);
    hipLaunchKernelGGL(k_list91, dim3(gs), dim3(256), 0, s, f, len, nseg, cnt, dP);
    hipLaunchKernelGGL(k_seek_step, dim3(1024), dim3(256), 0, s, f, len, dP, K, rec_off, flags, n, a);
    for (int round = 0; round < 40; round++) {  // walks of up to 2^40 steps
        hipLaunchKernelGGL(k_seek_jump, dim3(1024), dim3(256), 0, s, a, b, K);
        std::swap(a, b);
    }
    P.resize(K);
    R.resize(K);
    if (hipMemcpyAsync(P.data(), dP, K * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(R.data(), a, K * 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        return done(-1);
    for (uint64_t& r : R) r = (r & kSeekTerm) ? (r & ~kSeekTerm) : kSeekOther;  // unfinished walks: the kernel
    return done(hipGetLastError() == hipSuccess ? 0 : -1);
}

// ------------------------------------------------------------------------------------------
// DiskKeyIndex lookups (sstables/disk_key_index.go:87-140), one lane per query key: the reference's
// binarySearch over byte offsets [0, size) of an uncompressed index.rio, each probe findAt(h) =
// SeekNext(h) + proto.Unmarshal into an IndexEntry, compared with bytes.Compare. Every lane runs
// the exact probe sequence of a freshly loaded index (SeekNext is not monotone in h because of the
// scan's skip rule, so a table of record starts alone would not reproduce it).
// ------------------------------------------------------------------------------------------
// bytes.Compare(file[a, a + an), key[0, bn)): the file side through the lane's window
__device__ __forceinline__ int bytes_compare_dev(WinBytes& wb, uint64_t a, uint64_t an, const uint8_t* b, uint64_t bn) {
    const uint64_t m = an < bn ? an : bn;
    for (uint64_t k = 0; k < m; k++) {
        const uint32_t x = wb(a + k), y = b[k];
        if (x != y) return x < y ? -1 : 1;
    }
    return an < bn ? -1 : (an > bn ? 1 : 0);
}

// findAt: 0 and the entry's fields (key_off absolute in f), or a status. All bytes come through the
// lane's 16-byte window: one load per 16 bytes scanned or parsed instead of one per byte (the
// kernel is bound by L2 requests, not by latency).
__device__ __forceinline__ int index_find_at(WinBytes& wb, uint64_t len, uint32_t ver, uint64_t h, uint64_t seek_len,
                                             const uint32_t* T, uint64_t& ko, uint64_t& kl, uint64_t& vo, uint64_t& cs) {
    ReadAtResult r{};
    Hdr hd;
    uint64_t ro;
    const int e = seek_next_t(
        wb, len, h, seek_len,
        [&](uint64_t at) __attribute__((always_inline)) {
            return read_at_locate(wb, len, ver, RIO_COMP_NONE, at, r, hd, T);
        },
        ro);
    if (e) return e;
    const uint64_t pl = r.nil ? 0 : r.len;
    const uint64_t po = r.nil ? 0 : r.payload_off;
    if (!pb_index_entry_t(wb, po, pl, ko, kl, vo, cs)) return RIO_ERR_PROTO;
    ko += po;
    return RIO_OK;
}

__device__ __forceinline__ bool eof_class(int e) {
    return e == RIO_EOF || e == RIO_EOF_ZERO_TAIL || e == RIO_EOF_HEADER || e == RIO_EOF_PAYLOAD || e == RIO_EOF_CODEC;
}

// minimum waves per SIMD for k_index_search (0 = the compiler's choice: 129 VGPRs, 3 waves). Measured on
// the idx bench (M lookups/s): 3 waves 155.6, 4 189.3, 5 199.0, 6 21.2 (3393 scratch ops in the probe
// loop), 8 228.9 (64 VGPRs, 384 B scratch, 281 scratch ops). The spill placement is the compiler's and
// changes with the bound; re-measure after touching this kernel.
#ifndef RIO_IDX_OCC
#define RIO_IDX_OCC 8
#endif
#if RIO_IDX_OCC
__global__ void __launch_bounds__(256, RIO_IDX_OCC) k_index_search(
#else
__global__ void __launch_bounds__(256) k_index_search(
#endif
    const uint8_t* f, uint64_t len, uint64_t seek_len, const uint8_t* keys, const uint64_t* key_off, uint64_t nq,
    const uint32_t* perm, rio_index_hit* hits) {
    __shared__ uint32_t T[1024];  // CRC-32C tables (T[0..255] = the byte table)
    crc32c_tab_init(T);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t ver, comp;
    const int he = file_header_dev(f, len, ver, comp);
    for (uint64_t qq = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; qq < nq; qq += stride) {
        const uint64_t q = perm ? perm[qq] : qq;  // queries in key order (rio_sort.hip), results in place
        rio_index_hit out{};
        const uint8_t* key = keys + key_off[q];
        const uint64_t klen = key_off[q + 1] - key_off[q];
        int e = he;
        if (e == RIO_OK && comp != RIO_COMP_NONE) e = RIO_ERR_UNSUPPORTED;
        uint64_t ko = 0, kl = 0, vo = 0, cs = 0;
        WinBytes wb{f};
        if (e == RIO_OK) {
            uint64_t i = 0, j = len;
            while (i < j) {
                const uint64_t h = (i + j) >> 1;
                e = index_find_at(wb, len, ver, h, seek_len, T, ko, kl, vo, cs);
                if (e) break;
                if (bytes_compare_dev(wb, ko, kl, key, klen) < 0) i = h + 1; else j = h;
            }
            if (e == RIO_OK) {
                e = index_find_at(wb, len, ver, i, seek_len, T, ko, kl, vo, cs);
                if (e == RIO_OK) {
                    out.offset = i;
                    out.found = i < len && bytes_compare_dev(wb, ko, kl, key, klen) == 0;
                    if (out.found) {
                        out.value_offset = vo;
                        out.checksum = cs;
                    }
                }
            }
            if (eof_class(e)) {  // binarySearch: an io.EOF probe means "not found" at offset size
                e = RIO_OK;
                out.offset = len;
            }
        }
        out.status = e;
        hits[q] = out;
    }
}

// DiskKeyIndex lookups on a compressed index.rio (rio_index_open builds the view): the same binarySearch
// per query lane, each probe findAt(h) answered from the decoded records and the SeekNext map instead
// of the raw file: the first 0x91 at or after h fixes SeekNext's answer (windows of 4096 bytes), which
// is record R[k] (its IndexEntry parsed from the decoded arena), io.EOF (no 0x91 left, or a walk that
// runs past the last one), the record's codec error, or a trial outside the decoded sequence (handed
// back: RIO_ERR_UNSUPPORTED for that query).
__device__ __forceinline__ int index_view_find_at(const uint8_t* out, const uint64_t* out_off, const uint8_t* flags,
                                                  uint64_t n, const uint64_t* P, uint64_t K, const uint64_t* R,
                                                  uint64_t h, uint64_t& ko, uint64_t& kl, uint64_t& vo, uint64_t& cs) {
    const uint64_t k = lower_u64(P, K, h);
    if (k >= K) return RIO_EOF;
    const uint64_t r = R[k];
    if (r == kSeekEof) return RIO_EOF;
    if (r >= n) return RIO_ERR_UNSUPPORTED;
    if (flags[r] & RIO_FLAG_CORRUPT) return RIO_ERR_DECOMPRESS;
    if (flags[r] & RIO_FLAG_EOF) return RIO_EOF_CODEC;  // (the map walks past those)
    const uint64_t base = out_off[r], pl = out_off[r + 1] - base;  // a nil record: no bytes
    if (!pb_index_entry(out + base, pl, ko, kl, vo, cs)) return RIO_ERR_PROTO;
    ko += base;
    return RIO_OK;
}

__device__ __forceinline__ int bytes_compare_mem(const uint8_t* a, uint64_t an, const uint8_t* b, uint64_t bn) {
    const uint64_t m = an < bn ? an : bn;
    for (uint64_t k = 0; k < m; k++)
        if (a[k] != b[k]) return a[k] < b[k] ? -1 : 1;
    return an < bn ? -1 : (an > bn ? 1 : 0);
}

__global__ void __launch_bounds__(256) k_index_search_view(const uint8_t* out, const uint64_t* out_off,
                                                           const uint8_t* flags, uint64_t n, const uint64_t* P,
                                                           uint64_t K, const uint64_t* R, uint64_t len,
                                                           const uint8_t* keys, const uint64_t* key_off, uint64_t nq,
                                                           const uint32_t* perm, rio_index_hit* hits) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t qq = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; qq < nq; qq += stride) {
        const uint64_t q = perm ? perm[qq] : qq;
        rio_index_hit o{};
        const uint8_t* key = keys + key_off[q];
        const uint64_t klen = key_off[q + 1] - key_off[q];
        uint64_t ko = 0, kl = 0, vo = 0, cs = 0, i = 0, j = len;
        int e = RIO_OK;
        while (i < j) {
            const uint64_t h = (i + j) >> 1;
            e = index_view_find_at(out, out_off, flags, n, P, K, R, h, ko, kl, vo, cs);
            if (e) break;
            if (bytes_compare_mem(out + ko, kl, key, klen) < 0) i = h + 1; else j = h;
        }
        if (e == RIO_OK) {
            e = index_view_find_at(out, out_off, flags, n, P, K, R, i, ko, kl, vo, cs);
            if (e == RIO_OK) {
                o.offset = i;
                o.found = i < len && bytes_compare_mem(out + ko, kl, key, klen) == 0;
                if (o.found) {
                    o.value_offset = vo;
                    o.checksum = cs;
                }
            }
        }
        if (eof_class(e)) {  // binarySearch: an io.EOF probe means "not found" at offset size
            e = RIO_OK;
            o.offset = len;
        }
        o.status = e;
        hits[q] = o;
    }
}

hipError_t launch_index_search_view(const uint8_t* out, const uint64_t* out_off, const uint8_t* flags, uint64_t n,
                                    const uint64_t* P, uint64_t K, const uint64_t* R, uint64_t len, const uint8_t* keys,
                                    const uint64_t* key_off, uint64_t nq, const uint32_t* perm, rio_index_hit* hits,
                                    hipStream_t s) {
    if (nq == 0) return hipSuccess;
    const uint64_t blocks = (nq + 255) / 256;
    hipLaunchKernelGGL(k_index_search_view, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0, s, out,
                       out_off, flags, n, P, K, R, len, keys, key_off, nq, perm, hits);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Host-side launchers (called by rio_capi.cpp)
// ------------------------------------------------------------------------------------------
static inline unsigned blocks_for(uint64_t n, unsigned bs) {
    uint64_t b = (n + bs - 1) / bs;
    return (unsigned)(b == 0 ? 1 : b);
}

// Stage timing rides on the kernels' own dispatches (hipExtLaunchKernelGGL's start / stop events): a separate
// hipEventRecord puts a marker packet between two kernels and cost ~5.6 us of idle queue each (rocprofv3 trace of a
// C2 step, profiles/r5/r5bh_ext_events_ab.txt); without events the launches are plain.
template <typename K, typename A>
static void launch_ev(K kernel, dim3 g, dim3 b, hipStream_t s, hipEvent_t start, hipEvent_t stop, const A& P) {
    if (!start && !stop) {
        hipLaunchKernelGGL(kernel, g, b, 0, s, P);
        return;
    }
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
        hipExtLaunchKernelGGL(kernel, g, b, 0, s, start, stop, 0, P);
        return;
    }
    // under stream capture the events become record nodes around the kernel
    if (start) (void)hipEventRecord(start, s);
    hipLaunchKernelGGL(kernel, g, b, 0, s, P);
    if (stop) (void)hipEventRecord(stop, s);
}

// Framing: k_walk (file header, state reset, chunk walk), k_scan_blocks (both scan levels). walk_start / walk_stop /
// scan_stop: the stage events (any may be null).
hipError_t launch_frame_ev(const FrameParams& P, hipStream_t s, hipEvent_t walk_start, hipEvent_t walk_stop,
                           hipEvent_t scan_stop) {
    if (P.walk_lane)
        launch_ev(k_walk_lane, dim3(blocks_for(P.n_chunks, kWalkLaneBlock)), dim3(kWalkLaneBlock), s, walk_start, walk_stop, P);
    else
        launch_ev(k_walk, dim3(blocks_for(P.n_chunks, kWalkWaves)), dim3(64 * kWalkWaves), s, walk_start, walk_stop, P);
    launch_ev(k_scan_blocks, dim3(blocks_for(P.n_chunks, kScanBlock)), dim3(kScanBlock), s, nullptr, scan_stop, P);
    return hipGetLastError();
}
hipError_t launch_frame(const FrameParams& P, hipStream_t s, hipEvent_t* ev) {
    return ev ? launch_frame_ev(P, s, ev[0], ev[1], ev[2]) : launch_frame_ev(P, s, nullptr, nullptr, nullptr);
}

// Host API phase A: framing, then the zero-tail test and the sizes (k_finalize) for the caller.
// k_place: 16 lanes per chunk for the lane walk's chunks (RIO_PLACE16=0: a wave always)
#ifndef RIO_PLACE16
#define RIO_PLACE16 1
#endif
static void launch_place(const FrameParams& P, hipStream_t s, hipEvent_t start = nullptr, hipEvent_t stop = nullptr) {
    if (RIO_PLACE16 && P.walk_lane)
        launch_ev(k_place<16>, dim3(blocks_for(P.n_chunks, 16)), dim3(256), s, start, stop, P);
    else
        launch_ev(k_place<64>, dim3(blocks_for(P.n_chunks, 4)), dim3(256), s, start, stop, P);
}

hipError_t launch_phase_a(const FrameParams& P, hipStream_t s, hipEvent_t* ev) {
    launch_frame(P, s, ev);
    hipLaunchKernelGGL(k_zero, dim3(256), dim3(256), 0, s, P);
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(64), 0, s, P);
    return hipGetLastError();
}

hipError_t launch_snappy_decode(const FrameParams& P, hipStream_t s, bool main);  // rio_snappy.hip
hipError_t launch_snappy_batch(const FrameBatch& B, hipStream_t s);             // rio_snappy.hip
hipError_t launch_gzip_decode(const FrameParams& P, hipStream_t s);              // rio_gzip.hip
hipError_t launch_gzip_resize(const FrameParams& P, hipStream_t s);              // rio_gzip.hip
hipError_t launch_lzw_decode(const FrameParams& P, hipStream_t s);               // rio_lzw.hip
hipError_t launch_lzw_resize(const FrameParams& P, hipStream_t s);               // rio_lzw.hip

// gzip redo round: records holding several members (Go's multistream reader) are sized by
// k_gz_resize; then the scan, placement and gzip decoders run again with the corrected sizes. Every
// kernel of the round exits at once unless a record needed it.
static void launch_gzip_redo(const FrameParams& P0, hipStream_t s) {
    FrameParams P = P0;
    P.redo = RIO_COMP_GZIP;
    launch_gzip_resize(P, s);
    hipLaunchKernelGGL(k_scan_blocks, dim3(blocks_for(P.n_chunks, kScanBlock)), dim3(kScanBlock), 0, s, P);
    launch_place(P, s);
    launch_gzip_decode(P, s);
}

// the same round for lzw records whose decoded size is not the header's u
static void launch_lzw_redo(const FrameParams& P0, hipStream_t s) {
    FrameParams P = P0;
    P.redo = RIO_COMP_LZW;
    launch_lzw_resize(P, s);
    hipLaunchKernelGGL(k_scan_blocks, dim3(blocks_for(P.n_chunks, kScanBlock)), dim3(kScanBlock), 0, s, P);
    launch_place(P, s);
    launch_lzw_decode(P, s);
}

// the decoders of one file: by the compression hint, or all of them (each exits unless the file is
// its own)
static void launch_decoders(const FrameParams& P, hipStream_t s, bool snappy_main) {
    const uint32_t c = P.comp_hint;
    const bool any = c == RIO_COMP_UNKNOWN;
    if (any || c == RIO_COMP_NONE || c == RIO_COMP_SNAPPY)
        hipLaunchKernelGGL(k_copy_records, dim3(RIO_COPY_GRID), dim3(256), 0, s, P);
    if ((any || c == RIO_COMP_SNAPPY) && snappy_main) launch_snappy_decode(P, s, true);
    if (any || c == RIO_COMP_GZIP) {
        launch_gzip_decode(P, s);
        launch_gzip_redo(P, s);
    }
    if (any || c == RIO_COMP_LZW) {
        launch_lzw_decode(P, s);
        launch_lzw_redo(P, s);
    }
}

// Decode: placement (+ capacity check, zero tail), the decoders, k_finish (verify + result).
// stage events: [3] at the placement's end, [4] at k_finish's start, so the decode stage is the decoders' span;
// `done` (the context's order event) completes with k_finish
hipError_t launch_phase_b(const FrameParams& P, hipStream_t s, hipEvent_t* ev, hipEvent_t done) {
    launch_place(P, s, nullptr, ev ? ev[3] : nullptr);
    launch_decoders(P, s, true);
    launch_ev(k_finish, dim3(64), dim3(256), s, ev ? ev[4] : nullptr, done, P);
#if RIO_SCAN_PROBE
    hipLaunchKernelGGL(k_probe_dump, dim3(1), dim3(1), 0, s, P.walk_lane ? P.n_chunks : (uint64_t)0,
                       P.walk_lane ? (uint64_t)0 : P.n_chunks);
#endif
    return hipGetLastError();
}

// rio_device_decode_batch: phase B of every file of the batch; the Snappy decoders run once over all
// of them (k_snappy_pipe_batch / k_snappy_coop_batch), the other decode kernels per file
// stage events: [2] at the first placement's start (the framing of every file ends at [1]), [3] at the last
// placement's end, [4] at k_finish_batch's start
hipError_t launch_phase_b_batch(const FrameBatch& B, hipStream_t s, hipEvent_t* ev, hipEvent_t done) {
    for (uint32_t f = 0; f < B.n; f++)
        launch_place(B.f[f], s, (ev && f == 0) ? ev[2] : nullptr, (ev && f + 1 == B.n) ? ev[3] : nullptr);
    launch_snappy_batch(B, s);
    for (uint32_t f = 0; f < B.n; f++) launch_decoders(B.f[f], s, false);
    launch_ev(k_finish_batch, dim3(64, B.n), dim3(256), s, ev ? ev[4] : nullptr, done, B);
    return hipGetLastError();
}

hipError_t launch_read_at(const uint8_t* f, uint64_t len, uint64_t off, uint8_t* out, uint64_t out_cap,
                          ReadAtResult* res, hipStream_t s) {
    hipLaunchKernelGGL(k_read_at, dim3(1), dim3(64), 0, s, f, len, off, out, out_cap, res);
    return hipGetLastError();
}

hipError_t launch_seek_next(const uint8_t* f, uint64_t len, uint64_t off, uint64_t seek_len, uint8_t* out,
                            uint64_t out_cap, ReadAtResult* res, uint64_t* rec_off, hipStream_t s) {
    hipLaunchKernelGGL(k_seek_next, dim3(1), dim3(64), 0, s, f, len, off, seek_len, out, out_cap, res, rec_off);
    return hipGetLastError();
}

hipError_t launch_index_search(const uint8_t* f, uint64_t len, uint64_t seek_len, const uint8_t* keys,
                               const uint64_t* key_off, uint64_t nq, const uint32_t* perm, rio_index_hit* hits,
                               hipStream_t s) {
    if (nq == 0) return hipSuccess;
    const uint64_t blocks = (nq + 255) / 256;
    hipLaunchKernelGGL(k_index_search, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0, s, f, len,
                       seek_len, keys, key_off, nq, perm, hits);
    return hipGetLastError();
}

}  // namespace rio
