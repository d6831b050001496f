// rio_gzip.hip — gzip-compressed records decoded on the device (GzipCompressor.DecompressWithBuf,
// recordio/compressor/gzip_compression.go:54-69: Go compress/gzip Reader over compress/flate,
// called per record by FileReader.ReadNext, file_reader.go:115-125).
//
// Semantics restated from the published formats and Go's reader rules:
//   * RFC 1952 member: ID 1f 8b, CM 8, FLG with FEXTRA / FNAME / FCOMMENT (NUL-terminated, Go's
//     512-byte buffer limit) / FHCRC (low 16 bits of the header's CRC-32), 8-byte trailer
//     CRC-32/IEEE + ISIZE of the member's output.
//   * RFC 1951 blocks: stored (LEN / NLEN), fixed and dynamic Huffman. Go's Huffman acceptance:
//     HLIT <= 286, HDIST <= 30, every code complete except a single 1-bit code, empty distance
//     codes allowed until used; symbols 286/287 and distance codes 30/31 are corrupt; a distance
//     beyond the member's output so far is corrupt.
//   * Several members per record (Go's Reader is multistream): after a member's trailer the next
//     header follows; nothing after a trailer ends the record; anything else that is not a whole
//     header is an error. Each member's CRC-32 and ISIZE cover its own output, and DEFLATE distances
//     never reach into an earlier member (the decompressor is reset per member).
// Every failure is the codec-error class (RIO_ERR_DECOMPRESS).
//
// Sizes: the framing sized each record from its last four payload bytes (the last member's ISIZE),
// which is the record's size when it holds one member. A record whose output does not fit that size
// (several members, or a corrupt single member) is not stored: it is marked for k_gz_resize, which
// counts the output of every member without storing it (and classifies the record as corrupt where
// Go would fail). Then the scan, the placement and these decoders run once more with the counted
// sizes (launch_gzip_redo); every kernel of that round exits at once when no record needed it.
//
// k_gzip_inflate<kWin>: one wavefront per record (grid-stride over records). Huffman decoding is
// inherently serial, so the whole wave runs the decoder in lock step on wave-uniform state (bit
// buffer, tables read from LDS as broadcasts); the lanes split the wide work: loading the input
// into an LDS ring 1 KiB at a time, building the decode tables (ballot-based counting and
// sorting), match copies (64 bytes per round, `k mod dist` for overlapping copies) and flushing
// the LDS output window to HBM 1 KiB at a time. Three instantiations: records decoding to <= 1 KiB and <= 2 KiB
// keep the whole record in a 1 / 2 KiB window (7 / 5 waves per SIMD), larger ones use the 32 KiB DEFLATE
// window.
// k_gzip_crc: one lane per record, CRC-32/IEEE of the decoded bytes against the trailer.
#include <hip/hip_runtime.h>

#include "rio_device.h"
#include "rio_dev_util.h"

namespace rio {

namespace {
constexpr uint32_t kGzWaves = 4;          // waves per workgroup
constexpr uint32_t kGzIn = 2048;          // LDS input ring per wave (two 1 KiB refill blocks)
constexpr uint32_t kGzTinyIn = 1024;      // tiny class: two 512-B refill blocks
constexpr uint32_t kGzTinyWin = 1024;     // records with decoded size <= this: whole record in 1 KiB
constexpr uint32_t kGzSmallWin = 2048;    // records with decoded size <= this: whole record in LDS
constexpr uint32_t kGzLargeWin = 32768;   // DEFLATE window (maximum distance)
constexpr uint32_t kFastBits = 9;         // decode-table bits
constexpr uint32_t kFastSize = 1u << kFastBits;
// 1: literal runs decoded several symbols per fast-table read (below, in gz_record)
#ifndef RIO_GZ_RUN
#define RIO_GZ_RUN 1
#endif
constexpr uint64_t kPayFail = 1ull << 63;    // rec_pay marker: no CRC check by k_gzip_crc (inflate failed,
                                              // or several members, whose CRCs the inflate checked)
constexpr uint64_t kPayResize = 1ull << 62;  // rec_pay marker: output larger than the framing's size
constexpr uint64_t kPayLen = ~(kPayFail | kPayResize);
// RFC 1951 3.2.7 code-length code order; in constant memory so the uniform index is a scalar load
// (a local array indexed at run time lived in scratch)
__constant__ uint8_t kClenOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// per-wave decode tables
template <uint32_t kDB = kFastBits>
struct GzTables {
    uint16_t lfast[kFastSize];  // litlen (also the code-length code): sym | len << 9, 0 = longer code
    uint16_t dfast[1u << kDB];  // distance (kDB index bits: the tiny class keeps 7, distances there are short)
    uint16_t lsym[288];         // symbols sorted by (code length, symbol)
    uint16_t dsym[32];
    uint16_t lcnt[16];          // codes per length
    uint16_t dcnt[16];
    uint8_t lens[288 + 32 + 8];  // code lengths being read (litlen then distance)
};

template <uint32_t kWin, uint32_t kIn, uint32_t kDB = kFastBits>
struct GzLds {
    GzTables<kDB> t;
    uint8_t in[kIn] __attribute__((aligned(16)));
    uint8_t win[kWin] __attribute__((aligned(16)));
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ uint32_t lane_mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// A record is decoded by a group of G lanes: G = 64, the whole wave on wave-uniform state (scalar
// registers); G = 16, four records per wave, the group-uniform state in vector registers (every lane
// of a group computes the same value). The group's view of the wave primitives:
template <uint32_t G>
struct Grp {
    static_assert(G == 64 || G == 16, "group of 16 or 64 lanes");
    __device__ static __forceinline__ uint32_t gl(uint32_t lane) { return lane & (G - 1); }
    // a value every lane of the group holds (G = 64: into a scalar register)
    __device__ static __forceinline__ uint32_t uni(uint32_t v) {
        if constexpr (G == 64) return __builtin_amdgcn_readfirstlane(v); else return v;
    }
    // lane l of the group (l group-uniform)
    __device__ static __forceinline__ uint32_t rl(uint32_t v, uint32_t l, uint32_t lane) {
        if constexpr (G == 64) return __builtin_amdgcn_readlane(v, l);
        else return (uint32_t)__shfl((int)v, (int)((lane & ~(G - 1)) + l), 64);
    }
    // the group's ballot, bit k = lane k of the group
    __device__ static __forceinline__ uint64_t ballot(bool p, uint32_t lane) {
        if constexpr (G == 64) return __ballot(p);
        else return (__ballot(p) >> (lane & ~(G - 1))) & ((1ull << G) - 1);
    }
    // set bits of m below this lane (m a group ballot)
    __device__ static __forceinline__ uint32_t mbcnt(uint64_t m, uint32_t lane) {
        if constexpr (G == 64) return lane_mbcnt(m);
        else return (uint32_t)__builtin_popcountll(m & ((1ull << gl(lane)) - 1ull));
    }
};

// Wave-uniform bit reader over the record's DEFLATE stream [0, slen), staged through an LDS ring of
// kIn bytes refilled kIn / 2 bytes at a time.
template <uint32_t kIn, uint32_t G = 64>
struct BitIn {
    static constexpr uint32_t kBlk = kIn / 2;
    static_assert(kBlk <= 16 * G, "one pass of the group stages a block");
    const uint8_t* src;  // stream start in HBM
    uint8_t* ring;
    uint32_t slen;
    uint32_t loaded;  // stream bytes [loaded - kIn, loaded) are in the ring
    uint32_t pos;     // next stream byte pulled into bb
    uint64_t bb;
    uint32_t nb;

    // bits consumed so far (read-ahead past slen is zero-filled; overrun is checked by the caller)
    __device__ __forceinline__ uint64_t consumed() const { return 8ull * pos - nb; }

    // make stream bytes [p, p + 8) resident (kBlk-byte blocks, 16 bytes per lane)
    __device__ void stage(uint32_t p, uint32_t lane) {
        if (p >= loaded || p + kIn < loaded) loaded = p & ~(kBlk - 1);  // jump (stored block skip)
        while (loaded < p + 8 && loaded < slen) {
            const uint32_t off = loaded + Grp<G>::gl(lane) * 16;
            if (Grp<G>::gl(lane) * 16 < kBlk && off < slen) *reinterpret_cast<uint4*>(ring + (off & (kIn - 1))) = ldu16(src + off);
            loaded += kBlk;
        }
        __builtin_amdgcn_wave_barrier();
    }
    __device__ void refill(uint32_t lane) {
        while (nb <= 32) {
            stage(pos, lane);
            const uint32_t a = pos & ~3u;
            const uint32_t w0 = *reinterpret_cast<const uint32_t*>(ring + (a & (kIn - 1)));
            const uint32_t w1 = *reinterpret_cast<const uint32_t*>(ring + ((a + 4) & (kIn - 1)));
            uint32_t v = Grp<G>::uni(__builtin_amdgcn_alignbyte(w1, w0, pos & 3u));
            const uint32_t valid = pos < slen ? slen - pos : 0u;
            if (valid < 4) v &= valid == 0 ? 0u : (0xFFFFFFFFu >> (32u - 8u * valid));
            bb |= (uint64_t)v << nb;
            nb += 32;
            pos += 4;
        }
    }
    __device__ __forceinline__ uint32_t bits(uint32_t n) {  // n <= 32
        const uint32_t v = (uint32_t)(bb & ((1ull << n) - 1ull));
        bb >>= n;
        nb -= n;
        return v;
    }
    __device__ __forceinline__ bool overrun() const { return consumed() > 8ull * slen; }
};

// Canonical Huffman tables from code lengths lens[0..n) (Go huffmanDecoder.init acceptance).
// Returns false for an invalid (over-subscribed or incomplete) code; an all-zero code is accepted
// and fails when used.
// Lane l in [1, 16) owns code length l (its count, first canonical code and first sorted index);
// uses with a constant l read it back with readlane into a scalar register, so no per-lane arrays
// of wave-uniform values occupy VGPRs.
template <uint32_t G = 64, uint32_t kBits = kFastBits>
__device__ bool gz_build(const uint8_t* lens, uint32_t n, uint16_t* cnt, uint16_t* sym, uint16_t* fast,
                         uint32_t lane_w) {
    using Gr = Grp<G>;
    const uint32_t lane = Gr::gl(lane_w);
    uint32_t my_c = 0;  // codes of length `lane`
    for (uint32_t g = 0; g < n; g += G) {
        const uint32_t s = g + lane;
        const uint32_t L = s < n ? lens[s] : 0u;
#pragma unroll
        for (int l = 1; l < 16; l++) {
            const uint32_t k = (uint32_t)__builtin_popcountll(Gr::ballot(L == (uint32_t)l, lane_w));
            my_c += lane == (uint32_t)l ? k : 0u;
        }
    }
    uint32_t maxl = 0;
#pragma unroll
    for (int l = 1; l < 16; l++) maxl = Gr::rl(my_c, l, lane_w) ? (uint32_t)l : maxl;
    // canonical codes (RFC 1951 3.2.2): first code and first sorted index of every length
    uint32_t code = 0, acc = 0, my_next = 0, my_idx = 0;
#pragma unroll
    for (int l = 1; l < 16; l++) {
        const uint32_t c = Gr::rl(my_c, l, lane_w);
        code <<= 1;
        my_next = lane == (uint32_t)l ? code : my_next;
        my_idx = lane == (uint32_t)l ? acc : my_idx;
        if ((uint32_t)l <= maxl) code += c;
        acc += c;
    }
    if (lane < 16) cnt[lane] = (uint16_t)(lane ? my_c : 0u);
    __builtin_amdgcn_wave_barrier();
    if (maxl == 0) {
        for (uint32_t e = lane; e < (1u << kBits); e += G) fast[e] = 0;
        __builtin_amdgcn_wave_barrier();
        return true;
    }
    // complete code, or Go's exception: a single code of length 1
    const uint32_t full = code >> (15 - maxl);  // codes counted at length maxl
    if (full != (1u << maxl) && !(full == 1 && maxl == 1)) return false;
    // symbols sorted by (length, symbol): rank of each symbol among equal lengths via ballots
    uint32_t my_off = my_idx;  // next free sorted slot of length `lane`
    for (uint32_t g = 0; g < n; g += G) {
        const uint32_t s = g + lane;
        const uint32_t L = s < n ? lens[s] : 0u;
#pragma unroll
        for (int l = 1; l < 16; l++) {
            const uint64_t m = Gr::ballot(L == (uint32_t)l, lane_w);
            const uint32_t base = Gr::rl(my_off, l, lane_w);
            if (L == (uint32_t)l) sym[base + Gr::mbcnt(m, lane_w)] = (uint16_t)s;
            my_off += lane == (uint32_t)l ? (uint32_t)__builtin_popcountll(m) : 0u;
        }
    }
    __builtin_amdgcn_wave_barrier();
    // fast table: entry e = the next kFastBits stream bits (first bit = code MSB)
    // G = 16: the group's per-length values read once (through the LDS crossbar), not per entry
    uint32_t nxl[kBits + 1], cl[kBits + 1], il[kBits + 1];
    if constexpr (G != 64) {
#pragma unroll
        for (int l = 1; l <= (int)kBits; l++) {
            nxl[l] = Gr::rl(my_next, l, lane_w);
            cl[l] = Gr::rl(my_c, l, lane_w);
            il[l] = Gr::rl(my_idx, l, lane_w);
        }
    }
    for (uint32_t e = lane; e < (1u << kBits); e += G) {
        uint32_t v = 0, ent = 0;
#pragma unroll
        for (int l = 1; l <= (int)kBits; l++) {
            v = (v << 1) | ((e >> (l - 1)) & 1u);
            const uint32_t nx = G == 64 ? __builtin_amdgcn_readlane(my_next, l) : nxl[l];
            const uint32_t c = G == 64 ? __builtin_amdgcn_readlane(my_c, l) : cl[l];
            const uint32_t ix = G == 64 ? __builtin_amdgcn_readlane(my_idx, l) : il[l];
            if (ent == 0 && v - nx < c) ent = (uint32_t)sym[ix + v - nx] | ((uint32_t)l << 9);
        }
        fast[e] = (uint16_t)ent;
    }
    __builtin_amdgcn_wave_barrier();
    return true;
}

// One symbol; -1 if the bits match no code (incomplete / empty code).
template <uint32_t kIn, uint32_t G, uint32_t kBits = kFastBits>
__device__ __forceinline__ int gz_sym(BitIn<kIn, G>& B, const uint16_t* fast, const uint16_t* cnt, const uint16_t* sym) {
    using Gr = Grp<G>;
    const uint32_t e = Gr::uni(fast[(uint32_t)B.bb & ((1u << kBits) - 1)]);
    if (e) {
        B.bits(e >> 9);
        return (int)(e & 511u);
    }
    uint32_t code = 0, first = 0, index = 0;
    for (uint32_t l = 1; l < 16; l++) {
        code |= (uint32_t)(B.bb >> (l - 1)) & 1u;
        const uint32_t c = Gr::uni(cnt[l]);
        if (code - first < c) {
            B.bits(l);
            return (int)Gr::uni(sym[index + code - first]);
        }
        index += c;
        first = (first + c) << 1;
        code <<= 1;
    }
    return -1;
}

// DEFLATE length / distance bases (RFC 1951 3.2.5)
__device__ __forceinline__ uint32_t len_base(uint32_t s, uint32_t& eb) {  // s in [257, 285]
    const uint32_t i = s - 257;
    if (i < 8) { eb = 0; return 3 + i; }
    if (i == 28) { eb = 0; return 258; }
    eb = (i - 4) >> 2;
    return ((4u + (i & 3u)) << eb) + 3u;
}
__device__ __forceinline__ uint32_t dist_base(uint32_t s, uint32_t& eb) {  // s in [0, 29]
    if (s < 4) { eb = 0; return s + 1; }
    eb = (s - 2) >> 1;
    return ((2u + (s & 1u)) << eb) + 1u;
}

enum : int { kGzOk = 0, kGzCorrupt = 1, kGzUnsupported = 2, kGzResize = 3, kGzOkChecked = 4 };

// CRC-32/IEEE table for the per-member checks of records of several members (k_gzip_crc checks a
// record against its one trailer; these records are rare, so one lane runs the table loop)
struct CrcTab {
    uint32_t t[256];
    constexpr CrcTab() : t() {
        for (uint32_t k = 0; k < 256; k++) {
            uint32_t c = k;
            for (int j = 0; j < 8; j++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
            t[k] = c;
        }
    }
};
__constant__ CrcTab kCrc = CrcTab();

// running CRC-32 register (pre/post-inverted by the caller) over n bytes of the LDS window from w0
// (`win`) or of global memory (`g`); lane 0 computes, every lane gets the result
template <uint32_t kWin, uint32_t G = 64>
__device__ uint32_t gz_crc_run(uint32_t c, const uint8_t* win, uint32_t w0, const uint8_t* g, uint32_t n,
                               uint32_t lane) {
    if (Grp<G>::gl(lane) == 0)
        for (uint32_t k = 0; k < n; k++) c = kCrc.t[(c ^ (win ? win[(w0 + k) & (kWin - 1)] : g[k])) & 0xFFu] ^ (c >> 8);
    __builtin_amdgcn_wave_barrier();
    return Grp<G>::rl(c, 0, lane);
}

// Inflate one record's gzip members into `out` (dlen bytes, the size the framing or k_gz_resize gave
// it). kWhole: the window holds the whole record (flushed once at the end). kCount (k_gz_resize):
// the record is decoded through the window but nothing is stored, every member's CRC-32 and ISIZE
// are checked, *total = the output of every member; a record Go's reader fails on is kGzCorrupt.
// Output past dlen is never stored: kGzResize (k_gz_resize decides).
template <uint32_t kWin, uint32_t kIn, bool kCount = false, uint32_t G = 64, uint32_t kDB = kFastBits>
__device__ int gz_record(GzLds<kWin, kIn, kDB>& S, const uint8_t* src, uint32_t slen, uint8_t* out, uint32_t dlen,
                         uint32_t lane, uint64_t* total = nullptr) {
    using Gr = Grp<G>;
    const uint32_t gl = Gr::gl(lane);
    constexpr bool kWhole = kWin < kGzLargeWin && !kCount;
    constexpr uint32_t kMaxOut = 0xFFFFFFF0u;  // counted sizes past this are handed back
    const uint32_t cap = kCount ? kMaxOut : dlen;
    GzTables<kDB>& T = S.t;
    BitIn<kIn, G> B{src, S.in, slen, 0, 0, 0ull, 0};
    uint32_t d = 0, flushed = 0, dm = 0;  // dm: output position where the current member starts
    uint32_t mcrc = 0xFFFFFFFFu;          // kCount: CRC-32 register of the member's flushed bytes
    bool multi = false;
    auto flush = [&](uint32_t upto) {  // window bytes [flushed, upto) -> HBM, 16 per lane
        if (kCount) {  // nothing stored: the bytes leaving the window go into the member's CRC
            mcrc = gz_crc_run<kWin, G>(mcrc, S.win, flushed, nullptr, upto - flushed, lane);
            flushed = upto;
            return;
        }
        while (flushed < upto) {
            const uint32_t q = flushed + gl * 16;
            if (q < upto) {
                const uint4 v = *reinterpret_cast<const uint4*>(S.win + (q & (kWin - 1)));
                if (q + 16 <= upto)
                    stu16(out + q, v);
                else
                    st_partial(out + q, v, upto - q);
            }
            flushed = umin(upto, flushed + 16 * G);
        }
    };
  for (;;) {  // members
    B.refill(lane);
    // ---- member header (gzip reader.go readHeader: io.ReadFull of 10 bytes) ----
    if (slen - umin(slen, (uint32_t)(B.consumed() >> 3)) < 10) return kGzCorrupt;
    const uint32_t id = B.bits(16), cm = B.bits(8), flg = B.bits(8);
    if (id != 0x8B1Fu || cm != 8u) return kGzCorrupt;
    B.refill(lane);
    const uint32_t mt = B.bits(32);
    B.refill(lane);
    const uint32_t xo = B.bits(16);  // XFL, OS
    // header CRC-32 (FHCRC) over every header byte read so far
    uint32_t hcrc = 0xFFFFFFFFu;
    auto hbyte = [&](uint32_t b) {
        hcrc ^= b;
#pragma unroll
        for (int k = 0; k < 8; k++) hcrc = (hcrc >> 1) ^ (0xEDB88320u & (0u - (hcrc & 1u)));
    };
    hbyte(0x1F); hbyte(0x8B); hbyte(8); hbyte(flg);
    for (int k = 0; k < 4; k++) hbyte((mt >> (8 * k)) & 0xFF);
    hbyte(xo & 0xFF); hbyte(xo >> 8);
    if (flg & 4u) {  // FEXTRA: XLEN + data
        B.refill(lane);
        const uint32_t xlen = B.bits(16);
        hbyte(xlen & 0xFF); hbyte(xlen >> 8);
        for (uint32_t k = 0; k < xlen; k++) {
            B.refill(lane);
            hbyte(B.bits(8));
        }
        if (B.overrun()) return kGzCorrupt;
    }
    for (uint32_t f = 8; f <= 16; f <<= 1) {  // FNAME, FCOMMENT: NUL-terminated, < 512 bytes
        if (!(flg & f)) continue;
        for (uint32_t k = 0;; k++) {
            if (k >= 512) return kGzCorrupt;
            B.refill(lane);
            const uint32_t b = B.bits(8);
            if (B.overrun()) return kGzCorrupt;
            hbyte(b);
            if (b == 0) break;
        }
    }
    if (flg & 2u) {  // FHCRC
        B.refill(lane);
        const uint32_t h16 = B.bits(16);
        if (h16 != ((hcrc ^ 0xFFFFFFFFu) & 0xFFFFu)) return kGzCorrupt;
    }
    if (B.overrun()) return kGzCorrupt;

    // ---- DEFLATE blocks (flate inflate.go) ----
    bool fin = false;
    while (!fin) {
        B.refill(lane);
        fin = B.bits(1) != 0;
        const uint32_t type = B.bits(2);
        if (B.overrun()) return kGzCorrupt;
        if (type == 0) {  // stored: byte-align, LEN, NLEN, raw bytes
            const uint32_t p = (uint32_t)((B.consumed() + 7) >> 3);
            B.pos = p;
            B.nb = 0;
            B.bb = 0;
            B.refill(lane);
            const uint32_t ln = B.bits(16), nl = B.bits(16);
            if (B.overrun() || (ln ^ 0xFFFFu) != nl) return kGzCorrupt;
            const uint32_t p0 = p + 4;
            if (ln > slen - umin(slen, p0)) return kGzCorrupt;
            if (ln > cap - d) return kCount ? kGzUnsupported : kGzResize;
            // 1 KiB at a time, flushing in between: the window never overruns unflushed bytes
            for (uint32_t k0 = 0; k0 < ln; k0 += 1024) {
                const uint32_t m = umin(1024u, ln - k0);
                for (uint32_t k = gl; k < m; k += G) S.win[(d + k) & (kWin - 1)] = src[p0 + k0 + k];
                __builtin_amdgcn_wave_barrier();
                d += m;
                if (!kWhole && d - flushed >= 1024) flush(d & ~1023u);
            }
            B.pos = p0 + ln;
            B.nb = 0;
            B.bb = 0;
            continue;
        }
        if (type == 3) return kGzCorrupt;
        if (type == 1) {  // fixed Huffman (RFC 1951 3.2.6)
            for (uint32_t s = gl; s < 288 + 32; s += G)
                T.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
            __builtin_amdgcn_wave_barrier();
            gz_build<G>(T.lens, 288, T.lcnt, T.lsym, T.lfast, lane);
            gz_build<G, kDB>(T.lens + 288, 32, T.dcnt, T.dsym, T.dfast, lane);
        } else {  // dynamic (readHuffman)
            B.refill(lane);
            const uint32_t nlit = B.bits(5) + 257, ndist = B.bits(5) + 1, nclen = B.bits(4) + 4;
            if (nlit > 286 || ndist > 30) return kGzCorrupt;
            // code-length code lengths, in the RFC's order, into lens[0..19)
            for (uint32_t k = gl; k < 19; k += G) T.lens[k] = 0;
            __builtin_amdgcn_wave_barrier();
            for (uint32_t k = 0; k < nclen; k++) {
                B.refill(lane);
                const uint32_t v = B.bits(3);
                if (gl == 0) T.lens[kClenOrder[k]] = (uint8_t)v;
            }
            if (B.overrun()) return kGzCorrupt;
            __builtin_amdgcn_wave_barrier();
            if (!gz_build<G>(T.lens, 19, T.lcnt, T.lsym, T.lfast, lane)) return kGzCorrupt;
            // litlen + distance code lengths with the code-length code (runs 16 / 17 / 18); they
            // overwrite lens[0..19), whose code now lives in lfast / lcnt / lsym
            uint32_t i = 0, prev = 0;
            const uint32_t total = nlit + ndist;
            uint8_t* L = T.lens;
            while (i < total) {
                B.refill(lane);
#if RIO_GZ_RUN
              int x;
              if constexpr (G == 64) {
                // runs of plain code lengths (symbols 0..15) as in the data loop: every offset looked
                // up at once, the chain followed through the lanes, the lengths stored in one write
                {
                    const uint32_t lim = (uint32_t)umin((uint64_t)B.nb, (uint64_t)8 * slen - umin((uint64_t)8 * slen, (uint64_t)B.consumed()));
                    const uint32_t e = T.lfast[(uint32_t)(B.bb >> lane) & (kFastSize - 1)];
                    uint32_t o = 0, cnt = 0, eo = 0, last = prev;
                    uint64_t m = 0;
                    while (o < lim) {
                        eo = __builtin_amdgcn_readlane(e, o);
                        const uint32_t ln = eo >> 9;
                        if (ln == 0 || ln > lim - o || (eo & 511u) >= 16 || i + cnt >= total) break;
                        m |= 1ull << o;
                        last = eo & 511u;
                        cnt++;
                        o += ln;
                    }
                    if ((m >> lane) & 1ull) L[i + lane_mbcnt(m)] = (uint8_t)e;
                    i += cnt;
                    prev = last;
                    B.bb = o >= 64 ? 0ull : B.bb >> o;
                    B.nb -= o;
                    const uint32_t ln = o < lim ? eo >> 9 : 0u;
                    if (ln != 0 && ln <= lim - o && i < total) {  // a repeat code, complete in the lookup
                        B.bits(ln);
                        B.refill(lane);
                        x = (int)(eo & 511u);
                    } else {
                        __builtin_amdgcn_wave_barrier();
                        if (cnt) continue;
                        x = gz_sym(B, T.lfast, T.lcnt, T.lsym);
                    }
                }
              } else {
                x = gz_sym(B, T.lfast, T.lcnt, T.lsym);
              }
#else
                const int x = gz_sym(B, T.lfast, T.lcnt, T.lsym);
#endif
                if (x < 0 || B.overrun()) return kGzCorrupt;
                uint32_t rep = 1, val = (uint32_t)x;
                if (x == 16) {
                    if (i == 0) return kGzCorrupt;
                    rep = 3 + B.bits(2);
                    val = prev;
                } else if (x == 17) {
                    rep = 3 + B.bits(3);
                    val = 0;
                } else if (x == 18) {
                    rep = 11 + B.bits(7);
                    val = 0;
                }
                if (B.overrun() || i + rep > total) return kGzCorrupt;
                for (uint32_t k = gl; k < rep; k += G) L[i + k] = (uint8_t)val;
                __builtin_amdgcn_wave_barrier();
                i += rep;
                prev = val;
            }
            // distance lengths live at lens[nlit..): move them behind the 288 litlen slots
            {
                // every source byte read before any is written (the ranges may overlap)
                constexpr uint32_t kJ = (32 + G - 1) / G;
                uint8_t v[kJ];
#pragma unroll
                for (uint32_t j = 0; j < kJ; j++) {
                    const uint32_t k = gl + j * G;
                    v[j] = k < ndist ? L[nlit + k] : 0;
                }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (uint32_t j = 0; j < kJ; j++)
                    if (gl + j * G < 32) L[288 + gl + j * G] = v[j];
            }
            __builtin_amdgcn_wave_barrier();
            if (!gz_build<G>(L, nlit, T.lcnt, T.lsym, T.lfast, lane)) return kGzCorrupt;
            if (!gz_build<G, kDB>(L + 288, ndist, T.dcnt, T.dsym, T.dfast, lane)) return kGzCorrupt;
        }
        // ---- compressed data (huffmanBlock) ----
#ifdef RIO_GZ_EXP
        if (RIO_GZ_EXP == 1) return kGzOkChecked;  // timing only: headers and tables, no data
#endif
        for (;;) {
            B.refill(lane);
#if RIO_GZ_RUN
            int s;
            if constexpr (G == 64) {
            // Literal runs, several symbols per table read: lane l looks up the code starting l bits
            // into the bit buffer (all 64 offsets at once), then the chain from offset 0 is followed
            // through the lanes (readlane: scalar, no LDS round trip per symbol) while it yields
            // literals whose codes lie inside the buffered stream bits; the run's bytes are stored by
            // their lanes in one LDS write. The symbol the chain stops at is decoded from the same
            // lookup when its code is a complete fast-table code, else by gz_sym after a refill.
            // (Matches decoded from the same lookup as well measured slower: the extra uniform state
            // spills scalar registers inside the loop; C2-gzip 52.1 -> 66.0 ms.)
            {
                const uint32_t lim = (uint32_t)umin((uint64_t)B.nb, (uint64_t)8 * slen - umin((uint64_t)8 * slen, (uint64_t)B.consumed()));
                const uint32_t e = T.lfast[(uint32_t)(B.bb >> lane) & (kFastSize - 1)];
                uint32_t o = 0, cnt = 0, eo = 0;
                uint64_t m = 0;
                while (o < lim) {
                    eo = __builtin_amdgcn_readlane(e, o);
                    const uint32_t ln = eo >> 9;
                    if (ln == 0 || ln > lim - o || (eo & 511u) >= 256 || d + cnt >= cap) break;
                    m |= 1ull << o;
                    cnt++;
                    o += ln;
                }
                if ((m >> lane) & 1ull) S.win[(d + lane_mbcnt(m)) & (kWin - 1)] = (uint8_t)e;
                d += cnt;
                B.bb = o >= 64 ? 0ull : B.bb >> o;  // (o may be 64: B.bits takes n <= 32)
                B.nb -= o;
                const uint32_t ln = o < lim ? eo >> 9 : 0u;
                if (ln != 0 && ln <= lim - o) {  // the stop symbol's code is complete in the lookup
                    B.bits(ln);
                    B.refill(lane);  // a length symbol's extra bits follow (gz_sym's callers refill first)
                    s = (int)(eo & 511u);
                } else {
                    __builtin_amdgcn_wave_barrier();
                    if (cnt) {
                        if (!kWhole && d - flushed >= 1024) flush(d & ~1023u);
                        continue;  // refill, then go on with the run
                    }
                    s = gz_sym(B, T.lfast, T.lcnt, T.lsym);
                }
            }
            } else {
                s = gz_sym(B, T.lfast, T.lcnt, T.lsym);
            }
#else
            const int s = gz_sym(B, T.lfast, T.lcnt, T.lsym);
#endif
            if (s < 0 || B.overrun()) return kGzCorrupt;
            if (s < 256) {
                if (d >= cap) return kCount ? kGzUnsupported : kGzResize;
                if (gl == 0) S.win[d & (kWin - 1)] = (uint8_t)s;
                d++;
            } else if (s == 256) {
                break;
            } else {
                if (s > 285) return kGzCorrupt;
                uint32_t eb;
                const uint32_t len = len_base((uint32_t)s, eb) + B.bits(eb);
                B.refill(lane);
                const int ds = gz_sym<kIn, G, kDB>(B, T.dfast, T.dcnt, T.dsym);
                if (ds < 0 || ds >= 30) return kGzCorrupt;
                uint32_t deb;
                const uint32_t dist = dist_base((uint32_t)ds, deb) + B.bits(deb);
                if (B.overrun() || dist > d - dm) return kGzCorrupt;  // not into an earlier member
                if (len > cap - d) return kCount ? kGzUnsupported : kGzResize;
                // source bytes all precede d: k mod dist repeats the last `dist` bytes
                const float rc = 1.0f / (float)dist;
                for (uint32_t k0 = 0; k0 < len; k0 += G) {
                    const uint32_t k = k0 + gl;
                    if (k < len) {
                        int q = (int)((float)k * rc);
                        int r = (int)k - q * (int)dist;
                        r += r < 0 ? (int)dist : 0;
                        r -= r >= (int)dist ? (int)dist : 0;
                        const uint8_t b = S.win[(d - dist + (uint32_t)r) & (kWin - 1)];
                        S.win[(d + k) & (kWin - 1)] = b;
                    }
                    __builtin_amdgcn_wave_barrier();
                }
                d += len;
            }
            __builtin_amdgcn_wave_barrier();
            if (!kWhole && d - flushed >= 1024) flush(d & ~1023u);
        }
    }
    // ---- trailer: byte-aligned CRC-32 + ISIZE of this member ----
    const uint32_t tp = (uint32_t)((B.consumed() + 7) >> 3);
    if (tp + 8 > slen) return kGzCorrupt;  // truncated trailer (io.ErrUnexpectedEOF)
    B.pos = tp;
    B.nb = 0;
    B.bb = 0;
    B.refill(lane);
    const uint32_t want_crc = B.bits(32), isize = B.bits(32);
    if (isize != d - dm) return kGzCorrupt;  // gzip.ErrChecksum (size)
    multi = multi || tp + 8 < slen;
    if (kCount || multi) {
        // this member's CRC-32 here (k_gzip_crc sees the record's last trailer only)
        __builtin_amdgcn_wave_barrier();
        uint32_t got;
        if (kCount) {
            flush(d);
            got = mcrc ^ 0xFFFFFFFFu;
            mcrc = 0xFFFFFFFFu;
        } else if (kWhole) {
            got = gz_crc_run<kWin, G>(0xFFFFFFFFu, S.win, dm, nullptr, d - dm, lane) ^ 0xFFFFFFFFu;
        } else {
            // bytes already flushed from the arena, the rest from the window (no extra flush: the
            // flush position stays 1 KiB aligned, so no 16-byte read straddles the window's end)
            const uint32_t g_end = umax(dm, flushed);
            uint32_t c = 0xFFFFFFFFu;
            if (g_end > dm) {
                __threadfence_block();  // the member's stores complete before lane 0 reads them back
                c = gz_crc_run<kWin, G>(c, nullptr, 0, out + dm, g_end - dm, lane);
            }
            got = gz_crc_run<kWin, G>(c, S.win, g_end, nullptr, d - g_end, lane) ^ 0xFFFFFFFFu;
        }
        if (got != want_crc) return kGzCorrupt;  // gzip.ErrChecksum
    }
    if (tp + 8 == slen) break;  // nothing after the trailer: the reader's clean io.EOF
    // the next member's header follows (Go's multistream Reader)
    dm = d;
  }
    if (kCount) {
        *total = d;
        return kGzOk;
    }
    if (d != dlen) return kGzResize;  // several members, or a shorter output than the size claimed
    __builtin_amdgcn_wave_barrier();
    flush(d);
    return multi ? kGzOkChecked : kGzOk;  // one member: CRC-32 by k_gzip_crc
}

__device__ __forceinline__ bool gzip_active(const FrameParams& P, const ScanState* st) {
    return st->hdr_status == RIO_OK && !st->capacity_fail && st->compression == RIO_COMP_GZIP;
}

// a record that does not inflate is flagged (ReadNext returns the gzip reader's error for it and goes
// on); one the device does not handle (several members) ends the sequence for the reference reader
__device__ __forceinline__ void gz_fail(const FrameParams& P, uint64_t i, int rc) {
    P.rec_pay[i] |= kPayFail;
    if (rc == kGzUnsupported)
        atomicMin((unsigned long long*)&P.state->unsupported_rec, (unsigned long long)i);
    else
        mark_bad(P, i);
}
}  // namespace

// waves per workgroup of the four-records-per-wave class: two (28.7 KB of LDS, 5 workgroups = 40
// records per CU). A/B on MI355X, C2-gzip: 4 waves 46.7 ms (2 workgroups fit), 2 waves 41.9, 1 wave 64.1
#ifndef RIO_GZ_TW
#define RIO_GZ_TW 2
#endif
// minimum workgroups per CU the tiny four-records-per-wave kernel is built for (register budget:
// 3 -> 133 VGPRs, no scratch, 41.9 ms; 4 -> 128 + 16 B scratch, 42.3; 5 -> 96 + 176 B, 42.8; 6 -> 49.4)
#ifndef RIO_GZ_TMIN
#define RIO_GZ_TMIN 3
#endif
// waves per SIMD the LDS allows: tiny 5.1 KB per wave -> 7 workgroups of 4 waves, small 7.2 KB -> 5
#ifndef RIO_GZ_TINY_WGS
#define RIO_GZ_TINY_WGS 7
#endif
// records per wave of the tiny class (RIO_GZ_GROUP lanes per record: 16 = four records per wave,
// 64 = the wave on one record)
#ifndef RIO_GZ_GROUP
#define RIO_GZ_GROUP 16
#endif
constexpr uint32_t kGzTinyG = RIO_GZ_GROUP;
template <uint32_t kWin>
constexpr uint32_t gz_group() { return kWin == kGzTinyWin ? kGzTinyG : 64u; }
template <uint32_t kWin>
constexpr int gz_wgs() {
    return kWin == kGzTinyWin ? (kGzTinyG == 64 ? RIO_GZ_TINY_WGS : RIO_GZ_TMIN) : kWin == kGzSmallWin ? 5 : 1;
}
// input ring per record: a block is staged by one pass of the group (16 bytes per lane)
template <uint32_t kWin>
#ifndef RIO_GZ_TIN
#define RIO_GZ_TIN 16
#endif
#ifndef RIO_GZ_DBITS
#define RIO_GZ_DBITS 7
#endif
constexpr uint32_t gz_in() { return kWin == kGzTinyWin ? (kGzTinyG == 64 ? kGzTinyIn : RIO_GZ_TIN * kGzTinyG) : kGzIn; }
// distance fast-table bits: records of <= 1 KiB reach back < 1 KiB (distance codes <= 19, short codes)
template <uint32_t kWin>
constexpr uint32_t gz_dbits() { return kWin == kGzTinyWin && kGzTinyG != 64 ? RIO_GZ_DBITS : kFastBits; }
template <uint32_t kWin>
using GzLdsOf = GzLds<kWin, gz_in<kWin>(), gz_dbits<kWin>()>;
template <uint32_t kWin>
constexpr uint32_t gz_waves() { return kWin == kGzTinyWin && kGzTinyG != 64 ? RIO_GZ_TW : kGzWaves; }
template <uint32_t kWin>
constexpr size_t gz_lds_bytes() { return (size_t)gz_waves<kWin>() * (64 / gz_group<kWin>()) * sizeof(GzLdsOf<kWin>); }
template <uint32_t kWin>
constexpr uint32_t gz_grid() {
    return kWin == kGzTinyWin ? (kGzTinyG == 64 ? 256 * RIO_GZ_TINY_WGS : 256 * (8 / RIO_GZ_TW + (RIO_GZ_TW == 2))) :
           kWin == kGzSmallWin ? 1280 : 256;
}

template <uint32_t kWin>
__global__ void __launch_bounds__(64 * gz_waves<kWin>(), gz_wgs<kWin>()) k_gzip_inflate(FrameParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    ScanState* st = P.state;
    if (!gzip_active(P, st) || (P.redo && !st->gz_redo)) return;
    constexpr uint32_t G = gz_group<kWin>(), kPer = 64 / G;  // lanes per record, records per wave
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, grp = lane / G;
    const bool lead = (lane & (G - 1)) == 0;
    using Lds = GzLdsOf<kWin>;
    Lds& S = *reinterpret_cast<Lds*>(lds + (wv * kPer + grp) * sizeof(Lds));
    const uint64_t n = st->n_records;
    constexpr uint32_t kW = gz_waves<kWin>();
    const uint64_t groups = (uint64_t)gridDim.x * kW * kPer;
    for (uint64_t i = ((uint64_t)blockIdx.x * kW + wv) * kPer + grp; i < n; i += groups) {
        if (P.flags[i] & (RIO_FLAG_NIL | RIO_FLAG_CORRUPT | RIO_FLAG_EOF)) continue;  // nil / failed at framing
        const uint64_t o0 = P.out_off[i], dlen = P.out_off[i + 1] - o0;
        // size classes: (0, 1 KiB], (1 KiB, 2 KiB] held whole in LDS, larger ones through the DEFLATE window
        const uint32_t cls = dlen <= kGzTinyWin ? kGzTinyWin : dlen <= kGzSmallWin ? kGzSmallWin : kGzLargeWin;
        if (cls != kWin) continue;
        const uint64_t pay = P.rec_pay[i];
        const uint64_t slen = (pay & kPayLen) >> 8;
        if (slen >= 0xFFFFFFF0ull || dlen >= 0xFFFFFFF0ull) {
            if (lead) gz_fail(P, i, kGzUnsupported);
            continue;
        }
        const int rc = gz_record<kWin, gz_in<kWin>(), false, G, gz_dbits<kWin>()>(S, P.file + P.rec_off[i] + (pay & 0xFF), (uint32_t)slen,
                                                              P.out + o0, (uint32_t)dlen, lane);
        if (lead) {
            if (rc == kGzOkChecked) {
                P.rec_pay[i] = pay | kPayFail;  // every member's CRC checked here
            } else if (rc == kGzResize && !P.redo) {
                P.rec_pay[i] = pay | kPayFail | kPayResize;  // sized by k_gz_resize, decoded in the redo round
                st->gz_resize = 1u;
            } else if (rc != kGzOk) {
                gz_fail(P, i, rc == kGzResize ? kGzCorrupt : rc);  // (redo round: the counted size is final)
            }
        }
    }
}

// CRC-32/IEEE of every inflated record against its trailer (gzip reader.go Read: ErrChecksum).
__global__ void __launch_bounds__(256) k_gzip_crc(FrameParams P) {
    __shared__ uint32_t tab[256];
    for (uint32_t k = threadIdx.x; k < 256; k += blockDim.x) {
        uint32_t c = k;
        for (int j = 0; j < 8; j++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
        tab[k] = c;
    }
    __syncthreads();
    const ScanState* st = P.state;
    if (!gzip_active(P, st) || (P.redo && !st->gz_redo)) return;
    const uint64_t n = st->n_records;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (P.flags[i] & (RIO_FLAG_NIL | RIO_FLAG_CORRUPT | RIO_FLAG_EOF)) continue;
        const uint64_t pay = P.rec_pay[i];
        if (pay & kPayFail) continue;
        const uint64_t slen = (pay & kPayLen) >> 8;
        const uint8_t* t = P.file + P.rec_off[i] + (pay & 0xFF) + slen - 8;
        const uint32_t want = t[0] | (uint32_t)t[1] << 8 | (uint32_t)t[2] << 16 | (uint32_t)t[3] << 24;
        const uint8_t* o = P.out + P.out_off[i];
        const uint64_t len = P.out_off[i + 1] - P.out_off[i];
        uint32_t c = 0xFFFFFFFFu;
        uint64_t k = 0;
        for (; k < len && ((uintptr_t)(o + k) & 15u); k++) c = tab[(c ^ o[k]) & 0xFFu] ^ (c >> 8);
        for (; k + 16 <= len; k += 16) {
            const uint4 v = *reinterpret_cast<const uint4*>(o + k);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 16; j++) c = tab[(c ^ (w[j >> 2] >> (8 * (j & 3)))) & 0xFFu] ^ (c >> 8);
        }
        for (; k < len; k++) c = tab[(c ^ o[k]) & 0xFFu] ^ (c >> 8);
        if ((c ^ 0xFFFFFFFFu) != want) mark_bad(P, i);  // gzip.ErrChecksum
    }
}

// Sizes of the records the decoders marked kPayResize: every member's output counted (nothing stored),
// one wave per record, the chunk's scratch length and byte sum corrected for the redo scan; a record
// Go's reader fails on is flagged corrupt (its size stays the framing's). One wave per chunk (its
// records are slots [0, owned) of ChunkPlace, as in k_place). A file whose placement came from the
// sequential repair (rare) is handed back at the first such record instead.
__global__ void __launch_bounds__(64 * kGzWaves) k_gz_resize(FrameParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    ScanState* st = P.state;
    if (!st->gz_resize || !gzip_active(P, st)) return;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    if (!st->slow && blockIdx.x == 0 && threadIdx.x == 0) {  // read by the redo round's kernels only
        st->gz_redo = 1u;
        st->scan_ticket = 0;
        st->first_bad = kNone;  // recounted by the redo placement and decoders
        st->n_bad = 0;
    }
    using Lds = GzLds<kGzLargeWin, kGzIn>;  // the DEFLATE window: the CRCs need the bytes
    Lds& S = *reinterpret_cast<Lds*>(lds + wv * sizeof(Lds));
    for (uint64_t c = (uint64_t)blockIdx.x * kGzWaves + wv; c < P.n_chunks; c += (uint64_t)gridDim.x * kGzWaves) {
    const ChunkPlace pl = P.place[c];
    uint64_t* sl = P.scratch_len + c * P.slots;
    for (uint64_t k = 0; k < pl.owned; k++) {
        const uint64_t i = pl.base_idx + k;
        const uint64_t pay = P.rec_pay[i];
        if (!(pay & kPayResize)) continue;
        if (st->slow) {
            if (lane == 0) atomicMin((unsigned long long*)&st->unsupported_rec, (unsigned long long)i);
            continue;
        }
        uint64_t total = 0;
        const int rc = gz_record<kGzLargeWin, kGzIn, true>(S, P.file + P.rec_off[i] + (pay & 0xFF),
                                                              (uint32_t)((pay & kPayLen) >> 8), nullptr, 0, lane, &total);
        if (lane == 0) {
            if (rc == kGzOk) {
                const uint64_t old = sl[k] & kLenMask;
                sl[k] = (sl[k] & ~kLenMask) | total;
                P.chunks[c].bytes += total - old;  // (this wave is the chunk's only writer)
            } else if (rc == kGzCorrupt) {
                sl[k] |= kBadBit;
            } else {
                atomicMin((unsigned long long*)&st->unsupported_rec, (unsigned long long)i);
            }
        }
    }
    }
}

hipError_t launch_gzip_resize(const FrameParams& P, hipStream_t s) {
    // one workgroup per CU (the DEFLATE windows fill the LDS), chunks grid-stride: a file with no
    // such record costs one short launch
    hipLaunchKernelGGL(k_gz_resize, dim3(256), dim3(64 * kGzWaves), kGzWaves * sizeof(GzLds<kGzLargeWin, kGzIn>),
                       s, P);
    return hipGetLastError();
}

hipError_t launch_gzip_decode(const FrameParams& P, hipStream_t s) {
    hipLaunchKernelGGL(k_gzip_inflate<kGzTinyWin>, dim3(gz_grid<kGzTinyWin>()), dim3(64 * gz_waves<kGzTinyWin>()),
                       gz_lds_bytes<kGzTinyWin>(), s, P);
    hipLaunchKernelGGL(k_gzip_inflate<kGzSmallWin>, dim3(gz_grid<kGzSmallWin>()), dim3(64 * kGzWaves),
                       gz_lds_bytes<kGzSmallWin>(), s, P);
    hipLaunchKernelGGL(k_gzip_inflate<kGzLargeWin>, dim3(gz_grid<kGzLargeWin>()), dim3(64 * kGzWaves),
                       gz_lds_bytes<kGzLargeWin>(), s, P);
    hipLaunchKernelGGL(k_gzip_crc, dim3(512), dim3(256), 0, s, P);
    return hipGetLastError();
}

}  // namespace rio
