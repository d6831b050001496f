// rio_snappy.hip — Snappy block decode of every framed record (golang/snappy v1.0.0 semantics,
// decode.go + decode_other.go; called per record by FileReader.ReadNext, file_reader.go:115-125).
//
// k_snappy_pipe: one lane per record (SIMT across consecutive records), software-pipelined so that
// no lane ever waits on a memory load issued in the same iteration (snappy_lane, below).
//
//   * The record is emitted as a sequence of pieces of <= 16 bytes. A PARSER runs kD pieces ahead
//     of the EMITTER; pieces travel through kD register slots.
//   * Every iteration every lane issues exactly three vector-memory operations, in a fixed order:
//     one flush store, one far-history load, one input-chunk load. Lanes with nothing to do point
//     the operation at their wave's 64-byte sink line, so the address unit coalesces all
//     placeholder lanes of an instruction into one request. On CDNA vmcnt retires loads and stores
//     in issue order, so a uniform schedule is what lets the compiler wait for exactly the loads
//     issued kD iterations earlier instead of draining the queue whenever some lane of the wave
//     touched memory.
//   * The flush is cooperative: 64 contiguous bytes of 16 records per wave store. Lane-private
//     16-byte stores to 64 records run at ~1.5 TB/s on MI355X, the 16-record form at ~4.2 TB/s
//     (scripts/mem_probe.hip); loads do not care (5.5 vs 6.0 TB/s).
//   * History: the last 256 decoded bytes of each record live in LDS; copies reaching further back
//     (offset > kFarOff) are loaded from the output arena at PARSE time, kD iterations before use —
//     the flush schedule guarantees those bytes were stored already (flush lag < 128 bytes, parser
//     lead <= 16*(kD-1) bytes: kFarOff >= 16*(kD-1) + 16 + 128).
//   * Input: aligned 16-byte chunks loaded kD iterations ahead land in a 64-byte LDS ring.
//   * LDS images are dword columns (round 3): row k of lane l is one dword, and all of a lane's rows
//     sit in its own bank, so every per-lane dword access of a wave is conflict-free; the address
//     selects the dword and a piece needs only a byte shift (v_alignbyte_b32), placed
//     destination-aligned (see snappy_lane).
// Wave-per-record decoder (coop_*, k_snappy_coop_batch): files or arenas past 32-bit positions and
// streams >= 4 GiB; 64-bit addressing, one 64-byte output window per round with lane = byte.
// Files whose every record is a single literal (k_place sets ScanState::any_mixed otherwise) are
// copied by k_copy_records (rio_kernels.hip) and the kernels here exit at once.
#include <hip/hip_runtime.h>

#include "rio_device.h"
#include "rio_dev_util.h"

namespace rio {

namespace {
constexpr uint32_t kInCh = 4;                    // input ring: 4 chunks = 64 bytes per lane
constexpr uint32_t kD = 4;                       // pipeline depth in iterations
// chunks per wave: the balance against the per-chunk drain and setup (A/B on MI355X, records per lane
// per chunk: C3 64-B records 19 -> 9: decode 0.906 -> 0.870 ms; 4: 0.922, 1: 1.92; C2 stays at 1; one chunk of
// ceil(n / lanes) records per lane on C2: +10 %, round 6)
constexpr uint64_t kChunksPerWave = 8;
// copies reaching further back than kFarOff read the output arena (flushed: see snappy_lane); the
// flush is pipelined one step (+16 bytes of lag). Anything from that bound (208) up to what the
// history ring still holds (233, static_assert below) is correct; 232 turns the copies of offset
// 209-232 into ring copies (A/B on MI355X, two rounds: C2 decode -0.6/-0.9 %, C4 -0.7/-0.9 %, C3 equal)
constexpr uint32_t kFarOff = 232;
constexpr uint32_t kNoChunk = ~0u;               // slot carries no input chunk
constexpr uint32_t kLitEff = ~0u;                // "offset" of a literal element (see snappy_lane)
// the flush store is issued after the step's loads: one more step of flush lag for a far load to see (+16)
static_assert(kFarOff >= 16 * (kD - 1) + 16 + 128 + 16 + 16, "far history must be flushed before the parser reads it");
static_assert(kSnappyBlock % 64 == 0, "whole waves");

// materialize x in a VGPR here: the selects that use it can no longer be turned into branches that
// compute x on one side only (an empty asm with a register constraint; no instruction is emitted)
__device__ __forceinline__ void pin_v(uint32_t& x) { asm volatile("" : "+v"(x)); }

__device__ __forceinline__ uint4 sel4(bool c, uint4 a, uint4 b) {
    return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

// Cache policy. Flush stores: non-temporal below kPlainStoreMin bytes per record (round 3: the arena stores no longer
// push the lanes' input lines out of L2: C2 HBM reads 4.1 -> 3.4 GB per launch), plain from it (round 5: C4's far
// copies find their sources in L2 / MALL, decode 13.21 -> 12.19 ms). Far and input loads plain: non-temporal far loads
// +5 % (C2) / +11 % (C4), non-temporal input loads +10-13 % (they lose the paired loads' line reuse), sc0 / sc1 far loads
// even (round 6, C2 and C4).
// Compares are cheap to remove: two waves of a SIMD issue ~1.7 v_add / v_and / v_or / v_xor / v_lshrrev per 4-cycle slot
// but ~1.15 of the 3-operand integer ops (v_cndmask_e64, v_bfi, v_alignbyte ...) and ~0.95 v_cmp (scripts/op_probe.hip,
// profiles/r5/r5w_op_probe.txt): the record-end test is one OR and one compare, the offset doubling has no range compare,
// the emit's ring / far selects use the parse's masks (C2 decode -2 %, r5x).
// mean decoded bytes per record from which a wave's flush stores are plain (snappy_lane's kPlain)
constexpr uint64_t kPlainStoreMin = 4096;

// Buffer descriptors: the input prefetch, the flush store and the far-history load use 32-bit offsets from the wave's
// own file / arena base (wave-uniform descriptors in SGPRs); a lane with nothing to load or store passes an offset past
// the descriptor's range, which the range check drops (no sink line, no 64-bit address arithmetic). A wave's records
// span less than 0xF0000000 bytes of file and arena (snappy_lane checks; a wave past that decodes its records one
// thread each), so every real offset fits 32 bits and kOob is out of range, whatever the file's size.
constexpr uint32_t kOob = 0xFFFFFFC0u;
// Far windows inside the copy's line (files of plain-store records: C4; kLine in snappy_lane): a far piece's 16-byte window
// [q - r, q - r + 16) that straddles a 128-byte line costs two L2 -> fabric requests though the piece's own bytes
// [q, q + n) may sit in one line; then the window moves: back to the line's last 16 bytes (kind 4, shifted down at
// the emit) or, when the bytes lie in the next line, to q itself (kind 3, shifted up). 5.6 % of C4's far requests
// (host count over its streams, profiles/r6).
// Paired input loads: in the single-record-per-lane loop (kMulti = false: C2's and C4's shape) the input prefetch
// loads two adjacent 16-byte chunks (32 bytes) on even steps and none on odd steps, so the second load of a pair
// finds its line already requested by the first: half the L1 misses of the lane-private input stream for the same
// instruction count (round 5: C2 decode -1.7 %, C4 -0.5 %; the multi-record loop (C3) +3.5 %, so it keeps one chunk
// per step). ONE load per step serving either the far piece or the next input chunk (2 vector-memory operations per
// step instead of 3) measured +4 % on C2 and +5-12 % on C4 (round 6, profiles/r6): it loses the pairing.
// lane k's 64-bit value (k wave-uniform) into scalars
__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t k) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)k);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)k);
    return ((uint64_t)hi << 32) | lo;
}
typedef uint32_t v4u32b __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, uint64_t bytes) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(bytes < 0xFFFFFF00ull ? bytes : 0xFFFFFF00ull));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, (int)n,
                                             0x00020000);
}
}  // namespace

// Files the 32-bit lane-stream positions cannot cover take the wave-per-record decoder.
__device__ __forceinline__ bool snappy_wide(const FrameParams& P, const ScanState* st) {
    return st->huge_streams;  // per-wave buffer bases: any file and arena size (snappy_lane)
}

// ------------------------------------------------------------------------------------------
// k_snappy_coop: one wave per record, all 64 lanes on that record (files of large records: C4's
// 64 KiB values; and files past the lane decoder's 32-bit positions). A record is decoded in
// rounds of up to 64 elements:
//   1. parse: the next 256 stream bytes go to LDS; every lane computes, for 4 positions q, where an
//      element starting at q would end (J0[q] = next element start, >= 256: outside the window);
//      five pointer-doubling levels J_k = J_{k-1} o J_{k-1} follow, and lane e finds element e of
//      the chain as J composed along the bits of e. Lane e then decodes its element's header and
//      applies golang/snappy's checks (decode_other.go: header and literal inside the stream, copy
//      offset in [1, produced], output room) — produced = an exclusive scan of element lengths.
//   2. materialise the round's output in 64-byte windows, lane = output byte: the element covering
//      each byte comes from a prefix-max over "element starts here" marks; a literal byte is read
//      from the file, a copy byte from position s = dst - off + (x mod off) < dst (the periodic
//      extension of an overlapping copy): the current window (resolved through the lanes, always
//      an earlier element: a short dependency chain), a 1 KiB LDS history ring, or the output arena
//      (older bytes; their stores are drained by the vmcnt bound before every store, and the loads
//      bypass L1).
// A record that fails a check is flagged (mark_bad) where the check fails; its bytes are unspecified.
// ------------------------------------------------------------------------------------------
namespace {
constexpr uint32_t kCoopWaves = 4;
constexpr uint32_t kCoopGrid = 2048;  // x 4 waves: 32 waves per CU (latency-bound: LDS + shuffle chains)
constexpr uint32_t kCoopWin = 256;    // parse window (stream bytes)
constexpr uint32_t kCoopLevels = 6;   // 2^6 = 64 elements per round
constexpr uint32_t kCoopRing = 1024;  // history ring per wave
constexpr uint32_t kInDw = 72;        // window image: 288 bytes from (base & ~3)
constexpr uint32_t kOut = 0xFFFFu;    // "no next element inside the window"
// a mapped output window of the pipeline: the byte's source kind and what it needs
constexpr uint32_t kSlotLds = 0, kSlotGlobal = 1, kSlotRing = 2, kSlotLane = 3, kSlotIdle = 4;
struct CoopSlot {
    uint8_t g;      // global load in flight (far history or a literal byte past the LDS window)
    uint32_t v;     // literal byte from the LDS window
    uint32_t code;  // kind << 24 | ring position or source lane
};
struct CoopLds {
    uint32_t in[2][kInDw];                // parse window images (double-buffered: the next one lands
                                          // while the current round's literals are read)
    uint16_t J[kCoopLevels][kCoopWin];    // next-element tables
    uint8_t slot[64];                     // element starts in the current output window
    uint8_t ring[kCoopRing];              // decoded history of the current record
};

__device__ __forceinline__ bool coop_active(const FrameParams& P, const ScanState* st) {
    if (st->hdr_status != RIO_OK || st->capacity_fail || st->compression != RIO_COMP_SNAPPY || !st->any_mixed)
        return false;
    return st->huge_streams || snappy_wide(P, st) || (st->n_records && st->total_bytes / st->n_records >= P.coop_min);
}

// element header from its first 8 bytes (lo = bytes 0..3, hi = 4..7): header length, output length
// (64-bit: a 4-byte literal length may be 2^32), copy offset
__device__ __forceinline__ void coop_elem(uint32_t lo, uint32_t hi, uint32_t& hl, uint64_t& len, uint32_t& off,
                                          bool& lit) {
    const uint32_t tag = lo & 0xFFu, t = tag & 3u, x = tag >> 2;
    const uint32_t b1 = (lo >> 8) & 0xFFu, b12 = (lo >> 8) & 0xFFFFu;
    const uint32_t b1234 = (lo >> 8) | (hi << 24);
    lit = t == 0;
    if (t == 0) {
        if (x < 60) {
            hl = 1;
            len = x + 1;
        } else {
            const uint32_t nb = x - 59;  // 1..4 length bytes
            hl = 1 + nb;
            const uint32_t v = nb == 4 ? b1234 : (b1234 & ((1u << (8 * nb)) - 1u));
            len = (uint64_t)v + 1;
        }
        off = 0;
    } else if (t == 1) {
        hl = 2;
        len = 4 + (x & 7u);
        off = ((tag & 0xE0u) << 3) | b1;
    } else if (t == 2) {
        hl = 3;
        len = 1 + x;
        off = b12;
    } else {
        hl = 5;
        len = 1 + x;
        off = b1234;
    }
}

// bytes [u, u + 8) of a window image (u relative to its aligned base)
__device__ __forceinline__ void coop_bytes8(const uint32_t* in, uint32_t u, uint32_t& lo, uint32_t& hi) {
    const uint32_t k = u >> 2, r = u & 3u;
    const uint32_t d0 = in[k], d1 = in[k + 1], d2 = in[k + 2];
    lo = __builtin_amdgcn_alignbyte(d1, d0, r);
    hi = __builtin_amdgcn_alignbyte(d2, d1, r);
}

// wave-wide inclusive scans on DPP (row shifts within 16-lane rows, then row broadcasts 15 / 31):
// VALU latency instead of the LDS round trips of __shfl_up
template <bool kMax>
__device__ __forceinline__ uint32_t wave_incl(uint32_t v) {
    auto op = [](uint32_t a, uint32_t b) { return kMax ? (a > b ? a : b) : a + b; };
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));  // row_shr:1
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));  // row_shr:2
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));  // row_shr:4
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));  // row_shr:8
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return v;
}

__device__ __forceinline__ uint64_t wave_excl_u64(uint64_t v, uint32_t lane, uint64_t& total) {
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        x += lane >= (uint32_t)d ? y : 0ull;
    }
    total = __shfl(x, 63, 64);
    return x - v;
}

// the 288 window bytes from aligned address a: one dword per lane + 8 (clamped inside the padded file)
struct WinRegs {
    uint32_t w0, w1;
};
__device__ __forceinline__ WinRegs coop_fetch(const FrameParams& P, uint64_t a, uint32_t lane, uint64_t dw_end) {
    const uint64_t g0 = a + 4ull * lane, g1 = g0 + 256;
    WinRegs r;
    r.w0 = *reinterpret_cast<const uint32_t*>(P.file + (g0 < dw_end ? g0 : dw_end));
    r.w1 = lane < kInDw - 64 ? *reinterpret_cast<const uint32_t*>(P.file + (g1 < dw_end ? g1 : dw_end)) : 0u;
    return r;
}
__device__ __forceinline__ void coop_land(uint32_t* in, const WinRegs& r, uint32_t lane) {
    in[lane] = r.w0;
    if (lane < kInDw - 64) in[64 + lane] = r.w1;
}

// decode one record: stream [start, start + slen) of the file, dlen bytes to out
__device__ bool coop_record(const FrameParams& P, CoopLds& S, uint32_t lane, uint64_t start, uint32_t slen,
                            uint32_t dlen, uint8_t* out, uint8_t* sink) {
    const uint64_t dw_end = ((P.len + RIO_DEVICE_PAD) & ~3ull) - 4;  // last readable dword
    const bool small_out = dlen < (1u << 25);  // element lengths of a round fit 32-bit scans
    uint32_t pos = 0;  // stream position of the next element
    uint32_t d = 0;    // bytes produced
    uint32_t buf = 0;
    coop_land(S.in[0], coop_fetch(P, (start + pos) & ~3ull, lane, dw_end), lane);
    while (pos < slen) {
        const uint32_t* in = S.in[buf];
        const uint64_t base = start + pos;
        const uint32_t sh = (uint32_t)(base & 3u);
        const uint32_t lim = slen - pos < 0xFFF0u ? slen - pos : 0xFFF0u;  // stream bytes from the window start
        __builtin_amdgcn_wave_barrier();
        // ---- 1. parse: J0 for q = 4 lane + j, then pointer doubling ----
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
            const uint32_t q = 4 * lane + j;
            uint32_t lo, hi, hl, off;
            uint64_t len;
            bool lit;
            coop_bytes8(in, q + sh, lo, hi);
            coop_elem(lo, hi, hl, len, off, lit);
            uint32_t nx = kOut;
            if (q < lim && hl <= lim - q) {
                const uint64_t e = (uint64_t)q + hl + (lit ? len : 0);
                if (e <= lim) nx = (uint32_t)(e < kOut - 1 ? e : kOut - 1);
            }
            S.J[0][q] = (uint16_t)nx;
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (uint32_t k = 1; k < kCoopLevels; k++) {
            uint16_t v[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) {
                const uint32_t t = S.J[k - 1][4 * lane + j];
                v[j] = t < kCoopWin ? S.J[k - 1][t] : (uint16_t)t;
            }
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) S.J[k][4 * lane + j] = v[j];
            __builtin_amdgcn_wave_barrier();
        }
        // element e = lane of this round: the chain position next^e(0)
        uint32_t p = 0;
#pragma unroll
        for (uint32_t k = 0; k < kCoopLevels; k++)
            if (((lane >> k) & 1u) && p < kCoopWin) p = S.J[k][p];
        const bool valid = p < (lim < kCoopWin ? lim : kCoopWin);
        uint32_t lo = 0, hi = 0, hl = 0, off = 0;
        uint64_t len = 0;
        bool lit = false;
        if (valid) {
            coop_bytes8(in, p + sh, lo, hi);
            coop_elem(lo, hi, hl, len, off, lit);
        }
        bool bad = valid && (hl > lim - p || (lit && len > lim - p - hl));
        const uint64_t olen = valid ? (len < (uint64_t)dlen + 1 ? len : (uint64_t)dlen + 1) : 0;
        uint64_t total, excl;
        if (small_out) {  // olen <= 2^25: the round's sum fits 32 bits
            const uint32_t inc = wave_incl<false>((uint32_t)olen);
            excl = inc - (uint32_t)olen;
            total = (uint32_t)__shfl(inc, 63, 64);
        } else {
            excl = wave_excl_u64(olen, lane, total);
        }
        const uint64_t de = d + excl;
        bad = bad || (valid && (de + olen > dlen || (!lit && (off == 0 || off > de))));
        if (__any(bad)) return false;
        const uint32_t m = __builtin_popcountll(__ballot(valid));
        const uint32_t ext = p + hl + (lit ? (uint32_t)len : 0u);  // stream end of element e (window-relative)
        const uint32_t next_pos = pos + (uint32_t)__shfl(ext, m - 1, 64);
        // prefetch the next round's window while this one materialises
        WinRegs nxt{0, 0};
        const bool more = next_pos < slen;
        if (more) nxt = coop_fetch(P, (start + next_pos) & ~3ull, lane, dw_end);
        const uint32_t e_dst = (uint32_t)de, e_len = (uint32_t)olen;
        // literal: window position of its bytes; copy: offset
        const uint32_t e_a = lit ? p + hl : off;
        // ---- 2. materialise [d, d + total) in 64-byte windows, lane = byte ----
        // Software-pipelined by kCoopD windows: window j + kCoopD is mapped (covering element, byte
        // source, its global load issued) while window j is finished (ring / in-window sources
        // resolved, stored). Every map issues exactly one vector load and every finish one store
        // (placeholders go to the wave's sink line), so the compiler waits for exactly the load
        // issued kCoopD windows earlier; that wait also retires every store older than it, which is
        // what makes far history (> kCoopRing bytes back, at least 12 windows old) safe to load.
        const uint32_t Wend = d + (uint32_t)total;
        const uint32_t nwin = ((uint32_t)total + 63) >> 6;
        const uint32_t in_avail = kInDw * 4 - 8 - sh;  // window bytes a literal may take from LDS
        uint32_t ei = 0;  // element covering the next window to map
        auto map = [&](CoopSlot& T, uint32_t j) __attribute__((always_inline)) {
            const uint32_t W = d + 64 * j;
            uint32_t type = kSlotIdle, v = 0, sp = 0;
            const uint8_t* ap = sink + lane;
            if (W < Wend) {  // wave-uniform
                S.slot[lane] = 0;
                __builtin_amdgcn_wave_barrier();
                if (lane == 0) S.slot[0] = (uint8_t)(ei + 1);
                if (valid && e_dst > W && e_dst < W + 64) S.slot[e_dst - W] = (uint8_t)(lane + 1);
                __builtin_amdgcn_wave_barrier();
                const uint32_t k = wave_incl<true>(S.slot[lane]) - 1;
                const uint32_t dk = __shfl(e_dst, k, 64), lk = __shfl(e_len, k, 64), ak = __shfl(e_a, k, 64);
                const bool litk = __shfl(lit ? 1 : 0, k, 64) != 0;
                const uint32_t b = W + lane;
                const uint32_t x = b - dk;
                if (b >= Wend) {
                    type = kSlotIdle;
                } else if (litk) {
                    const uint32_t u = ak + x;  // window-relative stream position
                    if (u < in_avail) {
                        type = kSlotLds;
                        v = (in[(u + sh) >> 2] >> (8 * ((u + sh) & 3u))) & 0xFFu;
                    } else {
                        type = kSlotGlobal;
                        ap = P.file + base + u;
                    }
                } else {
                    uint32_t q = x;
                    if (x >= ak) {  // inside the copy's own period: x mod off (x < 64, off < 64 here)
                        const uint32_t qq = (uint32_t)((float)x * __frcp_rn((float)ak));
                        int r = (int)x - (int)(qq * ak);
                        r += r < 0 ? (int)ak : 0;
                        r -= r >= (int)ak ? (int)ak : 0;
                        q = (uint32_t)r;
                    }
                    sp = dk - ak + q;  // < dk: an earlier element's byte
                    if (sp >= W) {
                        type = kSlotLane;
                        sp -= W;  // the source lane
                    } else if (W - sp <= kCoopRing) {
                        type = kSlotRing;
                    } else {
                        type = kSlotGlobal;
                        ap = out + sp;
                    }
                }
                const uint32_t Wn = W + 64;
                if (Wn < Wend) {
                    const uint32_t k63 = __shfl(k, 63, 64), end63 = __shfl(dk + lk, 63, 64);
                    ei = end63 > Wn ? k63 : k63 + 1;
                }
            }
            T.g = __builtin_nontemporal_load(ap);  // L2: bypasses this CU's L1 (far history was written here)
            T.v = v;
            T.code = (type << 24) | sp;
        };
        auto finish = [&](CoopSlot& T, uint32_t j) __attribute__((always_inline)) {
            const uint32_t type = T.code >> 24, sp = T.code & 0xFFFFFFu;
            const uint32_t b = d + 64 * j + lane;
            uint32_t val = type == kSlotGlobal ? (uint32_t)T.g : T.v;
            if (type == kSlotRing) val = S.ring[sp & (kCoopRing - 1)];
            bool pend = type == kSlotLane;
            const uint32_t srcl = pend ? sp : lane;
            while (__any(pend)) {
                const uint32_t sv = __shfl(val, srcl, 64);
                const bool sp2 = __shfl(pend ? 1 : 0, srcl, 64) != 0;
                if (pend && !sp2) {
                    val = sv;
                    pend = false;
                }
            }
            const bool active = type != kSlotIdle;
            *(active ? out + b : sink + lane) = (uint8_t)val;
            if (active) S.ring[b & (kCoopRing - 1)] = (uint8_t)val;
        };
        CoopSlot T0, T1, T2, T3;
        map(T0, 0);
        map(T1, 1);
        map(T2, 2);
        map(T3, 3);
        for (uint32_t j = 0; j < nwin; j += 4) {
            finish(T0, j);
            map(T0, j + 4);
            finish(T1, j + 1);
            map(T1, j + 5);
            finish(T2, j + 2);
            map(T2, j + 6);
            finish(T3, j + 3);
            map(T3, j + 7);
        }
        d = Wend;
        pos = next_pos;
        buf ^= 1u;
        if (more) coop_land(S.in[buf], nxt, lane);
    }
    return d == dlen;
}

// every record of one file, records strided over all waves of the grid
__device__ __forceinline__ void coop_file(const FrameParams& P, CoopLds& S, uint32_t lane, uint64_t wave,
                                          uint64_t nw) {
    const ScanState* st = P.state;
    if (!coop_active(P, st)) return;
    const uint64_t n = st->n_records;
    if (st->huge_streams) {
        // a record stream past 32-bit positions (never produced by an encoder: a record over 4 GiB):
        // every record by one thread, byte loops straight to HBM
        for (uint64_t i = wave * 64 + lane; i < n; i += nw * 64) {
            if (P.flags[i] & (RIO_FLAG_NIL | RIO_FLAG_CORRUPT | RIO_FLAG_EOF)) continue;
            const uint64_t o0 = P.out_off[i], o1 = P.out_off[i + 1];
            uint64_t start, slen;
            rec_stream(P, i, start, slen);
            if (!snappy_decode_thread(P.file + start, slen, P.out + o0, o1 - o0))
                mark_bad(P, i);
        }
        return;
    }
    uint8_t* sink = P.sink + (wave % ((uint64_t)kSnappyGrid * (kSnappyBlock / 64))) * 64;  // placeholder line
    for (uint64_t i = wave; i < n; i += nw) {
        if (P.flags[i] & (RIO_FLAG_NIL | RIO_FLAG_CORRUPT | RIO_FLAG_EOF)) continue;
        const uint4 dsc = P.rec_desc[i];
        const uint64_t start = ((uint64_t)dsc.y << 32) | dsc.x;
        if (!coop_record(P, S, lane, start, dsc.z, dsc.w, P.out + P.out_off[i], sink) && lane == 0) mark_bad(P, i);
    }
}
}  // namespace

// ------------------------------------------------------------------------------------------
// snappy_lane: the lane decoder (round 3: dword-column LDS images). Each step of a lane emits the
// piece its parser produced kD steps earlier, takes part in the cooperative flush, parses the next
// piece, issues its far-history (or next descriptor) load and its input prefetch. Byte placement:
//   * Row k of a lane's history / input image is one dword; a lane's rows are 1 KiB apart and all
//     in its own bank, so any per-lane dword access of a wave is conflict-free, wherever the lanes
//     are. The LDS address selects the dword; only the byte shift inside it is VALU work
//     (v_alignbyte_b32). Round 2's [chunk][lane][16 B] image needed a select network over three
//     16-byte chunks per piece (funnel32: 44 VALU) and a second one for the parser (funnel16).
//   * A piece is placed destination-aligned: with r = d & 3, the four dwords of output bytes
//     [d - r, d - r + 16) are written (pieces are capped at 16 - r bytes), the r bytes below d
//     merged from the row as it stands (one v_bfi_b32). The source rows [q - r, q - r + 20) are
//     read as five dwords and shifted by (q - r) & 3.
//   * Literal bytes are read at parse time from the input image at the literal's own position
//     (five rows, shift (s - r) & 3) and travel in the slot; far-copy bytes are loaded from the
//     arena already destination-aligned (16 bytes at q - r), so they need no shift.
// The four waves' rows are interleaved: row k of wave w, lane l is the dword at k * 1024 + w * 256
// + 4 l of its image. The history image (64 rows, 64 KiB) starts at byte kColI of the workgroup's
// LDS and its local addresses are 16-bit: the next row is one v_pk_add_u16 (the ring wraps with the
// address); the input image (16 rows) is the first 16 KiB.
// Measured on MI355X against round 2's decoder (same pipeline, one box, 308-test parity subset
// green): static VALU per step 268 -> 217, executed VALU per C2 launch 4.95e8 -> 3.98e8 (PMC),
// decode C2 1.19 -> 1.13 ms, C3 0.86 -> 0.80, C4 13.9 -> 13.6 (gpurun_out/r3k).
// ------------------------------------------------------------------------------------------
namespace {
constexpr uint32_t kColRows = 64;  // history rows per lane: 256 bytes
constexpr uint32_t kColInRows = 16;                // input rows per lane: 64 bytes = kInCh chunks
constexpr uint32_t kColWaves = kSnappyBlock / 64;
constexpr uint32_t kColRow = kColWaves * 256;      // bytes per row of the four waves (1 KiB)
constexpr uint32_t kColH = kColRows * kColRow;     // history image (64 KiB: 16-bit local addresses)
constexpr uint32_t kColI = kColInRows * kColRow;   // input image (16 KiB)
constexpr uint32_t kColLds = kColH + kColI;
constexpr uint32_t kCoopSlice = kColH / kColWaves; // a wave's contiguous slice for the wave decoder
static_assert(kColH == 65536, "history addresses wrap at 16 bits");
static_assert(kColInRows == 4 * kInCh, "input image holds the input ring's chunks");
static_assert(sizeof(CoopLds) <= kCoopSlice, "wave decoder LDS must fit a history slice");
// live history: ring-copy sources reach kFarOff + 3 bytes below the destination, the emit writes
// the 16 bytes from d - r; the flush reads complete blocks at most 127 bytes below d
static_assert(kFarOff + 3 + 16 + 4 <= kColRows * 4, "history image must hold the copy reach");

struct ColSlot {
    uint4 in;        // input chunk in_c (load in flight)
    uint4 in2;       // paired loads: input chunk in_c + 1
    uint4 aux;       // far-copy bytes [q - r, q - r + 16) or the next record's descriptor (in flight)
    uint32_t x0, x1, x2, x3, x4;  // literal: input rows from (src - r) & ~3 (read at parse)
    uint32_t in_c;
    uint32_t n;      // piece length, 0 = bubble
    uint32_t kind;   // 0 literal, 1 ring copy, 2 far copy, 3 far copy loaded from q (see the emit)
    uint32_t q;      // ring copy: source output position; literal: byte shift of x0..x4
    uint32_t desc;   // aux carries the next record's descriptor
    uint32_t ringm, farm;  // kind 1 / kind 2 as all-ones masks (the emit selects by v_bfi, no compare)
};
__device__ __forceinline__ ColSlot col_empty_slot() {
    ColSlot S;
    S.in = zero4();
    S.in2 = zero4();
    S.aux = zero4();
    S.x0 = S.x1 = S.x2 = S.x3 = S.x4 = 0;
    S.in_c = kNoChunk;
    S.n = 0;
    S.kind = 1;
    S.ringm = ~0u;
    S.farm = 0;
    S.q = 0;
    S.desc = 0;
    return S;
}
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t col_ld(const uint8_t* L, uint32_t a) {
    return *reinterpret_cast<const uint32_t*>(L + a);
}
__device__ __forceinline__ void col_st(uint8_t* L, uint32_t a, uint32_t v) { *reinterpret_cast<uint32_t*>(L + a) = v; }

// history / input dword at a local address (the history image follows the input image)
__device__ __forceinline__ uint32_t col_hld(const uint8_t* L, uint32_t a) { return col_ld(L + kColI, a); }
__device__ __forceinline__ void col_hst(uint8_t* L, uint32_t a, uint32_t v) { col_st(L + kColI, a, v); }

// Decode the record range [r0, r1) of this lane as one stream (as snappy_lane_t). L is the
// workgroup's LDS base (input image, then history image).
// kMulti = false: every lane holds at most one record (r1 <= r0 + 1; C2's shape), so the next-record
// descriptor fetch, its latch and the record switch are compiled out. kLow = true: some lane's
// first record starts in the arena's first 3 bytes (the caller passes it wave-uniform), so a far
// copy there may need the kind-3 load from q (see the far-history load); every other wave has no
// such lane and its far loads go through the arena descriptor.
template <bool kMulti, bool kLow, bool kPlain = false>
__device__ __forceinline__ bool snappy_lane(const FrameParams& P, uint64_t r0, uint64_t r1, uint4 d0, uint64_t o0, uint8_t* L,
                                            uint32_t wave, uint32_t lane, uint8_t* sink, uint64_t* bad_rec) {
    const uint32_t wl = wave * 256u + lane * 4u;  // row 0 of this lane (both images)
    // history / input row of a byte position (mod the ring), and the next row with wrap
    auto hrow = [&](uint32_t b) __attribute__((always_inline)) { return ((b << 8) & (kColH - kColRow)) | wl; };
    // v_pk_add_u16: the low half wraps at 64 KiB, the high half (0) stays 0
    auto hnext = [&](uint32_t a) __attribute__((always_inline)) {
        const u16x2 v = __builtin_bit_cast(u16x2, a) + u16x2{(uint16_t)kColRow, 0};
        return __builtin_bit_cast(uint32_t, v);
    };
    auto irow = [&](uint32_t b) __attribute__((always_inline)) { return ((b << 8) & (kColI - kColRow)) | wl; };
    auto inext = [&](uint32_t a) __attribute__((always_inline)) { return (a + kColRow) & (kColI - 1u); };

    constexpr bool kPair = !kMulti;  // paired input prefetch
    // flush stores: plain (kPlain) for records of kPlainStoreMin bytes and more (C4's 64 KiB records: far
    // copies then find their sources in L2 / MALL, decode -7.7 %), non-temporal otherwise (C2 the same
    // speed with 2.84 instead of 3.62 GB of reads per launch; C3 plain +1.8 %)
    constexpr bool kStoreNT = !kPlain;
    const bool live = r0 < r1;
    uint8_t* const out = P.out;
    // d0 / o0: rec_desc and out_off of r0, loaded by the caller (zero when !live)
    uint8_t* const gout = out + o0;
    // a far copy's 16 bytes are loaded from q - r: below the arena for a source in its first
    // bytes (only the lane of a file's first record can meet this: kind 3)
    const bool low_base = o0 < 3;
    const uint8_t* const gout_m3 = gout - 3;  // never dereferenced below out: see low_base
    const uint64_t start0 = ((uint64_t)d0.y << 32) | d0.x;
    const uint64_t base = start0 & ~15ull;
    const uint4* sa = reinterpret_cast<const uint4*>(P.file + base);
    const uint32_t lastc = live && base < P.len ? (uint32_t)umin((P.len - 1 - base) >> 4, (uint64_t)0x0FFFFFFF) : 0u;
    // (only a file or arena of 3.75 GiB or more can hold such a wave: the common case skips the loads)
    if (P.len >= 0xF0000000ull || P.state->total_bytes >= 0xF0000000ull) {
        // the wave's input and output spans from its lowest record to the end of lane 63's last one
        // (records are consecutive in the file and the arena); past what 32-bit offsets reach (a
        // chunk of very large records), each lane decodes its records one thread each instead
        const uint64_t n = P.state->n_records;
        const uint64_t end_in = r1 < n ? P.rec_off[r1] : P.len, end_out = P.out_off[umin(r1, n)];
        const uint64_t b_in = rl64(base, 0u), b_out = rl64(o0, 0u);
        const uint64_t s_in = rl64(end_in, 63u) - umin(b_in, rl64(end_in, 63u));
        const uint64_t s_out = rl64(end_out, 63u) - umin(b_out, rl64(end_out, 63u));
        if (s_in >= 0xF0000000ull || s_out >= 0xF0000000ull) {  // wave-uniform
            bool okw = true;
            for (uint64_t i = r0; i < r1; i++) {
                if (P.flags[i] & (RIO_FLAG_NIL | RIO_FLAG_CORRUPT | RIO_FLAG_EOF)) continue;
                uint64_t st, sl;
                rec_stream(P, i, st, sl);
                const uint64_t a = P.out_off[i], z = P.out_off[i + 1];
                okw = snappy_decode_thread(P.file + st, sl, out + a, z - a) && okw;
            }
            *bad_rec = r0;
            return okw;
        }
    }
    // prime the input image with chunks [0, 4)
    uint32_t whi = live ? umin(kInCh, lastc + 1) : 0u;
    for (uint32_t c = 0; c < whi; c++) {
        const uint4 v = sa[c];
        const uint32_t a = wl | (c << 12);
        col_st(L, a, v.x);
        col_st(L, a + kColRow, v.y);
        col_st(L, a + 2 * kColRow, v.z);
        col_st(L, a + 3 * kColRow, v.w);
    }
    uint32_t cn = live ? whi : 0xFFFFFFFFu;

    uint64_t k = r0;
    uint32_t s = (uint32_t)(start0 - base), s_end = s + d0.z;
    uint32_t pd = 0, rd_start = 0, rd_end = d0.w;
    // eff: the current element's copy offset, or kLitEff for a literal (no copy offset is that large:
    // a valid one is <= the bytes produced)
    uint32_t rem = 0, eff = 0;
    bool bad = false, pdone = !live;
    uint4 nd = zero4();
    uint32_t nds = (kMulti && live && r0 + 1 < r1) ? 0u : 3u;
    uint32_t d = 0, fb = 0;

    // the buffer descriptors start at the wave's lowest record (lane 0's: a wave takes consecutive
    // records), so the 32-bit offsets are relative to it and any file or arena size works; the arena
    // base stays 16 bytes below the wave's first output byte (a far copy reads from q - r, r <= 3),
    // except within the arena's first 16 bytes, where it is the arena itself (kLow's kind 3 covers q - r
    // below it, as before)
    const uint64_t w_in = rl64(base, 0u);
    const uint64_t o0l = rl64(o0, 0u);
    // lane 0 is the wave's lowest record (see the INVARIANT at k_snappy_pipe)
#ifdef RIO_DEBUG_LANES
    if (live && (base < w_in || o0 < o0l)) __builtin_trap();
#endif
    const uint64_t w_out = o0l >= 16 ? o0l - 16 : 0;
    const __amdgpu_buffer_rsrc_t rsrc_file = uniform_rsrc(P.file + w_in, P.len + RIO_DEVICE_PAD - umin(w_in, P.len));
    const __amdgpu_buffer_rsrc_t rsrc_out = uniform_rsrc(P.out + w_out, P.state->total_bytes + 16 - umin(w_out, P.state->total_bytes));
    const uint32_t base32 = (uint32_t)(base - w_in), o32 = (uint32_t)(o0 - w_out);
    // the arena descriptor base's position in its 128-byte line (wave-uniform)
    const uint32_t line0 = (uint32_t)reinterpret_cast<uintptr_t>(P.out + w_out) & 127u;
    uint32_t obase[4];  // the flush owners' arena offsets
#pragma unroll
    for (uint32_t jj = 0; jj < 4; jj++)
        obase[jj] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((16u * jj + (lane >> 2)) * 4), (int)o32);

    ColSlot S0 = col_empty_slot(), S1 = col_empty_slot(), S2 = col_empty_slot(), S3 = col_empty_slot();
    uint32_t drain = 0, qsrc = 0;
    // the next emit's source rows (ring copy) and shift, and the row holding bytes [d & ~3, d)
    uint32_t wL0 = 0, wL1 = 0, wL2 = 0, wL3 = 0, wL4 = 0, wSh = 0, wP = 0;
    uint32_t aD = hrow(0);  // history row of d
    // the flush in flight: this step's owners' blocks, read during the previous step
    uint4 pfv = zero4();
    uint32_t pofb = 0, pfpos = 0;
    bool pready = false;
    // the parser's window: rows s >> 2 and (s >> 2) + 1, read one step ahead
    uint32_t Wa, Wb;
    {
        const uint32_t a = irow(s);
        Wa = col_ld(L, a);
        Wb = col_ld(L, inext(a));
    }

    auto step = [&](ColSlot& S, const ColSlot& N, const uint32_t j) __attribute__((always_inline)) {
        drain += pdone ? 1u : 0u;
        if constexpr (kMulti) {
            nd = sel4(S.desc != 0, S.aux, nd);
            nds = S.desc ? 2u : nds;
        }
        const uint32_t pos = s;

        // 2. emit the piece parsed kD steps ago: destination dwords of bytes [d - r, d - r + 16)
        {
            const uint32_t rm = S.ringm, fm = S.farm;
            auto bsel = [](uint32_t m, uint32_t a, uint32_t b) __attribute__((always_inline)) { return (a & m) | (b & ~m); };
            uint32_t X0 = bsel(rm, wL0, S.x0), X1 = bsel(rm, wL1, S.x1), X2 = bsel(rm, wL2, S.x2), X3 = bsel(rm, wL3, S.x3),
                     X4 = bsel(rm, wL4, S.x4);
            const uint32_t sh = bsel(rm, wSh, S.q);
            uint32_t D0 = __builtin_amdgcn_alignbyte(X1, X0, sh), D1 = __builtin_amdgcn_alignbyte(X2, X1, sh),
                     D2 = __builtin_amdgcn_alignbyte(X3, X2, sh), D3 = __builtin_amdgcn_alignbyte(X4, X3, sh);
            D0 = bsel(fm, S.aux.x, D0);
            D1 = bsel(fm, S.aux.y, D1);
            D2 = bsel(fm, S.aux.z, D2);
            D3 = bsel(fm, S.aux.w, D3);
            // kind 3 (rare: a far source in the first bytes of the arena, lane of the file's first
            // record): aux holds bytes [q, q + 16), shifted up by r here
            constexpr bool kLine = kPlain && !kMulti;
            if ((kLow || kLine) && __builtin_expect(__any(S.kind == 3), 0)) {
                if (S.kind == 3) {
                    const uint32_t u = 4u - (d & 3u);
                    D0 = __builtin_amdgcn_alignbyte(S.aux.x, 0u, u);
                    D1 = __builtin_amdgcn_alignbyte(S.aux.y, S.aux.x, u);
                    D2 = __builtin_amdgcn_alignbyte(S.aux.z, S.aux.y, u);
                    D3 = __builtin_amdgcn_alignbyte(S.aux.w, S.aux.z, u);
                }
            }
            // kind 4 (kLine): aux holds bytes [q - r - S.q, + 16), S.q in [1, 15]: shifted down by S.q bytes (dword
            // rotate by S.q >> 2, then the byte shift; the bytes pulled in past aux's end are never the piece's)
            if (kLine && __any(S.kind == 4)) {
                if (S.kind == 4) {
                    const bool h2 = (S.q & 8u) != 0, h1 = (S.q & 4u) != 0;
                    const uint32_t T0 = h2 ? S.aux.z : S.aux.x, T1 = h2 ? S.aux.w : S.aux.y;
                    const uint32_t T2 = h2 ? 0u : S.aux.z, T3 = h2 ? 0u : S.aux.w;
                    const uint32_t R0 = h1 ? T1 : T0, R1 = h1 ? T2 : T1, R2 = h1 ? T3 : T2, R3 = h1 ? 0u : T3;
                    D0 = __builtin_amdgcn_alignbyte(R1, R0, S.q);
                    D1 = __builtin_amdgcn_alignbyte(R2, R1, S.q);
                    D2 = __builtin_amdgcn_alignbyte(R3, R2, S.q);
                    D3 = __builtin_amdgcn_alignbyte(0u, R3, S.q);
                }
            }
            // bytes below d keep the row's content (v_bfi_b32); the shift uses the low 5 bits: 8 (d & 3)
            const uint32_t hm = 0xFFFFFFFFu << ((d << 3) & 31u);
            D0 = (D0 & hm) | (wP & ~hm);
            const uint32_t a1 = hnext(aD), a2 = hnext(a1), a3 = hnext(a2);
            col_hst(L, aD, D0);
            col_hst(L, a1, D1);
            col_hst(L, a2, D2);
            col_hst(L, a3, D3);
            d += S.n;
            // the NEXT slot: its destination row and (ring copy) its five source rows, read right
            // after this emit's writes so a whole step hides their latency
            const uint32_t r2 = d & 3u;
            aD = hrow(d);
            wP = col_hld(L, aD);
            const uint32_t src = N.q - r2;
            wSh = src;  // alignbyte takes the low 2 bits
            const uint32_t b0 = hrow(src), b1 = hnext(b0), b2 = hnext(b1), b3 = hnext(b2), b4 = hnext(b3);
            wL0 = col_hld(L, b0);
            wL1 = col_hld(L, b1);
            wL2 = col_hld(L, b2);
            wL3 = col_hld(L, b3);
            wL4 = col_hld(L, b4);
        }

        // 3. cooperative flush, pipelined one step: the NEXT step's owners (lanes 16 ((j + 1) % 4) ..
        // + 15) publish their flush state now and their blocks are read at the end of this step; the
        // blocks of this step's owners, read during the previous step, are stored after the parse.
        // So no LDS round trip sits in front of a store (the far threshold covers the step of lag).
        const uint4 fv_now = pfv;
        const uint32_t ofb_now = pofb, fpos_now = pfpos;
        const bool ready_now = pready;
        {
            const uint32_t fo = 16u * ((j + 1) & 3u) + (lane >> 2);
            pready = d - fb >= 64;
            pofb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(fo * 4), (int)(fb | (pready ? 0x80000000u : 0u)));
        }

        // 4. parse the next piece into this slot
        {
            // v_alignbyte_b32 and the shifts use the low bits of their shift operand only
            const uint32_t W0 = __builtin_amdgcn_alignbyte(Wb, Wa, pos);  // bytes s .. s + 3
            const uint32_t W1 = __builtin_amdgcn_alignbyte(Wb >> ((pos << 3) & 31u), W0, 1u);  // s + 1 .. s + 4
            const uint32_t tag = W0 & 0xFFu, t = tag & 3u, x = tag >> 2;
            const bool avail = umin((pos + 15) >> 4, lastc) < whi;
            const bool is0 = t == 0, is1 = t == 1;
            const bool is2 = t == 2;
            const bool lng = x >= 60;
            const uint32_t lmask = 0xFFFFFFFFu >> (((63u - x) << 3) & 31u);
            uint32_t lit_long = (W1 & lmask) + 1u, lit_short = x + 1u;
            uint32_t c1_len = (x & 7u) + 4u, c1_off = ((tag & 0xE0u) << 3) | (W1 & 0xFFu);
            uint32_t c2_off = W1 & 0xFFFFu;
            pin_v(lit_long);
            pin_v(lit_short);
            pin_v(c1_len);
            pin_v(c1_off);
            pin_v(c2_off);
            const uint32_t lit_len = lng ? lit_long : lit_short;
            const uint32_t len = is0 ? lit_len : (is1 ? c1_len : lit_short);
            const uint32_t lit_hl = lng ? x - 58u : 1u;
            const uint32_t cp_hl = is1 ? 2u : (is2 ? 3u : 5u);
            const uint32_t hl = is0 ? lit_hl : cp_hl;
            const uint32_t off = is0 ? kLitEff : (is1 ? c1_off : (is2 ? c2_off : W1));
            const uint32_t sleft = s_end - s;
            const uint32_t lim = is0 ? sleft - hl : pd - rd_start;
            const uint32_t key = (is0 ? len : off) - 1u;
            const bool hbad = (hl > sleft) | (key >= lim) | (len > rd_end - pd);
            const bool hdr = !pdone && rem == 0 && s < s_end && avail;
            const bool badn = hdr && hbad, ok = hdr && !hbad;
            bad = bad || badn;
            const uint32_t sh = ok ? hl : 0u;
            const uint32_t rem1 = ok ? len : rem, eff1 = ok ? off : eff;
            const bool lit1 = eff1 == kLitEff;
            const bool go = !pdone && !badn && rem1 != 0 && (!lit1 || avail);
            // destination-aligned pieces: at most 16 - r bytes (r = pd & 3); a literal's bytes also
            // stay inside the window [s, s + 16) the availability check covers, so a piece that starts
            // with its element's header is capped at 16 - hl (copies too: only copies longer than
            // 13 bytes ever take an extra piece for it); a copy's piece at most its offset
            const uint32_t r = pd & 3u;
            const uint32_t cap = 16u - umax(sh, r);
            const uint32_t n = go ? umin(rem1, umin(cap, eff1)) : 0u;
            S.n = n;
            const bool farc = !lit1 && n != 0 && eff1 > kFarOff;
            S.kind = lit1 ? 0u : (farc ? 2u : 1u);
            S.ringm = (lit1 || farc) ? 0u : ~0u;
            S.farm = farc ? ~0u : 0u;
            qsrc = pd - eff1;
            // literal rows from (s + sh - r) & ~3 (the bytes below s + sh are masked at the emit)
            const uint32_t ls = s + sh - r;
            const uint32_t c0 = irow(ls), c1 = inext(c0), c2 = inext(c1), c3 = inext(c2), c4 = inext(c3);
            S.x0 = col_ld(L, c0);
            S.x1 = col_ld(L, c1);
            S.x2 = col_ld(L, c2);
            S.x3 = col_ld(L, c3);
            S.x4 = col_ld(L, c4);
            // literal: the shift (low 2 bits) of x0..x4; a far copy's q goes unused at the emit
            S.q = (lit1 || farc) ? ls : qsrc;
            s += sh + (lit1 ? n : 0u);
            rem = rem1 - n;
            pd += n;
            // a piece that covered its whole offset doubles it (the source is periodic in eff1; n <= 16,
            // so eff stays <= 32, a ring copy); the record end tested as one OR (one compare, not three)
            eff = eff1 + ((n == eff1) ? n : 0u);
            s = badn ? s_end : s;
            uint32_t at_z = rem | (s ^ s_end) | (uint32_t)pdone;
            pin_v(at_z);
            if (at_z == 0) {
                const bool bad_len = pd != rd_end;
                bad = bad || bad_len;
                rem = bad_len ? rd_end - pd : rem;
                eff = bad_len ? 16u : eff;  // the rest of the record: a ring copy (bytes unspecified)
                const bool more = kMulti && k + 1 < r1;
                const bool sw = !bad_len && more && nds == 2;
                pdone = pdone || (!bad_len && !more);
                k += sw ? 1u : 0u;
                const uint64_t nstart = ((uint64_t)nd.y << 32) | nd.x;
                s = sw ? (uint32_t)(nstart - base) : s;
                s_end = sw ? s + nd.z : s_end;
                rd_start = sw ? pd : rd_start;
                rd_end = sw ? pd + nd.w : rd_end;
                nds = sw ? (k + 1 < r1 ? 0u : 3u) : nds;
            }
        }
        // this step's owners' blocks, stored after the step's loads (after the input prefetch), so a wait for this
        // step's loads three steps on does not also wait for this store: vmcnt retires stores and loads in issue order
        auto flush_store = [&]() __attribute__((always_inline)) {
            const v4u32b w = {fv_now.x, fv_now.y, fv_now.z, fv_now.w};
            __builtin_amdgcn_raw_buffer_store_b128(w, rsrc_out, (ofb_now >> 31) ? obase[j & 3u] + fpos_now : kOob, 0,
                                                   kStoreNT ? 2 : 0);
        };
        fb += ((lane >> 4) == (j & 3u) && ready_now) ? 64u : 0u;

        // far history (destination-aligned: from q - r), or the next record's descriptor, or a placeholder
        {
            const bool want_desc = kMulti && S.kind != 2 && nds == 0;
            S.desc = want_desc ? 1u : 0u;
            nds = want_desc ? 1u : nds;
            const uint32_t r = (pd - S.n) & 3u;  // the piece's destination alignment
            if constexpr (!kMulti && !kLow) {
                // no descriptor to fetch and no source below the arena: the arena descriptor alone
                uint32_t fo = o32 + qsrc - r;
                if constexpr (kPlain) {
                    // the window's place in its line; a straddling window moves inside the piece's own line
                    const uint32_t a = (line0 + fo) & 127u, back = a - 112u;
                    const bool strad = S.kind == 2 && a > 112u;
                    const bool inB = strad && a + r + S.n <= 128u && fo >= back;  // bytes in the window's first line
                    const bool inA = strad && a + r >= 128u;                     // bytes in the next line: from q
                    fo = inB ? fo - back : (inA ? fo + r : fo);
                    S.kind = inB ? 4u : (inA ? 3u : S.kind);
                    S.q = inB ? back : S.q;
                }
                const v4u32b v = __builtin_amdgcn_raw_buffer_load_b128(rsrc_out, S.kind >= 2 ? fo : kOob, 0, 0);
                S.aux = make_uint4(v.x, v.y, v.z, v.w);
            } else {
                // 16 bytes from q - r would start below the arena: load from q, shift at the emit (kind 3)
                const bool below = kLow && low_base && S.kind == 2 && qsrc < r;
                S.kind = below ? 3u : S.kind;
                const uint8_t* ap = S.kind >= 2 ? gout_m3 + (qsrc + 3u - (below ? 0u : r))
                                                : (want_desc ? reinterpret_cast<const uint8_t*>(P.rec_desc + (k + 1)) : sink);
                S.aux = ldu16(ap);
            }
        }

        // 5. input prefetch
        if constexpr (kPair) {
          if ((j & 1u) == 0) {  // a pair (cn, cn + 1) when the ring has room for both
            const uint32_t a = s >> 4;
            const bool take = cn <= lastc && cn + 1 < a + kInCh;
            const v4u32b v = __builtin_amdgcn_raw_buffer_load_b128(rsrc_file, take ? base32 + 16u * cn : kOob, 0, 0);
            const v4u32b v2 = __builtin_amdgcn_raw_buffer_load_b128(rsrc_file, take ? base32 + 16u * cn + 16u : kOob, 0, 0);
            S.in = make_uint4(v.x, v.y, v.z, v.w);
            S.in2 = make_uint4(v2.x, v2.y, v2.z, v2.w);
            S.in_c = take ? cn : kNoChunk;
            cn += take ? 2u : 0u;
          } else {
            S.in_c = kNoChunk;
          }
        } else {
            const uint32_t a = s >> 4;
            const bool take = cn <= lastc && cn < a + kInCh;
            const v4u32b v = __builtin_amdgcn_raw_buffer_load_b128(rsrc_file, take ? base32 + 16u * cn : kOob, 0, 0);
            S.in = make_uint4(v.x, v.y, v.z, v.w);
            S.in_c = take ? cn : kNoChunk;
            cn += take ? 1u : 0u;
        }

        flush_store();

        // 6. land the next slot's input chunk(s), then read the next step's parser window
        if constexpr (kPair) {
          if ((j & 1u) == 1) {  // the slot landing now was filled on an even step
            const bool landed = N.in_c != kNoChunk;
            if (landed) {
                const uint32_t a = wl | ((N.in_c & (kInCh - 1)) << 12);
                const uint32_t a2 = wl | (((N.in_c + 1) & (kInCh - 1)) << 12);
                col_st(L, a, N.in.x);
                col_st(L, a + kColRow, N.in.y);
                col_st(L, a + 2 * kColRow, N.in.z);
                col_st(L, a + 3 * kColRow, N.in.w);
                col_st(L, a2, N.in2.x);
                col_st(L, a2 + kColRow, N.in2.y);
                col_st(L, a2 + 2 * kColRow, N.in2.z);
                col_st(L, a2 + 3 * kColRow, N.in2.w);
            }
            whi = landed ? N.in_c + 2 : whi;
          }
        } else {
            const bool landed = N.in_c != kNoChunk;
            if (landed) {
                const uint32_t a = wl | ((N.in_c & (kInCh - 1)) << 12);
                col_st(L, a, N.in.x);
                col_st(L, a + kColRow, N.in.y);
                col_st(L, a + 2 * kColRow, N.in.z);
                col_st(L, a + 3 * kColRow, N.in.w);
            }
            whi = landed ? N.in_c + 1 : whi;
        }
        // 7. the next owners' blocks (rows fpos >> 2 .. + 3 of column fo: 16-byte aligned, no wrap
        // inside), the next parser window
        {
            const uint32_t fo = 16u * ((j + 1) & 3u) + (lane >> 2);
            pfpos = (pofb & 0x7FFFFFFFu) + 16u * (lane & 3u);
            const uint32_t fa = ((pfpos << 8) & (kColH - kColRow)) | (wave * 256u + fo * 4u);
            pfv = make_uint4(col_hld(L, fa), col_hld(L, fa + kColRow), col_hld(L, fa + 2 * kColRow),
                             col_hld(L, fa + 3 * kColRow));
            const uint32_t a = irow(s);
            Wa = col_ld(L, a);
            Wb = col_ld(L, inext(a));
        }
    };

    static_assert(kD == 4, "unrolled for four slots");
    do {
        step(S0, S1, 0);
        step(S1, S2, 1);
        step(S2, S3, 2);
        step(S3, S0, 3);
    } while (__any(drain < kD));
    // the stream's tail (< 128 bytes) from the lane's own rows
    for (uint32_t q = fb; q < d; q += 16) {
        const uint32_t a = hrow(q);
        const uint4 v = make_uint4(col_hld(L, a), col_hld(L, hnext(a)), col_hld(L, hnext(hnext(a))),
                                   col_hld(L, hnext(hnext(hnext(a)))));
        if (q + 16 <= d)
            stu16(gout + q, v);
        else
            st_partial(gout + q, v, d - q);
    }
    *bad_rec = r0;
    return !bad;
}
}  // namespace

// rio_device_decode_batch: the files one after the other, every wave of the grid on each (a wave
// that finishes its share of file f goes on to file f + 1 at once: no grid-wide step)
__global__ void __launch_bounds__(64 * kCoopWaves) k_snappy_coop_batch(FrameBatch B) {
    __shared__ CoopLds lds[kCoopWaves];
    const uint32_t wv = threadIdx.x >> 6;
    for (uint32_t f = 0; f < B.n; f++)
        coop_file(B.f[f], lds[wv], threadIdx.x & 63u, (uint64_t)blockIdx.x * kCoopWaves + wv,
                  (uint64_t)gridDim.x * kCoopWaves);
}

// rio_device_decode_batch: one launch for every lane-decoder file of the batch. The lanes of the grid
// are split over the files by record count (whole waves per file, so the file's parameters stay
// wave-uniform scalars), which is what fills the chip when each file alone has fewer records than
// lanes (BASELINE configs[3]: 8 files of 16384 x 64 KiB records).
__device__ __forceinline__ bool pipe_active(const FrameParams& P) {
    const ScanState* st = P.state;
    return st->hdr_status == RIO_OK && !st->capacity_fail && st->compression == RIO_COMP_SNAPPY && st->any_mixed &&
           !snappy_wide(P, st) && !(st->n_records && st->total_bytes / st->n_records >= P.coop_min);
}

// INVARIANT (both launch sites, k_snappy_pipe and k_snappy_pipe_batch): the lanes of a wave
// take consecutive, ascending records (lane l's first record = the wave's first + l * records per lane),
// so lane 0 holds the wave's lowest file offset (base) and arena offset (o0), and lane 63's last record
// ends the wave's spans. snappy_lane's kLow choice (rl64(o0, 0) < 3), its buffer bases (rl64(base, 0),
// rl64(o0, 0)) and its span guard all rely on it: a strided or load-balanced record-to-lane mapping
// would need the minimum over the live lanes instead. RIO_DEBUG_LANES checks it at run time.
__global__ void __launch_bounds__(kSnappyBlock) k_snappy_pipe(FrameParams P) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kColLds];
    ScanState* st = P.state;
    if (st->hdr_status != RIO_OK || st->capacity_fail || st->compression != RIO_COMP_SNAPPY) return;
    if (!st->any_mixed) return;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    if (coop_active(P, st)) {
        coop_file(P, *reinterpret_cast<CoopLds*>(lds + kColI + wave * kCoopSlice), lane,
                  (uint64_t)blockIdx.x * (kSnappyBlock / 64) + wave, (uint64_t)gridDim.x * (kSnappyBlock / 64));
        return;
    }
    const uint64_t n = st->n_records;
    const bool plain = n && st->total_bytes / n >= kPlainStoreMin;  // flush store policy (kPlainStoreMin)
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t g = (uint64_t)wave * gridDim.x + blockIdx.x;
    uint8_t* sink = P.sink + g * 64;
    const uint64_t rpc = n >= kChunksPerWave * 64 * waves ? n / (kChunksPerWave * 64 * waves) : 1;
    const uint64_t per = 64 * rpc, nchunks = (n + per - 1) / per;
    uint64_t chunk = g;
    while (chunk < nchunks) {
        const uint64_t r0 = umin(chunk * per + lane * rpc, n), r1 = umin(r0 + rpc, n);
        uint64_t bad_rec = 0;
        bool ok;
        // lane 0 holds the wave's lowest arena offset (consecutive ascending records per lane, the
        // INVARIANT above): a wave whose lanes all start at >= 3 never needs kind 3
        const bool live0 = r0 < r1;
        const uint4 d0 = live0 ? P.rec_desc[r0] : zero4();
        const uint64_t o0 = live0 ? P.out_off[r0] : 0;
        const bool low = rl64(live0 ? o0 : ~0ull, 0u) < 3;
        if (rpc == 1 && plain)
            ok = low ? snappy_lane<false, true, true>(P, r0, r1, d0, o0, lds, wave, lane, sink, &bad_rec)
                     : snappy_lane<false, false, true>(P, r0, r1, d0, o0, lds, wave, lane, sink, &bad_rec);
        else if (rpc == 1)
            ok = low ? snappy_lane<false, true>(P, r0, r1, d0, o0, lds, wave, lane, sink, &bad_rec)
                     : snappy_lane<false, false>(P, r0, r1, d0, o0, lds, wave, lane, sink, &bad_rec);
        else
            ok = low ? snappy_lane<true, true>(P, r0, r1, d0, o0, lds, wave, lane, sink, &bad_rec)
                     : snappy_lane<true, false>(P, r0, r1, d0, o0, lds, wave, lane, sink, &bad_rec);
        if (!ok) {
            const uint32_t at = atomicAdd(&st->n_fail_lanes, 1u);
            if (at < kFailLanes) {
                P.fail_lanes[2 * at] = r0;
                P.fail_lanes[2 * at + 1] = r1;
            }
        }
        uint32_t next = 0;
        if (lane == 0) next = atomicAdd(&st->pipe_next, 1u);
        chunk = waves + __shfl(next, 0);
    }
}

__global__ void __launch_bounds__(kSnappyBlock) k_snappy_pipe_batch(FrameBatch B) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kColLds];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t wg = (uint64_t)wave * gridDim.x + blockIdx.x;
    uint64_t N = 0;
    for (uint32_t f = 0; f < B.n; f++)
        if (pipe_active(B.f[f])) N += B.f[f].state->n_records;
    if (N == 0) return;
    uint64_t rpl = (N + 64 * waves - 1) / (64 * waves);
    for (;;) {
        uint64_t need = 0;
        for (uint32_t f = 0; f < B.n; f++)
            if (pipe_active(B.f[f])) need += (B.f[f].state->n_records + 64 * rpl - 1) / (64 * rpl);
        if (need <= waves) break;
        rpl++;
    }
    const uint64_t per_wave = 64 * rpl;
    uint64_t w0 = 0;
    for (uint32_t f = 0; f < B.n; f++) {
        const FrameParams& P = B.f[f];
        if (!pipe_active(P)) continue;
        const uint64_t n = P.state->n_records, wf = (n + per_wave - 1) / per_wave;
        if (wg < w0 + wf) {
            // consecutive ascending records per lane (the INVARIANT at k_snappy_pipe)
            const uint64_t t = ((wg - w0) << 6) | lane;
            const uint64_t r0 = umin(t * rpl, n), r1 = umin(r0 + rpl, n);
            uint8_t* sink = P.sink + wg * 64;
            uint64_t bad_rec = 0;
            bool ok;
            const bool live0 = r0 < r1;
            const uint4 d0 = live0 ? P.rec_desc[r0] : zero4();
            const uint64_t o0 = live0 ? P.out_off[r0] : 0;
            const bool low = rl64(live0 ? o0 : ~0ull, 0u) < 3;
            const bool plain = n && P.state->total_bytes / n >= kPlainStoreMin;  // wave-uniform (one file)
            if (rpl == 1 && plain)
                ok = low ? snappy_lane<false, true, true>(P, r0, r1, d0, o0, lds, wave, lane, sink, &bad_rec)
                         : snappy_lane<false, false, true>(P, r0, r1, d0, o0, lds, wave, lane, sink, &bad_rec);
            else if (rpl == 1)
                ok = low ? snappy_lane<false, true>(P, r0, r1, d0, o0, lds, wave, lane, sink, &bad_rec)
                         : snappy_lane<false, false>(P, r0, r1, d0, o0, lds, wave, lane, sink, &bad_rec);
            else
                ok = low ? snappy_lane<true, true>(P, r0, r1, d0, o0, lds, wave, lane, sink, &bad_rec)
                         : snappy_lane<true, false>(P, r0, r1, d0, o0, lds, wave, lane, sink, &bad_rec);
            if (!ok) {
                const uint32_t at = atomicAdd(&P.state->n_fail_lanes, 1u);
                if (at < kFailLanes) {
                    P.fail_lanes[2 * at] = r0;
                    P.fail_lanes[2 * at + 1] = r1;
                }
            }
            return;
        }
        w0 += wf;
    }
}

hipError_t launch_snappy_batch(const FrameBatch& B, hipStream_t s) {
    hipLaunchKernelGGL(k_snappy_pipe_batch, dim3(kSnappyGrid), dim3(kSnappyBlock), 0, s, B);
    hipLaunchKernelGGL(k_snappy_coop_batch, dim3(kCoopGrid), dim3(64 * kCoopWaves), 0, s, B);
    return hipGetLastError();
}

// main = false: the caller runs the lane and wave decoders for this file itself (a batch)
hipError_t launch_snappy_decode(const FrameParams& P, hipStream_t s, bool main) {
    // 4 waves x 20 KiB = 80 KiB per workgroup: 2 workgroups (8 waves) per CU
    if (main) {
        hipLaunchKernelGGL(k_snappy_pipe, dim3(kSnappyGrid), dim3(kSnappyBlock), 0, s, P);
    }
    return hipGetLastError();
}

}  // namespace rio
