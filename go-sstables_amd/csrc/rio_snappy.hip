// rio_snappy.hip — Snappy block decode of every framed record (golang/snappy v1.0.0 semantics,
// decode.go + decode_other.go; called per record by FileReader.ReadNext, file_reader.go:115-125).
//
// k_snappy_pipe: one lane per record (SIMT across consecutive records), software-pipelined so that
// no lane ever waits on a memory load issued in the same iteration.
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
//   * The flush is cooperative (see snappy_wave): 64 contiguous bytes of 16 records per wave
//     store. Lane-private 16-byte stores to 64 records run at ~1.5 TB/s on MI355X, the 16-record
//     form at ~4.2 TB/s (scripts/mem_probe.hip); loads do not care (5.5 vs 6.0 TB/s).
//   * History: the last 256 decoded bytes of each record live in an LDS ring; copies reaching
//     further back (offset > kFarOff) are loaded from the output arena at PARSE time, kD
//     iterations before use — the flush schedule guarantees those bytes were stored already
//     (flush lag < 128 bytes, parser lead <= 16*(kD-1) bytes: kFarOff >= 16*(kD-1) + 16 + 128).
//   * Input: aligned 16-byte chunks loaded kD iterations ahead land in a 64-byte LDS ring.
//   * LDS image per wave is chunk-interleaved ([chunk][lane][16 B]): every 16-byte access by a
//     wave touches each bank once, whatever positions the lanes are at.
// Wave-per-record decoder (coop_*, k_snappy_coop_batch): files or arenas past 32-bit positions and
// streams >= 4 GiB; 64-bit addressing, one 64-byte output window per round with lane = byte.
// Files whose every record is a single literal (k_place sets ScanState::any_mixed otherwise) are
// copied by k_copy_records (rio_kernels.hip) and the kernels here exit at once.
#include <hip/hip_runtime.h>

#include "rio_device.h"
#include "rio_dev_util.h"

namespace rio {

namespace {
constexpr uint32_t kOutCh = 16;                  // history ring: 16 chunks = 256 bytes per lane
constexpr uint32_t kInCh = 4;                    // input ring: 4 chunks = 64 bytes per lane
constexpr uint32_t kD = 4;                       // pipeline depth in iterations
// chunks per wave: the balance against the per-chunk drain and setup (A/B on MI355X, records per lane
// per chunk: C3 64-B records 19 -> 9: decode 0.906 -> 0.870 ms; 4: 0.922, 1: 1.92; C2 stays at 1)
#ifndef RIO_CHUNKS_PER_WAVE
#define RIO_CHUNKS_PER_WAVE 8
#endif
// copies reaching further back than kFarOff read the output arena (flushed: see snappy_lane)
constexpr uint32_t kFarOff = 16 * (kD - 1) + 16 + 128;
constexpr uint32_t kNoChunk = ~0u;               // slot carries no input chunk
static_assert(kFarOff >= 16 * (kD - 1) + 16 + 128, "far history must be flushed before the parser reads it");
// v9: a ring copy's source window starts >= 16 * (chunk(d) - kFarOff / 16), and ring chunk chunk(d) + 2
// (= chunk(d) - 14 mod 16) serves as the staging chunk of literal / far bytes: it must be dead
static_assert(kOutCh == 16 && kFarOff <= 16 * 13, "staging chunk must hold no live history");
static_assert(kSnappyBlock % 64 == 0, "whole waves");

// bytes [r, r + 16) of the 32-byte little-endian concatenation (a, b), r in [0, 16): dword
// selection by r >> 2 (two select levels) + v_alignbyte_b32 for the byte shift
__device__ __forceinline__ uint4 funnel16(uint4 a, uint4 b, uint32_t r) {
    const uint32_t sh = r & 3u;
    const bool h1 = (r & 4u) != 0, h2 = (r & 8u) != 0;
    const uint32_t p0 = h1 ? a.y : a.x, p1 = h1 ? a.z : a.y, p2 = h1 ? a.w : a.z, p3 = h1 ? b.x : a.w,
                   p4 = h1 ? b.y : b.x, p5 = h1 ? b.z : b.y, p6 = h1 ? b.w : b.z;
    const uint32_t e0 = h2 ? p2 : p0, e1 = h2 ? p3 : p1, e2 = h2 ? p4 : p2, e3 = h2 ? p5 : p3, e4 = h2 ? p6 : p4;
    return make_uint4(__builtin_amdgcn_alignbyte(e1, e0, sh), __builtin_amdgcn_alignbyte(e2, e1, sh),
                      __builtin_amdgcn_alignbyte(e3, e2, sh), __builtin_amdgcn_alignbyte(e4, e3, sh));
}

// materialize x in a VGPR here: the selects that use it can no longer be turned into branches that
// compute x on one side only (an empty asm with a register constraint; no instruction is emitted)
__device__ __forceinline__ void pin_v(uint32_t& x) { asm volatile("" : "+v"(x)); }

__device__ __forceinline__ uint4 sel4(bool c, uint4 a, uint4 b) {
    return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

// bytes [f, f + 16) and [f + 16, f + 32) of the 48-byte little-endian concatenation (A, B, C),
// f in [0, 16): one dword-select network shared by both halves, then v_alignbyte_b32
__device__ __forceinline__ void funnel32(uint4 A, uint4 B, uint4 C, uint32_t f, uint4& L, uint4& H) {
    const uint32_t sh = f & 3u;
    const bool h1 = (f & 4u) != 0, h2 = (f & 8u) != 0;
    // written out (no arrays): an indexed form is lowered to a private-memory table lookup
    uint32_t p0 = h1 ? A.y : A.x, p1 = h1 ? A.z : A.y, p2 = h1 ? A.w : A.z, p3 = h1 ? B.x : A.w,
             p4 = h1 ? B.y : B.x, p5 = h1 ? B.z : B.y, p6 = h1 ? B.w : B.z, p7 = h1 ? C.x : B.w,
             p8 = h1 ? C.y : C.x, p9 = h1 ? C.z : C.y, p10 = h1 ? C.w : C.z;
    pin_v(p0), pin_v(p1), pin_v(p2), pin_v(p3), pin_v(p4), pin_v(p5), pin_v(p6), pin_v(p7), pin_v(p8), pin_v(p9),
        pin_v(p10);
    const uint32_t e0 = h2 ? p2 : p0, e1 = h2 ? p3 : p1, e2 = h2 ? p4 : p2, e3 = h2 ? p5 : p3, e4 = h2 ? p6 : p4,
                   e5 = h2 ? p7 : p5, e6 = h2 ? p8 : p6, e7 = h2 ? p9 : p7, e8 = h2 ? p10 : p8;
    L = make_uint4(__builtin_amdgcn_alignbyte(e1, e0, sh), __builtin_amdgcn_alignbyte(e2, e1, sh),
                   __builtin_amdgcn_alignbyte(e3, e2, sh), __builtin_amdgcn_alignbyte(e4, e3, sh));
    H = make_uint4(__builtin_amdgcn_alignbyte(e5, e4, sh), __builtin_amdgcn_alignbyte(e6, e5, sh),
                   __builtin_amdgcn_alignbyte(e7, e6, sh), __builtin_amdgcn_alignbyte(e8, e7, sh));
}

// bytes [0, r) from `st`, [r, 16) from `v` (r in [0, 16)): two 64-bit masks, then bit selects
__device__ __forceinline__ uint4 merge_at(uint4 st, uint4 v, uint32_t r) {
    const uint32_t s8 = 8u * r;
    const uint64_t all = ~0ull;
    const uint64_t mlo = s8 >= 64 ? 0ull : (all << s8), mhi = s8 >= 64 ? (all << ((s8 - 64) & 63)) : all;
    const uint32_t m0 = (uint32_t)mlo, m1 = (uint32_t)(mlo >> 32), m2 = (uint32_t)mhi, m3 = (uint32_t)(mhi >> 32);
    return make_uint4((v.x & m0) | (st.x & ~m0), (v.y & m1) | (st.y & ~m1), (v.z & m2) | (st.z & ~m2),
                      (v.w & m3) | (st.w & ~m3));
}

// cache policy (RIO_NT): 1 = non-temporal flush stores, 2 = non-temporal far loads. Default 1: the
// arena stores no longer push the lanes' input lines out of L2 between their 16-byte reads (C2
// decode: HBM reads 4.1 -> 3.4 GB and writes 1.12 -> 1.03 GB per launch, 0.9 % slower, because far
// copies then miss L2 more often; C4: 3 % faster). 2 and 3 were slower (+5 %, +8 %).
#ifndef RIO_NT
#define RIO_NT 1
#endif
__device__ __forceinline__ void st_out(uint8_t* p, uint4 v) {
    if (RIO_NT & 1) stu16_nt(p, v); else stu16(p, v);
}
__device__ __forceinline__ uint4 ld_far(const uint8_t* p) { return (RIO_NT & 2) ? ldu16_nt(p) : ldu16(p); }

// per-lane view of the wave's chunk-interleaved LDS images. History and input ring are separate
// __shared__ objects, so the compiler knows they never alias and may issue the parser's input-ring
// reads while the emitter's history writes are still queued.
struct LaneLds {
    uint8_t* h;  // wave history image + lane * 16
    uint8_t* i;  // wave input-ring image + lane * 16
    __device__ uint4* out(uint32_t pos) const { return reinterpret_cast<uint4*>(h + ((pos >> 4) & (kOutCh - 1)) * 1024); }
    __device__ uint4* in(uint32_t c) const { return reinterpret_cast<uint4*>(i + (c & (kInCh - 1)) * 1024); }
};

// one pipeline slot: a parsed piece plus the two loads issued with it
struct Slot {
    uint4 in;       // input chunk in_c (load in flight; sink bytes when in_c == kNoChunk)
    uint4 aux;      // far-history bytes (kind 2) or the next record's descriptor (desc): in flight
    uint4 lit;      // literal bytes (kind == 0)
    uint32_t in_c;  // chunk index of `in`
    uint32_t n;     // piece length, 0 = bubble
    uint32_t q;     // source output position (kind 1)
    uint32_t kind;  // 0 literal, 1 ring copy, 2 far copy
    uint32_t desc;  // aux carries the next record's descriptor
};
__device__ __forceinline__ Slot empty_slot() {
    Slot S;
    S.in = zero4();
    S.in_c = kNoChunk;
    S.aux = zero4();
    S.lit = zero4();
    S.n = 0;
    S.q = 0;
    S.kind = 1;
    S.desc = 0;
    return S;
}
}  // namespace

// Files the 32-bit lane-stream positions cannot cover take the wave-per-record decoder.
__device__ __forceinline__ bool snappy_wide(const FrameParams& P, const ScanState* st) {
    return st->huge_streams || P.len >= 0xFFFFFF00ull || st->total_bytes >= 0xFFFFFF00ull;
}

// Decode the contiguous record range [r0, r1) of this lane as ONE stream: consecutive records are
// contiguous in the output arena and separated only by their headers in the file, so the lane's
// pipeline never drains between records; positions are relative to the lane's aligned input base
// and to its output base out_off[r0]. Copy offsets stay record-relative (golang/snappy bounds per
// record); the next record's descriptor travels in the far-load slot of a step without a far copy.
// The loop runs until every lane of the wave is done: finished lanes keep stepping as bubbles because
// the flush is cooperative — at step j the 16 lanes 16*(j%4) .. +15 are "owners" and every quad of
// lanes writes one owner's next complete 64-byte block (16 B per lane, 64 contiguous bytes of one
// stream): a wave store touches 16 streams instead of 64, which the L2 absorbs ~3x faster.
// Returns false with *bad_rec = the failing record if a record does not decode.
// kMulti = false: every lane of the wave has at most one record (C2's chunks), so the record switch
// and the next-descriptor fetch are compiled out of the step.
template <bool kMulti>
__device__ __forceinline__ bool snappy_lane_t(const FrameParams& P, uint64_t r0, uint64_t r1, uint8_t* wl, uint8_t* wi,
                                              uint32_t lane, uint8_t* sink, uint64_t* bad_rec) {
    const LaneLds L{wl + lane * 16, wi + lane * 16};
    const bool live = r0 < r1;
    uint8_t* const out = P.out;
    const uint4 d0 = live ? P.rec_desc[r0] : zero4();
    const uint64_t o0 = live ? P.out_off[r0] : 0;  // lane output base (arena offset)
    uint8_t* const gout = out + o0;
    const uint64_t start0 = ((uint64_t)d0.y << 32) | d0.x;
    const uint64_t base = start0 & ~15ull;  // lane input base (file offset, 16-B aligned)
    const uint4* sa = reinterpret_cast<const uint4*>(P.file + base);
    // chunks the prefetcher may read: up to the file end (+pad), never more than the lane needs
    const uint32_t lastc = live && base < P.len ? (uint32_t)min((P.len - 1 - base) >> 4, (uint64_t)0x0FFFFFFF) : 0u;
    // prime the input ring with chunks [0, 4)
    uint32_t whi = live ? min(kInCh, lastc + 1) : 0u;  // chunks [0, whi) have landed
    for (uint32_t c = 0; c < whi; c++) *L.in(c) = sa[c];
    uint32_t cn = live ? whi : 0xFFFFFFFFu;  // next chunk to load (never for an idle lane)

    // record state: current record k, its input [s, s_end) and output [rd_start, rd_end)
    uint64_t k = r0;
    uint32_t s = (uint32_t)(start0 - base), s_end = s + d0.z;
    uint32_t pd = 0, rd_start = 0, rd_end = d0.w;
    uint32_t rem = 0, eff = 0;
    bool islit = false, bad = false, pdone = !live;
    // next record's descriptor: 0 needed, 1 in flight, 2 landed, 3 none (last record)
    uint4 nd = zero4();
    uint32_t nds = (live && r0 + 1 < r1) ? 0u : 3u;
    // emitter state: d = bytes emitted, fb = flushed bytes (multiple of 64)
    uint32_t d = 0, fb = 0;
    uint4 stage = zero4();

    // output base of the owner each lane flushes for at step j (owner = 16 (j % 4) + lane / 4): the
    // owners never change, so their bases are exchanged once instead of every step
    uint8_t* obase[4];
#pragma unroll
    for (uint32_t jj = 0; jj < 4; jj++) {
        const int src = (int)((16u * jj + (lane >> 2)) * 4);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)o0);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(o0 >> 32));
        obase[jj] = out + (((uint64_t)hi << 32) | lo);
    }

    Slot S0 = empty_slot(), S1 = empty_slot(), S2 = empty_slot(), S3 = empty_slot();
    uint32_t drain = 0, qsrc = 0;
    // v9: the next emit's source window (three ring chunks) and its funnel shift
    uint4 wA = zero4(), wB = zero4(), wC = zero4();
    uint32_t wF = 0, wN = 0;
    // the parser's input window [s, s + 16), read one step ahead (end of the previous step) so that
    // its LDS latency hides behind the emit and flush
    // (the two raw chunks travel; the funnel runs where the parser needs the bytes)
    uint4 Wa = *L.in(s >> 4), Wb = *L.in((s >> 4) + 1);

    auto step = [&](Slot& S, const Slot& N, const uint32_t j) __attribute__((always_inline)) {
        drain += pdone ? 1u : 0u;
        // 1. the next record's descriptor, if this slot fetched it
        if constexpr (kMulti) {
            nd = sel4(S.desc != 0, S.aux, nd);
            nds = S.desc ? 2u : nds;
        }
        const uint32_t pos = s;

        // 2. emit the piece parsed kD iterations ago (a bubble appends nothing)
        // Destination-aligned: a literal's or far copy's 16 bytes are first stored to the dead ring
        // chunk chunk(d) + 2, so every piece is "bytes [w, w + 32) of the ring, w = source - r" with
        // r = d & 15: one funnel over three ring chunks yields the destination chunk and its
        // successor already aligned; bytes below r come from the staged head, bytes past the piece
        // are garbage that later pieces overwrite (never flushed: flushes take complete blocks < d).
        {
            const uint32_t r = d & 15u;
            uint4 lo, hi;
            funnel32(wA, wB, wC, wF, lo, hi);  // this piece's window, read during the previous step
            lo = merge_at(stage, lo, r);
            *L.out(d) = lo;
            *L.out(d + 16) = hi;
            stage = sel4(r + S.n >= 16, hi, lo);
            d += S.n;
            // The NEXT slot: d does not move before its emit, so its staging chunk and source window
            // are known now. Stage its literal / far bytes, then read its window: the reads' latency
            // hides behind this step's flush and parse instead of sitting on the emit chain.
            const uint32_t r2 = d & 15u, cs = (d >> 4) + 2u;
            *L.out(cs << 4) = sel4(N.kind == 0, N.lit, N.aux);
            const uint32_t w = (N.kind == 1 ? N.q : (cs << 4) + N.q) - r2;
            wN = w;
            wF = w & 15u;
        }

        // 3. cooperative flush: lane writes 16 bytes of owner o's next 64-byte block if complete
        {
            const uint32_t o = 16u * (j & 3u) + (lane >> 2), part = lane & 3u;
            const bool ready = d - fb >= 64;
            const uint32_t ofb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(o * 4), (int)(fb | (ready ? 0x80000000u : 0u)));
            const uint32_t pos = (ofb & 0x7FFFFFFFu) + 16u * part;
            const uint4 fv = *reinterpret_cast<const uint4*>(wl + ((pos >> 4) & (kOutCh - 1)) * 1024 + o * 16);
            // the next emit's window after the flush data: the store waits for fv only, the window
            // reads stay in flight through the store and the parse
            wA = *L.out(wN);
            wB = *L.out(wN + 16u);
            wC = *L.out(wN + 32u);
            st_out((ofb >> 31) ? obase[j & 3u] + pos : sink, fv);
            fb += ((lane >> 4) == (j & 3u) && ready) ? 64u : 0u;
        }

        // 4. parse the next piece into this slot (selects only: lanes diverge in data, not flow)
        {
            const uint4 W = funnel16(Wa, Wb, pos & 15u);  // input bytes [s, s + 16)
            // element header at s (golang/snappy decode_other.go tag forms): every form is computed
            // and combined with selects, so divergent tags cost no exec-mask branches
            const uint32_t W1 = __builtin_amdgcn_alignbyte(W.y, W.x, 1);  // the 4 bytes after the tag
            const uint32_t tag = W.x & 0xFFu, t = tag & 3u, x = tag >> 2;
            const bool avail = min((pos + 15) >> 4, lastc) < whi;
            const bool is0 = t == 0, is1 = t == 1;
            const bool is2 = t == 2;
            // literal: x < 60 -> length x + 1; x in [60, 63] -> x - 59 little-endian length bytes follow
            const bool lng = x >= 60;
            const uint32_t lmask = 0xFFFFFFFFu >> (((63u - x) << 3) & 31u);
            // every alternative computed unconditionally, then selected: the compiler otherwise
            // turned these nested ternaries into exec-mask branches (3 per step)
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
            const uint32_t off = is1 ? c1_off : (is2 ? c2_off : W1);
            // golang/snappy bounds, per record: header bytes present; literal source room or copy
            // offset in [1, bytes produced] (length / offset 0 wrap to the maximum key); output room
            const uint32_t sleft = s_end - s;
            const uint32_t lim = is0 ? sleft - hl : pd - rd_start;
            const uint32_t key = (is0 ? len : off) - 1u;
            const bool hbad = (hl > sleft) | (key >= lim) | (len > rd_end - pd);
            const bool hdr = !pdone && rem == 0 && s < s_end && avail;
            const bool badn = hdr && hbad, ok = hdr && !hbad;
            bad = bad || badn;
            const uint32_t sh = ok ? hl : 0u;
            const uint32_t rem1 = ok ? len : rem, eff1 = ok ? off : eff;
            const bool lit1 = ok ? t == 0 : islit;
            // a literal piece takes the window bytes after the header; a copy piece reaches back
            // at most `eff` bytes (overlapping copies double their reach: a multiple of the offset)
            const bool go = !pdone && !badn && rem1 != 0 && (!lit1 || avail);
            const uint32_t n = go ? min(rem1, lit1 ? 16u - sh : min(16u, eff1)) : 0u;
            S.n = n;
            S.kind = n == 0 ? 1u : (lit1 ? 0u : (eff1 > kFarOff ? 2u : 1u));
            qsrc = pd - eff1;
            // the literal starts sh bytes into W; the emitter's funnel absorbs that shift (S.q = sh),
            // a far copy's bytes sit at the start of the staging chunk (S.q = 0)
            S.q = S.kind == 1 ? qsrc : (S.kind == 0 ? sh : 0u);
            S.lit = W;
            s += sh + (lit1 ? n : 0u);
            rem = rem1 - n;
            pd += n;
            eff = (!lit1 && eff1 < 16 && n == eff1) ? 2 * eff1 : eff1;
            islit = lit1;
            // a record that does not decode is not the end of the lane: its remaining input is skipped
            // and the rest of its announced output is filled (16-byte ring pieces of unspecified
            // bytes), then the next record starts; k_finish re-checks the lane and flags it
            s = badn ? s_end : s;
            // record boundary: stream consumed -> the record must be complete; switch to the next
            // (its descriptor landed) or finish the range
            // (a real branch: a lane ends a record every ~130 steps, so most steps of a wave skip it;
            // it holds no memory operation, so the wave's memory schedule stays uniform)
            // one condition in a VGPR, one branch: written with && the compiler nested three
            // branches (and their exec-mask merges) into every step
            uint32_t at_end = (uint32_t)!pdone & (uint32_t)(rem == 0) & (uint32_t)(s == s_end);
            pin_v(at_end);
            if (at_end) {
                const bool bad_len = pd != rd_end;  // snappy: d != len(dst) => ErrCorrupt
                bad = bad || bad_len;
                // fill (rd_end > pd: output room is checked per element)
                rem = bad_len ? rd_end - pd : rem;
                eff = bad_len ? 16u : eff;
                islit = islit && !bad_len;
                if constexpr (kMulti) {
                    const bool more = k + 1 < r1;
                    const bool sw = !bad_len && more && nds == 2;
                    pdone = pdone || (!bad_len && !more);
                    k += sw ? 1u : 0u;
                    const uint64_t nstart = ((uint64_t)nd.y << 32) | nd.x;
                    s = sw ? (uint32_t)(nstart - base) : s;
                    s_end = sw ? s + nd.z : s_end;
                    rd_start = sw ? pd : rd_start;
                    rd_end = sw ? pd + nd.w : rd_end;
                    nds = sw ? (k + 1 < r1 ? 0u : 3u) : nds;
                } else {
                    pdone = pdone || !bad_len;
                }
            }
        }
        // far history (flushed: see header), or the next record's descriptor, or a placeholder load
        {
            const bool want_desc = kMulti && S.kind != 2 && nds == 0;
            S.desc = want_desc ? 1u : 0u;
            nds = want_desc ? 1u : nds;
            const uint8_t* ap = S.kind == 2 ? gout + qsrc
                                            : (want_desc ? reinterpret_cast<const uint8_t*>(P.rec_desc + (k + 1)) : sink);
            S.aux = ld_far(ap);
        }

        // 5. input prefetch: the next chunk if the ring has room for it when it lands
        {
            const uint32_t a = s >> 4;
            const bool take = cn <= lastc && cn < a + kInCh;
            S.in = *reinterpret_cast<const uint4*>(take ? reinterpret_cast<const uint8_t*>(sa + cn) : sink);
            S.in_c = take ? cn : kNoChunk;
            cn += take ? 1u : 0u;
        }

        // 6. land the next slot's input chunk (loaded kD - 1 iterations ago), then read the next
        // step's parser window
        {
            const bool landed = N.in_c != kNoChunk;
            if (landed) *L.in(N.in_c) = N.in;
            whi = landed ? N.in_c + 1 : whi;
            Wa = *L.in(s >> 4);
            Wb = *L.in((s >> 4) + 1);
        }
    };

    // one exit per kD steps, taken by the whole wave: every path around the loop issues the same
    // memory operations, so the compiler's wait counts stay exact
    static_assert(kD == 4, "unrolled for four slots");
    do {
        step(S0, S1, 0);
        step(S1, S2, 1);
        step(S2, S3, 2);
        step(S3, S0, 3);
    } while (__any(drain < kD));
    // the stream's tail (< 128 bytes), lane by lane; written even after a failure: the bytes of
    // the records before the failing one must be complete
    for (uint32_t q = fb; q < d; q += 16) {
        const uint4 v = *L.out(q);
        if (q + 16 <= d)
            stu16(gout + q, v);
        else
            st_partial(gout + q, v, d - q);
    }
    *bad_rec = r0;
    return !bad;
}

__device__ __forceinline__ bool snappy_lane(const FrameParams& P, uint64_t r0, uint64_t r1, uint8_t* wl, uint8_t* wi,
                                            uint32_t lane, uint8_t* sink, uint64_t* bad_rec) {
    return snappy_lane_t<true>(P, r0, r1, wl, wi, lane, sink, bad_rec);
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
// k_snappy_pipe runs the wave decoder in the wave's history image
static_assert(sizeof(CoopLds) <= kOutCh * 1024, "wave decoder LDS must fit a history image");

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
            const uint64_t pay = P.rec_pay[i];
            const uint64_t o0 = P.out_off[i], o1 = P.out_off[i + 1];
            if (!snappy_decode_thread(P.file + P.rec_off[i] + (pay & 0xFF), pay >> 8, P.out + o0, o1 - o0))
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

// rio_device_decode_batch: the files one after the other, every wave of the grid on each (a wave
// that finishes its share of file f goes on to file f + 1 at once: no grid-wide step)
__global__ void __launch_bounds__(64 * kCoopWaves) k_snappy_coop_batch(FrameBatch B) {
    __shared__ CoopLds lds[kCoopWaves];
    const uint32_t wv = threadIdx.x >> 6;
    for (uint32_t f = 0; f < B.n; f++)
        coop_file(B.f[f], lds[wv], threadIdx.x & 63u, (uint64_t)blockIdx.x * kCoopWaves + wv,
                  (uint64_t)gridDim.x * kCoopWaves);
}

__global__ void __launch_bounds__(kSnappyBlock) k_snappy_pipe(FrameParams P) {
    __shared__ __attribute__((aligned(16))) uint8_t hist[kSnappyBlock / 64][kOutCh * 1024];
    __shared__ __attribute__((aligned(16))) uint8_t inring[kSnappyBlock / 64][kInCh * 1024];
    ScanState* st = P.state;
    if (st->hdr_status != RIO_OK || st->capacity_fail || st->compression != RIO_COMP_SNAPPY) return;
    if (!st->any_mixed) return;  // every record is one literal: k_copy_records copies them
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    if (coop_active(P, st)) {  // large records / past 32-bit positions: the wave-per-record decoder
        coop_file(P, *reinterpret_cast<CoopLds*>(hist[wave]), lane, (uint64_t)blockIdx.x * (kSnappyBlock / 64) + wave,
                  (uint64_t)gridDim.x * (kSnappyBlock / 64));
        return;
    }
    const uint64_t n = st->n_records;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t g = (uint64_t)wave * gridDim.x + blockIdx.x;  // waves numbered across workgroups first
    uint8_t* sink = P.sink + g * 64;                               // the wave's placeholder line
    // Records go to waves in chunks of 64 lanes x rpc consecutive records (each lane one contiguous
    // range: one stream, no drain between its records). Chunk g is wave g's; a wave that finishes
    // takes the next unclaimed chunk, so waves whose records decode slower, or that start later, do
    // not hold the kernel's tail. About eight chunks per wave.
    constexpr uint64_t kCpw = RIO_CHUNKS_PER_WAVE;
    const uint64_t rpc = n >= kCpw * 64 * waves ? n / (kCpw * 64 * waves) : 1;
    const uint64_t per = 64 * rpc, nchunks = (n + per - 1) / per;
    uint64_t chunk = g;
    while (chunk < nchunks) {
        const uint64_t r0 = min(chunk * per + lane * rpc, n), r1 = min(r0 + rpc, n);
        uint64_t bad_rec = 0;
        if (!snappy_lane(P, r0, r1, hist[wave], inring[wave], lane, sink, &bad_rec)) {
            // a record of this lane did not decode: k_finish re-decodes the lane's records one
            // thread each and flags the failing ones
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

// rio_device_decode_batch: one launch for every lane-decoder file of the batch. The lanes of the grid
// are split over the files by record count (whole waves per file, so the file's parameters stay
// wave-uniform scalars), which is what fills the chip when each file alone has fewer records than
// lanes (BASELINE configs[3]: 8 files of 16384 x 64 KiB records).
__device__ __forceinline__ bool pipe_active(const FrameParams& P) {
    const ScanState* st = P.state;
    return st->hdr_status == RIO_OK && !st->capacity_fail && st->compression == RIO_COMP_SNAPPY && st->any_mixed &&
           !snappy_wide(P, st) && !(st->n_records && st->total_bytes / st->n_records >= P.coop_min);
}

__global__ void __launch_bounds__(kSnappyBlock) k_snappy_pipe_batch(FrameBatch B) {
    __shared__ __attribute__((aligned(16))) uint8_t hist[kSnappyBlock / 64][kOutCh * 1024];
    __shared__ __attribute__((aligned(16))) uint8_t inring[kSnappyBlock / 64][kInCh * 1024];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t wg = (uint64_t)wave * gridDim.x + blockIdx.x;  // waves numbered across workgroups first
    uint64_t N = 0;
    for (uint32_t f = 0; f < B.n; f++)
        if (pipe_active(B.f[f])) N += B.f[f].state->n_records;
    if (N == 0) return;
    // the fewest records per lane whose whole-wave shares (ceil per file) fit the grid: every wave
    // of the grid is resident at once (2 per SIMD), so a share past it would run as a second round
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
            const uint64_t t = ((wg - w0) << 6) | lane;
            const uint64_t r0 = min(t * rpl, n), r1 = min(r0 + rpl, n);
            uint8_t* sink = P.sink + wg * 64;
            uint64_t bad_rec = 0;
            if (!snappy_lane(P, r0, r1, hist[wave], inring[wave], lane, sink, &bad_rec)) {
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
