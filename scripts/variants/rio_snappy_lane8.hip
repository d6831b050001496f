// rio_snappy.hip — Snappy block decode of every framed record (golang/snappy v1.0.0 semantics,
// decode.go + decode_other.go; called per record by FileReader.ReadNext, file_reader.go:115-125).
//
// k_snappy_lane: one lane decodes a contiguous range of records as ONE stream (SIMT across 64
// consecutive ranges), software-pipelined so that no lane waits on a global load issued in the same
// step. One step = one piece of at most 8 output bytes (the element streams of text-like 1 KiB
// records average 8.4 bytes per element, so wider pieces would mostly run half empty).
//
//   * LDS is laid out in DWORD ROWS: row k holds dword k of every lane's ring ([row][lane][4 B]).
//     A lane's 4-byte-aligned dwords at any position are 256 B apart and every wave-wide dword access
//     hits 64 distinct banks whatever position each lane is at. Eight bytes at any byte position are
//     three consecutive dwords and ONE v_alignbyte per output dword: no select trees, unlike a layout
//     of 16-byte chunks (the previous decoder spent ~130 of its 250 VALU per step on them).
//   * Output history: the last 128 bytes of the lane's stream (32 rows). Copies reaching further
//     back (offset > kFar) load their 8 bytes from the output arena at PARSE time, kD steps before
//     use; the flush schedule guarantees those bytes were stored (static_asserts below).
//   * Input: 16-byte chunks loaded kD steps ahead land in a 64-byte ring (16 rows). The parser reads
//     a 12-byte window at its position: the element header and up to 8 literal bytes.
//   * Every step issues exactly three vector-memory operations in a fixed order (flush store, far /
//     descriptor load, input load); idle lanes aim them at the wave's 64-byte sink line. CDNA retires
//     vmcnt in issue order, so a uniform schedule lets the compiler wait for exactly the loads issued
//     kD steps earlier.
//   * Cooperative flush: at step j the 32 lanes of half (j & 1) are owners; each pair of lanes writes
//     one owner's next complete 32-byte block (16 B per lane), so a store instruction touches 32
//     records, not 64 (lane-private 16-B stores to 64 records ran at 1.5 TB/s on MI355X, 4.2 TB/s for
//     64-B blocks of 16 records: scripts/mem_probe.hip).
//   * 13 KiB of LDS per wave: four-wave workgroups, three per CU = 3 waves per SIMD (the previous
//     20 KiB per wave gave 2, and PMC showed each wave issuing VALU in only half its cycles).
// k_snappy_global: records of lanes whose stream spans 2 GiB or more (32-bit positions) decode with
// byte loops straight to HBM, one thread per record.
// Files whose every record is a single literal (k_place sets ScanState::any_mixed otherwise) are
// copied by k_snappy_literal (rio_kernels.hip) and both kernels here exit at once.
#include <hip/hip_runtime.h>

#include "rio_device.h"
#include "rio_dev_util.h"

// experiment kept for A/B timing only (scripts/variants/build.sh): 8-byte pieces, dword-row LDS
namespace rio {
constexpr unsigned kSnappyWavesPerBlock = 4;
constexpr unsigned kSnappyWaves = 256 * 3 * kSnappyWavesPerBlock;
}

namespace rio {

namespace {
constexpr uint32_t kOR = 32;                         // output history: 32 dword rows = 128 B per lane
constexpr uint32_t kIR = 16;                         // input ring: 16 dword rows = 4 chunks of 16 B
constexpr uint32_t kInCh = kIR / 4;
constexpr uint32_t kInBase = kOR * 256;              // LDS byte offset of the input ring
constexpr uint32_t kDummy = kInBase + kIR * 256;     // 4 rows absorbing placeholder landings
constexpr uint32_t kWaveLds = kDummy + 4 * 256;      // 13 KiB per wave
constexpr uint32_t kD = 4;                           // steps between a load and its use
constexpr uint32_t kBlk = 32;                        // cooperative flush block (bytes)
constexpr uint32_t kFar = 112;                       // copies with a larger offset read the arena
constexpr uint32_t kNoChunk = ~0u;
constexpr uint32_t kLagMax = 39;                     // d - fb when a far load issues (see flush)
constexpr uint64_t kWideSpan = 1ull << 31;           // lane streams at least this long: k_snappy_global
// A far copy's 8 source bytes must be flushed when its load issues (after the step's flush): the
// parser leads the emitter by at most 8 (kD - 1) bytes and the flush lags it by at most kLagMax.
static_assert(kFar >= 8 * (kD - 1) + 8 + kLagMax, "far history must be flushed before the parser reads it");
// A ring copy reads [d - kFar, d - kFar + 8) at emit time; the previous step's three dword writes
// end at most 12 bytes past d, so the ring still holds every position >= d + 12 - 4 kOR.
static_assert(kFar + 12 <= 4 * kOR, "ring copies must stay inside the history ring");
static_assert(kOR * 256 == 8192 && kIR * 256 == 4096, "ring address masks below assume 8 KiB / 4 KiB rings");

// materialize x in a VGPR here: selects that use it can no longer be turned into branches that
// compute x on one side only (an empty asm with a register constraint; no instruction is emitted)
__device__ __forceinline__ void pin_v(uint32_t& x) { asm volatile("" : "+v"(x)); }

// v_perm_b32 selector of bytes k .. k + 3 of a {hi, lo} dword pair plus `base` (k <= 4): k * 0x01010101
// by a 24-bit multiply-add and a shift (v_mul_lo_u32 is a quarter-rate instruction)
__device__ __forceinline__ uint32_t bytes_sel(uint32_t k, uint32_t base) {
    return __umul24(k, 0x010101u) + base + (k << 24);
}

__device__ __forceinline__ uint32_t lds_ld(const uint8_t* L, uint32_t a) { return *reinterpret_cast<const uint32_t*>(L + a); }
__device__ __forceinline__ void lds_st(uint8_t* L, uint32_t a, uint32_t v) { *reinterpret_cast<uint32_t*>(L + a) = v; }

// byte offset (in the history ring) of the dword holding output position p, and the next row
__device__ __forceinline__ uint32_t out_row(uint32_t p, uint32_t lb) { return (((p >> 2) & (kOR - 1)) << 8) | lb; }
__device__ __forceinline__ uint32_t out_next(uint32_t a) { return (a + 256u) & 0x1FFFu; }
__device__ __forceinline__ uint32_t in_row(uint32_t p, uint32_t lb) { return (((p >> 2) & (kIR - 1)) << 8) | lb; }
__device__ __forceinline__ uint32_t in_next(uint32_t a) { return (a + 256u) & 0xFFFu; }

// 16-byte global load bypassing the per-CU L1 (nt): far history is read back from the arena the same
// wave stores to, and a line cached before all of its bytes were flushed must not serve a later read
__device__ __forceinline__ uint4 ld_aux(const uint8_t* p) { return ldu16_nt(p); }

// one pipeline slot: a parsed piece plus the two loads issued with it
struct Slot {
    uint4 in;       // input chunk in_c (load in flight; sink bytes when in_c == kNoChunk)
    uint4 aux;      // far-copy bytes (.x .y) or the next record's descriptor (load in flight)
    uint2 lit;      // literal bytes
    uint32_t in_c;  // chunk index of `in`
    uint32_t q;     // source output position (ring / far copy)
    uint32_t m;     // n | kind << 8 | desc << 16; n = piece length (0 = bubble), kind 0 literal,
                    // 1 ring copy, 2 far copy; desc: aux carries the next record's descriptor
};
__device__ __forceinline__ Slot empty_slot() {
    Slot S;
    S.in = zero4();
    S.aux = zero4();
    S.lit = make_uint2(0, 0);
    S.in_c = kNoChunk;
    S.q = 0;
    S.m = 1u << 8;
    return S;
}

// Records [r0, r1) of lane t (T lanes): one record per lane while there are fewer records than lanes
// (packed into the first waves), else balanced contiguous ranges.
__device__ __forceinline__ void lane_range(uint64_t n, uint64_t T, uint64_t t, uint64_t& r0, uint64_t& r1) {
    if (n <= T) {
        r0 = min(t, n);
        r1 = min(t + 1, n);
    } else {
        r0 = t * n / T;
        r1 = (t + 1) * n / T;
    }
}

// The byte ranges a wave's records [r0, r1) occupy in the file (16-B aligned start) and the arena.
struct WaveSpan {
    uint64_t in0, in1, out0, out1;
};
__device__ __forceinline__ WaveSpan wave_span(const FrameParams& P, uint64_t r0, uint64_t r1) {
    WaveSpan w;
    w.in0 = (P.rec_off[r0] + (P.rec_pay[r0] & 0xFF)) & ~15ull;  // 64-bit sizes: rec_desc has 32-bit ones
    w.in1 = P.rec_off[r1 - 1] + (P.rec_pay[r1 - 1] & 0xFF) + (P.rec_pay[r1 - 1] >> 8);
    w.out0 = P.out_off[r0];
    w.out1 = P.out_off[r1];
    return w;
}
// a wave streams its lanes' records with 32-bit buffer offsets: spans of 2 GiB or more (a record of a
// few GiB) go to k_snappy_global instead
__device__ __forceinline__ bool wave_wide(const WaveSpan& w) {
    return w.in1 + RIO_DEVICE_PAD - w.in0 >= kWideSpan || w.out1 - w.out0 >= kWideSpan;
}

// Buffer descriptors (raw, stride 0): an access whose offset lies past num_records is dropped by the
// address unit (loads return zeros) without a memory request. Lanes with nothing to load or store
// use kOob, so a wave instruction costs only its active lanes' requests.
constexpr uint32_t kOob = 0x80000000u;
constexpr int kNt = 2;  // cache policy: non-temporal (loads bypass the CU's L1)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint64_t bytes) {
    // inputs made provably wave-uniform (T20: no waterfall loops around the buffer ops)
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const uint32_t n = __builtin_amdgcn_readfirstlane((uint32_t)bytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}
template <int kAux = 0>
__device__ __forceinline__ uint4 buf_ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    const v4 v = __builtin_bit_cast(v4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAux));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void buf_st16(__amdgpu_buffer_rsrc_t r, uint32_t off, uint4 v) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    const v4 w = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(w, r, off, 0, 0);
}
}  // namespace

// Decode the contiguous record range [r0, r1) of this lane as ONE stream: consecutive records are
// contiguous in the output arena and separated only by their headers in the file, so the pipeline
// never drains between records. Positions are relative to the lane's aligned input base and to its
// output base out_off[r0]; copy offsets stay record-relative (golang/snappy bounds per record). The
// next record's descriptor travels in the far-load slot of a step without a far copy. The loop runs
// until every lane of the wave is done: finished lanes keep stepping as bubbles and as flush helpers.
// Returns false with *bad_rec = the failing record if a record does not decode.
__device__ __forceinline__ bool snappy_lane(const FrameParams& P, uint64_t r0, uint64_t r1, uint8_t* L, uint32_t lane,
                                            const WaveSpan& W, uint64_t r0w, uint64_t* bad_rec) {
    const uint32_t lb = lane * 4;
    const bool live = r0 < r1;
    const uint32_t nk = (uint32_t)(r1 - r0);
    // the wave's input, arena and descriptor ranges as buffers (32-bit lane offsets below)
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(P.file + W.in0, W.in1 + RIO_DEVICE_PAD - W.in0);
    const __amdgpu_buffer_rsrc_t rout = make_rsrc(P.out + W.out0, W.out1 - W.out0);
    const __amdgpu_buffer_rsrc_t rdesc = make_rsrc(P.rec_desc + r0w, (uint64_t)(P.rec_cap + 1 - r0w) * 16);
    const uint4 d0 = live ? P.rec_desc[r0] : zero4();
    const uint64_t o0 = live ? P.out_off[r0] : W.out0;
    const uint32_t lo = (uint32_t)(o0 - W.out0);  // lane output base in rout
    const uint64_t start0 = live ? ((uint64_t)d0.y << 32) | d0.x : W.in0;
    const uint64_t base = start0 & ~15ull;  // lane input base (file offset, 16-B aligned)
    const uint32_t base_lo = (uint32_t)base;
    const uint32_t li = (uint32_t)(base - W.in0);  // lane input base in rin
    // chunks the prefetcher may read: up to the file end (+pad)
    const uint32_t lastc = live && base < P.len ? (uint32_t)min((P.len - 1 - base) >> 4, (uint64_t)0x0FFFFFFF) : 0u;
    // prime the input ring with chunks [0, 4)
    uint32_t whi = live ? min(kInCh, lastc + 1) : 0u;  // chunks [0, whi) have landed
#pragma unroll
    for (uint32_t c = 0; c < kInCh; c++) {
        const uint4 v = buf_ld16(rin, c < whi ? li + 16 * c : kOob);
        const uint32_t a = kInBase + ((c << 10) | lb);
        lds_st(L, a, v.x);
        lds_st(L, a + 256, v.y);
        lds_st(L, a + 512, v.z);
        lds_st(L, a + 768, v.w);
    }
    uint32_t cn = live ? whi : 0xFFFFFFFFu;  // next chunk to load (never for an idle lane)

    // record state: record r0 + kk, its input [s, s_end) and output [rd_start, rd_end)
    uint32_t kk = 0;
    uint32_t s = (uint32_t)(start0 - base), s_end = s + d0.z;
    uint32_t pd = 0, rd_start = 0, rd_end = d0.w;
    uint32_t rem = 0, eff = 0;
    bool islit = false, bad = false, pdone = !live;
    // next record's descriptor: 0 needed, 1 in flight (ndl), 2 landed, 3 none (last record)
    uint4 nd = zero4(), ndl = zero4();
    uint32_t nds = (live && nk > 1) ? 0u : 3u;
    const uint32_t kd0 = (uint32_t)(r0 - r0w) + 1;  // descriptor index of record r0 + 1 in rdesc
    // emitter: d = bytes emitted, fb = bytes flushed (multiple of kBlk), stage = the dword holding d
    uint32_t d = 0, fb = 0, stage = 0;

    // output base of the owner each lane flushes for at steps of parity h (owner 32 h + lane / 2)
    uint32_t obase[2];
#pragma unroll
    for (uint32_t h = 0; h < 2; h++)
        obase[h] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((32u * h + (lane >> 1)) * 4), (int)lo);

    Slot S0 = empty_slot(), S1 = empty_slot(), S2 = empty_slot(), S3 = empty_slot();
    uint32_t drain = 0;

    auto step = [&](Slot& S, const uint32_t j) __attribute__((always_inline)) {
        drain += pdone ? 1u : 0u;
        // 1. land the input chunk loaded kD steps ago, and the next record's descriptor
        {
            // branch-free: a slot without a chunk writes its placeholder bytes to the dummy rows
            const bool landed = S.in_c != kNoChunk;
            const uint32_t a = landed ? kInBase + (((S.in_c & (kInCh - 1)) << 10) | lb) : kDummy + lb;
            lds_st(L, a, S.in.x);
            lds_st(L, a + 256, S.in.y);
            lds_st(L, a + 512, S.in.z);
            lds_st(L, a + 768, S.in.w);
            whi = landed ? S.in_c + 1 : whi;
        }
        // the next record's descriptor: one load per kD steps (step 0), landed kD steps later
        if (j == 0) {
            const bool dl = nds == 1;
            nd = make_uint4(dl ? ndl.x : nd.x, dl ? ndl.y : nd.y, dl ? ndl.z : nd.z, dl ? ndl.w : nd.w);
            nds = dl ? 2u : nds;
            const bool want = nds == 0;
            ndl = buf_ld16(rdesc, want ? (kd0 + kk) * 16 : kOob);
            nds = want ? 1u : nds;
        }

        // 2. emit the piece parsed kD steps ago at output position d (a bubble appends nothing)
        {
            const uint32_t n = S.m & 0xFFu, kind = (S.m >> 8) & 3u;
            const uint32_t qa0 = out_row(S.q, lb), qa1 = out_next(qa0), qa2 = out_next(qa1);
            const uint32_t h0 = lds_ld(L, qa0), h1 = lds_ld(L, qa1), h2 = lds_ld(L, qa2);
            const uint32_t rq = S.q & 3u;
            uint32_t hx = __builtin_amdgcn_alignbyte(h1, h0, rq), hy = __builtin_amdgcn_alignbyte(h2, h1, rq);
            pin_v(hx);
            pin_v(hy);
            const bool ring = kind == 1, litk = kind == 0;
            const uint32_t vx = ring ? hx : (litk ? S.lit.x : S.aux.x);
            const uint32_t vy = ring ? hy : (litk ? S.lit.y : S.aux.y);
            // place the 8 bytes at d: dwords d/4 .. d/4 + 2 (bytes past d + n are overwritten later)
            const uint32_t r = d & 3u, r8 = r * 8u;
            const uint32_t w0 = __builtin_amdgcn_ubfe(stage, 0, r8) | (vx << r8);
            uint32_t w1a = __builtin_amdgcn_alignbyte(vy, vx, 0u - r);  // bytes 4 - r .. 7 - r (r > 0)
            pin_v(w1a);
            const uint32_t w1 = r == 0 ? vy : w1a;
            const uint32_t w2 = __builtin_amdgcn_ubfe(vy, 32u - r8, r8);
            const uint32_t da0 = out_row(d, lb), da1 = out_next(da0), da2 = out_next(da1);
            lds_st(L, da0, w0);
            lds_st(L, da1, w1);
            lds_st(L, da2, w2);
            const uint32_t e = r + n;
            stage = e >= 8 ? w2 : (e >= 4 ? w1 : w0);
            d += n;
        }

        // 3. cooperative flush: the lane pair (2i, 2i + 1) writes owner 32 h + i's next 32-byte
        //    block if complete. Between two checks of an owner d grows <= 16, so d - fb <= 47 at a
        //    check and <= 39 after any step's flush (kLagMax).
        {
            const uint32_t h = j & 1u;
            const uint32_t o = 32u * h + (lane >> 1), part = lane & 1u;
            const bool ready = d - fb >= kBlk;
            const uint32_t ofb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(o * 4), (int)(fb | (ready ? 0x80000000u : 0u)));
            const uint32_t pos = (ofb & 0x7FFFFFFFu) + 16u * part;
            const uint32_t fa = out_row(pos, o * 4);  // rows of pos .. pos + 15: 4-row aligned, no wrap
            const uint4 fv = make_uint4(lds_ld(L, fa), lds_ld(L, fa + 256), lds_ld(L, fa + 512), lds_ld(L, fa + 768));
            buf_st16(rout, (ofb >> 31) ? obase[h] + pos : kOob, fv);
            fb += ((lane >> 5) == h && ready) ? kBlk : 0u;
        }

        // 4. parse the next piece into this slot (selects only: lanes diverge in data, not flow)
        uint32_t kind;
        {
            const uint32_t ia0 = in_row(s, lb), ia1 = in_next(ia0), ia2 = in_next(ia1);
            const uint32_t w0 = lds_ld(L, kInBase + ia0), w1 = lds_ld(L, kInBase + ia1), w2 = lds_ld(L, kInBase + ia2);
            const uint32_t r = s & 3u;
            const bool avail = min((s + 11u) >> 4, lastc) < whi;  // window bytes [s, s + 12) landed
            // element header at s (decode_other.go): tag and the four bytes after it
            const uint32_t tag = __builtin_amdgcn_alignbyte(w1, w0, r) & 0xFFu;
            const uint32_t W1 = __builtin_amdgcn_perm(w1, w0, bytes_sel(r, 0x04030201u));
            const uint32_t t = tag & 3u, x = tag >> 2;
            const bool lit = t == 0, lng = x >= 60;
            // value bytes after the tag: literal 60..63 -> 1..4 length bytes, copy-1/2/4 -> 1/2/4.
            // Every alternative is computed and pinned, then selected: the compiler otherwise turns
            // the nested ternaries into exec-mask branches.
            uint32_t nb_lit = lng ? x - 59u : 0u, nb_cp = t == 3 ? 4u : t;
            pin_v(nb_lit);
            pin_v(nb_cp);
            const uint32_t nb = lit ? nb_lit : nb_cp;
            uint32_t val_part = __builtin_amdgcn_ubfe(W1, 0, 8u * nb);  // nb < 4 (width 32 reads as 0)
            pin_v(val_part);
            const uint32_t val = nb >= 4 ? W1 : val_part;
            const uint32_t hl = nb + 1u;
            uint32_t len_lit = lng ? val + 1u : x + 1u, len_c1 = (x & 7u) + 4u, len_cx = x + 1u;
            pin_v(len_lit);
            pin_v(len_c1);
            const uint32_t len = lit ? len_lit : (t == 1 ? len_c1 : len_cx);
            uint32_t off_c1 = val | ((tag >> 5) << 8);
            pin_v(off_c1);
            const uint32_t off = t == 1 ? off_c1 : val;
            // golang/snappy bounds, per record: header bytes present; literal source room or copy
            // offset in [1, bytes produced] (length / offset 0 wrap to the maximum key); output room
            const uint32_t sleft = s_end - s;
            const uint32_t lim = lit ? sleft - hl : pd - rd_start;
            const uint32_t key = (lit ? len : off) - 1u;
            const bool hbad = (hl > sleft) | (key >= lim) | (len > rd_end - pd);
            const bool hdr = !pdone && rem == 0 && s < s_end && avail;
            const bool badn = hdr && hbad, ok = hdr && !hbad;
            bad = bad || badn;
            pdone = pdone || badn;
            const uint32_t sh = ok ? hl : 0u;
            const uint32_t rem1 = ok ? len : rem, eff1 = ok ? off : eff;
            const bool lit1 = ok ? lit : islit;
            // literal bytes: 8 window bytes from u = r + sh (u <= 8; bytes past the window's 12 are
            // never used: the piece is capped at 12 - u)
            const uint32_t u = r + sh;
            const bool hw = u > 4;
            uint32_t u4 = u - 4u;
            pin_v(u4);
            const uint32_t psel = bytes_sel(hw ? u4 : u, 0x03020100u);
            const uint32_t plo = hw ? w1 : w0, phi = hw ? w2 : w1;
            S.lit = make_uint2(__builtin_amdgcn_perm(phi, plo, psel), __builtin_amdgcn_perm(w2, phi, psel));
            // a literal piece takes window bytes; a copy piece reaches back at most `eff` bytes
            // (overlapping copies double their reach: a multiple of the offset)
            const bool go = !pdone && rem1 != 0 && (!lit1 || avail);
            const uint32_t cap = lit1 ? min(8u, 12u - u) : min(8u, eff1);
            const uint32_t n = go ? min(rem1, cap) : 0u;
            kind = n == 0 ? 1u : (lit1 ? 0u : (eff1 > kFar ? 2u : 1u));
            S.q = pd - eff1;
            s += sh + (lit1 ? n : 0u);
            rem = rem1 - n;
            pd += n;
            eff = (!lit1 && eff1 < 8u && n == eff1) ? 2u * eff1 : eff1;
            islit = lit1;
            S.m = n | (kind << 8);
            // record boundary: stream consumed -> the record must be complete (snappy: d !=
            // len(dst) => ErrCorrupt); switch to the next record (its descriptor landed) or finish
            {
                const bool at_end = !pdone && rem == 0 && s == s_end;
                const bool bad_len = at_end && pd != rd_end;
                const bool more = kk + 1 < nk;
                bad = bad || bad_len;
                pdone = pdone || bad_len || (at_end && !more);
                const bool sw = at_end && !bad_len && more && nds == 2;
                kk += sw ? 1u : 0u;
                const uint32_t ns = nd.x - base_lo;  // the lane span is < 2^31: 32-bit difference
                s = sw ? ns : s;
                s_end = sw ? ns + nd.z : s_end;
                rd_start = sw ? pd : rd_start;
                rd_end = sw ? pd + nd.w : rd_end;
                nds = sw ? (kk + 1 < nk ? 0u : 3u) : nds;
            }
        }
        // far history (flushed: see the static_asserts)
        S.aux = buf_ld16<kNt>(rout, kind == 2 ? lo + S.q : kOob);
        // 5. input prefetch: the next chunk if the ring has room for it when it lands
        {
            const bool take = cn <= lastc && cn < (s >> 4) + kInCh;
#ifdef RIO_IN_NT
            S.in = buf_ld16<kNt>(rin, take ? li + 16 * cn : kOob);
#else
            S.in = buf_ld16(rin, take ? li + 16 * cn : kOob);
#endif
            S.in_c = take ? cn : kNoChunk;
            cn += take ? 1u : 0u;
        }
    };

    // one exit per kD steps, taken by the whole wave: every path around the loop issues the same
    // memory operations, so the compiler's wait counts stay exact
    static_assert(kD == 4, "unrolled for four slots");
    do {
        step(S0, 0);
        step(S1, 1);
        step(S2, 2);
        step(S3, 3);
    } while (__any(drain < kD));
    // the stream's tail (< 48 bytes), lane by lane; written even after a failure: the bytes of the
    // records before the failing one must be complete
    uint8_t* const gout = P.out + o0;
    for (uint32_t q = fb; q < d; q += 16) {
        const uint32_t fa = out_row(q, lb);
        const uint4 v = make_uint4(lds_ld(L, fa), lds_ld(L, fa + 256), lds_ld(L, fa + 512), lds_ld(L, fa + 768));
        if (q + 16 <= d)
            stu16(gout + q, v);
        else
            st_partial(gout + q, v, d - q);
    }
    *bad_rec = r0 + kk;
    return !bad;
}

// Waves whose records span 2 GiB of input or output leave them to k_snappy_global.
__global__ void __launch_bounds__(64 * kSnappyWavesPerBlock) k_snappy_lane(FrameParams P) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kSnappyWavesPerBlock * kWaveLds];
    ScanState* st = P.state;
    if (st->hdr_status != RIO_OK || st->capacity_fail || st->compression != RIO_COMP_SNAPPY) return;
    if (!st->any_mixed) return;  // every record is one literal: k_snappy_literal copies them
    const uint64_t n = st->n_records;
    const uint32_t lane = threadIdx.x & 63u, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t T = (uint64_t)kSnappyWaves * 64;
    const uint64_t wave = (uint64_t)wv * gridDim.x + blockIdx.x;  // consecutive waves on different CUs
    uint64_t r0w, r1w, x;
    lane_range(n, T, wave * 64, r0w, x);
    lane_range(n, T, wave * 64 + 63, x, r1w);
    if (r0w >= n) return;  // the whole wave is idle
    const WaveSpan W = wave_span(P, r0w, r1w);
    if (wave_wide(W)) {
        atomicOr(&st->huge_streams, 1u);  // k_snappy_global decodes this wave's records
        return;
    }
    uint64_t r0, r1;
    lane_range(n, T, wave * 64 + lane, r0, r1);
    uint64_t bad_rec = 0;
    if (!snappy_lane(P, r0, r1, lds + wv * kWaveLds, lane, W, r0w, &bad_rec))
        atomicMin((unsigned long long*)&st->decode_err_rec, (unsigned long long)(2 * bad_rec));
}

// Records of waves whose streams span 2 GiB or more: every record decoded by one thread with byte
// loops straight to HBM (the same wave assignment as k_snappy_lane decides which).
__global__ void __launch_bounds__(256) k_snappy_global(FrameParams P) {
    ScanState* st = P.state;
    if (st->hdr_status != RIO_OK || st->capacity_fail || st->compression != RIO_COMP_SNAPPY || !st->huge_streams ||
        !st->any_mixed)
        return;
    const uint64_t n = st->n_records;
    const uint64_t T = (uint64_t)kSnappyWaves * 64;
    for (uint64_t w = blockIdx.x; w < kSnappyWaves; w += gridDim.x) {
        uint64_t r0w, r1w, x;
        lane_range(n, T, w * 64, r0w, x);
        lane_range(n, T, w * 64 + 63, x, r1w);
        if (r0w >= n || !wave_wide(wave_span(P, r0w, r1w))) continue;
        for (uint64_t i = r0w + threadIdx.x; i < r1w; i += blockDim.x) {
            if (P.flags[i] & RIO_FLAG_NIL) continue;
            const uint64_t pay = P.rec_pay[i], slen = pay >> 8;
            const uint64_t o0 = P.out_off[i], o1 = P.out_off[i + 1];
            if (!snappy_decode_thread(P.file + P.rec_off[i] + (pay & 0xFF), slen, P.out + o0, o1 - o0))
                atomicMin((unsigned long long*)&st->decode_err_rec, (unsigned long long)(2 * i));
        }
    }
}

hipError_t launch_snappy_decode(const FrameParams& P, hipStream_t s) {
    hipLaunchKernelGGL(k_snappy_lane, dim3(kSnappyWaves / kSnappyWavesPerBlock), dim3(64 * kSnappyWavesPerBlock), 0, s, P);
    hipLaunchKernelGGL(k_snappy_global, dim3(64), dim3(256), 0, s, P);
    return hipGetLastError();
}

}  // namespace rio
