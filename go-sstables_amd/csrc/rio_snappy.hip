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
//   * History: the last 256 decoded bytes of each record live in an LDS ring; copies reaching
//     further back (offset > kFarOff) are loaded from the output arena at PARSE time, kD
//     iterations before use — the flush schedule guarantees those bytes were stored already
//     (flush lag < 32 bytes, parser lead <= 16*(kD-1) bytes, kFarOff >= 16*kD + 32).
//   * Input: aligned 16-byte chunks loaded kD iterations ahead land in a 64-byte LDS ring.
//   * LDS image per wave is chunk-interleaved ([chunk][lane][16 B]): every 16-byte access by a
//     wave touches each bank once, whatever positions the lanes are at.
// k_snappy_global: records whose compressed stream exceeds 32-bit positions (never produced by a
// real encoder) decode with byte loops straight to HBM.
#include <hip/hip_runtime.h>

#include "rio_device.h"
#include "rio_dev_util.h"

namespace rio {

namespace {
constexpr uint32_t kOutCh = 16;                  // history ring: 16 chunks = 256 bytes per lane
constexpr uint32_t kInCh = 4;                    // input ring: 4 chunks = 64 bytes per lane
constexpr uint32_t kWaveLds = (kOutCh + kInCh) * 64 * 16;  // 20 KiB per wave
constexpr uint32_t kFarOff = kOutCh * 16 - 48;   // copies reaching further back read HBM
constexpr uint32_t kD = 3;                       // pipeline depth in iterations
constexpr uint32_t kNoChunk = ~0u;               // slot carries no input chunk
static_assert(kFarOff >= 16 * kD + 32, "far history must be flushed before the parser reads it");
static_assert(kSnappyBlock % 64 == 0, "whole waves");

// per-lane view of the wave's chunk-interleaved LDS image
struct LaneLds {
    uint8_t* p;  // wave image + lane * 16
    __device__ uint4* out(uint32_t pos) const { return reinterpret_cast<uint4*>(p + ((pos >> 4) & (kOutCh - 1)) * 1024); }
    __device__ uint4* in(uint32_t c) const { return reinterpret_cast<uint4*>(p + (kOutCh + (c & (kInCh - 1))) * 1024); }
    // 16 bytes of history at output position q
    __device__ uint4 out16(uint32_t q) const {
        const uint32_t r = q & 15u;
        const uint4 x0 = *out(q), x1 = *out(q + 16);
        return or4(shr_bytes(x0, r), shl_bytes(x1, 16 - r));
    }
    // 16 bytes of input at aligned-frame position pos
    __device__ uint4 in16(uint32_t pos) const {
        const uint32_t r = pos & 15u, c = pos >> 4;
        const uint4 x0 = *in(c), x1 = *in(c + 1);
        return or4(shr_bytes(x0, r), shl_bytes(x1, 16 - r));
    }
};

// one pipeline slot: a parsed piece plus the two loads issued with it
struct Slot {
    uint4 in;       // input chunk in_c (load in flight; sink bytes when in_c == kNoChunk)
    uint4 far;      // far-history bytes (load in flight; placeholder unless kind == 2)
    uint4 lit;      // literal bytes (kind == 0)
    uint32_t in_c;  // chunk index of `in`
    uint32_t n;     // piece length, 0 = bubble
    uint32_t q;     // source output position (kind 1)
    uint32_t kind;  // 0 literal, 1 ring copy, 2 far copy
};
}  // namespace

// Decode one record. src: element stream (after the length preamble) of slen bytes; the decoded
// length dlen was validated against the preamble by framing.
__device__ bool snappy_pipe(const uint8_t* src, uint32_t slen, const LaneLds& L, uint8_t* gout, uint32_t dlen,
                            uint8_t* sink) {
    if (slen == 0) return dlen == 0;
    const uint32_t so = (uint32_t)((uintptr_t)src & 15u);
    const uint4* sa = reinterpret_cast<const uint4*>(src - so);
    const uint32_t lastc = (so + slen - 1) >> 4;  // last input chunk holding stream bytes
    // prime the input ring with chunks [0, 4)
    uint32_t whi = min(kInCh, lastc + 1);  // chunks [0, whi) have landed in LDS
    for (uint32_t c = 0; c < whi; c++) *L.in(c) = sa[c];
    uint32_t cn = whi;  // next chunk to load

    // parser state
    uint32_t s = 0, pd = 0, rem = 0, eff = 0;
    bool islit = false, pdone = false, bad = false;
    // emitter state
    uint32_t d = 0, fl = 0;
    uint4 stage = zero4();

    Slot S0, S1, S2;
    {
        const uint4 c0 = sa[0];
        for (Slot* S : {&S0, &S1, &S2}) {
            S->in = c0;
            S->in_c = kNoChunk;
            S->far = zero4();
            S->lit = zero4();
            S->n = 0;
            S->q = 0;
            S->kind = 0;
        }
    }
    uint32_t drain = 0;

    auto step = [&](Slot& S) {
        // 1. land the input chunk loaded kD iterations ago
        if (S.in_c != kNoChunk) {
            *L.in(S.in_c) = S.in;
            whi = S.in_c + 1;
        }

        // 2. emit the piece parsed kD iterations ago (a bubble appends nothing)
        {
            uint4 v = L.out16(S.q);
            v = make_uint4(S.kind == 2 ? S.far.x : v.x, S.kind == 2 ? S.far.y : v.y, S.kind == 2 ? S.far.z : v.z,
                           S.kind == 2 ? S.far.w : v.w);
            v = make_uint4(S.kind == 0 ? S.lit.x : v.x, S.kind == 0 ? S.lit.y : v.y, S.kind == 0 ? S.lit.z : v.z,
                           S.kind == 0 ? S.lit.w : v.w);
            const uint32_t n = S.n, r = d & 15u;
            v = keep_bytes(v, n);
            const uint4 lo = or4(stage, shl_bytes(v, r));
            const uint4 hi = shr_bytes(v, 16 - r);
            *L.out(d) = lo;       // chunk holding d: staged head + new bytes
            *L.out(d + 16) = hi;  // next chunk: only bytes not yet final
            const bool roll = r + n >= 16;
            stage = make_uint4(roll ? hi.x : lo.x, roll ? hi.y : lo.y, roll ? hi.z : lo.z, roll ? hi.w : lo.w);
            d += n;
        }

        // 3. flush one completed 16-byte chunk (placeholder: the sink line)
        {
            const bool full = fl + 16 <= d;
            const uint4 fv = *L.out(fl);
            stu16(full ? gout + fl : sink, fv);
            fl += full ? 16u : 0u;
        }

        // 4. parse the next piece into this slot
        uint32_t n = 0, q = 0, kind = 0;
        uint4 lit = zero4();
        if (!pdone) {
            if (rem == 0) {  // element header: bytes s .. s+4 must have landed
                const uint32_t pos = so + s;
                if (min((pos + 4) >> 4, lastc) < whi) {
                    const uint4 W = L.in16(pos);
                    const uint32_t tag = W.x & 0xFF, t = tag & 3, x = tag >> 2;
                    const uint64_t w64 = ((uint64_t)W.y << 32) | W.x;
                    const uint32_t lit_hl = x < 60 ? 1u : x - 58u;
                    const uint32_t ext = (uint32_t)((w64 >> 8) & ((1ull << ((8 * (lit_hl - 1)) & 63)) - 1));
                    const uint32_t len = t == 0 ? (x < 60 ? x : ext) + 1 : (t == 1 ? 4 + (x & 7) : x + 1);
                    const uint32_t hl = t == 0 ? lit_hl : (t == 1 ? 2u : (t == 2 ? 3u : 5u));
                    const uint32_t o1 = ((tag & 0xE0u) << 3) | ((W.x >> 8) & 0xFF);
                    const uint32_t o2 = (W.x >> 8) & 0xFFFF;
                    const uint32_t o4 = (W.x >> 8) | (W.y << 24);
                    const uint32_t off = t == 1 ? o1 : (t == 2 ? o2 : o4);
                    islit = t == 0;
                    // golang/snappy bounds: header bytes, literal source, copy offset, output room
                    bad = hl > slen - s || len > dlen - pd ||
                          (islit ? (len == 0 || len > slen - s - hl) : (off == 0 || off > pd));
                    if (bad) {
                        pdone = true;
                    } else {
                        s += hl;
                        rem = len;
                        eff = off;
                    }
                }
            }
            if (rem != 0) {
                if (islit) {  // literal piece: its bytes must have landed
                    const uint32_t pos = so + s;
                    if (min((pos + 15) >> 4, lastc) < whi) {
                        n = min(rem, 16u);
                        lit = L.in16(pos);
                        s += n;
                    }
                } else {  // copy piece; overlapping copies double their reach (a multiple of the offset)
                    n = min(min(rem, 16u), eff);
                    q = pd - eff;
                    kind = eff > kFarOff ? 2u : 1u;
                    eff = (eff < 16 && n == eff) ? 2 * eff : eff;
                }
                rem -= n;
                pd += n;
            }
            if (rem == 0 && s >= slen) pdone = true;
        }
        S.n = n;
        S.q = q;
        S.kind = kind;
        S.lit = lit;
        // far history (flushed: see header) or a placeholder load
        S.far = ldu16(kind == 2 ? gout + q : sink);

        // 5. input prefetch: the next chunk if the ring has room for it when it lands
        {
            const uint32_t a = (so + s) >> 4;
            const bool take = cn <= lastc && cn < a + kInCh;
            S.in = *reinterpret_cast<const uint4*>(take ? reinterpret_cast<const uint8_t*>(sa + cn) : sink);
            S.in_c = take ? cn : kNoChunk;
            cn += take ? 1u : 0u;
        }
    };

    // one exit per kD steps: every path around the loop issues the same memory operations, so the
    // compiler's wait counts stay exact (extra steps after the drain only emit bubbles)
    static_assert(kD == 3, "unrolled for three slots");
    do {
        drain += pdone ? 1u : 0u;
        step(S0);
        drain += pdone ? 1u : 0u;
        step(S1);
        drain += pdone ? 1u : 0u;
        step(S2);
    } while (drain < kD);
    if (bad || d != dlen || pd != dlen) return false;
    for (uint32_t k = fl; k < d; k += 16) {
        const uint4 v = *L.out(k);
        if (k + 16 <= d)
            stu16(gout + k, v);
        else
            st_partial(gout + k, v, d - k);
    }
    return true;
}

__global__ void __launch_bounds__(kSnappyBlock) k_snappy_pipe(FrameParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    ScanState* st = P.state;
    if (st->hdr_status != RIO_OK || st->capacity_fail || st->compression != RIO_COMP_SNAPPY) return;
    const uint64_t n = st->n_records;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const LaneLds L{lds + wave * kWaveLds + lane * 16};
    const uint64_t gtid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint8_t* sink = P.sink + (gtid >> 6) * 64;  // the wave's placeholder line
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = gtid; i < n; i += stride) {
        if (P.flags[i] & RIO_FLAG_NIL) continue;
        const uint64_t pay = P.rec_pay[i], slen = pay >> 8;
        if (slen > 0xFFFFFFFFull) continue;  // k_snappy_global
        const uint64_t o0 = P.out_off[i], olen = P.out_off[i + 1] - o0;
        const uint8_t* src = P.file + P.rec_off[i] + (pay & 0xFF);
        if (!snappy_pipe(src, (uint32_t)slen, L, P.out + o0, (uint32_t)olen, sink))
            atomicMin((unsigned long long*)&st->decode_err_rec, (unsigned long long)i);
    }
}

__global__ void __launch_bounds__(256) k_snappy_global(FrameParams P) {
    ScanState* st = P.state;
    if (st->hdr_status != RIO_OK || st->capacity_fail || st->compression != RIO_COMP_SNAPPY) return;
    const uint64_t n = st->n_records;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (P.flags[i] & RIO_FLAG_NIL) continue;
        const uint64_t pay = P.rec_pay[i], slen = pay >> 8;
        if (slen <= 0xFFFFFFFFull) continue;  // k_snappy_pipe
        const uint64_t o0 = P.out_off[i], o1 = P.out_off[i + 1];
        if (!snappy_decode_thread(P.file + P.rec_off[i] + (pay & 0xFF), slen, P.out + o0, o1 - o0))
            atomicMin((unsigned long long*)&st->decode_err_rec, (unsigned long long)i);
    }
}

hipError_t launch_snappy_decode(const FrameParams& P, hipStream_t s) {
    // 4 waves x 20 KiB = 80 KiB per workgroup: 2 workgroups (8 waves) per CU
    hipLaunchKernelGGL(k_snappy_pipe, dim3(kSnappyGrid), dim3(kSnappyBlock), (kSnappyBlock / 64) * kWaveLds, s, P);
    hipLaunchKernelGGL(k_snappy_global, dim3(64), dim3(256), 0, s, P);
    return hipGetLastError();
}

}  // namespace rio
