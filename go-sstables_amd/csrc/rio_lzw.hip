// rio_lzw.hip — LZW-compressed records decoded on the device (LzwCompressor.DecompressWithBuf,
// recordio/compressor/lzw_compressor.go:52-63: Go compress/lzw reader, LSB bit order, litWidth 8,
// called per record by FileReader.ReadNext, file_reader.go:115-125).
//
// Go's reader (restated in oracle/rio_oracle.c, orc_lzw_decode): codes of 9..12 bits, LSB first;
// 256 = clear (width 9, hi 257, no previous code), 257 = eof (the record ends; bytes after it are
// ignored); a code above hi is "lzw: invalid code"; running out of bytes before eof is
// io.ErrUnexpectedEOF. Both failures are the codec-error class (RIO_FLAG_CORRUPT).
// Counting code k of an epoch from the last clear (or the stream start), hi before code k is
// min(257 + k, 4095) and the width grows after codes 254 / 766 / 1790, so the width and the bit
// position of code k are closed-form in k. Code k >= 1 (k <= 3838) defines entry 257 + k = code k - 1's
// output followed by the first byte of code k's output, i.e. |S_{k-1}| + 1 output bytes starting where
// S_{k-1} starts. Decoding is therefore LZ77 over the record's own output:
//   code < 256  -> one literal byte;
//   code c >= 258 -> len[c - 258] + 1 bytes copied from output position pos[c - 258] (overlapping the
//                  destination by one byte when c is the entry being defined: Go's "code == hi").
//
// k_lzw_decode: one wave per record, grid-stride. Rounds of 64 codes: lane l reads code k0 + l at its
// closed-form bit position; the first clear / eof / invalid / missing code ends the round's valid
// prefix; code lengths resolve by pointer jumping over the lanes (a length depends on an earlier
// code's), positions by a wave prefix sum, and (pos, len) of every code of the epoch stay in LDS for
// the later rounds. The round's output is then materialised in 64-byte windows with lane = byte: the
// byte's code from a prefix-max over "code starts here" marks, then a literal, or a copy source that
// is either an earlier byte of the same window (resolved through the lanes) or an earlier window's
// byte read back from the output arena after the wave's stores have drained (L1-bypassing loads).
// Sizes: the framing sized each record by its header's u (the reference's buffer size, equal to the
// decoded length for every file its writer produces). A record whose output differs is not stored: it
// is marked for k_lzw_resize, which counts it, and the scan, placement and this decoder run again with
// the counted sizes (the gzip redo round of rio_kernels.hip).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "rio_device.h"
#include "rio_dev_util.h"

namespace rio {

namespace {
constexpr uint32_t kLzMaxK = 3840;             // codes of an epoch a later code may reference (258 + k <= 4095)
// size classes: a record of slen payload bytes holds at most 8 slen / 9 codes, so records up to
// kLzSmallLen bytes never index past kLzSmallK codes and take a table of 6 KiB (25 waves per CU
// instead of 6)
constexpr uint32_t kLzSmallK = 1024, kLzSmallLen = kLzSmallK * 9 / 8;
constexpr uint32_t kLzSmallGrid = 256 * 32;
constexpr uint64_t kLzResize = 1ull << 62;     // rec_pay marker: output size differs from the framing's
constexpr uint64_t kLzLen = ~(3ull << 62);
constexpr uint32_t kLzGrid = 1536;             // one-wave workgroups: 23 KiB of LDS each, 6 per CU
enum : uint32_t { kLit = 0, kCopy = 1, kClear = 2, kEnd = 3, kBad = 4, kMissing = 5 };
enum : int { kLzOk = 0, kLzResize_ = 1, kLzCorrupt = 2, kLzUnsupported = 3 };

// positions as 16-bit values in the small class (records decoding to < 64 KiB): 4 KiB of LDS per
// wave, 8 waves per SIMD
template <uint32_t kMaxK>
using LzPos = typename std::conditional<kMaxK == 1024, uint16_t, uint32_t>::type;
template <uint32_t kMaxK>
struct LzLds {
    LzPos<kMaxK> pos[kMaxK];  // record output position of code k of the current epoch
    uint16_t len[kMaxK];      // its output length (<= 3840)
    uint8_t slot[64];         // code starts of the current output window
};

// width and epoch bit offset of code k (writer.go incHi / reader.go decode: 9 bits for codes 0..254,
// 10 for 255..766, 11 for 767..1790, 12 after)
__device__ __forceinline__ uint32_t lz_width(uint32_t k) { return k < 255 ? 9u : k < 767 ? 10u : k < 1791 ? 11u : 12u; }
__device__ __forceinline__ uint64_t lz_bits(uint32_t k) {
    const uint64_t a = umin(k, 255u), b = umin(k, 767u) - a, c = umin(k, 1791u) - a - b, d = (uint64_t)k - a - b - c;
    return 9 * a + 10 * b + 11 * c + 12 * d;
}

// wave-wide inclusive scans on DPP (row shifts within 16-lane rows, then row broadcasts 15 / 31):
// VALU latency instead of the LDS round trips of __shfl_up (as the Snappy wave decoder's)
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
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t v, uint32_t) { return wave_incl<false>(v); }
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v, uint32_t) { return wave_incl<true>(v); }

// one record: stream p[0, slen) -> out[0, dlen). kCount: nothing stored, *total = decoded length.
template <bool kCount, uint32_t kMaxK>
__device__ int lz_record(LzLds<kMaxK>& S, const uint8_t* p, uint32_t slen, uint8_t* out, uint32_t dlen, uint32_t lane,
                         uint64_t* total) {
    const uint64_t nbits = 8ull * slen;
    // the payload's aligned base: every code is read from two aligned dwords (the padded file makes
    // reads past the payload safe)
    const uint8_t* pa = reinterpret_cast<const uint8_t*>((uintptr_t)p & ~(uintptr_t)3);
    const uint32_t pa_sh = (uint32_t)((uintptr_t)p & 3u);
    uint64_t ebit = 0;  // bit position of the epoch's code 0
    uint32_t k0 = 0;    // index (within the epoch) of the round's first code
    uint64_t d = 0;     // bytes produced
    for (;;) {
        const uint32_t k = k0 + lane;
        const uint32_t w = lz_width(k);
        const uint64_t bp = ebit + lz_bits(k);
        const bool avail = bp + w <= nbits;
        uint32_t code = 0;
        if (avail) {
            const uint64_t byte = (bp >> 3) + pa_sh;
            const uint32_t* q = reinterpret_cast<const uint32_t*>(pa + (byte & ~3ull));
            const uint32_t lo = q[0], hi = q[1];
            const uint32_t win = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(byte & 3u));  // bytes [byte, byte + 4)
            code = (win >> (bp & 7u)) & ((1u << w) - 1u);
        }
        const uint32_t hi = umin(257u + k, 4095u);
        const uint32_t kind = !avail ? kMissing : code < 256 ? kLit : code == 256 ? kClear : code == 257 ? kEnd
                              : code <= hi ? kCopy : kBad;
        const uint64_t spec = __ballot(kind >= kClear);
        const uint32_t nv = spec ? (uint32_t)__builtin_ctzll(spec) : 64u;  // valid codes: lanes [0, nv)
        const bool valid = lane < nv;
        // lengths: len_k = 1 (literal), or len_j + 1 with j = code - 258 < k; pointer jumping over the
        // lanes for j inside this round (len_l = acc + len_par until done)
        const uint32_t j = code - 258u;
        uint32_t acc = 0, par = lane;
        bool done = true;
        if (valid) {
            if (kind == kLit) {
                acc = 1;
            } else if (j < k0) {
                acc = (uint32_t)S.len[j] + 1u;
            } else {
                acc = 1;
                par = j - k0;
                done = false;
            }
        }
        while (__any(!done)) {
            const uint32_t pacc = __shfl(acc, par, 64), ppar = __shfl(par, par, 64);
            const bool pdone = __shfl(done ? 1 : 0, par, 64) != 0;
            if (!done) {
                acc += pacc;
                if (pdone) done = true; else par = ppar;
            }
        }
        const uint32_t incl = wave_incl_add(acc, lane);
        const uint32_t T = __shfl(incl, 63, 64);
        const uint64_t pos = d + incl - acc;
        // copy source: an earlier round's code from LDS, or a lane of this round
        const uint32_t jl = valid && kind == kCopy && j >= k0 ? j - k0 : lane;
        const uint64_t pos_j = __shfl(pos, jl, 64);
        uint64_t src = 0;
        if (valid && kind == kCopy) src = j < k0 ? (uint64_t)S.pos[j] : pos_j;
        __builtin_amdgcn_wave_barrier();
        if (valid && k < kMaxK) {
            S.pos[k] = (LzPos<kMaxK>)pos;
            S.len[k] = (uint16_t)acc;
        }
        const uint64_t d2 = d + T;
        if (!kCount) {
            if (d2 > dlen) return kLzResize_;  // more output than the framing's size (k_lzw_resize decides)
            // ---- materialise [d, d2) in 64-byte windows, lane = byte ----
            uint32_t ei = 0;  // code (lane) covering the window's first byte
            const uint32_t lit = kind == kLit ? code : 0x100u;
            for (uint64_t W = d; W < d2; W += 64) {
                S.slot[lane] = 0;
                __builtin_amdgcn_wave_barrier();
                if (lane == 0) S.slot[0] = (uint8_t)(ei + 1);
                if (valid && pos > W && pos < W + 64) S.slot[pos - W] = (uint8_t)(lane + 1);
                __builtin_amdgcn_wave_barrier();
                const uint32_t kk = wave_incl_max(S.slot[lane], lane) - 1u;
                const uint64_t pk = __shfl(pos, kk, 64), sk = __shfl(src, kk, 64);
                const uint32_t lk = __shfl(lit, kk, 64), ak = __shfl(acc, kk, 64);
                const uint64_t b = W + lane;
                const bool active = b < d2;
                // the previous windows' stores have drained before any of them is read back
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                uint32_t val = 0, srcl = lane;
                bool pend = false;
                if (active) {
                    if (lk < 0x100u) {
                        val = lk;
                    } else {
                        const uint64_t s = sk + (b - pk);  // < b
                        if (s >= W) {
                            pend = true;
                            srcl = (uint32_t)(s - W);
                        } else {
                            val = __builtin_nontemporal_load(out + s);  // L2: bypasses this CU's L1
                        }
                    }
                }
                while (__any(pend)) {  // sources inside the window: always an earlier lane
                    const uint32_t sv = __shfl(val, srcl, 64);
                    const bool sp = __shfl(pend ? 1 : 0, srcl, 64) != 0;
                    if (pend && !sp) {
                        val = sv;
                        pend = false;
                    }
                }
                if (active) out[b] = (uint8_t)val;
                // the code covering the next window's first byte
                const uint32_t k63 = __shfl(kk, 63, 64);
                const uint64_t end63 = __shfl(pk + ak, 63, 64);
                ei = end63 > W + 64 ? k63 : k63 + 1;
                __builtin_amdgcn_wave_barrier();
            }
        }
        d = d2;
        if (nv == 64) {
            k0 += 64;
            continue;
        }
        const uint32_t stop = __shfl(kind, nv, 64);
        if (stop == kClear) {  // reset: the next epoch's code 0 follows the clear code
            ebit += lz_bits(k0 + nv) + lz_width(k0 + nv);
            k0 = 0;
            continue;
        }
        if (stop != kEnd) return kLzCorrupt;  // invalid code / io.ErrUnexpectedEOF
        if (kCount) {
            *total = d;
            return kLzOk;
        }
        return d == dlen ? kLzOk : kLzResize_;
    }
}

__device__ __forceinline__ bool lzw_active(const FrameParams& P, const ScanState* st) {
    return st->hdr_status == RIO_OK && !st->capacity_fail && st->compression == RIO_COMP_LZW;
}
}  // namespace

template <uint32_t kMaxK>
__global__ void __launch_bounds__(64) k_lzw_decode(FrameParams P) {
    __shared__ LzLds<kMaxK> S;
    constexpr bool kSmall = kMaxK == kLzSmallK;
    ScanState* st = P.state;
    if (!lzw_active(P, st) || (P.redo && !st->gz_redo)) return;
    const uint32_t lane = threadIdx.x;
    const uint64_t n = st->n_records;
    for (uint64_t i = blockIdx.x; i < n; i += gridDim.x) {
        if (P.flags[i] & (RIO_FLAG_NIL | RIO_FLAG_CORRUPT | RIO_FLAG_EOF)) continue;  // nil / failed at framing
        const uint64_t o0 = P.out_off[i], dlen = P.out_off[i + 1] - o0;
        const uint64_t pay = P.rec_pay[i];
        const uint64_t slen = (pay & kLzLen) >> 8;
        if ((slen <= kLzSmallLen && dlen < 65536) != kSmall) continue;  // the other size class's
        if (slen >= 0xFFFFFFF0ull || dlen >= 0xFFFFFFF0ull) {  // past 32-bit positions: the reference reader's
            if (lane == 0) atomicMin((unsigned long long*)&st->unsupported_rec, (unsigned long long)i);
            continue;
        }
        const int rc = lz_record<false, kMaxK>(S, P.file + P.rec_off[i] + (pay & 0xFF), (uint32_t)slen, P.out + o0,
                                        (uint32_t)dlen, lane, nullptr);
        if (lane == 0) {
            if (rc == kLzResize_ && !P.redo) {
                P.rec_pay[i] = pay | kLzResize;  // sized by k_lzw_resize, decoded in the redo round
                st->gz_resize = 1u;
            } else if (rc != kLzOk) {
                mark_bad(P, i);  // (redo round: the counted size is final)
            }
        }
    }
}

// Sizes of the records k_lzw_decode marked: decoded length counted (nothing stored), the chunk's
// scratch length and byte sum corrected for the redo scan; a record Go's reader fails on is flagged
// corrupt (its size stays the framing's). One wave per chunk (its records are slots [0, owned) of
// ChunkPlace, as in k_place). A file whose placement came from the sequential repair is handed back
// at the first such record instead. (k_gz_resize's structure; the redo flags are shared.)
__global__ void __launch_bounds__(64) k_lzw_resize(FrameParams P) {
    __shared__ LzLds<kLzMaxK> S;
    ScanState* st = P.state;
    if (!st->gz_resize || !lzw_active(P, st)) return;
    const uint32_t lane = threadIdx.x;
    if (!st->slow && blockIdx.x == 0 && lane == 0) {  // read by the redo round's kernels only
        st->gz_redo = 1u;
        st->scan_ticket = 0;
        st->first_bad = kNone;  // recounted by the redo placement and decoder
        st->n_bad = 0;
    }
    for (uint64_t c = blockIdx.x; c < P.n_chunks; c += gridDim.x) {
        const ChunkPlace pl = P.place[c];
        uint64_t* sl = P.scratch_len + c * P.slots;
        for (uint64_t k = 0; k < pl.owned; k++) {
            const uint64_t i = pl.base_idx + k;
            const uint64_t pay = P.rec_pay[i];
            if (!(pay & kLzResize)) continue;
            if (st->slow) {
                if (lane == 0) atomicMin((unsigned long long*)&st->unsupported_rec, (unsigned long long)i);
                continue;
            }
            uint64_t total = 0;
            const int rc = lz_record<true, kLzMaxK>(S, P.file + P.rec_off[i] + (pay & 0xFF), (uint32_t)((pay & kLzLen) >> 8),
                                           nullptr, 0, lane, &total);
            if (lane == 0) {
                if (rc == kLzOk && total < 0xFFFFFFF0ull) {
                    const uint64_t old = sl[k] & kLenMask;
                    sl[k] = (sl[k] & ~kLenMask) | total;
                    P.chunks[c].bytes += total - old;  // (this wave is the chunk's only writer)
                } else if (rc == kLzCorrupt) {
                    sl[k] |= kBadBit;
                } else {
                    atomicMin((unsigned long long*)&st->unsupported_rec, (unsigned long long)i);
                }
            }
        }
    }
}

hipError_t launch_lzw_decode(const FrameParams& P, hipStream_t s) {
    hipLaunchKernelGGL(k_lzw_decode<kLzSmallK>, dim3(kLzSmallGrid), dim3(64), 0, s, P);
    hipLaunchKernelGGL(k_lzw_decode<kLzMaxK>, dim3(kLzGrid), dim3(64), 0, s, P);
    return hipGetLastError();
}

hipError_t launch_lzw_resize(const FrameParams& P, hipStream_t s) {
    hipLaunchKernelGGL(k_lzw_resize, dim3(kLzGrid), dim3(64), 0, s, P);
    return hipGetLastError();
}

}  // namespace rio
