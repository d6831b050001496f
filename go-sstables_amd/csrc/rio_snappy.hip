// rio_snappy.hip — Snappy block decode of every framed record (golang/snappy v1.0.0 semantics,
// decode.go + decode_other.go; called per record by FileReader.ReadNext, file_reader.go:115-125).
//
// k_snappy_ring<R>: one lane per record (SIMT across consecutive records). Each lane keeps the
// last R decoded bytes of its record in an LDS ring and emits the record as a sequence of
// <=16-byte pieces; a piece comes either from a 16-byte register window over the compressed
// element stream (literals) or from history (copies: the LDS ring, or HBM for offsets beyond the
// ring). Completed history is flushed to the output arena in R/4-byte bursts, so the lane's loads
// never queue behind a store per element (vmcnt counts loads and stores in issue order on CDNA).
// The loop has one exit and computes both piece sources, selecting between them: divergent
// element types cost selects, not exec-mask branch nests.
// k_snappy_global: records whose compressed stream exceeds 32-bit positions (never produced by a
// real encoder) decode with byte loops straight to HBM.
#include <hip/hip_runtime.h>

#include "rio_device.h"
#include "rio_dev_util.h"

namespace rio {

// 16 bytes at output position q from the ring (two aligned chunk reads + funnel)
template <uint32_t R>
__device__ __forceinline__ uint4 ring_read16(const uint8_t* H, uint32_t q) {
    constexpr uint32_t M = R - 1;
    const uint32_t c0 = q & ~15u, r = q & 15u;
    const uint4 x0 = *reinterpret_cast<const uint4*>(H + (c0 & M));
    const uint4 x1 = *reinterpret_cast<const uint4*>(H + ((c0 + 16) & M));
    return or4(shr_bytes(x0, r), shl_bytes(x1, 16 - r));
}

// L1-bypassing 16-byte load of bytes this lane flushed earlier (sc1: served by L2)
__device__ __forceinline__ uint4 ld16_sc1(const uint8_t* p) {
    uint4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}

template <uint32_t R>
__device__ bool snappy_ring(const uint8_t* src, uint32_t slen, uint8_t* H, uint8_t* gout, uint32_t dlen) {
    constexpr uint32_t M = R - 1;
    constexpr uint32_t kFlushAt = R / 2;  // flush when this many bytes are unflushed
    constexpr uint32_t kFlush = R / 4;    // bytes per flush (multiple of 16)
    constexpr uint32_t kRingOff = R - 48; // copies with offset <= this read the ring
    static_assert((R & M) == 0 && R >= 128, "ring size");
    uint32_t s = 0, d = 0, fl = 0, rem = 0, off = 0, wv = 0;
    bool lit = false, bad = false;
    uint4 W = zero4(), stage = zero4();
    while (rem != 0 || s < slen) {
        if (rem == 0) {  // next element: decode its tag from the window (selects)
            if (wv < 5) {
                W = ldu16(src + s);
                wv = 16;
            }
            const uint32_t tag = W.x & 0xFF, t = tag & 3, x = tag >> 2;
            const uint64_t w64 = ((uint64_t)W.y << 32) | W.x;
            const uint32_t lit_hl = x < 60 ? 1u : x - 58u;
            const uint32_t ext = (uint32_t)((w64 >> 8) & ((1ull << ((8 * (lit_hl - 1)) & 63)) - 1));
            const uint32_t len = t == 0 ? (x < 60 ? x : ext) + 1 : (t == 1 ? 4 + (x & 7) : x + 1);
            const uint32_t hl = t == 0 ? lit_hl : (t == 1 ? 2u : (t == 2 ? 3u : 5u));
            const uint32_t o1 = ((tag & 0xE0u) << 3) | ((W.x >> 8) & 0xFF);
            const uint32_t o2 = (W.x >> 8) & 0xFFFF;
            const uint32_t o4 = (W.x >> 8) | (W.y << 24);
            off = t == 1 ? o1 : (t == 2 ? o2 : o4);
            lit = t == 0;
            // golang/snappy bounds: header bytes, literal source, copy offset, output room
            bad = hl > slen - s || len > dlen - d ||
                  (lit ? (len == 0 || len > slen - s - hl) : (off == 0 || off > d));
            if (bad) break;
            s += hl;
            W = shr_bytes(W, hl);
            wv -= hl;
            rem = len;
        }
        const uint32_t n = min(rem, 16u);
        if (lit && wv < n) {
            W = ldu16(src + s);
            wv = 16;
        }
        const uint32_t q = d - off;
        uint4 v = ring_read16<R>(H, q & M);
        if (!lit && off > kRingOff) v = ld16_sc1(gout + q);
        if (!lit && off < n) {  // overlapping copy: replicate the period-`off` pattern in registers
            v = keep_bytes(v, off);
            for (uint32_t k = off; k < 16; k *= 2) v = or4(v, shl_bytes(v, k));
            off *= (16 + off - 1) / off;  // later pieces: a multiple of the period >= 16
        }
        v = make_uint4(lit ? W.x : v.x, lit ? W.y : v.y, lit ? W.z : v.z, lit ? W.w : v.w);
        const uint32_t adv = lit ? n : 0u;
        s += adv;
        W = shr_bytes(W, adv);
        wv -= adv;
        // append n bytes at d: merge with the staged head of the current 16-byte chunk; both
        // chunk writes are unconditional (the second holds only bytes not yet final)
        const uint32_t r = d & 15u, F = d - r;
        v = keep_bytes(v, n);
        const uint4 lo = or4(stage, shl_bytes(v, r));
        const uint4 hi = shr_bytes(v, 16 - r);
        *reinterpret_cast<uint4*>(H + (F & M)) = lo;
        *reinterpret_cast<uint4*>(H + ((F + 16) & M)) = hi;
        const bool roll = r + n >= 16;
        stage = make_uint4(roll ? hi.x : lo.x, roll ? hi.y : lo.y, roll ? hi.z : lo.z, roll ? hi.w : lo.w);
        d += n;
        rem -= n;
        if (d - fl >= kFlushAt) {
#pragma unroll
            for (uint32_t k = 0; k < kFlush; k += 16)
                stu16(gout + fl + k, *reinterpret_cast<const uint4*>(H + ((fl + k) & M)));
            fl += kFlush;
        }
    }
    if (bad || d != dlen) return false;
    for (uint32_t k = fl; k < d; k += 16) {
        const uint4 v = *reinterpret_cast<const uint4*>(H + (k & M));
        if (k + 16 <= d)
            stu16(gout + k, v);
        else
            st_partial(gout + k, v, d - k);
    }
    return true;
}

template <uint32_t R>
__global__ void __launch_bounds__(256) k_snappy_ring(FrameParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    ScanState* st = P.state;
    if (st->hdr_status != RIO_OK || st->capacity_fail || st->compression != RIO_COMP_SNAPPY) return;
    const uint64_t n = st->n_records;
    uint8_t* H = lds + threadIdx.x * (R + 16);  // +16: skews slot banks
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (P.flags[i] & RIO_FLAG_NIL) continue;
        const uint64_t pay = P.rec_pay[i], slen = pay >> 8;
        if (slen > 0xFFFFFFFFull) continue;  // k_snappy_global
        const uint64_t o0 = P.out_off[i], olen = P.out_off[i + 1] - o0;
        const uint8_t* src = P.file + P.rec_off[i] + (pay & 0xFF);
        if (!snappy_ring<R>(src, (uint32_t)slen, H, P.out + o0, (uint32_t)olen))
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
        if (slen <= 0xFFFFFFFFull) continue;  // k_snappy_ring
        const uint64_t o0 = P.out_off[i], o1 = P.out_off[i + 1];
        if (!snappy_decode_thread(P.file + P.rec_off[i] + (pay & 0xFF), slen, P.out + o0, o1 - o0))
            atomicMin((unsigned long long*)&st->decode_err_rec, (unsigned long long)i);
    }
}

constexpr uint32_t kRing = 256;

hipError_t launch_snappy_decode(const FrameParams& P, hipStream_t s) {
    // 256 lanes x (256+16)-byte rings = 68 KiB LDS per workgroup: 2 workgroups (8 waves) per CU
    static const unsigned grid = [] {
        const char* g = getenv("RIO_DECODE_GRID");
        return g && *g ? (unsigned)atoi(g) : 512u;
    }();
    hipLaunchKernelGGL(k_snappy_ring<kRing>, dim3(grid), dim3(256), 256 * (kRing + 16), s, P);
    hipLaunchKernelGGL(k_snappy_global, dim3(64), dim3(256), 0, s, P);
    return hipGetLastError();
}

}  // namespace rio
