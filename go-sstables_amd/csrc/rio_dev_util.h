// rio_dev_util.h — device helpers shared by the recordio kernels (varints, 128-bit byte shifts,
// unaligned 16-byte global access, the single-thread Snappy decoder). Internal to librio.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "rio.h"

namespace rio {

// Same-type min / max. HIP's global min/max are overloaded for int, unsigned, 64-bit and floating
// types; a call with mixed operands (say uint32_t and int, or a readfirstlane result) can resolve to
// the double overload and silently convert (round 3: the parser/emitter hang). Every
// kernel calls these instead; tests/test_kernel_lint.py rejects a bare min( / max( in csrc/*.hip.
template <typename A, typename B>
__host__ __device__ __forceinline__ A umin(A a, B b) {
    static_assert(std::is_same<A, B>::value, "rio::umin: operands of different types; cast explicitly");
    static_assert(std::is_integral<A>::value, "rio::umin: integer operands only");
    return a < b ? a : b;
}
template <typename A, typename B>
__host__ __device__ __forceinline__ A umax(A a, B b) {
    static_assert(std::is_same<A, B>::value, "rio::umax: operands of different types; cast explicitly");
    static_assert(std::is_integral<A>::value, "rio::umax: integer operands only");
    return a > b ? a : b;
}

// encoding/binary.Uvarint semantics: >0 bytes read, 0 buffer too small, <0 overflow
__device__ inline int uvarint_buf(const uint8_t* p, uint64_t n, uint64_t& x) {
    uint64_t v = 0;
    uint32_t sh = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (i == 10) return -(int)(i + 1);
        uint32_t b = p[i];
        if (b < 0x80) {
            if (i == 9 && b > 1) return -(int)(i + 1);
            x = v | ((uint64_t)b << sh);
            return (int)(i + 1);
        }
        v |= (uint64_t)(b & 0x7F) << sh;
        sh += 7;
    }
    return 0;
}

// ---- 16-byte values: unaligned global access (gfx950 unaligned mode), byte shifts -----------
typedef uint4 __attribute__((aligned(1))) u4u;

// HIP_vector_type's copy operators take 16-aligned references; the access itself is the 1-aligned
// u4u (one global_load/store_dwordx4 in unaligned mode), which is what -Walign-mismatch flags
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Walign-mismatch"
__device__ __forceinline__ uint4 ldu16(const uint8_t* p) { return *reinterpret_cast<const u4u*>(p); }
__device__ __forceinline__ void stu16(uint8_t* p, uint4 v) { *reinterpret_cast<u4u*>(p) = v; }
#pragma clang diagnostic pop
// non-temporal (streaming) 16-byte access: bytes touched once should not displace lines the
// kernel comes back to (the decoder's input lines)
// (p any byte address: the 1-aligned vector type, as u4u for the plain forms)
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
typedef uint32_t v4u32u __attribute__((ext_vector_type(4), aligned(1)));
__device__ __forceinline__ uint4 ldu16_nt(const uint8_t* p) {
    const v4u32 v = __builtin_nontemporal_load(reinterpret_cast<const v4u32u*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void stu16_nt(uint8_t* p, uint4 v) {
    v4u32u w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<v4u32u*>(p));
}
__device__ __forceinline__ uint4 zero4() { return make_uint4(0, 0, 0, 0); }
__device__ __forceinline__ uint4 or4(uint4 a, uint4 b) { return make_uint4(a.x | b.x, a.y | b.y, a.z | b.z, a.w | b.w); }

__device__ __forceinline__ uint4 pack4(uint64_t lo, uint64_t hi) {
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

// 128-bit value >> 8k bits, k in [0, 16] (k = 16 gives 0); branch-free (selects only)
__device__ __forceinline__ uint4 shr_bytes(uint4 v, uint32_t k) {
    const uint64_t lo = ((uint64_t)v.y << 32) | v.x, hi = ((uint64_t)v.w << 32) | v.z;
    const uint32_t b = 8 * k;
    const uint64_t carry = b ? (hi << ((64 - b) & 63)) : 0ull;
    const uint64_t small_lo = (lo >> (b & 63)) | carry;
    const uint64_t big_lo = b < 128 ? (hi >> ((b - 64) & 63)) : 0ull;
    const uint64_t rlo = b < 64 ? small_lo : big_lo;
    const uint64_t rhi = b < 64 ? (hi >> (b & 63)) : 0ull;
    return pack4(rlo, rhi);
}

// 128-bit value << 8k bits, k in [0, 16]
__device__ __forceinline__ uint4 shl_bytes(uint4 v, uint32_t k) {
    const uint64_t lo = ((uint64_t)v.y << 32) | v.x, hi = ((uint64_t)v.w << 32) | v.z;
    const uint32_t b = 8 * k;
    const uint64_t carry = b ? (lo >> ((64 - b) & 63)) : 0ull;
    const uint64_t small_hi = (hi << (b & 63)) | carry;
    const uint64_t big_hi = b < 128 ? (lo << ((b - 64) & 63)) : 0ull;
    const uint64_t rhi = b < 64 ? small_hi : big_hi;
    const uint64_t rlo = b < 64 ? (lo << (b & 63)) : 0ull;
    return pack4(rlo, rhi);
}

// keep the first n bytes (n in [0, 16]), zero the rest
__device__ __forceinline__ uint4 keep_bytes(uint4 v, uint32_t n) {
    const uint64_t lo = ((uint64_t)v.y << 32) | v.x, hi = ((uint64_t)v.w << 32) | v.z;
    const uint32_t b = 8 * n;
    const uint64_t mlo = b >= 64 ? ~0ull : ((1ull << (b & 63)) - 1);
    const uint64_t mhi = b <= 64 ? 0ull : (b >= 128 ? ~0ull : ((1ull << ((b - 64) & 63)) - 1));
    return pack4(lo & mlo, hi & mhi);
}

// store the first n (< 16) bytes of v
__device__ __forceinline__ void st_partial(uint8_t* p, uint4 v, uint32_t n) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t k = 0; k < 16; k++)
        if (k < n) p[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
}

// golang/snappy v1.0.0 decode (decode.go / decode_other.go) of one record by one thread; used by
// the single-record (ReadNextAt / SeekNext) kernels.
__device__ inline bool snappy_decode_thread(const uint8_t* src, uint64_t slen, uint8_t* dst, uint64_t dlen) {
    uint64_t s = 0, d = 0;
    while (s < slen) {
        const uint32_t tag = src[s];
        uint64_t length, offset;
        if ((tag & 3) == 0) {
            uint32_t x = tag >> 2;
            if (x < 60) {
                s += 1;
            } else {
                const uint32_t nb = x - 59;
                s += 1 + nb;
                if (s > slen) return false;
                x = 0;
                for (uint32_t k = 0; k < nb; k++) x |= (uint32_t)src[s - nb + k] << (8 * k);
            }
            length = (uint64_t)x + 1;
            if (length > dlen - d || length > slen - s) return false;
            for (uint64_t k = 0; k < length; k++) dst[d + k] = src[s + k];
            d += length;
            s += length;
            continue;
        }
        if ((tag & 3) == 1) {
            s += 2;
            if (s > slen) return false;
            length = 4 + ((tag >> 2) & 7);
            offset = ((tag & 0xE0u) << 3) | src[s - 1];
        } else if ((tag & 3) == 2) {
            s += 3;
            if (s > slen) return false;
            length = 1 + (tag >> 2);
            offset = (uint64_t)src[s - 2] | (uint64_t)src[s - 1] << 8;
        } else {
            s += 5;
            if (s > slen) return false;
            length = 1 + (tag >> 2);
            offset = (uint64_t)src[s - 4] | (uint64_t)src[s - 3] << 8 | (uint64_t)src[s - 2] << 16 |
                     (uint64_t)src[s - 1] << 24;
        }
        if (offset == 0 || d < offset || length > dlen - d) return false;
        for (uint64_t k = 0; k < length; k++) dst[d + k] = dst[d - offset + k];
        d += length;
    }
    return d == dlen;
}

}  // namespace rio
