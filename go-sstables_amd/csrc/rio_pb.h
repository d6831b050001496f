// rio_pb.h — protobuf wire-format helpers shared by the device kernels (protowire rules as
// google.golang.org/protobuf's proto.Unmarshal applies them to sstables/proto/sstable.proto).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rio {

// byte sources: RawBytes reads memory directly; WinBytes keeps one aligned 16-byte window of the
// (RIO_DEVICE_PAD-padded) file per lane and reloads it only when a position leaves it
struct RawBytes {
    const uint8_t* f;
    __device__ __forceinline__ uint32_t operator()(uint64_t p) const { return f[p]; }
};
struct WinBytes {
    const uint8_t* f;
    uint64_t base = ~0ull;
    uint4 v;
    __device__ __forceinline__ uint32_t operator()(uint64_t p) {
        const uint64_t b = p & ~15ull;
        if (b != base) {
            v = *reinterpret_cast<const uint4*>(f + b);
            base = b;
        }
        const uint32_t k = (uint32_t)p & 15u, j = k >> 2;
        const uint32_t d = j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
        return (d >> (8 * (k & 3u))) & 0xFFu;
    }
};

// protowire.ConsumeVarint over bytes [base, base + n) of a source: <= 10 bytes, the 10th <= 1
template <class B>
__device__ __forceinline__ bool pb_varint_t(B& g, uint64_t base, uint64_t n, uint64_t& pos, uint64_t& v) {
    uint64_t x = 0;
    for (int i = 0; i < 10; i++) {
        if (pos >= n) return false;
        const uint32_t c = g(base + pos++);
        if (i == 9 && c > 1) return false;
        x |= (uint64_t)(c & 0x7F) << (7 * i);
        if (c < 0x80) {
            v = x;
            return true;
        }
    }
    return false;
}

// skip one field value (protowire.ConsumeFieldValue); groups iteratively to their matching end tag
template <class B>
__device__ __forceinline__ bool pb_skip_t(B& g, uint64_t base, uint64_t n, uint64_t& pos, uint64_t num, uint32_t wt) {
    uint64_t v;
    if (wt == 0) return pb_varint_t(g, base, n, pos, v);
    if (wt == 1) {
        if (n - pos < 8) return false;
        pos += 8;
        return true;
    }
    if (wt == 5) {
        if (n - pos < 4) return false;
        pos += 4;
        return true;
    }
    if (wt == 2) {
        if (!pb_varint_t(g, base, n, pos, v) || v > n - pos) return false;
        pos += v;
        return true;
    }
    if (wt != 3) return false;  // 4 unmatched end group, 6, 7 invalid
    // group: nested start / end tags must match; a stack of field numbers would be exact, the depth
    // plus the outermost number suffices for wire-valid input and rejects the rest
    uint32_t depth = 1;
    uint64_t stack[16];
    stack[0] = num;
    while (depth) {
        uint64_t tag;
        if (!pb_varint_t(g, base, n, pos, tag)) return false;
        const uint64_t fn = tag >> 3;
        const uint32_t t = (uint32_t)(tag & 7);
        if (fn < 1 || fn > 0x1FFFFFFFull) return false;
        if (t == 4) {
            if (stack[depth - 1] != fn) return false;
            depth--;
        } else if (t == 3) {
            if (depth == 16) return false;
            stack[depth++] = fn;
        } else if (t == 0) {
            if (!pb_varint_t(g, base, n, pos, v)) return false;
        } else if (t == 1 || t == 5) {
            const uint64_t w = t == 1 ? 8 : 4;
            if (n - pos < w) return false;
            pos += w;
        } else if (t == 2) {
            if (!pb_varint_t(g, base, n, pos, v) || v > n - pos) return false;
            pos += v;
        } else {
            return false;
        }
    }
    return true;
}

// proto.Unmarshal into a reset IndexEntry {key = 1, valueOffset = 2, checksum = 3}
// (sstables/proto/sstable.proto:5-9): last occurrence wins, a known field with another wire type
// and unknown fields are skipped. key_off is relative to b. Returns false for malformed input.
template <class B>
__device__ __forceinline__ bool pb_index_entry_t(B& g, uint64_t base, uint64_t len, uint64_t& ko, uint64_t& kl, uint64_t& vo,
                                        uint64_t& cs) {
    uint64_t pos = 0;
    ko = kl = vo = cs = 0;
    while (pos < len) {
        uint64_t tag, v;
        if (!pb_varint_t(g, base, len, pos, tag)) return false;
        const uint64_t fn = tag >> 3;
        const uint32_t wt = (uint32_t)(tag & 7);
        if (fn < 1 || fn > 0x1FFFFFFFull) return false;
        if (fn == 1 && wt == 2) {
            if (!pb_varint_t(g, base, len, pos, v) || v > len - pos) return false;
            ko = pos;
            kl = v;
            pos += v;
        } else if ((fn == 2 || fn == 3) && wt == 0) {
            if (!pb_varint_t(g, base, len, pos, v)) return false;
            if (fn == 2) vo = v; else cs = v;
        } else if (!pb_skip_t(g, base, len, pos, fn, wt)) {
            return false;
        }
    }
    return true;
}

// proto.Unmarshal into a reset DataEntry {value = 1} (sstables/proto/sstable.proto:12-14), the v0
// tables' value records: present = field 1 seen as bytes (last occurrence wins; present with length 0
// is Go's non-nil empty slice), [vo, vo + vl) relative to base. Returns false for malformed input.
template <class B>
__device__ __forceinline__ bool pb_data_entry_t(B& g, uint64_t base, uint64_t len, bool& present, uint64_t& vo,
                                                uint64_t& vl) {
    uint64_t pos = 0;
    present = false;
    vo = vl = 0;
    while (pos < len) {
        uint64_t tag, v;
        if (!pb_varint_t(g, base, len, pos, tag)) return false;
        const uint64_t fn = tag >> 3;
        const uint32_t wt = (uint32_t)(tag & 7);
        if (fn < 1 || fn > 0x1FFFFFFFull) return false;
        if (fn == 1 && wt == 2) {
            if (!pb_varint_t(g, base, len, pos, v) || v > len - pos) return false;
            present = true;
            vo = pos;
            vl = v;
            pos += v;
        } else if (!pb_skip_t(g, base, len, pos, fn, wt)) {
            return false;
        }
    }
    return true;
}

// pointer forms (b[0, n))
__device__ __forceinline__ bool pb_varint(const uint8_t* b, uint64_t n, uint64_t& pos, uint64_t& v) {
    RawBytes g{b};
    return pb_varint_t(g, 0, n, pos, v);
}
__device__ inline bool pb_index_entry(const uint8_t* b, uint64_t len, uint64_t& ko, uint64_t& kl, uint64_t& vo,
                                      uint64_t& cs) {
    RawBytes g{b};
    return pb_index_entry_t(g, 0, len, ko, kl, vo, cs);
}

}  // namespace rio
