// rio_pb.h — protobuf wire-format helpers shared by the device kernels (protowire rules as
// google.golang.org/protobuf's proto.Unmarshal applies them to sstables/proto/sstable.proto).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rio {

// protowire.ConsumeVarint over b[0, n): <= 10 bytes, the 10th <= 1
__device__ __forceinline__ bool pb_varint(const uint8_t* b, uint64_t n, uint64_t& pos, uint64_t& v) {
    uint64_t x = 0;
    for (int i = 0; i < 10; i++) {
        if (pos >= n) return false;
        const uint32_t c = b[pos++];
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
__device__ inline bool pb_skip(const uint8_t* b, uint64_t n, uint64_t& pos, uint64_t num, uint32_t wt) {
    uint64_t v;
    if (wt == 0) return pb_varint(b, n, pos, v);
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
        if (!pb_varint(b, n, pos, v) || v > n - pos) return false;
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
        if (!pb_varint(b, n, pos, tag)) return false;
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
            if (!pb_varint(b, n, pos, v)) return false;
        } else if (t == 1 || t == 5) {
            const uint64_t w = t == 1 ? 8 : 4;
            if (n - pos < w) return false;
            pos += w;
        } else if (t == 2) {
            if (!pb_varint(b, n, pos, v) || v > n - pos) return false;
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
__device__ inline bool pb_index_entry(const uint8_t* b, uint64_t len, uint64_t& ko, uint64_t& kl, uint64_t& vo,
                                      uint64_t& cs) {
    uint64_t pos = 0;
    ko = kl = vo = cs = 0;
    while (pos < len) {
        uint64_t tag, v;
        if (!pb_varint(b, len, pos, tag)) return false;
        const uint64_t fn = tag >> 3;
        const uint32_t wt = (uint32_t)(tag & 7);
        if (fn < 1 || fn > 0x1FFFFFFFull) return false;
        if (fn == 1 && wt == 2) {
            if (!pb_varint(b, len, pos, v) || v > len - pos) return false;
            ko = pos;
            kl = v;
            pos += v;
        } else if ((fn == 2 || fn == 3) && wt == 0) {
            if (!pb_varint(b, len, pos, v)) return false;
            if (fn == 2) vo = v; else cs = v;
        } else if (!pb_skip(b, len, pos, fn, wt)) {
            return false;
        }
    }
    return true;
}

}  // namespace rio
