// rio_sstable.hip — device side of an SSTable's load, validation and full scan on top of the
// recordio decode (sstables/sstable_reader.go, sstable_iterator.go, slice_key_index.go).
//
// An SSTable is data.rio (values: one recordio record per value, Snappy by default,
// sstable_writer.go:50-56,219-220) + index.rio (one protobuf IndexEntry {key = 1, valueOffset = 2,
// checksum = 3} per record, sstables/proto/sstable.proto:5-9, uncompressed by default). Both files
// are decoded by the recordio path (rio_device_decode); these kernels work on the decoded arenas:
//
// k_sst_index    one lane per index record: proto.Unmarshal into a reset IndexEntry
//                (SliceKeyIndexLoader.Load, slice_key_index.go:91-131): wire format restated from
//                protowire (varints <= 10 bytes, field numbers 1 .. 2^29-1, last occurrence wins,
//                known fields with another wire type and unknown fields skipped, groups skipped to
//                their end tag). Outputs key (offset / length into the index arena), valueOffset,
//                checksum; the first malformed record is reported.
// k_sst_validate one lane per index entry: the value is the data record whose file offset is the
//                entry's valueOffset (MMapReader.ReadNextAt, sstable_reader.go:85-92) — record i
//                for every table the writer produced (valueOffset = the offset its data write
//                returned, sstable_writer.go:126-132) — then CRC-64/ISO of the value
//                (checksumValue, :240-248) against the stored checksum, 0 meaning "no checksum"
//                (:100-108). Outputs every entry's CRC-64, the first mismatching entry, and the
//                first entry not in the writer's layout (valueOffset is not data record i's offset:
//                the scan's positional pairing and validation would diverge; the adapter keeps the
//                reference reader).
// k_sst_data_entry one lane per data record of a v0 table (metadata version 0, sstable_reader.go:
//                303-314): proto.Unmarshal into a DataEntry {value = 1} (sstable.proto:12-14), as
//                MMapProtoReader.ReadNextAt / ProtoReader.ReadNext do for every value
//                (recordio/proto/mmap_proto_reader.go:12-24). Outputs the value's [begin, end) in the data
//                arena (kValueNil both for an absent field: value nil), the first malformed record.
//                k_sst_validate then hashes these ranges instead of the whole records.
#include <hip/hip_runtime.h>

#include "rio_device.h"
#include "rio_dev_util.h"
#include "rio_pb.h"

namespace rio {


__global__ void __launch_bounds__(256) k_sst_index(const uint8_t* arena, const uint64_t* off, uint64_t n,
                                                   uint64_t* key_off, uint64_t* key_len, uint64_t* value_off,
                                                   uint64_t* checksum, unsigned long long* first_bad) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t base = off[i], len = off[i + 1] - base;
        const uint8_t* b = arena + base;
        uint64_t ko, kl, vo, cs;
        const bool ok = pb_index_entry(b, len, ko, kl, vo, cs);
        key_off[i] = base + ko;
        key_len[i] = kl;
        value_off[i] = vo;
        checksum[i] = cs;
        if (!ok) atomicMin(first_bad, (unsigned long long)i);
    }
}

// CRC-64/ISO, reflected, slice-by-8: tab[k][i] = CRC of byte i followed by k zero bytes, so one
// 8-byte step is eight independent LDS lookups instead of eight dependent ones.
__device__ __forceinline__ uint64_t crc64_step8(const uint64_t (*tab)[256], uint64_t c, uint64_t w) {
    c ^= w;
    return tab[7][c & 0xFF] ^ tab[6][(c >> 8) & 0xFF] ^ tab[5][(c >> 16) & 0xFF] ^ tab[4][(c >> 24) & 0xFF] ^
           tab[3][(c >> 32) & 0xFF] ^ tab[2][(c >> 40) & 0xFF] ^ tab[1][(c >> 48) & 0xFF] ^ tab[0][c >> 56];
}

__global__ void __launch_bounds__(256) k_sst_data_entry(const uint8_t* arena, const uint64_t* off, uint64_t n,
                                                        uint64_t* view, unsigned long long* first_bad) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
        const uint64_t base = off[j], len = off[j + 1] - base;
        RawBytes g{arena};
        bool present;
        uint64_t vo, vl;
        const bool ok = pb_data_entry_t(g, base, len, present, vo, vl);
        view[2 * j] = ok ? (present ? base + vo : RIO_VALUE_NIL) : RIO_VALUE_BAD;
        view[2 * j + 1] = ok ? (present ? base + vo + vl : RIO_VALUE_NIL) : RIO_VALUE_BAD;
        if (!ok) atomicMin(first_bad, (unsigned long long)j);
    }
}

// view == nullptr: the value of data record j is the whole record; else [view[2j], view[2j+1]) (v0
// DataEntry values; a nil or malformed one hashes as empty)
__global__ void __launch_bounds__(256) k_sst_validate(const uint8_t* data, const uint64_t* data_off,
                                                      const uint64_t* data_rec_off, uint64_t n_data,
                                                      const uint64_t* value_off, const uint64_t* checksum,
                                                      uint64_t n_index, uint64_t* crc_out,
                                                      unsigned long long* result, const uint64_t* view) {
    __shared__ uint64_t tab[8][256];  // 16 KiB
    for (uint32_t k = threadIdx.x; k < 256; k += blockDim.x) {
        uint64_t c = k;
        for (int j = 0; j < 8; j++) c = (c >> 1) ^ (0xD800000000000000ull & (0ull - (c & 1ull)));
        tab[0][k] = c;
    }
    __syncthreads();
    for (int t = 1; t < 8; t++) {
        for (uint32_t k = threadIdx.x; k < 256; k += blockDim.x)
            tab[t][k] = (tab[t - 1][k] >> 8) ^ tab[0][tab[t - 1][k] & 0xFF];
        __syncthreads();
    }
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_index; i += stride) {
        const uint64_t want = value_off[i];
        uint64_t j = i;
        if (!(i < n_data && data_rec_off[i] == want)) {
            // not the writer's layout (entry i <-> data record i): the full scan pairs entries and
            // records by position while validation follows valueOffset, so the device path hands
            // the table back; the search still gives validation its value
            uint64_t lo = 0, hi = n_data;
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1;
                if (data_rec_off[mid] < want) lo = mid + 1; else hi = mid;
            }
            if (lo >= n_data || data_rec_off[lo] != want) {
                crc_out[i] = 0;
                atomicMin(&result[1], (unsigned long long)i);
                continue;
            }
            j = lo;
            atomicMin(&result[1], (unsigned long long)i);
        }
        uint64_t vb = data_off[j], ve = data_off[j + 1];
        if (view) {
            vb = view[2 * j];
            ve = view[2 * j + 1];
            if (vb >= RIO_VALUE_BAD) vb = ve = 0;
        }
        const uint8_t* v = data + vb;
        const uint64_t len = ve - vb;
        uint64_t c = ~0ull, k = 0;
        // 64 bytes per iteration: four unaligned 16-byte loads in flight before the CRC steps
        for (; k + 64 <= len; k += 64) {
            uint4 w[4];
#pragma unroll
            for (int q = 0; q < 4; q++) w[q] = ldu16(v + k + 16 * q);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                c = crc64_step8(tab, c, ((uint64_t)w[q].y << 32) | w[q].x);
                c = crc64_step8(tab, c, ((uint64_t)w[q].w << 32) | w[q].z);
            }
        }
        for (; k + 16 <= len; k += 16) {
            const uint4 w = ldu16(v + k);
            c = crc64_step8(tab, c, ((uint64_t)w.y << 32) | w.x);
            c = crc64_step8(tab, c, ((uint64_t)w.w << 32) | w.z);
        }
        for (; k < len; k++) c = tab[0][(c ^ v[k]) & 0xFFu] ^ (c >> 8);
        c = ~c;
        crc_out[i] = c;
        if (checksum[i] != 0 && c != checksum[i]) atomicMin(&result[0], (unsigned long long)i);
    }
}

__global__ void k_sst_init(unsigned long long* r, int n) {
    if (threadIdx.x < (unsigned)n) r[threadIdx.x] = ~0ull;
}

hipError_t launch_sst_index(const uint8_t* arena, const uint64_t* off, uint64_t n, uint64_t* key_off,
                            uint64_t* key_len, uint64_t* value_off, uint64_t* checksum, uint64_t* result,
                            hipStream_t s) {
    unsigned long long* r = reinterpret_cast<unsigned long long*>(result);
    hipLaunchKernelGGL(k_sst_init, dim3(1), dim3(64), 0, s, r, 1);
    const uint64_t blocks = (n + 255) / 256;
    if (n) hipLaunchKernelGGL(k_sst_index, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, s, arena, off,
                              n, key_off, key_len, value_off, checksum, r);
    return hipGetLastError();
}

hipError_t launch_sst_data_entry(const uint8_t* arena, const uint64_t* off, uint64_t n, uint64_t* view,
                                 uint64_t* result, hipStream_t s) {
    unsigned long long* r = reinterpret_cast<unsigned long long*>(result);
    hipLaunchKernelGGL(k_sst_init, dim3(1), dim3(64), 0, s, r, 1);
    const uint64_t blocks = (n + 255) / 256;
    if (n)
        hipLaunchKernelGGL(k_sst_data_entry, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, s, arena, off,
                           n, view, r);
    return hipGetLastError();
}

hipError_t launch_sst_validate(const uint8_t* data, const uint64_t* data_off, const uint64_t* data_rec_off,
                               uint64_t n_data, const uint64_t* value_off, const uint64_t* checksum,
                               uint64_t n_index, uint64_t* crc_out, uint64_t* result, hipStream_t s,
                               const uint64_t* view) {
    unsigned long long* r = reinterpret_cast<unsigned long long*>(result);
    hipLaunchKernelGGL(k_sst_init, dim3(1), dim3(64), 0, s, r, 2);
    const uint64_t blocks = (n_index + 255) / 256;
    if (n_index)
        hipLaunchKernelGGL(k_sst_validate, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, s, data,
                           data_off, data_rec_off, n_data, value_off, checksum, n_index, crc_out, r, view);
    return hipGetLastError();
}

}  // namespace rio
