/*
 * rio_oracle.h — CPU restatement of the reference recordio readers (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 * It is the parity checker and the CPU baseline ("kind": "port"); it is never on the product path.
 *
 * Parity pinning: checked against every reference fixture under tests/golden/v{3,4}_compat (copied
 * data files of recordio/test_files) and the expectations the reference's own tests assert
 * (tests/golden/expectations.json, tests/test_oracle_golden.py). The Go reference cannot be built
 * here (no Go toolchain), so the fixtures + test assertions are the pin.
 * Status vocabulary: include/rio.h.
 */
#ifndef RIO_ORACLE_H
#define RIO_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_file_result {
    uint32_t version, compression;
    uint64_t n_records;
    uint64_t total_out_bytes;
    int32_t status;
    uint64_t status_offset;
    uint64_t detail0, detail1;
    uint8_t* out;       /* malloc'd, total_out_bytes */
    uint64_t* out_off;  /* malloc'd, n_records + 1 */
    uint64_t* rec_off;  /* malloc'd, n_records */
    uint8_t* flags;     /* malloc'd, n_records: RIO_FLAG_NIL / CORRUPT / EOF */
    uint64_t first_bad; /* first record whose payload does not decompress (UINT64_MAX: none) */
    uint64_t n_bad;
} orc_file_result;

uint32_t orc_crc32c(const uint8_t* p, uint64_t n);
/* readFileHeaderFromBuffer (common_reader.go:22-44) on the first 8 bytes */
int orc_file_header(const uint8_t* f, uint64_t len, uint32_t* version, uint32_t* compression,
                    uint64_t* detail);
/* FileReader Open + ReadNext loop until the first error that is not a codec error (file_reader.go:
 * 26-131, 389-447; v1/v2 legacy paths :282-360, read only so the reference's SSTable fixtures can pin
 * the checker). A payload that does not decompress was consumed before the codec ran (:113-122,
 * :430-439), so the loop goes on: such a record gets RIO_FLAG_CORRUPT (RIO_FLAG_EOF for gzip's empty
 * payload) and the output length the device reserves for it (usable snappy preamble / plausible gzip
 * ISIZE, else 0), filled with zeros. */
int orc_file_reader_decode(const uint8_t* f, uint64_t len, orc_file_result* res);
void orc_file_result_free(orc_file_result* res);
/* MMapReader.ReadNextAt (mmap_reader.go:130-203 v4, 298-356 v3). *out is malloc'd (NULL for nil). */
int orc_read_next_at(const uint8_t* f, uint64_t len, uint64_t offset, uint8_t** out,
                     uint64_t* out_len, int* is_nil, uint64_t* detail0, uint64_t* detail1);
/* MMapReader.SeekNext (mmap_reader.go:58-128) with window seek_len (4096 by default, :370); on a
 * trial ReadNextAt error *rec_offset is that trial's offset */
int orc_seek_next(const uint8_t* f, uint64_t len, uint64_t offset, uint64_t seek_len,
                  uint64_t* rec_offset, uint8_t** out, uint64_t* out_len, int* is_nil);
/* snappy.Decode of golang/snappy v1.0.0 (decode.go + decode_other.go). *out malloc'd. */
int orc_snappy_decode(const uint8_t* src, uint64_t n, uint8_t** out, uint64_t* out_len);
/* lzw.NewReader(LSB, 8) drained (LzwCompressor.DecompressWithBuf, lzw_compressor.go:52-63) and
 * lzw.NewWriter(LSB, 8) Write + Close (:12-26; dst capacity >= 2 n + 16). *out malloc'd. */
int orc_lzw_decode(const uint8_t* src, uint64_t n, uint8_t** out, uint64_t* out_len);
uint64_t orc_lzw_encode(uint8_t* dst, const uint8_t* src, uint64_t n);
/* bytes an lzw record may decode to per payload byte, above which the device does not size a
 * record by its header's u (a 9-bit code yields at most 4096 bytes) */
#define ORC_LZW_MAX_RATIO 4096ull
void orc_free(void* p);
/* multi-threaded CPU baseline: record-parallel ReadNextAt over a known offset table; returns
 * decoded bytes (0 on error). threads <= 0 => 1. */
uint64_t orc_parallel_read_at(const uint8_t* f, uint64_t len, const uint64_t* rec_off, uint64_t n,
                              int threads);

/* sstables: CRC-64/ISO of a value (checksumValue, sstable_reader.go:240-248) */
uint64_t orc_crc64_iso(const uint8_t* p, uint64_t n);
/* sstables: proto.Unmarshal of an IndexEntry record (sstables/proto/sstable.proto:5-9); the key is
 * b[key_off, key_off + key_len). 0 ok, -1 malformed. */
int orc_index_entry(const uint8_t* b, uint64_t n, uint64_t* key_off, uint64_t* key_len, uint64_t* value_off,
                    uint64_t* checksum);
/* sstables: index load + validateDataFile + Scan over in-memory images (CPU baseline of config 5);
 * entries scanned, *first_bad = first checksum mismatch or UINT64_MAX */
/* DiskKeyIndex.binarySearch over a fresh index (disk_key_index.go:87-127); ORC_ERR_PROTO = 21 */
int orc_disk_index_search(const uint8_t* f, uint64_t len, const uint8_t* key, uint64_t klen, uint64_t seek_len,
                          uint64_t* offset, int* found, uint64_t* value_off, uint64_t* checksum);
/* FileWriter.Write over a batch with golang/snappy v1.0.0 (write-side checker / CPU baseline) */
uint64_t orc_snappy_encode(uint8_t* dst, const uint8_t* src, uint64_t n);
uint64_t orc_encode_file(const uint8_t* records, const uint64_t* off, const uint8_t* flags, uint64_t n, uint32_t comp,
                         uint8_t* out, uint64_t cap, uint64_t* rec_off);
int orc_data_entry(const uint8_t* b, uint64_t n, int* present, uint64_t* value_off, uint64_t* value_len);
uint64_t orc_sst_scan(const uint8_t* index, uint64_t ilen, const uint8_t* data, uint64_t dlen, uint64_t* first_bad);

#ifdef __cplusplus
}
#endif
#endif
