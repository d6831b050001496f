/*
 * rio.h — C-ABI of the MI355X-native recordio decode path (v3/v4, and the legacy v1/v2 layouts).
 *
 * This is the drop-in boundary a Go `recordio` adapter (behind `//go:build cgo && rocm`) binds
 * with cgo; see INTEGRATION.md for the binding. Plain pointers and sizes only, no torch/HIP types
 * in any signature (a HIP stream is passed as `void*`). The library never retains a caller pointer
 * after a call returns.
 *
 * Reference interfaces replaced (github.com/thomasjungblut/go-sstables, paths relative to the repo):
 *   recordio.ReaderI  {Open, Close, ReadNext, SkipNext}          recordio/recordio.go:83-89
 *   recordio.ReadAtI  {Open, Close, Size, ReadNextAt, SeekNext}   recordio/recordio.go:91-105
 *   NewFileReaderWithPath / NewFileReader                         recordio/file_reader.go:490-524
 *   NewMemoryMappedReaderWithPath                                 recordio/mmap_reader.go:364-371
 *   FileReader.ReadNext v4 / v3 (sequential whole-file semantics) recordio/file_reader.go:61-131, 389-447
 *     readNextV2 / readNextV1                                     recordio/file_reader.go:322-388, 282-320
 *   MMapReader.ReadNextAt v4 / v3                                 recordio/mmap_reader.go:130-203, 298-356
 *     readNextAtV2 / readNextAtV1                                 recordio/mmap_reader.go:242-296, 205-240
 *   MMapReader.SeekNext                                           recordio/mmap_reader.go:58-128
 *   readFileHeaderFromBuffer                                      recordio/common_reader.go:22-44
 *   readRecordHeaderV1 / V2                                       recordio/common_reader.go:46-81
 *   readRecordHeaderV3 / V4 + checksumByteReader                  recordio/common_reader.go:83-151,
 *                                                                 recordio/checksum_byte_reader.go:11-60
 *   SnappyCompressor.DecompressWithBuf (golang/snappy v1.0.0)     recordio/compressor/snappy_compression.go:22-24
 *   NewSSTableReader load / validateDataFile / Scan (rio_sst_*)   sstables/sstable_reader.go:250-345, 205-238, 119-159
 *   DiskKeyIndex binarySearch (rio_index_*)                       sstables/disk_key_index.go:87-140
 *   wal.Replayer.Replay (rio_replay_*)                            wal/replayer.go:18-77
 *   FileWriter.Write + fillRecordHeaderV4 (input generator only)  recordio/file_writer.go:160-233
 */
#ifndef RIO_H
#define RIO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------------------------ */
/* Format constants (recordio/recordio.go:11-43)                                               */
/* ------------------------------------------------------------------------------------------ */
#define RIO_VERSION1 1u
#define RIO_VERSION2 2u
#define RIO_VERSION3 3u
#define RIO_VERSION4 4u
#define RIO_MAGIC 0x130691u /* MagicNumberSeparatorLong, uvarint bytes 91 8d 4c */
#define RIO_FILE_HEADER_BYTES 8u
#define RIO_RECORD_HEADER_V1_BYTES 20u /* RecordHeaderSizeBytesV1V2: LE u32 magic, LE u64 u, LE u64 c */
#define RIO_RECORD_HEADER_V3_MAX 31u /* RecordHeaderV3MaxSizeBytes */
#define RIO_RECORD_HEADER_V4_MAX 36u /* RecordHeaderV4MaxSizeBytes */
#define RIO_COMP_NONE 0u
#define RIO_COMP_GZIP 1u
#define RIO_COMP_SNAPPY 2u
#define RIO_COMP_LZW 3u
/* Device input buffers handed to rio_device_decode must have this many readable bytes past
 * `len` (the kernels load whole aligned 16-B words around headers; bytes past `len` are never
 * interpreted). */
#define RIO_DEVICE_PAD 64u

/* ------------------------------------------------------------------------------------------ */
/* Status codes: one per error class the reference's readers distinguish.                     */
/* `rio_status_is_eof(s)` answers `errors.Is(err, io.EOF)` for the error the reference returns. */
/* ------------------------------------------------------------------------------------------ */
typedef enum rio_status {
    RIO_OK = 0,
    /* header read hit EOF before its first byte: FileReader wraps io.EOF once
     * (file_reader.go:93), MMapReader.ReadNextAt returns a bare io.EOF (mmap_reader.go:153-155) */
    RIO_EOF = 1,
    /* FileReader only: magic mismatch and every byte after the consumed magic varint is zero
     * (DirectIO padding) -> bare io.EOF (file_reader.go:76-91) */
    RIO_EOF_ZERO_TAIL = 2,
    /* io.EOF on the first byte of a later header field (nil byte / u / c / crc varint) */
    RIO_EOF_HEADER = 3,
    /* payload read classified as io.EOF: FileReader io.ReadFull read 0 bytes (file_reader.go:104-107);
     * MMapReader any short ReadAt (mmap_reader.go:175-178) */
    RIO_EOF_PAYLOAD = 4,
    RIO_ERR_UNEXPECTED_EOF = 5,   /* io.ErrUnexpectedEOF (partial varint / partial payload) */
    RIO_ERR_MAGIC = 6,            /* MagicNumberMismatchErr (common_reader.go:19) */
    RIO_ERR_HEADER_CRC = 7,       /* HeaderChecksumMismatchErr (common_reader.go:20,140-148) */
    RIO_ERR_VARINT_OVERFLOW = 8,  /* binary.ReadUvarint overflow */
    RIO_ERR_HEADER_TOO_LONG = 9,  /* "checksum byte reader out of range" (checksum_byte_reader.go:25-27) */
    RIO_ERR_DECOMPRESS = 10,      /* codec error (snappy ErrCorrupt, gzip errors) */
    RIO_ERR_VERSION = 11,         /* "version mismatch, expected a value from 1 to 4 but was N" */
    RIO_ERR_COMPRESSION_TYPE = 12,/* "unknown compression type [N]" */
    RIO_ERR_SHORT_FILE_HEADER = 13,/* fewer than 8 bytes in the file */
    RIO_ERR_INVALID_OFFSET = 14,  /* "mmap: invalid ReadAt offset N" (offset > size) */
    RIO_ERR_UNSUPPORTED = 15,     /* a request the GPU path does not serve (SeekNext on v1 files
                                     mmap_reader.go:62-64; see DESIGN.md §8 for the rest) */
    RIO_ERR_CAPACITY = 16,        /* caller-provided output arrays too small */
    RIO_ERR_ARG = 17,             /* bad argument */
    RIO_ERR_HIP = 18,             /* HIP runtime failure */
    RIO_ERR_STATE = 19,           /* reader not opened / already closed / already opened */
    RIO_ERR_IO = 20,              /* file open / mmap / read failure */
    RIO_ERR_PROTO = 21,           /* proto.Unmarshal of an IndexEntry failed (invalid wire format) */
    /* the codec returned io.EOF: gzip.NewReader on an empty payload (gzip_compression.go:56-59).
     * FileReader.ReadNext returns it bare (file_reader.go:119-121), MMapReader.ReadNextAt wraps it
     * once ("failed decompressing record", mmap_reader.go:189-191); errors.Is(err, io.EOF) holds */
    RIO_EOF_CODEC = 22,
    RIO_STATUS_COUNT_ = 22
} rio_status;

const char* rio_strerror(int status);
int rio_status_is_eof(int status);
const char* rio_build_info(void);

/* ------------------------------------------------------------------------------------------ */
/* Whole-file decode result.                                                                   */
/* Sequential semantics: `n_records` records are delivered in file order, then `status`.       */
/* A clean end is one of the RIO_EOF family. Records with index < n_records are valid even if   */
/* status is an error: the reference's ReadNext loop returns them before the error.            */
/* A record whose payload fails to decompress does not end the sequence: FileReader.ReadNext     */
/* returns the codec error for it and the next call reads the record after it (the payload was   */
/* consumed, file_reader.go:101-125), so such a record is delivered with RIO_FLAG_CORRUPT (or    */
/* RIO_FLAG_EOF for gzip's empty payload) and the records after it are decoded. Its slice of     */
/* `out` has the length its payload announced (snappy preamble, gzip ISIZE; 0 when that is       */
/* unusable) and unspecified bytes. first_bad / n_bad summarise the flagged records.             */
/* ------------------------------------------------------------------------------------------ */
typedef struct rio_file_info {
    uint32_t version;         /* file header version (1..4) */
    uint32_t compression;     /* file header compression type (0..3) */
    uint64_t n_records;       /* records delivered before `status` */
    uint64_t total_out_bytes; /* sum of decoded record lengths of those records */
    int32_t status;           /* terminal status of the ReadNext loop */
    uint32_t reserved0;
    uint64_t status_offset;   /* file offset of the record header at which `status` was raised */
    uint64_t detail0;         /* HEADER_CRC: expected crc; VERSION/COMPRESSION_TYPE: value */
    uint64_t detail1;         /* HEADER_CRC: actual crc */
    uint64_t n_chunks;        /* framing chunks used (diagnostic) */
    uint64_t n_repairs;       /* chunks whose speculative entry had to be re-walked (diagnostic) */
    uint64_t first_bad;       /* first record flagged RIO_FLAG_CORRUPT / RIO_FLAG_EOF (~0: none) */
    uint64_t n_bad;           /* records so flagged (< n_records) */
} rio_file_info;

/* Per-record flag bits (rio_decode `flags`) */
#define RIO_FLAG_NIL 0x1u     /* record written as nil: ReadNext returns nil, not []byte{} */
#define RIO_FLAG_CORRUPT 0x2u /* the payload does not decompress: ReadNext returns the codec error
                                 (snappy ErrCorrupt / the gzip reader's error) for this record */
#define RIO_FLAG_EOF 0x4u     /* gzip: empty payload, gzip.NewReader's bare io.EOF for this record
                                 (gzip_compression.go:56-59, passed through by file_reader.go:118-121) */

/* ------------------------------------------------------------------------------------------ */
/* Context: one HIP device + stream + device arenas + pinned staging. NOT thread-safe: use one  */
/* per goroutine / host thread. Independent files on different devices need no communication. */
/* ------------------------------------------------------------------------------------------ */
typedef struct rio_ctx rio_ctx;

int rio_ctx_create(int device, rio_ctx** out);
void rio_ctx_destroy(rio_ctx* ctx);
int rio_device_count(int* out);
int rio_ctx_device(const rio_ctx* ctx); /* the context's device, -1 for NULL */
/* Pooled contexts for per-file readers (the Go adapter's FileReader.Open / Close,
 * file_reader.go:26-59): rio_ctx_acquire hands out an idle context of `device` from a process-wide
 * pool (creating one when none is idle), rio_ctx_release returns it (up to 4 idle per device are
 * kept, the rest destroyed). A fresh context grows every device arena on its first file (12-16 ms
 * for a 128 MiB file against 4.7 ms warm), so a reader per file should not create one. */
int rio_ctx_acquire(int device, rio_ctx** out);
void rio_ctx_release(rio_ctx* ctx);

/* ---- host-memory two-phase API (the cgo binding: one call pair per file) --------------------
 * rio_frame: H2D copy of the file through pinned staging, device framing (record boundaries,
 * header CRC, decoded sizes) and the scan; fills `info` (sizes the caller must allocate). For a
 * gzip file rio_frame also decodes it (a record of several gzip members is larger than its last
 * member's ISIZE, the framing's size, which only the decode finds out), so the sizes are exact.
 * rio_decode: device decode of every framed record + D2H of the results into caller buffers:
 *   out      [>= info->total_out_bytes]  concatenated record bytes
 *   out_off  [n_records + 1]             record i = out[out_off[i] .. out_off[i+1])
 *   rec_off  [n_records]                 file offset of record i's header (ReadNextAt offset)
 *   flags    [n_records]                 RIO_FLAG_NIL / RIO_FLAG_CORRUPT / RIO_FLAG_EOF
 * rio_decode fills info->first_bad / n_bad (records that fail to decompress are flagged, not cut). */
int rio_frame(rio_ctx* ctx, const uint8_t* file, uint64_t len, rio_file_info* info);
int rio_decode(rio_ctx* ctx, uint8_t* out, uint64_t out_cap, uint64_t* out_off, uint64_t* rec_off,
               uint8_t* flags, uint64_t rec_cap, rio_file_info* info);
/* rio_host_register / rio_host_unregister: page-lock a host buffer the caller reuses for file images
 * (hipHostRegister). rio_frame and rio_stream_open_host then copy such an image to the device by DMA
 * in place instead of through the pinned staging pieces; results are the same either way. No
 * reference counterpart: the cgo adapter would register its read buffer pool once.
 * Unregister such a range with rio_host_unregister; a range unlocked behind the library's back is
 * detected (hipPointerGetAttributes) and copied through staging. */
int rio_host_register(const void* p, uint64_t n);
int rio_host_unregister(const void* p);

/* ---- device-resident API: the file is already in HBM; everything runs on `stream` with no host
 * synchronisation (graph-capturable). Outputs are device pointers with the layout above; the
 * result struct is written to device memory `d_info`. `d_file` must have RIO_DEVICE_PAD readable
 * bytes past `len`. If the decoded size exceeds out_cap or rec_cap, d_info->status is
 * RIO_ERR_CAPACITY with the sizes needed in d_info and nothing usable is decoded (call again with
 * outputs of that size). A gzip file whose records of several members outgrow the framing's sizes
 * reports this only after its decode: a capacity-0 probe can undersize it, so loop on CAPACITY.
 * `stream` is a hipStream_t (NULL = the ctx stream). */
/* Calls of one ctx share its device scratch: a device-API call on a stream other than the previous
 * call's waits (stream-ordered) for that call. Arenas grow on demand (hipMalloc); before capturing
 * calls into a hipGraph, size them with rio_ctx_reserve (largest file length, record count and batch
 * size to come) so that nothing is allocated during capture, and capture on the stream of the
 * previous call. */
int rio_ctx_reserve(rio_ctx* ctx, uint64_t max_file_len, uint64_t max_records, uint32_t max_batch);
/* Device bytes the ctx's framing and decode arenas hold (grow-only; no reference counterpart): constant across
 * calls after rio_ctx_reserve, whichever walk the automatic choice takes for each file. */
uint64_t rio_ctx_arena_bytes(const rio_ctx* ctx);
int rio_device_decode(rio_ctx* ctx, const uint8_t* d_file, uint64_t len, uint8_t* d_out,
                      uint64_t out_cap, uint64_t* d_out_off, uint64_t* d_rec_off, uint8_t* d_flags,
                      uint64_t rec_cap, rio_file_info* d_info, void* stream);
/* Same as rio_device_decode for a file whose 8-byte header the caller has already read (an mmap'd or
 * uploaded file): `compression` is its compression type, so only that codec's decode kernels are
 * launched (a Snappy file: 6 launches). RIO_COMP_UNKNOWN launches every decoder, as
 * rio_device_decode does. A file whose header contradicts the hint comes back as RIO_ERR_ARG. */
#define RIO_COMP_UNKNOWN 0xFFFFFFFFu
int rio_device_decode_ex(rio_ctx* ctx, const uint8_t* d_file, uint64_t len, uint32_t compression, uint8_t* d_out,
                         uint64_t out_cap, uint64_t* d_out_off, uint64_t* d_rec_off, uint8_t* d_flags, uint64_t rec_cap,
                         rio_file_info* d_info, void* stream);
/* Batch form: n_files device-resident files, file k = d_files[k] (lens[k] bytes, 16-byte aligned,
 * RIO_DEVICE_PAD readable bytes past it) decoded into its own outputs (d_out[k] ... d_info[k], as for
 * rio_device_decode). The arrays of pointers are host arrays; everything runs on `stream` without
 * host synchronisation. Replaces a loop of FileReader / MMapReader opens over a directory or shard
 * (wal/replayer.go:18-77, BASELINE configs[3]): the large-record decoder runs once across the files. */
int rio_device_decode_batch(rio_ctx* ctx, uint32_t n_files, const uint8_t* const* d_files, const uint64_t* lens,
                            uint8_t* const* d_out, const uint64_t* out_cap, uint64_t* const* d_out_off,
                            uint64_t* const* d_rec_off, uint8_t* const* d_flags, const uint64_t* rec_cap,
                            rio_file_info* const* d_info, void* stream);
/* Upper bound on records in a file of `len` bytes (the smallest record is v2's empty one, 5 bytes:
 * magic, u = 0, c = 0; v3 / v4 / v1 take 6 / 7 / 20). */
uint64_t rio_max_records(uint64_t len);
/* Kernel-timing probe for benchmarks: per-stage device milliseconds (walk, scan, placement, decode) averaged
 * over the decodes recorded since rio_ctx_set_timing; fills up to n entries, returns the count (0 when timing
 * is off). rio_ctx_set_timing(ctx, slots): record HIP events around the stages of the next `slots` calls
 * (a ring; 0 = off, the default: the events cost ~3 us each per call). */
int rio_ctx_last_stage_ms(rio_ctx* ctx, float* ms, int n);
int rio_ctx_set_timing(rio_ctx* ctx, int enable);

/* ---- sstables on the device (sstables/sstable_reader.go). Both calls work on arenas produced by
 * rio_device_decode of index.rio / data.rio, run on `stream` (NULL = ctx stream), no host sync.
 *
 * rio_sst_index_parse replaces SliceKeyIndexLoader.Load's per-record proto.Unmarshal into an
 * IndexEntry (slice_key_index.go:91-131, sstables/proto/sstable.proto:5-9). Record i of the index
 * arena (d_index_out[d_index_off[i] .. d_index_off[i+1])) -> key bytes at
 * d_index_out[d_key_off[i] .. + d_key_len[i]), valueOffset, checksum (absent fields = 0).
 * d_result[0] = first malformed record (proto error: the reference's Load fails there) or ~0.
 *
 * rio_sst_validate replaces validateDataFile (sstable_reader.go:205-238) and the
 * SSTableFullScanIterator's optional hash check (sstable_iterator.go:77-111): for every index entry,
 * the value is the data record whose file offset is valueOffset (getValueAtOffset, :85-92), its
 * CRC-64/ISO (checksumValue, :240-248) goes to d_crc_out[i]. d_result[0] = first entry whose
 * non-zero checksum mismatches (ChecksumError), d_result[1] = first entry not in the writer's
 * layout (valueOffset != data record i's offset: keep the reference reader); ~0 = none. */
int rio_sst_index_parse(rio_ctx* ctx, const uint8_t* d_index_out, const uint64_t* d_index_off, uint64_t n,
                        uint64_t* d_key_off, uint64_t* d_key_len, uint64_t* d_value_off, uint64_t* d_checksum,
                        uint64_t* d_result, void* stream);
int rio_sst_validate(rio_ctx* ctx, const uint8_t* d_data_out, const uint64_t* d_data_off,
                     const uint64_t* d_data_rec_off, uint64_t n_data, const uint64_t* d_value_off,
                     const uint64_t* d_checksum, uint64_t n_index, uint64_t* d_crc_out, uint64_t* d_result,
                     void* stream);
/* v0 tables (metadata version 0: values are protobuf DataEntry {value = 1}, sstable_reader.go:303-314,
 * sstables/proto/sstable.proto:12-14). rio_sst_data_entries replaces the proto.Unmarshal of every value
 * record (MMapProtoReader.ReadNextAt / ProtoReader.ReadNext, recordio/proto/mmap_proto_reader.go:12-24)
 * on the decoded data arena: d_view[2j], d_view[2j+1] = [begin, end) of record j's DataEntry.value in
 * d_data_out, both RIO_VALUE_NIL when the field is absent (value nil) and RIO_VALUE_BAD when the
 * record is not a valid DataEntry ("proto: cannot parse invalid wire-format data").
 * d_result[0] = first malformed record or ~0. rio_sst_validate_view is rio_sst_validate over those
 * ranges (a nil or malformed value hashes as empty). */
#define RIO_VALUE_NIL (~0ull)
#define RIO_VALUE_BAD (~0ull - 1)
int rio_sst_data_entries(rio_ctx* ctx, const uint8_t* d_data_out, const uint64_t* d_data_off, uint64_t n_data,
                         uint64_t* d_view, uint64_t* d_result, void* stream);
int rio_sst_validate_view(rio_ctx* ctx, const uint8_t* d_data_out, const uint64_t* d_data_off,
                          const uint64_t* d_data_rec_off, uint64_t n_data, const uint64_t* d_view,
                          const uint64_t* d_value_off, const uint64_t* d_checksum, uint64_t n_index,
                          uint64_t* d_crc_out, uint64_t* d_result, void* stream);

/* ---- sstables, host-memory API (the cgo binding: one call per table) ------------------------
 * rio_sst_open replaces NewSSTableReader's load (sstable_reader.go:250-345) for the tables the device
 * path handles: H2D of index.rio and data.rio, device decode of both, IndexEntry parse and the CRC-64
 * of every value on the device (the two calls above), D2H of what the iterator needs. The handle owns
 * host copies; pointers from rio_sst_entry stay valid until rio_sst_free.
 * Returns RIO_ERR_UNSUPPORTED (no handle, `info` filled) when either file is one the device path hands
 * back (none of recordio v1..v4 is; the code stays for the adapter's contract). Otherwise the
 * handle is returned and `info` says which of the reference's load errors applies: index/data status
 * outside the EOF family (reading error), first_bad_proto (proto.Unmarshal error, slice_key_index.go:
 * 107-110), first_unplaced (not the writer's layout: keep the reference reader), first_bad_crc
 * (validateDataFile's ChecksumError, sstable_reader.go:205-238, unless SkipHashCheckOnLoad), and
 * data.first_bad (a value that does not decompress: validateDataFile's ReadNextAt error). Of
 * first_bad_crc and data.first_bad the smaller entry is the one validateDataFile stops at; on a tie it
 * is the read error (a flagged value's CRC is not meaningful). */
typedef struct rio_sst_info {
    rio_file_info index;      /* ReadNext loop over index.rio */
    rio_file_info data;       /* ReadNext loop over data.rio */
    uint64_t n_entries;       /* index records = IndexEntries */
    uint64_t first_bad_proto; /* ~0 = none */
    uint64_t first_bad_crc;   /* ~0 = none */
    uint64_t first_unplaced;  /* ~0 = none */
    uint64_t index_bad;       /* first index record that does not decompress (RIO_FLAG_CORRUPT): Load's
                                 ReadNext error there, before any later index status; ~0 = none.
                                 n_entries stops at the first flagged index record (gzip's bare io.EOF
                                 ends the index cleanly, slice_key_index.go:117-126) */
    uint64_t first_bad_value; /* v0 tables: first data record that is not a valid DataEntry; ~0 = none */
} rio_sst_info;
typedef struct rio_sst rio_sst;
int rio_sst_open(rio_ctx* ctx, const uint8_t* index_file, uint64_t index_len, const uint8_t* data_file,
                 uint64_t data_len, rio_sst** out, rio_sst_info* info);
/* flags: RIO_SST_V0_VALUES for a table whose metadata version is 0 (no meta.pb.bin, or version 0):
 * values are DataEntry protos (rio_sst_data_entries), rio_sst_entry returns DataEntry.value and
 * RIO_ERR_PROTO for a malformed one; validateDataFile does not run for such tables (:205-209), so
 * first_bad_crc is left ~0 and crc still holds each value's CRC-64. */
#define RIO_SST_V0_VALUES 1u
int rio_sst_open_ex(rio_ctx* ctx, const uint8_t* index_file, uint64_t index_len, const uint8_t* data_file,
                    uint64_t data_len, uint32_t flags, rio_sst** out, rio_sst_info* info);
/* Entry i in index order (SSTableFullScanIterator.Next, sstable_iterator.go:77-111): key, the value of
 * data record i (is_nil for a nil record), the stored valueOffset and checksum and the value's CRC-64.
 * Returns RIO_OK, RIO_ERR_ARG for i >= n_entries, the data file's terminal status when data record i
 * does not exist (the scan's dataReader.ReadNext error; key and checksum are still filled), or
 * RIO_ERR_DECOMPRESS / RIO_EOF_CODEC when data record i is flagged RIO_FLAG_CORRUPT / RIO_FLAG_EOF. */
int rio_sst_entry(const rio_sst* t, uint64_t i, const uint8_t** key, uint64_t* key_len, const uint8_t** value,
                  uint64_t* value_len, int* is_nil, uint64_t* value_offset, uint64_t* checksum, uint64_t* crc);
void rio_sst_free(rio_sst* t);

/* ---- recordio v4 encoding on the device (the write side: FileWriter.Write for a batch) --------
 * Replaces a loop of FileWriter.Write (recordio/file_writer.go:189-233; compaction output,
 * sstable_merger.go:36-169): record i = d_records[d_rec_off[i] .. d_rec_off[i+1]) (RIO_DEVICE_PAD
 * readable bytes past the arena end), d_flags[i] & RIO_FLAG_NIL marks a nil record (d_flags NULL =
 * none), compression RIO_COMP_NONE or RIO_COMP_SNAPPY (golang/snappy v1.0.0 block encoding). The
 * whole v4 file (8-byte header + records) goes to d_out, byte-identical to the reference writer; record
 * i's file offset (what Write returns) to d_out_rec_off[i], the file length to *d_out_len. With
 * out_cap >= rio_encode_bound(n, total_bytes) the file always fits; otherwise nothing is written
 * when *d_out_len > out_cap. Stream-ordered, no host sync. total_bytes = d_rec_off[n]. */
uint64_t rio_encode_bound(uint64_t n_records, uint64_t total_bytes, uint32_t compression);
int rio_device_encode(rio_ctx* ctx, const uint8_t* d_records, const uint64_t* d_rec_off, const uint8_t* d_flags,
                      uint64_t n, uint64_t total_bytes, uint32_t compression, uint8_t* d_out, uint64_t out_cap,
                      uint64_t* d_out_rec_off, uint64_t* d_out_len, void* stream);
/* host-memory form (the cgo binding): H2D of the records, device encode, D2H of the file image and
 * offsets; *out_len = file length (RIO_ERR_CAPACITY when it exceeds out_cap). Synchronises. */
int rio_encode_file(rio_ctx* ctx, const uint8_t* records, const uint64_t* rec_off, const uint8_t* flags, uint64_t n,
                    uint32_t compression, uint8_t* out, uint64_t out_cap, uint64_t* out_rec_off, uint64_t* out_len);

/* ---- DiskKeyIndex lookups (sstables/disk_key_index.go:87-140) --------------------------------
 * Batched DiskKeyIndex.Get / Contains / IteratorStartingAt: one result per query key, each the
 * reference's binarySearch over the byte offsets of an uncompressed index.rio with every probe
 * findAt(h) = SeekNext(h) + proto.Unmarshal(IndexEntry), exactly as a freshly loaded DiskKeyIndex
 * runs it (the reference's offsetCache is per index and may keep an empty entry at an offset whose
 * probe hit io.EOF; later lookups on the same Go object then see that entry: see DESIGN.md §8).
 *   status  RIO_OK (no error; `found` tells Get / Contains), else findAt's error: SeekNext's
 *           non-EOF error (e.g. RIO_ERR_UNEXPECTED_EOF) or RIO_ERR_PROTO. RIO_ERR_UNSUPPORTED for a
 *           v1 index (SeekNext's "unsupported on files with version lower than v2", mmap_reader.go:62-64),
 *           and from rio_device_index_search for a compressed one (keep the reference index); the
 *           rio_index handle answers compressed indexes from their decoded view.
 *   offset  binarySearch's offset (IteratorStartingAt starts there; size when an io.EOF probe ended it)
 *   value_offset / checksum  IndexVal when found. */
typedef struct rio_index_hit {
    uint64_t offset;
    uint64_t value_offset;
    uint64_t checksum;
    int32_t status;
    int32_t found;
} rio_index_hit;
/* device-resident: d_file (RIO_DEVICE_PAD readable bytes past len), query i = d_keys[d_key_off[i] ..
 * d_key_off[i+1]), results to d_hits[n]; seek_len 0 = 4096 (mmap_reader.go:370); no host sync */
int rio_device_index_search(rio_ctx* ctx, const uint8_t* d_file, uint64_t len, uint64_t seek_len,
                            const uint8_t* d_keys, const uint64_t* d_key_off, uint64_t n, rio_index_hit* d_hits,
                            void* stream);
/* host-memory handle (the cgo DiskIndexLoader.Load / Get binding): the index file stays resident in
 * HBM; each search copies the keys in and the hits out (synchronises). A compressed index.rio is
 * decoded once at open (records + the SeekNext map over the file) and searched from that view
 * (disk_key_index.go:173 reads it through an MMapReader, which decompresses every record). */
typedef struct rio_index rio_index;
int rio_index_open(rio_ctx* ctx, const uint8_t* file, uint64_t len, rio_index** out);
int rio_index_search(rio_index* idx, const uint8_t* keys, const uint64_t* key_off, uint64_t n, rio_index_hit* hits);
void rio_index_free(rio_index* idx);

/* ---- ordered replay of a file list (the WAL replay adapter) ----------------------------------
 * Replaces the per-file loop of wal.Replayer.Replay (wal/replayer.go:18-77; the caller walks the
 * directory and sorts the *.wal paths as :20-37 does). A worker thread with its own context maps and
 * decodes file k+1.. on `device` while the caller consumes file k; at most `depth` (0 = 2) decoded
 * files are held ahead. `workers` (0 = 2, at most depth) threads each own a context and stream, so
 * one file's H2D overlaps another's decode and D2H. rio_replay_next hands out the files strictly in list order: it returns
 * RIO_EOF after the last one; otherwise that file's rc (RIO_OK, RIO_ERR_IO when it cannot be opened or
 * mapped, RIO_ERR_HIP) with `info` and the arrays of rio_decode (out / out_off[n+1] / flags[n]), valid
 * until the next rio_replay_next or rio_replay_free. Deliver records < info.n_records, then map
 * info.status like FileReader.ReadNext's terminal error; when info.n_bad, stop at record
 * info.first_bad instead: RIO_FLAG_EOF ends this file (replayer.go:60-63), RIO_FLAG_CORRUPT ends the
 * replay with the codec error (:65-67). A file with info.status RIO_ERR_UNSUPPORTED
 * must be re-read whole by the reference reader before any of its records is delivered. */
typedef struct rio_replay rio_replay;
int rio_replay_open(int device, const char* const* paths, uint64_t n_paths, uint32_t depth, uint32_t workers,
                    rio_replay** out);
/* The same over several GPUs of one node (one host thread + context per GPU, no
 * communication): workers_per_device workers per device, worker w on devices[w % n_devices], file i
 * to worker i % W; files are still handed out strictly in list order. A device may be listed twice
 * (two workers' contexts on one GPU). depth (0 = 2) is raised to the worker count
 * workers_per_device * n_devices (0 = 2 per device), so every worker has a file in flight. */
int rio_replay_open_devices(const int* devices, uint32_t n_devices, const char* const* paths, uint64_t n_paths,
                            uint32_t depth, uint32_t workers_per_device, rio_replay** out);
int rio_replay_next(rio_replay* r, uint64_t* index, const uint8_t** out, const uint64_t** out_off,
                    const uint8_t** flags, rio_file_info* info);
void rio_replay_free(rio_replay* r);

/* ---- windowed sequential decode of one file (FileReader.ReadNext, file_reader.go:61-131, over a
 * file larger than the staging it should take: SURVEY §8b "one cgo call per window") -----------
 * The file is framed and decoded in windows of about `window_bytes` (0 = 128 MiB; a record larger
 * than a window doubles it) cut at record boundaries: one window's H2D overlaps the previous one's
 * decode and D2H on a second context. At most `depth` (0 = 4) decoded windows are held ahead.
 * rio_stream_next hands out the windows in file order: rc RIO_OK (or RIO_ERR_IO / RIO_ERR_HIP)
 * with the window's records — out / out_off[n+1] (window-relative) / rec_off[n] (file offsets of
 * the record headers) / flags[n], valid until the next rio_stream_next or rio_stream_free — and
 * `first_record`, the file-wide index of its first record. info.status is RIO_OK while more windows
 * follow; the last window carries the file's terminal status as the whole-file rio_frame /
 * rio_decode pair reports it (status_offset a file offset; the failing record's index is
 * first_record + info.n_records). info.first_bad / n_bad cover the window's flagged records
 * (first_bad a file-wide index). RIO_EOF after the last window. RIO_ERR_UNSUPPORTED: the adapter
 * continues with the reference reader after SkipNext over the records already delivered.
 * rio_stream_open_host reads from host memory instead of a path (the caller keeps it alive until
 * rio_stream_free). */
/* ---- a file set over several GPUs (independent files sharded over the GPUs of a node,
 * the 8 tables of an SSTable set, a WAL directory decoded without ordering): rio_fileset_decode
 * assigns the files to `devices` longest-processing-time first on their sizes, runs one host thread
 * with a pooled context per device (read, H2D, device decode, D2H into page-locked blocks) and
 * returns when every file is decoded. rio_fileset_get: file i's arrays (layout as rio_replay_next,
 * plus rec_off[n]), its info, the device that decoded it; rc RIO_OK or the file's RIO_ERR_IO /
 * RIO_ERR_HIP. Valid until rio_fileset_free. A device may be listed twice. */
typedef struct rio_fileset rio_fileset;
int rio_fileset_decode(const int* devices, uint32_t n_devices, const char* const* paths, uint64_t n_paths,
                       rio_fileset** out);
int rio_fileset_get(const rio_fileset* s, uint64_t i, const uint8_t** out, const uint64_t** out_off,
                    const uint64_t** rec_off, const uint8_t** flags, rio_file_info* info, int* device);
void rio_fileset_free(rio_fileset* s);

typedef struct rio_stream rio_stream;
int rio_stream_open(int device, const char* path, uint64_t window_bytes, uint32_t depth, rio_stream** out);
int rio_stream_open_host(int device, const uint8_t* data, uint64_t len, uint64_t window_bytes, uint32_t depth,
                         rio_stream** out);
int rio_stream_next(rio_stream* s, uint64_t* first_record, const uint8_t** out, const uint64_t** out_off,
                    const uint64_t** rec_off, const uint8_t** flags, rio_file_info* info);
void rio_stream_free(rio_stream* s);

/* ---- single-record decode at an arbitrary offset (MMapReader.ReadNextAt semantics) on the
 * device; `d_file` device-resident. The decoded record is written to `d_out` (capacity out_cap);
 * *len_out / *nil_out / status go to host memory (this call synchronises). */
int rio_device_read_at(rio_ctx* ctx, const uint8_t* d_file, uint64_t len, uint64_t offset,
                       uint8_t* d_out, uint64_t out_cap, uint64_t* len_out, int* nil_out,
                       uint64_t* detail0, uint64_t* detail1);

/* ------------------------------------------------------------------------------------------ */
/* Reader handles mirroring recordio.ReaderI / recordio.ReadAtI on top of the device path.     */
/* Returned data pointers: ReadNext until Close (windowed file readers: until the next        */
/* ReadNext); ReadNextAt / SeekNext as documented at their declarations. The Go adapter        */
/* slices/copies them into Go memory.                                                           */
/* ------------------------------------------------------------------------------------------ */
typedef struct rio_reader rio_reader;

int rio_reader_new_file(rio_ctx* ctx, const char* path, rio_reader** out); /* NewFileReaderWithPath */
int rio_reader_new_mmap(rio_ctx* ctx, const char* path, rio_reader** out); /* NewMemoryMappedReaderWithPath */
int rio_reader_open(rio_reader* r);
int rio_reader_close(rio_reader* r);
void rio_reader_free(rio_reader* r);
int rio_reader_header(rio_reader* r, uint32_t* version, uint32_t* compression);
uint64_t rio_reader_size(rio_reader* r);
/* detail values of the last error (HEADER_CRC: expected/actual; VERSION etc.: value) */
void rio_reader_last_detail(rio_reader* r, uint64_t* detail0, uint64_t* detail1, uint64_t* offset);
/* ReaderI. read_next on a record that does not decompress returns RIO_ERR_DECOMPRESS (RIO_EOF_CODEC
 * for gzip's empty payload) and the next call returns the record after it; skip_next passes over it. */
int rio_reader_read_next(rio_reader* r, const uint8_t** data, uint64_t* len, int* is_nil);
int rio_reader_skip_next(rio_reader* r);
/* ReadAtI (recordio.go:91-105), thread-safe: any number of threads may call these on one handle.
 * The first call decodes the whole file once; after that ReadNextAt at a record start, and SeekNext
 * (seek_len >= 4) whose scan lands on a decoded record, are a binary search on the calling thread
 * (no kernel, no lock) and *data points into the reader's decoded arena, valid until rio_reader_free.
 * Other offsets run the single-record kernels on a per-call stream; *data is then valid until the
 * calling thread's next ReadNextAt / SeekNext. Detail values are per thread (rio_reader_last_detail). */
int rio_reader_read_next_at(rio_reader* r, uint64_t offset, const uint8_t** data, uint64_t* len,
                            int* is_nil);
int rio_reader_seek_next(rio_reader* r, uint64_t offset, uint64_t* rec_offset, const uint8_t** data,
                         uint64_t* len, int* is_nil);
/* MMapReader.seekLen (mmap_reader.go:370, default 4096; tests shrink it to 10) */
int rio_reader_set_seek_len(rio_reader* r, uint64_t seek_len);
/* whole-file result of a file reader after its (lazy) device decode (RIO_ERR_STATE when windowed) */
int rio_reader_file_info(rio_reader* r, rio_file_info* info);
/* File readers decode files larger than 256 MiB in 128 MiB windows (rio_stream_*); before the first
 * ReadNext / SkipNext this sets the window (files larger than it are windowed), or ~0 for whole-file
 * decode always, or 0 for the automatic policy. Records and errors are the same either way. */
int rio_reader_set_window(rio_reader* r, uint64_t window_bytes);

/* ------------------------------------------------------------------------------------------ */
/* Input generator (host): byte-identical to FileWriter for v4 files (file_writer.go:160-233);   */
/* Snappy records use a golang/snappy v1.0.0-compatible block encoder. Not on the decode path.  */
/* ------------------------------------------------------------------------------------------ */
typedef struct rio_writer rio_writer;
int rio_writer_new(const char* path, uint32_t compression, rio_writer** out);
/* record == NULL writes a nil record; returns the record's offset in *offset */
int rio_writer_write(rio_writer* w, const uint8_t* record, uint64_t len, uint64_t* offset);
uint64_t rio_writer_size(rio_writer* w);
int rio_writer_close(rio_writer* w);
/* In-memory encoder used by the generators: appends one record to buf (capacity cap), returns
 * bytes written or 0 if it does not fit. record == NULL => nil record. */
uint64_t rio_encode_record_v4(uint8_t* buf, uint64_t cap, uint32_t compression,
                              const uint8_t* record, uint64_t len);
void rio_encode_file_header(uint8_t* buf8, uint32_t version, uint32_t compression);
uint64_t rio_snappy_max_encoded_len(uint64_t n);
uint64_t rio_snappy_encode(uint8_t* dst, uint64_t dst_cap, const uint8_t* src, uint64_t n);
/* Synthetic workloads of BASELINE.json. Writes a complete v4 file
 * image into buf; returns its length (0 if cap too small). kind: 0 = ref-random (one record of
 * bytes in [0,254] repeated, benchmark/recordio_read_test.go:32-42), 1 = text-like (seeded
 * Zipf words, distinct per record), 2 = random bytes distinct per record. */
uint64_t rio_generate(uint8_t* buf, uint64_t cap, uint32_t compression, uint64_t n_records,
                      uint64_t record_len, int kind, uint64_t seed, int threads);
uint64_t rio_generate_bound(uint32_t compression, uint64_t n_records, uint64_t record_len);

#ifdef __cplusplus
}
#endif
#endif /* RIO_H */
