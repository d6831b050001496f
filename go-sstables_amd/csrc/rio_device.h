// rio_device.h — structures shared by the HIP kernels (rio_kernels.hip) and the host runtime
// (rio_capi.cpp). Internal to librio; the public boundary is include/rio.h.
#pragma once
#include <stdint.h>

#include "rio.h"

namespace rio {

constexpr uint64_t kNone = ~0ull;       // "no speculative entry found in this chunk"
// scratch_len: decoded length | flag bits
constexpr uint64_t kNilBit = 1ull << 63;  // nil record
constexpr uint64_t kBadBit = 1ull << 62;  // payload fails already at framing (codec preamble / size)
constexpr uint64_t kEofBit = 1ull << 61;  // gzip: empty payload (gzip.NewReader's io.EOF)
constexpr uint64_t kLenMask = kEofBit - 1;
constexpr uint32_t kDescWide = 0xFFFFFFFFu;  // rec_desc z = w = kDescWide: sizes in rec_pay (rec_stream)
// lanes of the Snappy lane decoder that met a corrupt record are listed for k_finish (re-checked there)
constexpr uint32_t kFailLanes = 1024;

// Snappy decode launch shape (k_snappy_pipe): every wave owns one 64-byte sink line that absorbs
// the pipeline's placeholder loads and stores.
constexpr unsigned kSnappyBlock = 256;
// RIO_SNAPPY_GRID: the launch grid (experiment builds: make variant VDEFS=-DRIO_SNAPPY_GRID=768); the
// sink is sized for up to kSnappyGridMax workgroups whatever the variant, so a build that changes the
// grid in rio_snappy.hip alone stays inside the context's sink
#ifndef RIO_SNAPPY_GRID
#define RIO_SNAPPY_GRID 512
#endif
constexpr unsigned kSnappyGrid = RIO_SNAPPY_GRID;
constexpr unsigned kSnappyGridMax = 1024;
static_assert(kSnappyGrid <= kSnappyGridMax, "sink sized for kSnappyGridMax workgroups");
constexpr uint64_t kSinkBytes = (uint64_t)kSnappyBlock / 64 * kSnappyGridMax * 64;

// Framing chunk: a byte range [cs, ce) of the file; a chunk OWNS the records whose header starts
// in its range. Written by the walk kernel, consumed by the scan / place kernels.
struct ChunkSum {
    uint64_t entry;    // speculative first record start in [cs, ce) (kNone if none validated)
    uint64_t exit;     // first record start >= ce reached from `entry` (or err_off if status != OK)
    uint64_t bytes;    // decoded bytes of the records walked from `entry`
    uint64_t err_off;  // offset of the header that raised `status`
    uint64_t det0, det1;  // HEADER_CRC expected/actual; MAGIC: bytes consumed by the magic varint
    uint32_t count;    // records walked from `entry` (all stored in scratch)
    int32_t status;    // RIO_OK or the terminal status raised inside this chunk
};

// Key-point summary of a run of chunks: the composed chunk functions
// evaluated at the run's first speculative entry `key`; identity (pass-through) for inputs >= ce.
struct RunSum {
    uint64_t key;      // kNone: the run has no speculative entry (owns nothing unless broken)
    uint64_t out;      // chain position after the run when entered at `key`
    uint64_t cnt;      // records owned
    uint64_t bytes;    // decoded bytes owned
    uint64_t ce;       // end of the run's byte range (0 = identity element)
    uint32_t term;     // the chain terminated (status) inside the run
    uint32_t broken;   // a speculative entry did not chain: slow path required
    uint64_t term_chunk;  // chunk index that raised the terminal status
};

// Per-chunk placement decided by the scan: records [base_idx, base_idx + owned) of the file are
// this chunk's scratch slots [0, owned).
struct ChunkPlace {
    uint64_t base_idx;
    uint64_t base_bytes;
    uint64_t owned;
};

// Device-side scan state (one per decode call).
struct ScanState {
    uint32_t version, compression;
    int32_t hdr_status;     // file header status
    uint32_t slow;          // 1 => ChunkPlace array is authoritative (sequential repair ran)
    uint64_t n_records;
    uint64_t total_bytes;
    int32_t status;         // terminal status
    uint32_t zero_nonzero;  // zero-tail check result (1 = a non-zero byte found)
    uint64_t status_offset;
    uint64_t det0, det1;
    uint64_t zero_from;     // zero-tail check range start (kNone = no check)
    uint64_t n_repairs;
    uint64_t first_bad;        // first record flagged RIO_FLAG_CORRUPT / RIO_FLAG_EOF (kNone = none)
    uint64_t n_bad;            // records so flagged
    uint64_t unsupported_rec;  // first record the device path hands back (absurd gzip sizes)
    uint32_t n_fail_lanes;     // Snappy lane-decoder lanes listed in fail_lanes (> kFailLanes: all)
    uint32_t capacity_fail;
    uint32_t huge_streams;  // a record stream exceeds 32-bit positions: the wave decoder (coop_file) runs, one thread per record
    uint32_t any_mixed;     // snappy: some record is not one literal covering its output (k_place);
                            // 0 => every record is copied by k_copy_records instead of k_snappy_pipe
    uint32_t scan_ticket;   // k_scan_blocks: the last block to finish runs the top-level scan
    uint32_t finish_ticket; // k_finish: the last block to finish publishes the result
    uint32_t pipe_next;     // k_snappy_pipe: next record chunk handed to a wave that finished its own
    uint32_t gz_resize;     // gzip: some record holds several members whose output the framing's
                            // size (its last member's ISIZE) does not cover: k_gz_resize sizes them;
                            // lzw: some record's output is not its header's u (k_lzw_resize)
    uint32_t gz_redo;       // k_gz_resize / k_lzw_resize ran: the scan, placement and decoders run again
};

// Result of the single-record (ReadNextAt) kernel.
struct ReadAtResult {
    int32_t status;
    int32_t nil;
    uint64_t len;
    uint64_t det0, det1;
    uint64_t hdr_len;
    uint64_t payload_off;
};

// Launch configuration passed from the host runtime.
struct FrameParams {
    const uint8_t* file;
    uint64_t len;
    uint64_t chunk_bytes;
    uint64_t n_chunks;
    uint64_t slots;  // scratch slots per chunk
    uint64_t* scratch_off;   // [n_chunks * slots] record header offsets
    uint64_t* scratch_len;   // [n_chunks * slots] decoded length | kNilBit
    uint64_t* scratch_pay;   // [n_chunks * slots] payload descriptor (see rec_pay)
    // internal per-record payload descriptor [rec_cap]: bits 0..7 = bytes from the record header
    // start to the first payload byte the decoder consumes (header + snappy preamble), bits 8..63
    // = length of the consumed payload stream (snappy element stream / raw payload). Written for
    // gzip / lzw files and for records rec_desc cannot describe (see rec_stream)
    uint64_t* rec_pay;
    // internal per-record decode descriptor [rec_cap] (Snappy decode): x,y = file offset of the
    // element stream (lo, hi), z = stream length, w = decoded length
    uint4* rec_desc;
    uint8_t* sink;           // [kSinkBytes] placeholder-store target of the Snappy decode pipeline
    uint64_t* fail_lanes;    // [2 * kFailLanes] record ranges [r0, r1) of lanes that met a corrupt record
    // Snappy: files whose mean decoded record is at least this many bytes (and files past 32-bit
    // lane positions) take the wave-per-record decoder k_snappy_coop instead of k_snappy_pipe
    uint64_t coop_min;
    // the file header's compression type as the host knows it (RIO_COMP_UNKNOWN: every decoder is
    // launched and exits unless the file is its own); k_finish rejects a file that contradicts it
    uint32_t comp_hint;
    uint32_t zero_done;  // the zero-tail check already ran (host API phase A): k_place skips it
    uint32_t walk_lane;  // framing by k_walk_lane (one lane per chunk) instead of k_walk (one wave per chunk)
    uint64_t* walk_hint; // page-locked host word: the decode's mean bytes per record (finalize_info), read by
                         // the context when it picks the next decode's walk (null: not recorded)
    uint32_t redo;       // redo round of this codec (RIO_COMP_GZIP: k_gz_resize onwards, RIO_COMP_LZW:
                         // k_lzw_resize onwards; 0: first round): the kernel exits unless the file is
                         // that codec's and its resize kernel ran
    ChunkSum* chunks;
    RunSum* block_runs;      // [n_blocks] (scan level 1 output)
    RunSum* chunk_excl;      // [n_chunks] exclusive within-block prefix
    ChunkPlace* place;       // [n_chunks]
    uint64_t* block_in;      // [n_blocks] chain position entering each block
    RunSum* block_excl;      // [n_blocks] exclusive prefix over blocks
    uint64_t n_blocks;
    ScanState* state;
    // outputs
    uint8_t* out;
    uint64_t out_cap;
    uint64_t* out_off;
    uint64_t* rec_off;
    uint8_t* flags;
    uint64_t rec_cap;
    rio_file_info* info;  // device copy of the public result
};

// Files of one rio_device_decode_batch call, passed by value to the batched decode kernel (the
// kernel argument holds them all: no H2D copy, no host sync, graph-capturable).
constexpr uint32_t kMaxBatch = 16;
struct FrameBatch {
    FrameParams f[kMaxBatch];
    uint32_t n;
};

// rio_encode.hip: recordio v4 encoding of a batch of records (rio_device_encode)
struct EncParams {
    const uint8_t* rec;        // records arena
    const uint64_t* rec_off;   // [n + 1]
    const uint8_t* flags;      // [n] RIO_FLAG_NIL, or null
    uint64_t n;
    uint32_t compression;
    uint8_t* scratch;          // compressed payloads, record i at scr_off[i]
    uint64_t* scr_off;         // [n + 1]
    uint64_t* clen;            // [n] payload length in the file (c for snappy, u for none)
    uint16_t* gtab;            // global tables: kMaxTable entries per lane of k_snappy_encode<false>
    uint8_t* hdr;              // [n][kHdrSlot] header bytes; hdr[i * kHdrSlot + 63] = header length
    uint64_t* size;            // [n + 1] exclusive scan of the record sizes = file offsets - 8
    uint64_t* tmp;             // [n + 1] scan inputs (payload bounds, then record sizes)
    uint8_t* out;
    uint64_t out_cap;
    uint64_t* out_rec_off;     // [n] file offset of each record (what Write returns)
    uint64_t* out_len;         // [1] file length
    uint32_t lds_small;        // records <= 1 KiB on the LDS-table kernel
};

#ifdef __HIPCC__
// A record whose payload does not decode: flag it for ReadNext (RIO_FLAG_CORRUPT) and count it.
// Only the thread that decoded record i writes its flag byte.
__device__ inline void mark_bad(const FrameParams& P, uint64_t i, uint8_t flag = RIO_FLAG_CORRUPT) {
    P.flags[i] = (uint8_t)(P.flags[i] | flag);
    atomicMin((unsigned long long*)&P.state->first_bad, (unsigned long long)i);
    atomicAdd((unsigned long long*)&P.state->n_bad, 1ull);
}
// Record i's consumed stream (snappy element stream / raw payload): file offset and length. k_place
// writes rec_pay only for gzip / lzw files (their kernels keep markers in it) and for records whose
// sizes do not fit rec_desc's 32-bit fields (rec_desc then holds the kDescWide sentinel).
__device__ inline void rec_stream(const FrameParams& P, uint64_t i, uint64_t& start, uint64_t& slen) {
    const uint4 d = P.rec_desc[i];
    if (d.z == kDescWide && d.w == kDescWide) {
        const uint64_t pay = P.rec_pay[i];
        start = P.rec_off[i] + (pay & 0xFF);
        slen = pay >> 8;
    } else {
        start = ((uint64_t)d.y << 32) | d.x;
        slen = d.z;
    }
}
#endif

}  // namespace rio
