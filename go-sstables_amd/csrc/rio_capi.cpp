// rio_capi.cpp — host runtime and C-ABI of librio (include/rio.h).
//
// Owns HIP contexts (device, stream, grow-only device arenas, pinned staging) and the reader
// handles that mirror recordio.ReaderI / recordio.ReadAtI:
//   FileReader  Open/ReadNext/SkipNext/Close   recordio/file_reader.go:26-172, 272-279
//   MMapReader  Open/ReadNextAt/SeekNext/Size  recordio/mmap_reader.go:25-203, 358-371
// Every decode runs on the device (rio_kernels.hip); host code only moves bytes, parses the
// 8-byte file header at Open (readFileHeaderFromBuffer, common_reader.go:22-44) and iterates the
// decoded arena. There is no CPU decode fallback: a missing GPU is an error.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include <condition_variable>

#include "rio.h"
#include "rio_device.h"
#include "rio_host.h"

namespace rio {
hipError_t launch_phase_a(const FrameParams& P, hipStream_t s, hipEvent_t* ev);
hipError_t launch_frame(const FrameParams& P, hipStream_t s, hipEvent_t* ev);
hipError_t launch_frame_ev(const FrameParams& P, hipStream_t s, hipEvent_t walk_start, hipEvent_t walk_stop,
                           hipEvent_t scan_stop);
hipError_t launch_phase_b(const FrameParams& P, hipStream_t s, hipEvent_t* ev, hipEvent_t done = nullptr);
hipError_t launch_phase_b_batch(const FrameBatch& B, hipStream_t s, hipEvent_t* ev, hipEvent_t done = nullptr);
hipError_t launch_sst_index(const uint8_t* arena, const uint64_t* off, uint64_t n, uint64_t* key_off,
                            uint64_t* key_len, uint64_t* value_off, uint64_t* checksum, uint64_t* result,
                            hipStream_t s);
hipError_t launch_sst_validate(const uint8_t* data, const uint64_t* data_off, const uint64_t* data_rec_off,
                               uint64_t n_data, const uint64_t* value_off, const uint64_t* checksum,
                               uint64_t n_index, uint64_t* crc_out, uint64_t* result, hipStream_t s,
                               const uint64_t* view = nullptr);
hipError_t launch_sst_data_entry(const uint8_t* arena, const uint64_t* off, uint64_t n, uint64_t* view,
                                 uint64_t* result, hipStream_t s);
hipError_t launch_index_search(const uint8_t* f, uint64_t len, uint64_t seek_len, const uint8_t* keys,
                               const uint64_t* key_off, uint64_t nq, const uint32_t* perm, rio_index_hit* hits,
                               hipStream_t s);
size_t key_sort_tmp_bytes(uint64_t n);
hipError_t launch_key_sort(const uint8_t* keys, const uint64_t* key_off, uint64_t n, uint64_t* pfx_in, uint64_t* pfx_out,
                           uint32_t* idx_in, uint32_t* perm, void* tmp, size_t tmp_bytes, hipStream_t s);
hipError_t launch_encode(const EncParams& P, void* cub_tmp, size_t cub_bytes, hipStream_t s);
uint64_t enc_scratch_bytes(uint64_t n, uint64_t bytes, uint32_t compression);
uint64_t enc_table_bytes();
size_t enc_cub_bytes(uint64_t n);
hipError_t launch_read_at(const uint8_t* f, uint64_t len, uint64_t off, uint8_t* out, uint64_t out_cap,
                          ReadAtResult* res, hipStream_t s);
int build_seek_map(const uint8_t* f, uint64_t len, const uint64_t* rec_off, const uint8_t* flags, uint64_t n,
                   std::vector<uint64_t>& P, std::vector<uint64_t>& R, hipStream_t s);
hipError_t launch_index_search_view(const uint8_t* out, const uint64_t* out_off, const uint8_t* flags, uint64_t n,
                                    const uint64_t* P, uint64_t K, const uint64_t* R, uint64_t len, const uint8_t* keys,
                                    const uint64_t* key_off, uint64_t nq, const uint32_t* perm, rio_index_hit* hits,
                                    hipStream_t s);
hipError_t launch_seek_next(const uint8_t* f, uint64_t len, uint64_t off, uint64_t seek_len, uint8_t* out,
                            uint64_t out_cap, ReadAtResult* res, uint64_t* rec_off, hipStream_t s);
}  // namespace rio

using namespace rio;

// ------------------------------------------------------------------------------------------
// status helpers
// ------------------------------------------------------------------------------------------
extern "C" const char* rio_strerror(int s) {
    switch (s) {
    case RIO_OK: return "ok";
    case RIO_EOF: return "EOF";
    case RIO_EOF_ZERO_TAIL: return "EOF (zero-padded tail)";
    case RIO_EOF_HEADER: return "EOF inside record header";
    case RIO_EOF_PAYLOAD: return "EOF reading record payload";
    case RIO_ERR_UNEXPECTED_EOF: return "unexpected EOF";
    case RIO_ERR_MAGIC: return "magic number mismatch";
    case RIO_ERR_HEADER_CRC: return "header checksum mismatch";
    case RIO_ERR_VARINT_OVERFLOW: return "binary: varint overflows a 64-bit integer";
    case RIO_ERR_HEADER_TOO_LONG: return "checksum byte reader out of range";
    case RIO_ERR_DECOMPRESS: return "snappy: corrupt input";
    case RIO_ERR_VERSION: return "version mismatch";
    case RIO_ERR_COMPRESSION_TYPE: return "unknown compression type";
    case RIO_ERR_SHORT_FILE_HEADER: return "not enough bytes in the file header";
    case RIO_ERR_INVALID_OFFSET: return "mmap: invalid ReadAt offset";
    case RIO_ERR_UNSUPPORTED: return "not supported by the GPU decode path";
    case RIO_ERR_CAPACITY: return "output capacity too small";
    case RIO_ERR_ARG: return "invalid argument";
    case RIO_ERR_HIP: return "HIP runtime error";
    case RIO_ERR_STATE: return "reader state error";
    case RIO_ERR_IO: return "I/O error";
    case RIO_ERR_PROTO: return "proto: cannot parse invalid wire-format data";
    case RIO_EOF_CODEC: return "EOF from the codec (empty gzip payload)";
    default: return "unknown status";
    }
}

extern "C" int rio_status_is_eof(int s) {
    return s == RIO_EOF || s == RIO_EOF_ZERO_TAIL || s == RIO_EOF_HEADER || s == RIO_EOF_PAYLOAD || s == RIO_EOF_CODEC;
}

extern "C" const char* rio_build_info(void) { return "librio gfx950 recordio v3/v4 decode"; }

extern "C" uint64_t rio_max_records(uint64_t len) {
    return len <= RIO_FILE_HEADER_BYTES ? 1 : (len - RIO_FILE_HEADER_BYTES) / 5 + 1;  // v2's 5-byte empty record
}

#define HIP_TRY(x)                                  \
    do {                                            \
        hipError_t e_ = (x);                        \
        if (e_ != hipSuccess) return RIO_ERR_HIP;   \
    } while (0)

// ------------------------------------------------------------------------------------------
// context
// ------------------------------------------------------------------------------------------
namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(n, 256);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

uint64_t env_u64(const char* name, uint64_t dflt) {
    const char* v = getenv(name);
    if (!v || !*v) return dflt;
    return strtoull(v, nullptr, 0);
}

constexpr size_t kStage = 32ull << 20;  // pinned staging piece

}  // namespace

namespace {
// framing scratch + per-record decode descriptors of one file (a ctx has one set per file of a batch)
struct FileArenas {
    // meta: the scan state, the file info, the lanes' failure list, the block and chunk summaries and the chunk
    // placements of one call in one allocation (state and block summaries first, 256-byte aligned parts)
    DevBuf scratch_off, scratch_len, scratch_pay, rec_pay, rec_desc, meta;
    void release() {
        for (DevBuf* b : {&scratch_off, &scratch_len, &scratch_pay, &rec_pay, &rec_desc, &meta}) b->release();
    }
};
}  // namespace

struct rio_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // timing ring (empty by default): slot i holds the 5 stage events of the i-th decode since rio_ctx_set_timing
    std::vector<std::array<hipEvent_t, 5>> ev;
    uint64_t ev_cursor = 0;
    uint64_t chunk_bytes = 32768;
    bool chunk_auto = true;  // RIO_CHUNK_BYTES unset: larger wave-walk chunks for large records (kBigRecordChunk)
    // framing walk (RIO_WALK_LANE): 0 k_walk (one wave per chunk_bytes chunk), 1 k_walk_lane (one lane per
    // lane_chunk_bytes chunk, RIO_LANE_CHUNK_BYTES), 2 auto (default): the lane walk when the context's
    // previous decode had records of kLaneWalkMin..kLaneWalkMax bytes on average (512 B and up on files of 1 GiB and
    // more; walk_hint, written by that decode's finalize_info into page-locked host memory: no host
    // synchronisation), else the wave walk
    uint32_t walk_mode = 2;
    uint64_t lane_chunk_bytes = 16384;
    uint64_t lane_walk_min = 512;  // kLaneWalkSmallMin (RIO_LANE_WALK_MIN)
    uint64_t walk_slots = 5120;    // resident k_walk waves: CUs x 4 SIMDs x kWalkWavesPerSimd (wave_chunk_bytes)
    uint64_t* walk_hint = nullptr;
    uint64_t coop_min = ~0ull >> 8;
    hipEvent_t* next_events() {
        if (ev.empty()) return nullptr;
        return ev[ev_cursor++ % ev.size()].data();
    }
    hipEvent_t* same_events() {  // phase B of the call whose phase A took the last slot
        if (ev.empty() || ev_cursor == 0) return nullptr;
        return ev[(ev_cursor - 1) % ev.size()].data();
    }
    void set_ring(size_t n) {
        for (auto& s : ev)
            for (auto& e : s) hipEventDestroy(e);
        ev.assign(n, {});
        for (auto& s : ev)
            for (auto& e : s) hipEventCreate(&e);
        ev_cursor = 0;
    }
    // framing arenas
    FileArenas fa;                                   // the single-file calls
    std::vector<std::unique_ptr<FileArenas>> batch;  // rio_device_decode_batch: one set per file
    DevBuf sink;
    // host-API arenas
    DevBuf file, out, out_off, rec_off, flags, readat_out, readat_res, seek_off;
    // reader handles sharing this ctx take this around every device use (rio_reader_*)
    std::mutex mu;
    // rio_sst_open: parsed index fields (4 x n), per-entry CRC-64, kernel results
    DevBuf sst_fields, sst_crc, sst_res, sst_view;
    // rio_device_encode: compressed payloads, their offsets and lengths, hash tables, headers,
    // record sizes, scan temp; rio_encode_file: records, offsets, flags, file image, record offsets
    DevBuf enc_scr, enc_scr_off, enc_clen, enc_tab, enc_hdr, enc_size, enc_tmp, enc_cub;
    DevBuf enc_rec, enc_rec_off, enc_flags, enc_out, enc_out_off, enc_len;
    // index search: key prefixes, indices, permutation, radix sort temp
    DevBuf q_pfx, q_pfx_out, q_idx, q_perm, q_tmp;
    uint8_t* pinned[2] = {nullptr, nullptr};
    hipEvent_t pin_ev[2] = {};
    // device-API calls share the ctx's scratch: a call on another stream than the previous one waits
    // for it (order_ev, recorded after every device-API call)
    hipEvent_t order_ev = nullptr;
    hipStream_t order_stream = nullptr;
    bool order_valid = false;
    // last host-API framing (rio_frame -> rio_decode)
    FrameParams last{};
    bool framed = false;
    bool predecoded = false;  // gzip: rio_frame decoded the file already (ctx arenas hold the result)
    uint64_t file_len = 0;
    rio_file_info frame_info{};
};

// mean bytes per record for which the auto walk takes k_walk_lane (round 5 A/B on MI355X, 16 KiB lane chunks:
// 1 KiB incompressible records walk 0.269 -> 0.142 ms; 560-byte records even; 48-byte and 36 KiB records
// slower, so those keep k_walk)
constexpr uint64_t kLaneWalkMin = 768, kLaneWalkMax = 8192, kLaneWalkChunks = 32768;
// 512..767-byte records take the lane walk only on files of kLaneWalkSmallChunks lane chunks and more (~30 hops per
// lane want a wave per SIMD of lanes): C2's 561-byte records in 535 MiB measured even (walk 0.143 -> 0.155 ms, decode
// 0.999 -> 0.988), the same records in a 5 GB file walk 1.10 -> 0.67 ms (profiles/r5/r5be_lane_walk_min_ab.txt).
// RIO_LANE_WALK_MIN overrides kLaneWalkSmallMin.
constexpr uint64_t kLaneWalkSmallMin = 512, kLaneWalkSmallChunks = 65536;
// records of more than kLaneWalkMax bytes on average: wave-walk chunks of at least kBigRecordChunk (a 32 KiB chunk holds
// at most a few such records and the placement runs a wave per chunk with most lanes idle: C4 place 0.123 -> 0.076 ms,
// walk 0.61 -> 0.585, +1.2 %, profiles/r5/r5bl_c4_chunk_ab.txt); not when RIO_CHUNK_BYTES sets the size
constexpr uint64_t kBigRecordChunk = 65536;
// Small files walk smaller chunks: the smallest multiple of 4 KiB (the walk's fill round) whose chunk count fits one round
// of resident walk waves (CUs x 4 SIMDs x RIO_WALK_OCC = 5 waves: 5 120 on MI355X), at least kSmallFileChunkMin; files
// that need more than one round at the default size keep it. A 32 MiB file's 1 024 default chunks were one wave per SIMD,
// each walking 32 KiB as a chain of dependent fill rounds; a chunk count just past one round runs a second round for a
// few waves (round 6 on MI355X: 32 MiB of 1 KiB records 0.117 -> 0.084 ms at 8 KiB chunks; 100 MB 0.171 -> 0.15 ms at
// 20 KiB (5 059 waves), against 16 KiB (6 100: two rounds) and 19 KiB (5 325); profiles/r6/r6j_small_file_chunks.txt)
constexpr uint64_t kSmallFileChunkMin = 8192, kWalkWavesPerSimd = 5;
static uint64_t wave_chunk_bytes(const rio_ctx* ctx, uint64_t len) {
    const uint64_t cb = ctx->chunk_bytes;
    if (!ctx->chunk_auto) return cb;
    const uint64_t slots = ctx->walk_slots;
    const uint64_t want = ((len + slots - 1) / slots + 4095) & ~4095ull;
    return std::min(cb, std::max(want, kSmallFileChunkMin));
}

// bytes of a file's framing arenas at chunk size cb: scratch (per array) and meta
struct ArenaSizes {
    uint64_t n_chunks, slots, n_blocks, scratch, meta;
};
static ArenaSizes arena_sizes(uint64_t len, uint64_t cb) {
    ArenaSizes z;
    z.n_chunks = len > RIO_FILE_HEADER_BYTES ? (len - RIO_FILE_HEADER_BYTES + cb - 1) / cb : 0;
    z.slots = cb / 5 + 1;  // records starting in a chunk: the smallest is v2's 5 bytes
    z.n_blocks = (z.n_chunks + 255) / 256;
    const uint64_t nc = std::max<uint64_t>(z.n_chunks, 1), nb = std::max<uint64_t>(z.n_blocks, 1);
    z.scratch = nc * z.slots * 8;
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    z.meta = al(sizeof(ScanState)) + al(sizeof(rio_file_info)) + 2 * al(nb * sizeof(RunSum)) +
             al(2 * kFailLanes * sizeof(uint64_t)) + al(nc * sizeof(ChunkSum)) + al(nc * sizeof(RunSum)) +
             al(nc * sizeof(ChunkPlace));
    return z;
}

// reserve_all: size the arenas for every chunk size the automatic walk choice can pick for a file of len bytes
// (wave chunks, lane chunks, big-record wave chunks), not only the one the current hint selects, so a later call
// whose hint flips the walk never grows an arena (rio_ctx_reserve's promise)
static int ctx_frame_params(rio_ctx* ctx, const uint8_t* d_file, uint64_t len, FrameParams& P, FileArenas& A,
                            bool reserve_all = false) {
    memset(&P, 0, sizeof P);
    P.file = d_file;
    P.len = len;
    // the lane walk reads ~64 bytes per record and is latency-bound per lane; the wave walk reads every
    // byte (HBM-bound on records of ~1 KiB and more) and frames candidates 64 at a time (the better one for
    // small records, and for very large ones, whose chunks hold no header and the lane walk scans)
    // (and only with lanes to fill the chip: a file of fewer than kLaneWalkChunks lane chunks leaves the lane
    // walk's one-chain-per-lane latency exposed, C1's 103 MB: walk 0.076 -> 0.179 ms)
    bool lane = ctx->walk_mode == 1;
    if (ctx->walk_mode == 2 && ctx->walk_hint && len / ctx->lane_chunk_bytes >= kLaneWalkChunks) {
        const uint64_t m = *reinterpret_cast<volatile uint64_t*>(ctx->walk_hint);
        const uint64_t chunks = len / ctx->lane_chunk_bytes;
        lane = (m >= kLaneWalkMin && m <= kLaneWalkMax) ||
               (m >= ctx->lane_walk_min && m < kLaneWalkMin && chunks >= kLaneWalkSmallChunks);
    }
    uint64_t cb = lane ? ctx->lane_chunk_bytes : wave_chunk_bytes(ctx, len);
    if (!lane && ctx->chunk_auto && ctx->walk_hint && *reinterpret_cast<volatile uint64_t*>(ctx->walk_hint) > kLaneWalkMax)
        cb = std::max<uint64_t>(cb, kBigRecordChunk);
    P.walk_lane = lane ? 1u : 0u;
    P.walk_hint = ctx->walk_hint;
    P.chunk_bytes = cb;
    P.coop_min = ctx->coop_min;
    P.comp_hint = RIO_COMP_UNKNOWN;
    P.zero_done = 0;
    const ArenaSizes z = arena_sizes(len, cb);
    P.n_chunks = z.n_chunks;
    P.slots = z.slots;
    P.n_blocks = z.n_blocks;
    const uint64_t nc = std::max<uint64_t>(P.n_chunks, 1), nb = std::max<uint64_t>(P.n_blocks, 1);
    uint64_t scr = z.scratch, meta_need = z.meta;
    if (reserve_all) {
        for (uint64_t c : {wave_chunk_bytes(ctx, len), ctx->chunk_bytes, ctx->lane_chunk_bytes,
                           std::max<uint64_t>(ctx->chunk_bytes, kBigRecordChunk)}) {
            const ArenaSizes y = arena_sizes(len, c);
            scr = std::max(scr, y.scratch);
            meta_need = std::max(meta_need, y.meta);
        }
    }
    HIP_TRY(A.scratch_off.ensure(scr));
    HIP_TRY(A.scratch_len.ensure(scr));
    HIP_TRY(A.scratch_pay.ensure(scr));
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    const uint64_t o_info = al(sizeof(ScanState)), o_brun = o_info + al(sizeof(rio_file_info));
    const uint64_t o_bexc = o_brun + al(nb * sizeof(RunSum)), o_fail = o_bexc + al(nb * sizeof(RunSum));
    const uint64_t o_chk = o_fail + al(2 * kFailLanes * sizeof(uint64_t)), o_cexc = o_chk + al(nc * sizeof(ChunkSum));
    const uint64_t o_place = o_cexc + al(nc * sizeof(RunSum)), meta_bytes = o_place + al(nc * sizeof(ChunkPlace));
    HIP_TRY(A.meta.ensure(std::max(meta_bytes, meta_need)));
    HIP_TRY(ctx->sink.ensure(kSinkBytes));
    uint8_t* const mb = A.meta.as<uint8_t>();
    P.sink = ctx->sink.as<uint8_t>();
    P.fail_lanes = reinterpret_cast<uint64_t*>(mb + o_fail);
    P.scratch_off = A.scratch_off.as<uint64_t>();
    P.scratch_len = A.scratch_len.as<uint64_t>();
    P.scratch_pay = A.scratch_pay.as<uint64_t>();
    P.chunks = reinterpret_cast<ChunkSum*>(mb + o_chk);
    P.chunk_excl = reinterpret_cast<RunSum*>(mb + o_cexc);
    P.place = reinterpret_cast<ChunkPlace*>(mb + o_place);
    P.block_runs = reinterpret_cast<RunSum*>(mb + o_brun);
    P.block_excl = reinterpret_cast<RunSum*>(mb + o_bexc);
    P.state = reinterpret_cast<ScanState*>(mb);
    P.info = reinterpret_cast<rio_file_info*>(mb + o_info);
    return RIO_OK;
}

extern "C" int rio_device_count(int* out) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    if (out) *out = n;
    return n > 0 ? RIO_OK : RIO_ERR_HIP;
}

extern "C" int rio_ctx_create(int device, rio_ctx** out) {
    if (!out) return RIO_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return RIO_ERR_HIP;
    if (device < 0 || device >= n) return RIO_ERR_ARG;
    HIP_TRY(hipSetDevice(device));
    auto* c = new rio_ctx();
    c->device = device;
    c->chunk_bytes = env_u64("RIO_CHUNK_BYTES", 32768);
    c->chunk_auto = std::getenv("RIO_CHUNK_BYTES") == nullptr;
    // k_walk's candidate bounds take 32-bit differences inside a chunk (magic_mask): chunks stay below
    // 1 GiB; anything outside [64, 1 GiB] or not a multiple of 16 falls back to the default
    if (c->chunk_bytes < 64 || c->chunk_bytes > (1ull << 30) || (c->chunk_bytes & 15)) c->chunk_bytes = 32768;
    c->walk_mode = (uint32_t)std::min<uint64_t>(env_u64("RIO_WALK_LANE", 2), 2);
    c->lane_chunk_bytes = env_u64("RIO_LANE_CHUNK_BYTES", 16384);
    c->lane_walk_min = env_u64("RIO_LANE_WALK_MIN", kLaneWalkSmallMin);
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        c->walk_slots = (uint64_t)cus * 4 * kWalkWavesPerSimd;
    if (c->lane_chunk_bytes < 64 || c->lane_chunk_bytes > (1ull << 30) || (c->lane_chunk_bytes & 15))
        c->lane_chunk_bytes = 16384;
    if (hipHostMalloc(reinterpret_cast<void**>(&c->walk_hint), sizeof(uint64_t), hipHostMallocPortable) != hipSuccess) {
        (void)hipGetLastError();
        c->walk_hint = nullptr;  // no hint: the wave walk
    } else {
        *c->walk_hint = 0;
    }
    c->coop_min = env_u64("RIO_COOP_MIN", ~0ull >> 8);  // k_snappy_coop: wide files only
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return RIO_ERR_HIP;
    }
    // no stage events until rio_ctx_set_timing asks for them: the five timing events of a call cost a C2 step
    // 1.5 % and a C1-size step 13 % (profiles/r5/r5az_event_cost.txt)
    c->set_ring(0);
    *out = c;
    return RIO_OK;
}

extern "C" int rio_ctx_device(const rio_ctx* c) { return c ? c->device : -1; }

extern "C" void rio_ctx_destroy(rio_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    if (c->order_ev) {  // the last device-API call may have run on a caller's stream
        hipEventSynchronize(c->order_ev);
        hipEventDestroy(c->order_ev);
    }
    c->fa.release();
    for (auto& a : c->batch) a->release();
    for (DevBuf* b : {&c->sink, &c->file, &c->out, &c->out_off, &c->rec_off, &c->flags,
                      &c->readat_out, &c->readat_res, &c->seek_off, &c->sst_fields, &c->sst_crc, &c->sst_res, &c->sst_view, &c->enc_scr, &c->enc_scr_off, &c->enc_clen, &c->enc_tab,
                      &c->enc_hdr, &c->enc_size, &c->enc_tmp, &c->enc_cub, &c->enc_rec, &c->enc_rec_off, &c->enc_flags, &c->enc_out,
                      &c->enc_out_off, &c->enc_len, &c->q_pfx, &c->q_pfx_out, &c->q_idx, &c->q_perm, &c->q_tmp})
        b->release();
    for (int i = 0; i < 2; i++) {
        if (c->pinned[i]) hipHostFree(c->pinned[i]);
        if (c->pin_ev[i]) hipEventDestroy(c->pin_ev[i]);
    }
    c->set_ring(0);
    if (c->walk_hint) hipHostFree(c->walk_hint);
    hipStreamDestroy(c->stream);
    delete c;
}

// slots == 0 disables stage events; slots == n keeps the events of the last n decodes
extern "C" int rio_ctx_set_timing(rio_ctx* c, int slots) {
    if (!c || slots < 0) return RIO_ERR_ARG;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    c->set_ring((size_t)slots);
    return RIO_OK;
}

// Mean per-stage device milliseconds over the decodes recorded in the ring:
// [0] header + walk, [1] scan + zero-tail check, [2] placement, [3] decode kernels.
extern "C" int rio_ctx_last_stage_ms(rio_ctx* c, float* ms, int n) {
    if (!c || !ms || c->ev.empty() || c->ev_cursor == 0) return 0;
    const uint64_t used = std::min<uint64_t>(c->ev_cursor, c->ev.size());
    double acc[4] = {0, 0, 0, 0};
    for (uint64_t s = 0; s < used; s++) {
        auto& e = c->ev[s];
        hipEventSynchronize(e[4]);
        for (int k = 0; k < 4; k++) {
            float v = 0;
            hipEventElapsedTime(&v, e[k], e[k + 1]);
            acc[k] += v;
        }
    }
    int k = std::min(n, 4);
    for (int i = 0; i < k; i++) ms[i] = (float)(acc[i] / (double)used);
    return k;
}

// ------------------------------------------------------------------------------------------
// device-resident single call
// ------------------------------------------------------------------------------------------
// The device-API calls of one ctx use the same scratch arenas: a call on a stream other than the
// previous call's waits for that call first (stream-ordered, no host synchronisation).
static int order_before(rio_ctx* ctx, hipStream_t s) {
    if (ctx->order_valid && ctx->order_stream != s) HIP_TRY(hipStreamWaitEvent(s, ctx->order_ev, 0));
    return RIO_OK;
}
// the device-resident calls hand the order event to their last kernel (k_finish) as its completion event instead
// of recording it behind the call: no marker packet between this call and the next (profiles/r5/r5bi_order_event_ab.txt)
static int order_event(rio_ctx* ctx, hipEvent_t& e) {
    if (!ctx->order_ev) HIP_TRY(hipEventCreateWithFlags(&ctx->order_ev, hipEventDisableTiming));
    e = ctx->order_ev;
    return RIO_OK;
}
static void order_mark(rio_ctx* ctx, hipStream_t s) {
    ctx->order_stream = s;
    ctx->order_valid = true;
}
static int order_after(rio_ctx* ctx, hipStream_t s) {
    if (!ctx->order_ev) HIP_TRY(hipEventCreateWithFlags(&ctx->order_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(ctx->order_ev, s));
    ctx->order_stream = s;
    ctx->order_valid = true;
    return RIO_OK;
}

extern "C" int rio_ctx_reserve(rio_ctx* ctx, uint64_t max_file_len, uint64_t max_records, uint32_t max_batch) {
    if (!ctx || max_batch > kMaxBatch) return RIO_ERR_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    FrameParams P;
    if (int rc = ctx_frame_params(ctx, nullptr, max_file_len, P, ctx->fa, true)) return rc;
    HIP_TRY(ctx->fa.rec_pay.ensure((max_records + 1) * 8));
    HIP_TRY(ctx->fa.rec_desc.ensure((max_records + 1) * 16));
    while (ctx->batch.size() < max_batch) ctx->batch.emplace_back(new FileArenas());
    for (uint32_t j = 0; j < max_batch; j++) {
        FileArenas& A = *ctx->batch[j];
        if (int rc = ctx_frame_params(ctx, nullptr, max_file_len, P, A, true)) return rc;
        HIP_TRY(A.rec_pay.ensure((max_records + 1) * 8));
        HIP_TRY(A.rec_desc.ensure((max_records + 1) * 16));
    }
    if (!ctx->order_ev) HIP_TRY(hipEventCreateWithFlags(&ctx->order_ev, hipEventDisableTiming));
    return RIO_OK;
}
extern "C" uint64_t rio_ctx_arena_bytes(const rio_ctx* ctx) {
    if (!ctx) return 0;
    uint64_t t = ctx->sink.cap;
    auto add = [&](const FileArenas& A) {
        for (const DevBuf* b : {&A.scratch_off, &A.scratch_len, &A.scratch_pay, &A.rec_pay, &A.rec_desc, &A.meta}) t += b->cap;
    };
    add(ctx->fa);
    for (auto& a : ctx->batch) add(*a);
    return t;
}

extern "C" int rio_device_decode(rio_ctx* ctx, const uint8_t* d_file, uint64_t len, uint8_t* d_out,
                                 uint64_t out_cap, uint64_t* d_out_off, uint64_t* d_rec_off, uint8_t* d_flags,
                                 uint64_t rec_cap, rio_file_info* d_info, void* stream) {
    return rio_device_decode_ex(ctx, d_file, len, RIO_COMP_UNKNOWN, d_out, out_cap, d_out_off, d_rec_off, d_flags,
                                rec_cap, d_info, stream);
}

extern "C" int rio_device_decode_ex(rio_ctx* ctx, const uint8_t* d_file, uint64_t len, uint32_t compression,
                                    uint8_t* d_out, uint64_t out_cap, uint64_t* d_out_off, uint64_t* d_rec_off,
                                    uint8_t* d_flags, uint64_t rec_cap, rio_file_info* d_info, void* stream) {
    if (!ctx || !d_file || !d_out_off || !d_rec_off || !d_flags || !d_info) return RIO_ERR_ARG;
    if (compression > RIO_COMP_LZW && compression != RIO_COMP_UNKNOWN) return RIO_ERR_ARG;
    if ((reinterpret_cast<uintptr_t>(d_file) & 15) != 0) return RIO_ERR_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    FrameParams P;
    int rc = ctx_frame_params(ctx, d_file, len, P, ctx->fa);
    if (rc) return rc;
    P.out = d_out;
    P.out_cap = out_cap;
    P.out_off = d_out_off;
    P.rec_off = d_rec_off;
    P.flags = d_flags;
    P.rec_cap = rec_cap;
    P.info = d_info;
    HIP_TRY(ctx->fa.rec_pay.ensure((rec_cap + 1) * 8));
    P.rec_pay = ctx->fa.rec_pay.as<uint64_t>();
    HIP_TRY(ctx->fa.rec_desc.ensure((rec_cap + 1) * 16));
    P.rec_desc = ctx->fa.rec_desc.as<uint4>();
    P.comp_hint = compression;
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    if (int rc2 = order_before(ctx, s)) return rc2;
    hipEvent_t oe;
    if (int rc3 = order_event(ctx, oe)) return rc3;
    hipEvent_t* ev = ctx->next_events();
    HIP_TRY(launch_frame(P, s, ev));
    HIP_TRY(launch_phase_b(P, s, ev, oe));
    order_mark(ctx, s);
    return RIO_OK;
}

// Batch of device-resident files (BASELINE configs[3]: the 8 files of a GPU's shard in one step):
// framing per file, then the large-record Snappy decoder once over all of them, so that files of few
// large records still fill the chip. Up to kMaxBatch files per launch group; larger batches run as
// consecutive groups on the same stream.
extern "C" int rio_device_decode_batch(rio_ctx* ctx, uint32_t n_files, const uint8_t* const* d_files,
                                       const uint64_t* lens, uint8_t* const* d_out, const uint64_t* out_cap,
                                       uint64_t* const* d_out_off, uint64_t* const* d_rec_off, uint8_t* const* d_flags,
                                       const uint64_t* rec_cap, rio_file_info* const* d_info, void* stream) {
    if (!ctx || (n_files && (!d_files || !lens || !d_out || !out_cap || !d_out_off || !d_rec_off || !d_flags ||
                             !rec_cap || !d_info)))
        return RIO_ERR_ARG;
    for (uint32_t k = 0; k < n_files; k++)
        if (!d_files[k] || (reinterpret_cast<uintptr_t>(d_files[k]) & 15) || !d_out_off[k] || !d_rec_off[k] ||
            !d_flags[k] || !d_info[k])
            return RIO_ERR_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    if (int rc = order_before(ctx, s)) return rc;
    if (n_files == 0) return RIO_OK;  // nothing enqueued: the previous call's order event still stands
    hipEvent_t oe;
    if (int rc = order_event(ctx, oe)) return rc;
    while (ctx->batch.size() < std::min<uint32_t>(n_files, kMaxBatch)) ctx->batch.emplace_back(new FileArenas());
    hipEvent_t* ev = ctx->next_events();
    // the next call's walk hint comes from ONE file of the batch, the longest (the first of equal ones), so the choice
    // does not depend on which file's k_finish ran last
    uint32_t hint_file = 0;
    for (uint32_t k = 1; k < n_files; k++)
        if (lens[k] > lens[hint_file]) hint_file = k;
    for (uint32_t g = 0; g < n_files; g += kMaxBatch) {
        FrameBatch B{};
        B.n = std::min<uint32_t>(kMaxBatch, n_files - g);
        for (uint32_t j = 0; j < B.n; j++) {
            const uint32_t k = g + j;
            FileArenas& A = *ctx->batch[j];
            FrameParams& P = B.f[j];
            int rc = ctx_frame_params(ctx, d_files[k], lens[k], P, A);
            if (rc) return rc;
            P.out = d_out[k];
            P.out_cap = out_cap[k];
            P.out_off = d_out_off[k];
            P.rec_off = d_rec_off[k];
            P.flags = d_flags[k];
            P.rec_cap = rec_cap[k];
            P.info = d_info[k];
            HIP_TRY(A.rec_pay.ensure((rec_cap[k] + 1) * 8));
            P.rec_pay = A.rec_pay.as<uint64_t>();
            HIP_TRY(A.rec_desc.ensure((rec_cap[k] + 1) * 16));
            P.rec_desc = A.rec_desc.as<uint4>();
            if (k != hint_file) P.walk_hint = nullptr;
        }
        // stage events bracket the whole batch, on the kernels' own dispatches: [0] at the first file's walk start,
        // [1] at the last file's scan end, [2] .. [4] in launch_phase_b_batch (placement start / end, k_finish start)
        hipEvent_t* e = (ev && g == 0) ? ev : nullptr;
        hipEvent_t* last = (ev && g + kMaxBatch >= n_files) ? ev : nullptr;
        for (uint32_t j = 0; j < B.n; j++)
            HIP_TRY(launch_frame_ev(B.f[j], s, (e && j == 0) ? e[0] : nullptr, nullptr,
                                    (last && j + 1 == B.n) ? last[1] : nullptr));
        HIP_TRY(launch_phase_b_batch(B, s, last, g + kMaxBatch >= n_files ? oe : nullptr));
    }
    order_mark(ctx, s);
    return RIO_OK;
}

// ------------------------------------------------------------------------------------------
// host two-phase API (cgo)
// ------------------------------------------------------------------------------------------
static int ensure_pinned(rio_ctx* c) {
    for (int i = 0; i < 2; i++) {
        if (!c->pinned[i]) {
            HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->pinned[i]), kStage, hipHostMallocDefault));
            HIP_TRY(hipEventCreateWithFlags(&c->pin_ev[i], hipEventDisableTiming));
        }
    }
    return RIO_OK;
}

// Page-locked host ranges this library knows: rio_host_register's ranges and PinnedPool's
// blocks, base -> bytes. A DMA straight from host memory needs ALL of [p, p + n) page-locked; a
// pointer attribute only describes p itself.
namespace {
std::mutex g_pin_mu;
std::map<uintptr_t, uint64_t> g_pin;
bool pinned_known(uintptr_t a, uint64_t n) {
    std::lock_guard<std::mutex> g(g_pin_mu);
    auto it = g_pin.upper_bound(a);
    if (it == g_pin.begin()) return false;
    --it;
    return a >= it->first && a - it->first <= it->second && n <= it->second - (a - it->first);
}
}  // namespace
namespace rio {
void note_pinned(const void* p, uint64_t n) {
    std::lock_guard<std::mutex> g(g_pin_mu);
    g_pin[reinterpret_cast<uintptr_t>(p)] = n;
}
void forget_pinned(const void* p) {
    std::lock_guard<std::mutex> g(g_pin_mu);
    g_pin.erase(reinterpret_cast<uintptr_t>(p));
}
}  // namespace rio

// true when all of [p, p + n) is page-locked host memory: a range this library registered or
// allocated, or one allocation HIP reports (hipHostMalloc / hipHostRegister by the caller) that
// covers the whole range. The copy then goes by DMA directly, without the staging pieces; anything
// else (a partly registered image, a range running past its registration) takes the staging path.
// The probes' errors on pageable memory are cleared so a later hipGetLastError (kernel launch
// check) does not see them.
static bool host_pinned(const void* p, uint64_t n) {
    if (!p || n < (1u << 20)) return false;  // small copies: staging costs nothing
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    hipPointerAttribute_t at{};
    bool ok = hipPointerGetAttributes(&at, p) == hipSuccess && at.type == hipMemoryTypeHost;
    // the registry covers whole ranges the library locked itself, but only while HIP still reports the memory
    // page-locked: a range the caller unregistered with hipHostUnregister directly (or freed) is forgotten here
    // instead of being taken for DMA-able memory
    if (pinned_known(a, n)) {
        (void)hipGetLastError();
        if (ok) return true;
        std::lock_guard<std::mutex> g(g_pin_mu);
        auto it = g_pin.upper_bound(a);
        if (it != g_pin.begin()) g_pin.erase(std::prev(it));
        return false;
    }
    if (ok) {
        void* base = nullptr;
        size_t sz = 0;
        ok = hipMemGetAddressRange(&base, &sz, const_cast<void*>(p)) == hipSuccess && base &&
             reinterpret_cast<uintptr_t>(base) <= a && a - reinterpret_cast<uintptr_t>(base) <= sz &&
             n <= sz - (a - reinterpret_cast<uintptr_t>(base));
    }
    (void)hipGetLastError();
    return ok;
}

// pageable host -> device through two pinned staging pieces (copy of piece k+1 overlaps the DMA
// of piece k); pinned sources go directly
static int h2d_staged(rio_ctx* c, void* dst, const uint8_t* src, uint64_t n) {
    if (host_pinned(src, n)) {
        HIP_TRY(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, c->stream));
        return RIO_OK;
    }
    int rc = ensure_pinned(c);
    if (rc) return rc;
    uint64_t o = 0;
    int k = 0;
    while (o < n) {
        const uint64_t m = std::min<uint64_t>(kStage, n - o);
        HIP_TRY(hipEventSynchronize(c->pin_ev[k]));
        HostPool::get().copy(c->pinned[k], src + o, m);
        HIP_TRY(hipMemcpyAsync(static_cast<uint8_t*>(dst) + o, c->pinned[k], m, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipEventRecord(c->pin_ev[k], c->stream));
        o += m;
        k ^= 1;
    }
    return RIO_OK;
}

// device -> pageable host through pinned staging; pinned destinations directly
static int d2h_staged(rio_ctx* c, uint8_t* dst, const void* src, uint64_t n) {
    if (host_pinned(dst, n)) {
        HIP_TRY(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        return RIO_OK;
    }
    int rc = ensure_pinned(c);
    if (rc) return rc;
    uint64_t o = 0, prev_o = 0, prev_m = 0;
    int k = 0;
    bool have_prev = false;
    while (o < n) {
        const uint64_t m = std::min<uint64_t>(kStage, n - o);
        HIP_TRY(hipEventSynchronize(c->pin_ev[k]));
        HIP_TRY(hipMemcpyAsync(c->pinned[k], static_cast<const uint8_t*>(src) + o, m, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipEventRecord(c->pin_ev[k], c->stream));
        if (have_prev) {
            HIP_TRY(hipEventSynchronize(c->pin_ev[k ^ 1]));
            HostPool::get().copy(dst + prev_o, c->pinned[k ^ 1], prev_m);
        }
        have_prev = true;
        prev_o = o;
        prev_m = m;
        o += m;
        k ^= 1;
    }
    if (have_prev) {
        HIP_TRY(hipEventSynchronize(c->pin_ev[k ^ 1]));
        HostPool::get().copy(dst + prev_o, c->pinned[k ^ 1], prev_m);
    }
    return RIO_OK;
}

// host producer -> device through the two pinned staging pieces: producing piece k+1 overlaps
// the DMA of piece k (the pieces are filled in order)
static int h2d_fill(rio_ctx* c, void* dst, uint64_t n, rio::FillFn fill, void* user) {
    int rc = ensure_pinned(c);
    if (rc) return rc;
    uint64_t o = 0;
    int k = 0;
    while (o < n) {
        const uint64_t m = std::min<uint64_t>(kStage, n - o);
        HIP_TRY(hipEventSynchronize(c->pin_ev[k]));
        if ((rc = fill(user, c->pinned[k], o, m))) {
            (void)hipStreamSynchronize(c->stream);  // the other piece's DMA may still read staging
            return rc;
        }
        HIP_TRY(hipMemcpyAsync(static_cast<uint8_t*>(dst) + o, c->pinned[k], m, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipEventRecord(c->pin_ev[k], c->stream));
        o += m;
        k ^= 1;
    }
    return RIO_OK;
}

// `prefix` (prefix_len bytes, host) then `file` (len - prefix_len bytes): a window of a larger file
// behind its file header (rio::frame_direct)
static int frame_common(rio_ctx* ctx, uint64_t len, rio_file_info* info, const uint8_t* file, rio::FillFn fill,
                        void* user, const uint8_t* prefix = nullptr, uint64_t prefix_len = 0) {
    HIP_TRY(hipSetDevice(ctx->device));
    // the host API shares the ctx arenas with the device API: wait for a device-API call still
    // running on another stream, and make the next device-API call wait for this one
    if (int rc = order_before(ctx, ctx->stream)) return rc;
    ctx->framed = false;
    HIP_TRY(ctx->file.ensure(len + RIO_DEVICE_PAD));
    if (prefix_len) HIP_TRY(hipMemcpyAsync(ctx->file.p, prefix, prefix_len, hipMemcpyHostToDevice, ctx->stream));
    int rc = fill ? h2d_fill(ctx, ctx->file.p, len, fill, user)
                  : h2d_staged(ctx, ctx->file.as<uint8_t>() + prefix_len, file, len - prefix_len);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(ctx->file.as<uint8_t>() + len, 0, RIO_DEVICE_PAD, ctx->stream));
    FrameParams P;
    rc = ctx_frame_params(ctx, ctx->file.as<uint8_t>(), len, P, ctx->fa);
    if (rc) return rc;
    HIP_TRY(launch_phase_a(P, ctx->stream, ctx->next_events()));
    HIP_TRY(hipMemcpyAsync(&ctx->frame_info, P.info, sizeof(rio_file_info), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->predecoded = false;
    const rio_file_info& fi = ctx->frame_info;
    const bool expand = fi.compression == RIO_COMP_GZIP || fi.compression == RIO_COMP_LZW;
    if (expand && fi.status != RIO_ERR_VERSION && fi.status != RIO_ERR_COMPRESSION_TYPE &&
        fi.status != RIO_ERR_UNSUPPORTED && fi.status != RIO_ERR_SHORT_FILE_HEADER) {
        // gzip / lzw: decode now. The framing sizes a gzip record from its last member's ISIZE, an lzw
        // record from its header's u; a record of several gzip members (Go's multistream reader) is
        // larger, an lzw record under a header that lies differs, which only the decode finds out, and
        // the caller allocates from the sizes returned here. A decode that needs more room than the
        // framing's sizes reports RIO_ERR_CAPACITY with the sizes it needs: frame and decode again
        // into arenas of that size (the whole pipeline: framing resets the device state).
        uint64_t n = fi.n_records, nb = fi.total_out_bytes;
        rio_file_info fin{};
        for (int attempt = 0; attempt < 3; attempt++) {
            HIP_TRY(ctx->out.ensure(nb + 16));
            HIP_TRY(ctx->out_off.ensure((n + 1) * 8));
            HIP_TRY(ctx->rec_off.ensure(n * 8 + 8));
            HIP_TRY(ctx->flags.ensure(n + 8));
            HIP_TRY(ctx->fa.rec_pay.ensure((n + 1) * 8));
            HIP_TRY(ctx->fa.rec_desc.ensure((n + 1) * 16));
            if (attempt) HIP_TRY(launch_phase_a(P, ctx->stream, nullptr));
            FrameParams D = P;
            D.zero_done = 1;  // phase A ran k_zero
            D.comp_hint = fi.compression;
            D.out = ctx->out.as<uint8_t>();
            D.out_cap = nb;
            D.out_off = ctx->out_off.as<uint64_t>();
            D.rec_off = ctx->rec_off.as<uint64_t>();
            D.flags = ctx->flags.as<uint8_t>();
            D.rec_cap = n;
            D.rec_pay = ctx->fa.rec_pay.as<uint64_t>();
            D.rec_desc = ctx->fa.rec_desc.as<uint4>();
            HIP_TRY(launch_phase_b(D, ctx->stream, attempt ? nullptr : ctx->same_events()));
            HIP_TRY(hipMemcpyAsync(&fin, D.info, sizeof fin, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(hipStreamSynchronize(ctx->stream));
            P = D;
            if (fin.status != RIO_ERR_CAPACITY) break;
            n = fin.n_records;
            nb = fin.total_out_bytes;
        }
        if (fin.status == RIO_ERR_CAPACITY) return RIO_ERR_CAPACITY;
        ctx->frame_info = fin;
        ctx->predecoded = true;
    }
    *info = ctx->frame_info;
    ctx->last = P;
    ctx->framed = true;
    ctx->file_len = len;
    return order_after(ctx, ctx->stream);
}

extern "C" int rio_frame(rio_ctx* ctx, const uint8_t* file, uint64_t len, rio_file_info* info) {
    if (!ctx || (!file && len) || !info) return RIO_ERR_ARG;
    return frame_common(ctx, len, info, file, nullptr, nullptr);
}

namespace rio {
int frame_fill(rio_ctx* ctx, uint64_t len, FillFn fill, void* user, rio_file_info* info) {
    if (!ctx || !fill || !info) return RIO_ERR_ARG;
    return frame_common(ctx, len, info, nullptr, fill, user);
}
int frame_direct(rio_ctx* ctx, const uint8_t* prefix, uint64_t prefix_len, const uint8_t* src, uint64_t n,
                 rio_file_info* info) {
    if (!ctx || !info || (n && !src) || (prefix_len && !prefix)) return RIO_ERR_ARG;
    return frame_common(ctx, prefix_len + n, info, src, nullptr, nullptr, prefix, prefix_len);
}
bool is_host_pinned(const void* p, uint64_t n) { return host_pinned(p, n); }
}  // namespace rio

// page-lock a caller's host buffer (a file image it reuses): the H2D of rio_frame / rio_stream_open_host
// then reads it by DMA in place instead of through the staging pieces
extern "C" int rio_host_register(const void* p, uint64_t n) {
    if (!p || !n) return RIO_ERR_ARG;
    HIP_TRY(hipHostRegister(const_cast<void*>(p), n, hipHostRegisterDefault));
    rio::note_pinned(p, n);
    return RIO_OK;
}
extern "C" int rio_host_unregister(const void* p) {
    if (!p) return RIO_ERR_ARG;
    rio::forget_pinned(p);
    HIP_TRY(hipHostUnregister(const_cast<void*>(p)));
    return RIO_OK;
}

extern "C" int rio_decode(rio_ctx* ctx, uint8_t* out, uint64_t out_cap, uint64_t* out_off, uint64_t* rec_off,
                          uint8_t* flags, uint64_t rec_cap, rio_file_info* info) {
    if (!ctx || !info) return RIO_ERR_ARG;
    if (!ctx->framed) return RIO_ERR_STATE;
    HIP_TRY(hipSetDevice(ctx->device));
    const rio_file_info fi = ctx->frame_info;
    if (fi.status == RIO_ERR_VERSION || fi.status == RIO_ERR_COMPRESSION_TYPE || fi.status == RIO_ERR_UNSUPPORTED ||
        fi.status == RIO_ERR_SHORT_FILE_HEADER) {
        *info = fi;
        return RIO_OK;
    }
    const uint64_t n = fi.n_records, nb = fi.total_out_bytes;
    if (rec_cap < n || out_cap < nb || (n && (!out_off || !rec_off || !flags)) || (nb && !out)) return RIO_ERR_CAPACITY;
    if (int rc = order_before(ctx, ctx->stream)) return rc;
    if (ctx->predecoded) {  // gzip: rio_frame decoded the file (its sizes are the decoded ones)
        const FrameParams& P = ctx->last;
        int rc;
        if (nb && (rc = d2h_staged(ctx, out, P.out, nb))) return rc;
        if (out_off && (rc = d2h_staged(ctx, reinterpret_cast<uint8_t*>(out_off), P.out_off, (n + 1) * 8))) return rc;
        if (n) {
            if ((rc = d2h_staged(ctx, reinterpret_cast<uint8_t*>(rec_off), P.rec_off, n * 8))) return rc;
            if ((rc = d2h_staged(ctx, flags, P.flags, n))) return rc;
        }
        *info = fi;
        return order_after(ctx, ctx->stream);
    }
    HIP_TRY(ctx->out.ensure(nb + 16));
    HIP_TRY(ctx->out_off.ensure((n + 1) * 8));
    HIP_TRY(ctx->rec_off.ensure(n * 8 + 8));
    HIP_TRY(ctx->flags.ensure(n + 8));
    FrameParams P = ctx->last;
    P.zero_done = 1;               // phase A ran k_zero (rio_frame's status is final)
    P.comp_hint = fi.compression;  // from the file header rio_frame read
    P.out = ctx->out.as<uint8_t>();
    P.out_cap = nb;
    P.out_off = ctx->out_off.as<uint64_t>();
    P.rec_off = ctx->rec_off.as<uint64_t>();
    P.flags = ctx->flags.as<uint8_t>();
    P.rec_cap = n;
    HIP_TRY(ctx->fa.rec_pay.ensure((n + 1) * 8));
    P.rec_pay = ctx->fa.rec_pay.as<uint64_t>();
    HIP_TRY(ctx->fa.rec_desc.ensure((n + 1) * 16));
    P.rec_desc = ctx->fa.rec_desc.as<uint4>();
    HIP_TRY(launch_phase_b(P, ctx->stream, ctx->same_events()));
    rio_file_info fin{};
    HIP_TRY(hipMemcpyAsync(&fin, P.info, sizeof fin, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    int rc;
    if (fin.total_out_bytes && (rc = d2h_staged(ctx, out, P.out, fin.total_out_bytes))) return rc;
    if (out_off && (rc = d2h_staged(ctx, reinterpret_cast<uint8_t*>(out_off), P.out_off, (fin.n_records + 1) * 8))) return rc;
    if (fin.n_records) {
        if ((rc = d2h_staged(ctx, reinterpret_cast<uint8_t*>(rec_off), P.rec_off, fin.n_records * 8))) return rc;
        if ((rc = d2h_staged(ctx, flags, P.flags, fin.n_records))) return rc;
    }
    *info = fin;
    return order_after(ctx, ctx->stream);
}

// ------------------------------------------------------------------------------------------
// single-record decode (ReadNextAt) / seek (SeekNext) on a device-resident file
// ------------------------------------------------------------------------------------------
static int read_at_impl(rio_ctx* ctx, const uint8_t* d_file, uint64_t len, uint64_t offset, bool seek,
                        uint64_t seek_len, ReadAtResult* res, uint64_t* rec_offset) {
    HIP_TRY(ctx->readat_res.ensure(sizeof(ReadAtResult)));
    HIP_TRY(ctx->seek_off.ensure(8));
    if (ctx->readat_out.cap == 0) HIP_TRY(ctx->readat_out.ensure(1 << 20));
    for (int attempt = 0; attempt < 2; attempt++) {
        if (seek)
            HIP_TRY(launch_seek_next(d_file, len, offset, seek_len, ctx->readat_out.as<uint8_t>(), ctx->readat_out.cap,
                                     ctx->readat_res.as<ReadAtResult>(), ctx->seek_off.as<uint64_t>(), ctx->stream));
        else
            HIP_TRY(launch_read_at(d_file, len, offset, ctx->readat_out.as<uint8_t>(), ctx->readat_out.cap,
                                   ctx->readat_res.as<ReadAtResult>(), ctx->stream));
        HIP_TRY(hipMemcpyAsync(res, ctx->readat_res.p, sizeof(ReadAtResult), hipMemcpyDeviceToHost, ctx->stream));
        if (rec_offset) HIP_TRY(hipMemcpyAsync(rec_offset, ctx->seek_off.p, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        if (res->status != RIO_ERR_CAPACITY) return RIO_OK;
        HIP_TRY(ctx->readat_out.ensure(res->len + 16));
    }
    return RIO_OK;
}

extern "C" int rio_device_read_at(rio_ctx* ctx, const uint8_t* d_file, uint64_t len, uint64_t offset,
                                  uint8_t* d_out, uint64_t out_cap, uint64_t* len_out, int* nil_out,
                                  uint64_t* detail0, uint64_t* detail1) {
    if (!ctx || !d_file) return RIO_ERR_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    ReadAtResult r{};
    HIP_TRY(ctx->readat_res.ensure(sizeof(ReadAtResult)));
    HIP_TRY(launch_read_at(d_file, len, offset, d_out, out_cap, ctx->readat_res.as<ReadAtResult>(), ctx->stream));
    HIP_TRY(hipMemcpyAsync(&r, ctx->readat_res.p, sizeof r, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (len_out) *len_out = r.len;
    if (nil_out) *nil_out = r.nil;
    if (detail0) *detail0 = r.det0;
    if (detail1) *detail1 = r.det1;
    return r.status;
}

// ------------------------------------------------------------------------------------------
// reader handles
// ------------------------------------------------------------------------------------------
// MMapReader's view of a decoded file: the FileReader sequence of records (rio_frame + rio_decode,
// once per reader) and the SeekNext map (build_seek_map, rio_kernels.hip: every 0x91 position P[k]
// and the record R[k] a SeekNext walk reaching it ends at). ReadNextAt at a record start and SeekNext
// whose walk ends at a decoded record are answered from here by binary search on the calling thread:
// no kernel, no lock, no copy (the data pointer stays valid until rio_reader_free).
struct ReadAtIndex {
    std::vector<uint8_t> out, flags;
    std::vector<uint64_t> out_off, rec_off, P, R;
    uint64_t n = 0;
    // record index i with rec_off[i] == off, or n
    uint64_t find(uint64_t off) const {
        const uint64_t i = lower(off);
        return i < n && rec_off[i] == off ? i : n;
    }
    uint64_t lower(uint64_t off) const {
        return (uint64_t)(std::lower_bound(rec_off.begin(), rec_off.begin() + n, off) - rec_off.begin());
    }
    // ReadNextAt's result for record i (mmap_reader.go:130-203; the FileReader decoded the same bytes)
    int record(uint64_t i, const uint8_t** data, uint64_t* len, int* is_nil) const {
        if (flags[i] & RIO_FLAG_CORRUPT) return RIO_ERR_DECOMPRESS;
        if (flags[i] & RIO_FLAG_EOF) return RIO_EOF_CODEC;
        const bool nil = (flags[i] & RIO_FLAG_NIL) != 0;
        if (is_nil) *is_nil = nil ? 1 : 0;
        if (len) *len = nil ? 0 : out_off[i + 1] - out_off[i];
        if (data) *data = out.data() + out_off[i];
        return RIO_OK;
    }
};

struct rio_reader {
    rio_ctx* ctx = nullptr;
    std::string path;
    bool mmap_mode = false;
    std::atomic<bool> open{false}, closed{false};
    int fd = -1;
    const uint8_t* map = nullptr;
    uint64_t size = 0;
    uint32_t version = 0, compression = 0;
    std::mutex mu;
    // FILE mode: whole-file decode result
    bool decoded = false;
    int decode_rc = RIO_OK;
    rio_file_info info{};
    std::vector<uint8_t> out;
    std::vector<uint64_t> out_off, rec_off;
    std::vector<uint8_t> flags;
    uint64_t cursor = 0;
    bool past_end = false;
    // windowed decode (rio_stream) for files larger than `window`: ReadNext walks the current
    // window's view, then fetches the next; the whole-file decode is the one-window case
    uint64_t window = 0;  // 0: automatic (kAutoWindow above kAutoWindowFrom), ~0: never
    rio_stream* stream = nullptr;
    const uint8_t* w_out = nullptr;
    const uint64_t* w_off = nullptr;
    const uint8_t* w_flags = nullptr;
    uint64_t w_n = 0;
    bool w_last = true;
    // MMAP mode
    bool on_device = false;
    DevBuf dfile;
    std::atomic<uint64_t> seek_len{4096};
    // MMAP mode: the decoded file (built on the first ReadNextAt / SeekNext, then read-only)
    std::atomic<const ReadAtIndex*> ix{nullptr};
    std::unique_ptr<ReadAtIndex> ix_own;
};

// details of the last failed reader call, per calling thread (ReadAtI is used concurrently)
struct LastDetail {
    uint64_t d0 = 0, d1 = 0, off = 0;
};
static thread_local LastDetail tl_det;

static int reader_new(rio_ctx* ctx, const char* path, bool mm, rio_reader** out) {
    if (!ctx || !path || !out) return RIO_ERR_ARG;
    *out = nullptr;
    // NewFileReader / mmap.Open fail on a missing file (file_reader.go:507, mmap_reader.go:366)
    int fd = ::open(path, O_RDONLY);
    if (fd < 0) return RIO_ERR_IO;
    auto* r = new rio_reader();
    r->ctx = ctx;
    r->path = path;
    r->mmap_mode = mm;
    r->fd = fd;
    struct stat st;
    if (fstat(fd, &st) == 0) r->size = (uint64_t)st.st_size;
    *out = r;
    return RIO_OK;
}

extern "C" int rio_reader_new_file(rio_ctx* ctx, const char* path, rio_reader** out) {
    return reader_new(ctx, path, false, out);
}
extern "C" int rio_reader_new_mmap(rio_ctx* ctx, const char* path, rio_reader** out) {
    return reader_new(ctx, path, true, out);
}

extern "C" int rio_reader_open(rio_reader* r) {
    if (!r) return RIO_ERR_ARG;
    std::lock_guard<std::mutex> g(r->mu);
    if (r->open) return RIO_ERR_STATE;    // "already opened"
    if (r->closed) return RIO_ERR_STATE;  // "already closed"
    struct stat st;
    if (fstat(r->fd, &st) != 0) return RIO_ERR_IO;
    r->size = (uint64_t)st.st_size;
    if (r->size) {
        void* m = mmap(nullptr, r->size, PROT_READ, MAP_PRIVATE, r->fd, 0);
        if (m == MAP_FAILED) return RIO_ERR_IO;
        r->map = static_cast<const uint8_t*>(m);
    }
    if (r->size < RIO_FILE_HEADER_BYTES) return RIO_ERR_SHORT_FILE_HEADER;
    const uint8_t* f = r->map;
    r->version = f[0] | (uint32_t)f[1] << 8 | (uint32_t)f[2] << 16 | (uint32_t)f[3] << 24;
    r->compression = f[4] | (uint32_t)f[5] << 8 | (uint32_t)f[6] << 16 | (uint32_t)f[7] << 24;
    if (r->version > RIO_VERSION4 || r->version < RIO_VERSION1) {
        tl_det.d0 = r->version;
        return RIO_ERR_VERSION;
    }
    if (r->compression > RIO_COMP_LZW) {
        tl_det.d0 = r->compression;
        return RIO_ERR_COMPRESSION_TYPE;
    }
    r->open = true;
    return RIO_OK;
}

extern "C" int rio_reader_close(rio_reader* r) {
    if (!r) return RIO_ERR_ARG;
    std::lock_guard<std::mutex> g(r->mu);
    r->closed = true;
    r->open = false;
    if (r->map) munmap(const_cast<uint8_t*>(r->map), r->size);
    r->map = nullptr;
    if (r->stream) rio_stream_free(r->stream);
    r->stream = nullptr;
    r->w_n = 0;
    r->dfile.release();
    r->on_device = false;
    return RIO_OK;
}

extern "C" void rio_reader_free(rio_reader* r) {
    if (!r) return;
    rio_reader_close(r);
    if (r->fd >= 0) ::close(r->fd);
    delete r;
}

extern "C" int rio_reader_header(rio_reader* r, uint32_t* version, uint32_t* compression) {
    if (!r) return RIO_ERR_ARG;
    if (version) *version = r->version;
    if (compression) *compression = r->compression;
    return r->open ? RIO_OK : RIO_ERR_STATE;
}

extern "C" uint64_t rio_reader_size(rio_reader* r) { return r ? r->size : 0; }

extern "C" void rio_reader_last_detail(rio_reader* r, uint64_t* d0, uint64_t* d1, uint64_t* off) {
    if (!r) return;
    if (d0) *d0 = tl_det.d0;
    if (d1) *d1 = tl_det.d1;
    if (off) *off = tl_det.off;
}

// files past 32 MiB are read window by window (rio_stream_*): one window's H2D overlaps earlier windows'
// decode and D2H, where the one-shot pair moves the whole file in, then all records out (round 4)
constexpr uint64_t kAutoWindowFrom = 32ull << 20, kAutoWindow = 128ull << 20;

static uint64_t reader_window(const rio_reader* r) {
    if (r->window == ~0ull) return 0;
    const uint64_t w = r->window ? r->window : kAutoWindow;
    const uint64_t from = r->window ? w : kAutoWindowFrom;
    return r->size > RIO_FILE_HEADER_BYTES + from ? w : 0;
}

// the next window of a streamed file becomes the reader's view
static int stream_fetch(rio_reader* r) {
    uint64_t first = 0;
    const uint8_t *o = nullptr, *fl = nullptr;
    const uint64_t *off = nullptr, *ro = nullptr;
    rio_file_info fi{};
    int rc = rio_stream_next(r->stream, &first, &o, &off, &ro, &fl, &fi);
    if (rc == RIO_EOF) rc = RIO_ERR_STATE;  // the last window was taken already (not reached: w_last)
    if (rc) return rc;
    r->w_out = o;
    r->w_off = off;
    r->w_flags = fl;
    r->w_n = fi.n_records;
    r->w_last = fi.status != RIO_OK;
    r->cursor = 0;
    r->info = fi;
    return RIO_OK;
}

static int file_decode(rio_reader* r) {
    if (r->decoded) return r->decode_rc;
    r->decoded = true;
    if (const uint64_t w = reader_window(r)) {
        int rc = rio_stream_open(r->ctx->device, r->path.c_str(), w, 4, &r->stream);
        if (!rc) rc = stream_fetch(r);
        // a file the device path does not decode is refused at its first window, as below
        if (!rc && r->info.status == RIO_ERR_UNSUPPORTED && r->w_n == 0) rc = RIO_ERR_UNSUPPORTED;
        return r->decode_rc = rc;
    }
    rio_file_info fi{};
    std::lock_guard<std::mutex> cg(r->ctx->mu);
    int rc = rio_frame(r->ctx, r->map, r->size, &fi);
    if (rc) return r->decode_rc = rc;
    if (fi.status == RIO_ERR_UNSUPPORTED) return r->decode_rc = RIO_ERR_UNSUPPORTED;
    r->out.resize(fi.total_out_bytes + 1);
    r->out_off.resize(fi.n_records + 1);
    r->rec_off.resize(fi.n_records + 1);
    r->flags.resize(fi.n_records + 1);
    rc = rio_decode(r->ctx, r->out.data(), fi.total_out_bytes, r->out_off.data(), r->rec_off.data(), r->flags.data(),
                    fi.n_records, &fi);
    if (rc) return r->decode_rc = rc;
    r->info = fi;
    r->w_out = r->out.data();
    r->w_off = r->out_off.data();
    r->w_flags = r->flags.data();
    r->w_n = fi.n_records;
    r->w_last = true;
    return r->decode_rc = RIO_OK;
}

// position the view on the next record: true if there is one, else the view holds the terminal info
static int view_advance(rio_reader* r, bool& have) {
    while (r->cursor >= r->w_n && !r->w_last) {
        const int rc = stream_fetch(r);
        if (rc) return rc;
    }
    have = r->cursor < r->w_n;
    return RIO_OK;
}

extern "C" int rio_reader_set_window(rio_reader* r, uint64_t window_bytes) {
    if (!r) return RIO_ERR_ARG;
    std::lock_guard<std::mutex> g(r->mu);
    if (r->decoded) return RIO_ERR_STATE;
    r->window = window_bytes;
    return RIO_OK;
}

extern "C" int rio_reader_file_info(rio_reader* r, rio_file_info* info) {
    if (!r || !info) return RIO_ERR_ARG;
    std::lock_guard<std::mutex> g(r->mu);
    if (!r->open || r->closed || r->mmap_mode) return RIO_ERR_STATE;
    int rc = file_decode(r);
    if (rc) return rc;
    if (r->stream) return RIO_ERR_STATE;  // windowed: the whole-file totals are not known up front
    *info = r->info;
    return RIO_OK;
}

// terminal status as ReadNext reports it
static int terminal(rio_reader* r) {
    tl_det.d0 = r->info.detail0;
    tl_det.d1 = r->info.detail1;
    tl_det.off = r->info.status_offset;
    return r->info.status;
}

extern "C" int rio_reader_read_next(rio_reader* r, const uint8_t** data, uint64_t* len, int* is_nil) {
    if (!r) return RIO_ERR_ARG;
    std::lock_guard<std::mutex> g(r->mu);
    if (data) *data = nullptr;
    if (len) *len = 0;
    if (is_nil) *is_nil = 0;
    if (!r->open || r->closed || r->mmap_mode) return RIO_ERR_STATE;
    int rc = file_decode(r);
    if (rc) return rc;
    if (r->past_end) return RIO_EOF;
    bool have = false;
    if ((rc = view_advance(r, have))) return rc;
    if (!have) return terminal(r);
    const uint64_t i = r->cursor++;
    // a record whose payload does not decompress: ReadNext returns the codec error (or gzip's bare
    // io.EOF for an empty payload) and the next call goes on with the record after it
    if (r->w_flags[i] & (RIO_FLAG_CORRUPT | RIO_FLAG_EOF)) {
        tl_det.d0 = tl_det.d1 = 0;
        tl_det.off = r->info.status_offset;
        return (r->w_flags[i] & RIO_FLAG_EOF) ? RIO_EOF_CODEC : RIO_ERR_DECOMPRESS;
    }
    if (data) *data = r->w_out + r->w_off[i];
    if (len) *len = r->w_off[i + 1] - r->w_off[i];
    if (is_nil) *is_nil = (r->w_flags[i] & RIO_FLAG_NIL) ? 1 : 0;
    return RIO_OK;
}

// FileReader.SkipNext (file_reader.go:133-172): header parse + seek, no payload read, no
// zero-tail check. Divergence (documented): a nil record in a compressed file is skipped by its
// true extent, not by c bytes (the reference's :151-157 quirk).
extern "C" int rio_reader_skip_next(rio_reader* r) {
    if (!r) return RIO_ERR_ARG;
    std::lock_guard<std::mutex> g(r->mu);
    if (!r->open || r->closed || r->mmap_mode) return RIO_ERR_STATE;
    int rc = file_decode(r);
    if (rc) return rc;
    if (r->past_end) return RIO_EOF;
    bool have = false;
    if ((rc = view_advance(r, have))) return rc;
    if (have) {
        r->cursor++;
        return RIO_OK;
    }
    const int s = terminal(r);
    switch (s) {
    case RIO_EOF_ZERO_TAIL: return RIO_ERR_MAGIC;  // SkipNext does not test for a zero tail
    case RIO_ERR_UNEXPECTED_EOF:  // detail0 == 1: raised by the payload read, else inside a header varint
        if (r->info.detail0 != 1) return s;
        [[fallthrough]];
    case RIO_EOF_PAYLOAD:  // header parsed fine: SkipNext seeks past the payload
        r->past_end = true;
        return RIO_OK;
    default: return s;
    }
}

// ---- ReadAtI (MMapReader.ReadNextAt / SeekNext, mmap_reader.go:58-203) -----------------------
// The file is decoded once (rio_frame + rio_decode on the reader's ctx) into a ReadAtIndex. A
// ReadNextAt at a record start, and a SeekNext whose scan meets only bytes that cannot form a marker
// before a record's header, are answered from it on the calling thread (binary search, no kernel, no
// lock). Everything else (offsets inside records or past the decoded sequence, scans over 0x91
// bytes) runs the single-record kernels (k_read_at / k_seek_next) under the reader's lock, exactly
// as before; for gzip files those kernels locate the record and the host serves the payload from the
// index when the offset is a record start.
// Largest decoded size (and record count) the index is built for: a file past it keeps n = 0 and
// every ReadNextAt / SeekNext takes the single-record kernels (no whole-file host copy, no
// first-call decode of a huge file). The framing's sizes are what the records claim, so a damaged
// header cannot make this allocate more than the cap. RIO_READAT_INDEX_MAX overrides (bytes).
static uint64_t readat_index_cap() {
    static const uint64_t cap = env_u64("RIO_READAT_INDEX_MAX", 4ull << 30);
    return cap;
}

static void build_readat_index(rio_reader* r, ReadAtIndex& x) {
    rio_ctx* ctx = r->ctx;
    std::lock_guard<std::mutex> cg(ctx->mu);
    rio_file_info fi{};
    if (rio_frame(ctx, r->map, r->size, &fi) != RIO_OK) return;
    const uint64_t n0 = fi.n_records;
    if (fi.total_out_bytes > readat_index_cap() || n0 > readat_index_cap() / 16) return;
    try {
        x.out.assign(fi.total_out_bytes + 1, 0);
        x.out_off.assign(n0 + 1, 0);
        x.rec_off.assign(n0 + 1, 0);
        x.flags.assign(n0 + 1, 0);
    } catch (const std::bad_alloc&) {  // never through the C-ABI: the kernels answer instead
        x = ReadAtIndex{};
        return;
    }
    if (rio_decode(ctx, x.out.data(), fi.total_out_bytes, x.out_off.data(), x.rec_off.data(), x.flags.data(), n0, &fi) !=
        RIO_OK)
        return;
    if (fi.status == RIO_ERR_VERSION || fi.status == RIO_ERR_COMPRESSION_TYPE || fi.status == RIO_ERR_SHORT_FILE_HEADER)
        return;
    const uint64_t n = std::min<uint64_t>(fi.n_records, n0);
    // the device file, record offsets and flags of the decode are still in the ctx arenas
    if (build_seek_map(ctx->file.as<uint8_t>(), r->size, ctx->rec_off.as<uint64_t>(), ctx->flags.as<uint8_t>(), n, x.P,
                       x.R, ctx->stream))
        return;
    x.n = n;  // published only complete: a failed build leaves n = 0 (every call takes the kernels)
}

static const ReadAtIndex* readat_index(rio_reader* r) {
    if (const ReadAtIndex* x = r->ix.load(std::memory_order_acquire)) return x;
    std::lock_guard<std::mutex> g(r->mu);
    if (const ReadAtIndex* x = r->ix.load(std::memory_order_relaxed)) return x;
    auto x = std::make_unique<ReadAtIndex>();
    if (r->open && !r->closed) build_readat_index(r, *x);
    r->ix.store(x.get(), std::memory_order_release);
    r->ix_own = std::move(x);
    return r->ix_own.get();
}

static int ensure_on_device(rio_reader* r) {
    if (r->on_device) return RIO_OK;
    HIP_TRY(hipSetDevice(r->ctx->device));
    HIP_TRY(r->dfile.ensure(r->size + RIO_DEVICE_PAD));
    int rc = h2d_staged(r->ctx, r->dfile.p, r->map, r->size);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(r->dfile.as<uint8_t>() + r->size, 0, RIO_DEVICE_PAD, r->ctx->stream));
    HIP_TRY(hipStreamSynchronize(r->ctx->stream));
    r->on_device = true;
    return RIO_OK;
}

// record bytes of a kernel-path result: valid until this thread's next ReadNextAt / SeekNext
static thread_local std::vector<uint8_t> tl_rec;

// the single-record kernels (ReadNextAt at `offset`, or SeekNext scanning from it); *res_out gets the
// kernel's result (a gzip / lzw record it located but did not expand: payload_off, len)
static int readat_kernel(rio_reader* r, uint64_t offset, bool seek, uint64_t seek_len, uint64_t* ro_out,
                         const uint8_t** data, uint64_t* len, int* is_nil, ReadAtResult* res_out = nullptr) {
    std::lock_guard<std::mutex> g(r->mu);
    if (!r->open || r->closed) return RIO_ERR_STATE;
    std::lock_guard<std::mutex> cg(r->ctx->mu);
    int rc = ensure_on_device(r);
    if (rc) return rc;
    ReadAtResult res{};
    uint64_t ro = 0;
    rc = read_at_impl(r->ctx, r->dfile.as<uint8_t>(), r->size, offset, seek, seek_len, &res, seek ? &ro : nullptr);
    if (rc) return rc;
    if (ro_out) *ro_out = ro;
    if (res_out) *res_out = res;
    tl_det.d0 = res.det0;
    tl_det.d1 = res.det1;
    if (res.status != RIO_OK) return res.status;
    if (is_nil) *is_nil = res.nil;
    if (len) *len = res.nil ? 0 : res.len;
    tl_rec.resize(res.len + 1);
    if (!res.nil && res.len) HIP_TRY(hipMemcpy(tl_rec.data(), r->ctx->readat_out.p, res.len, hipMemcpyDeviceToHost));
    if (data) *data = tl_rec.data();
    return RIO_OK;
}

// A gzip / lzw record the whole-file decode never reached (MMapReader.ReadNextAt decodes any record
// start, mmap_reader.go:130-203, e.g. one after a header that fails its CRC, where FileReader stops):
// the single-record kernel located it (res: payload_off, len = payload bytes), and it is decoded here
// as a file of its own (the 8-byte file header, then the record's header and payload) through the
// whole-file path on the reader's context: the same inflate / lzw kernels, Go's multistream and size
// rules included. ReadNextAt's result for it: the record, or the codec's error class.
static thread_local std::vector<uint8_t> tl_x_out, tl_x_flags;
static thread_local std::vector<uint64_t> tl_x_off, tl_x_rec;
static int readat_expand(rio_reader* r, uint64_t rec, const ReadAtResult& res, const uint8_t** data, uint64_t* len,
                         int* is_nil) {
    const uint64_t end = res.payload_off + res.len;
    if (!r->map || res.nil || res.len == 0 || res.payload_off <= rec || end > r->size) return RIO_ERR_UNSUPPORTED;
    std::vector<uint8_t> img(RIO_FILE_HEADER_BYTES + (end - rec));
    memcpy(img.data(), r->map, RIO_FILE_HEADER_BYTES);
    memcpy(img.data() + RIO_FILE_HEADER_BYTES, r->map + rec, end - rec);
    std::lock_guard<std::mutex> g(r->mu);
    if (!r->open || r->closed) return RIO_ERR_STATE;
    std::lock_guard<std::mutex> cg(r->ctx->mu);
    rio_file_info fi{};
    int rc = rio_frame(r->ctx, img.data(), img.size(), &fi);
    if (rc) return rc;
    if (fi.n_records == 0) return RIO_ERR_UNSUPPORTED;  // (the kernel framed it: not reached)
    const uint64_t n = fi.n_records;
    // the sizes are what the (possibly damaged) headers claim: an lzw u may be 4096x its payload.
    // Bounded like the index (readat_index_cap), and an allocation failure is a status, never an
    // exception through the C-ABI
    if (fi.total_out_bytes > readat_index_cap() || n > readat_index_cap() / 16) return RIO_ERR_CAPACITY;
    try {
        tl_x_out.resize(fi.total_out_bytes + 1);
        tl_x_off.resize(n + 1);
        tl_x_rec.resize(n);
        tl_x_flags.resize(n);
    } catch (const std::exception&) {
        return RIO_ERR_CAPACITY;
    }
    rc = rio_decode(r->ctx, tl_x_out.data(), fi.total_out_bytes, tl_x_off.data(), tl_x_rec.data(), tl_x_flags.data(), n,
                    &fi);
    if (rc) return rc;
    if (fi.n_records == 0 || fi.status == RIO_ERR_UNSUPPORTED) return RIO_ERR_UNSUPPORTED;
    if (tl_x_flags[0] & RIO_FLAG_CORRUPT) return RIO_ERR_DECOMPRESS;
    if (tl_x_flags[0] & RIO_FLAG_EOF) return RIO_EOF_CODEC;
    if (is_nil) *is_nil = 0;
    if (len) *len = tl_x_off[1] - tl_x_off[0];
    if (data) *data = tl_x_out.data() + tl_x_off[0];
    return RIO_OK;
}

static int readat_check(rio_reader* r, const uint8_t** data, uint64_t* len, int* is_nil, bool seek) {
    if (data) *data = nullptr;
    if (len) *len = 0;
    if (is_nil) *is_nil = 0;
    if (!r->open || r->closed) return RIO_ERR_STATE;
    // SeekNext: "unsupported on files with version lower than v2" (mmap_reader.go:62-64)
    if (seek && r->version < RIO_VERSION2) return RIO_ERR_UNSUPPORTED;
    return RIO_OK;
}

extern "C" int rio_reader_read_next_at(rio_reader* r, uint64_t offset, const uint8_t** data, uint64_t* len,
                                       int* is_nil) {
    if (!r) return RIO_ERR_ARG;
    if (int rc = readat_check(r, data, len, is_nil, false)) return rc;
    tl_det = LastDetail{0, 0, offset};
    const ReadAtIndex* x = readat_index(r);
    const uint64_t i = x->find(offset);
    if (i < x->n) return x->record(i, data, len, is_nil);
    ReadAtResult res{};
    const int rc = readat_kernel(r, offset, false, 0, nullptr, data, len, is_nil, &res);
    const bool expand = r->compression == RIO_COMP_GZIP || r->compression == RIO_COMP_LZW;
    if (rc == RIO_ERR_UNSUPPORTED && expand) return readat_expand(r, offset, res, data, len, is_nil);
    return rc;
}

extern "C" int rio_reader_seek_next(rio_reader* r, uint64_t offset, uint64_t* rec_offset, const uint8_t** data,
                                    uint64_t* len, int* is_nil) {
    if (!r) return RIO_ERR_ARG;
    if (rec_offset) *rec_offset = 0;
    if (int rc = readat_check(r, data, len, is_nil, true)) return rc;
    tl_det = LastDetail{0, 0, offset};
    const uint64_t seek_len = r->seek_len.load(std::memory_order_relaxed);
    const ReadAtIndex* x = readat_index(r);
    uint64_t s = offset;  // the scan's position: a fresh SeekNext from s continues it exactly
    // with windows of >= 4 bytes the walk is fixed by the first 0x91 at or after s (build_seek_map).
    // Not at 3: mmap_reader.go:89-98 leaves the window once ix >= numRead, also right after the third
    // marker byte, so with seekLen 3 every marker ends the scan in io.EOF (k_seek_next reproduces it)
    if (seek_len >= 4 && s <= r->size && x->n) {
        const uint64_t k = (uint64_t)(std::lower_bound(x->P.begin(), x->P.end(), s) - x->P.begin());
        if (k < x->P.size() && x->R[k] < x->n) {  // else the single-record kernel answers (kSeekOther / io.EOF walks)
            const uint64_t i = x->R[k];
            if (rec_offset) *rec_offset = x->rec_off[i];
            tl_det.off = x->rec_off[i];
            return x->record(i, data, len, is_nil);
        }
    }
    for (;;) {
        uint64_t ro = 0;
        ReadAtResult res{};
        const int rc = readat_kernel(r, s, true, seek_len, &ro, data, len, is_nil, &res);
        if (rec_offset) *rec_offset = ro;
        tl_det.off = rc == RIO_ERR_INVALID_OFFSET ? offset : ro;
        // gzip / lzw: the kernel stops at a trial whose payload needs expanding; a record start is served
        // from the decoded index, any other record is expanded on its own (readat_expand); an io.EOF-class
        // trial (an empty gzip payload) continues the scan as mmap_reader.go:105-114 does
        const bool expand = r->compression == RIO_COMP_GZIP || r->compression == RIO_COMP_LZW;
        if (rc != RIO_ERR_UNSUPPORTED || !expand) return rc;
        const uint64_t i = x->find(ro);
        int rx;
        if (i < x->n) {
            rx = x->record(i, data, len, is_nil);
        } else {
            rx = readat_expand(r, ro, res, data, len, is_nil);
        }
        if (rx == RIO_EOF_CODEC) {
            s = ro + 3;
            continue;
        }
        return rx;
    }
}

extern "C" int rio_reader_set_seek_len(rio_reader* r, uint64_t seek_len) {
    if (!r || seek_len == 0) return RIO_ERR_ARG;
    r->seek_len.store(seek_len, std::memory_order_relaxed);
    return RIO_OK;
}

// ------------------------------------------------------------------------------------------
// sstables: index parse + value validation on decoded arenas (rio_sstable.hip)
// ------------------------------------------------------------------------------------------
extern "C" int rio_sst_index_parse(rio_ctx* ctx, const uint8_t* d_index_out, const uint64_t* d_index_off, uint64_t n,
                                   uint64_t* d_key_off, uint64_t* d_key_len, uint64_t* d_value_off,
                                   uint64_t* d_checksum, uint64_t* d_result, void* stream) {
    if (!ctx || !d_index_off || !d_result || (n && (!d_index_out || !d_key_off || !d_key_len || !d_value_off || !d_checksum)))
        return RIO_ERR_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    HIP_TRY(launch_sst_index(d_index_out, d_index_off, n, d_key_off, d_key_len, d_value_off, d_checksum, d_result, s));
    return RIO_OK;
}

extern "C" int rio_sst_validate(rio_ctx* ctx, const uint8_t* d_data_out, const uint64_t* d_data_off,
                                const uint64_t* d_data_rec_off, uint64_t n_data, const uint64_t* d_value_off,
                                const uint64_t* d_checksum, uint64_t n_index, uint64_t* d_crc_out, uint64_t* d_result,
                                void* stream) {
    if (!ctx || !d_result || (n_index && (!d_value_off || !d_checksum || !d_crc_out || !d_data_off || !d_data_rec_off)))
        return RIO_ERR_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    HIP_TRY(launch_sst_validate(d_data_out, d_data_off, d_data_rec_off, n_data, d_value_off, d_checksum, n_index,
                                d_crc_out, d_result, s));
    return RIO_OK;
}

extern "C" int rio_sst_data_entries(rio_ctx* ctx, const uint8_t* d_data_out, const uint64_t* d_data_off, uint64_t n_data,
                                    uint64_t* d_view, uint64_t* d_result, void* stream) {
    if (!ctx || !d_data_off || !d_result || (n_data && (!d_data_out || !d_view))) return RIO_ERR_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    HIP_TRY(launch_sst_data_entry(d_data_out, d_data_off, n_data, d_view, d_result, s));
    return RIO_OK;
}

extern "C" int rio_sst_validate_view(rio_ctx* ctx, const uint8_t* d_data_out, const uint64_t* d_data_off,
                                     const uint64_t* d_data_rec_off, uint64_t n_data, const uint64_t* d_view,
                                     const uint64_t* d_value_off, const uint64_t* d_checksum, uint64_t n_index,
                                     uint64_t* d_crc_out, uint64_t* d_result, void* stream) {
    if (!ctx || !d_result ||
        (n_index && (!d_value_off || !d_checksum || !d_crc_out || !d_data_off || !d_data_rec_off || !d_view)))
        return RIO_ERR_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    HIP_TRY(launch_sst_validate(d_data_out, d_data_off, d_data_rec_off, n_data, d_value_off, d_checksum, n_index,
                                d_crc_out, d_result, s, d_view));
    return RIO_OK;
}

// ------------------------------------------------------------------------------------------
// sstables: host-memory table handle (the cgo NewSSTableReader binding)
// ------------------------------------------------------------------------------------------
struct rio_sst {
    std::vector<uint8_t> index, data, index_flags, data_flags;
    std::vector<uint64_t> index_off, index_rec_off, data_off, data_rec_off;
    std::vector<uint64_t> key_off, key_len, value_off, checksum, crc;
    std::vector<uint64_t> view;  // v0 tables: DataEntry.value ranges per data record (rio_sst_data_entries)
    bool v0 = false;
    rio_sst_info info{};
};

// rio_frame + rio_decode into host vectors; the device arenas (ctx->out, out_off, rec_off) keep
// the decoded file until the next decode on this ctx
static int sst_decode_host(rio_ctx* ctx, const uint8_t* file, uint64_t len, std::vector<uint8_t>& out,
                           std::vector<uint64_t>& off, std::vector<uint64_t>& rec_off, std::vector<uint8_t>& flags,
                           rio_file_info& info) {
    int rc = rio_frame(ctx, file, len, &info);
    if (rc) return rc;
    const uint64_t n = info.n_records;
    out.assign(info.total_out_bytes + 1, 0);
    off.assign(n + 1, 0);
    rec_off.assign(n + 1, 0);
    flags.assign(n + 1, 0);
    rc = rio_decode(ctx, out.data(), info.total_out_bytes, off.data(), rec_off.data(), flags.data(), n, &info);
    if (rc) return rc;
    off.resize(info.n_records + 1);
    return RIO_OK;
}

static bool sst_header_level(int s) {
    return s == RIO_ERR_VERSION || s == RIO_ERR_COMPRESSION_TYPE || s == RIO_ERR_SHORT_FILE_HEADER;
}

extern "C" int rio_sst_open(rio_ctx* ctx, const uint8_t* index_file, uint64_t index_len, const uint8_t* data_file,
                            uint64_t data_len, rio_sst** out, rio_sst_info* info) {
    return rio_sst_open_ex(ctx, index_file, index_len, data_file, data_len, 0, out, info);
}

extern "C" int rio_sst_open_ex(rio_ctx* ctx, const uint8_t* index_file, uint64_t index_len, const uint8_t* data_file,
                               uint64_t data_len, uint32_t flags, rio_sst** out, rio_sst_info* info) {
    if (!ctx || !out || !info || (!index_file && index_len) || (!data_file && data_len)) return RIO_ERR_ARG;
    *out = nullptr;
    memset(info, 0, sizeof *info);
    HIP_TRY(hipSetDevice(ctx->device));
    auto* t = new rio_sst();
    t->v0 = (flags & RIO_SST_V0_VALUES) != 0;
    rio_sst_info& I = t->info;
    I.first_bad_proto = I.first_bad_crc = I.first_unplaced = I.index_bad = I.first_bad_value = ~0ull;
    int rc = sst_decode_host(ctx, index_file, index_len, t->index, t->index_off, t->index_rec_off, t->index_flags, I.index);
    uint64_t n = 0;
    if (!rc && !sst_header_level(I.index.status) && I.index.status != RIO_ERR_UNSUPPORTED) {
        // the index arena is on the device (ctx->out / ctx->out_off): parse it there
        n = I.index.n_records;
        // an index record that does not decompress ends Load's ReadNext loop (slice_key_index.go:
        // 117-126): ErrCorrupt fails the load there, gzip's bare io.EOF ends the index cleanly
        if (I.index.n_bad && I.index.first_bad < n) {
            if (t->index_flags[I.index.first_bad] & RIO_FLAG_CORRUPT) I.index_bad = I.index.first_bad;
            n = I.index.first_bad;
        }
        const uint64_t nn = std::max<uint64_t>(n, 1);
        if (ctx->sst_fields.ensure(nn * 32) || ctx->sst_crc.ensure(nn * 8) || ctx->sst_res.ensure(32)) rc = RIO_ERR_HIP;
        uint64_t* f = ctx->sst_fields.as<uint64_t>();
        uint64_t* res = ctx->sst_res.as<uint64_t>();
        if (!rc && launch_sst_index(ctx->out.as<uint8_t>(), ctx->out_off.as<uint64_t>(), n, f, f + nn, f + 2 * nn,
                                    f + 3 * nn, res, ctx->stream) != hipSuccess)
            rc = RIO_ERR_HIP;
        t->key_off.assign(nn, 0);
        t->key_len.assign(nn, 0);
        t->value_off.assign(nn, 0);
        t->checksum.assign(nn, 0);
        t->crc.assign(nn, 0);
        std::vector<uint64_t>* dst[4] = {&t->key_off, &t->key_len, &t->value_off, &t->checksum};
        for (int k = 0; k < 4 && !rc; k++)
            rc = d2h_staged(ctx, reinterpret_cast<uint8_t*>(dst[k]->data()), f + k * nn, nn * 8);
        if (!rc) rc = d2h_staged(ctx, reinterpret_cast<uint8_t*>(&I.first_bad_proto), res, 8);
        if (!rc) {
            // key offsets are absolute into the index arena, which t->index mirrors
            rc = sst_decode_host(ctx, data_file, data_len, t->data, t->data_off, t->data_rec_off, t->data_flags, I.data);
        }
        if (!rc && !sst_header_level(I.data.status) && I.data.status != RIO_ERR_UNSUPPORTED) {
            const uint64_t* view = nullptr;
            if (t->v0) {  // DataEntry values: their ranges in the data arena, then hashed as such
                const uint64_t nd = std::max<uint64_t>(I.data.n_records, 1);
                if (ctx->sst_view.ensure(nd * 16)) rc = RIO_ERR_HIP;
                if (!rc && launch_sst_data_entry(ctx->out.as<uint8_t>(), ctx->out_off.as<uint64_t>(), I.data.n_records,
                                                 ctx->sst_view.as<uint64_t>(), res + 3, ctx->stream) != hipSuccess)
                    rc = RIO_ERR_HIP;
                t->view.assign(2 * nd, 0);
                if (!rc) rc = d2h_staged(ctx, reinterpret_cast<uint8_t*>(t->view.data()), ctx->sst_view.p, nd * 16);
                if (!rc) rc = d2h_staged(ctx, reinterpret_cast<uint8_t*>(&I.first_bad_value), res + 3, 8);
                view = ctx->sst_view.as<uint64_t>();
            }
            if (!rc && launch_sst_validate(ctx->out.as<uint8_t>(), ctx->out_off.as<uint64_t>(), ctx->rec_off.as<uint64_t>(),
                                           I.data.n_records, f + 2 * nn, f + 3 * nn, n, ctx->sst_crc.as<uint64_t>(),
                                           res + 1, ctx->stream, view) != hipSuccess)
                rc = RIO_ERR_HIP;
            if (!rc) rc = d2h_staged(ctx, reinterpret_cast<uint8_t*>(t->crc.data()), ctx->sst_crc.p, nn * 8);
            uint64_t vr[2] = {~0ull, ~0ull};
            if (!rc) rc = d2h_staged(ctx, reinterpret_cast<uint8_t*>(vr), res + 1, 16);
            I.first_bad_crc = t->v0 ? ~0ull : vr[0];  // validateDataFile returns at once for v0 (:205-209)
            I.first_unplaced = vr[1];
        }
    }
    I.n_entries = n;
    *info = I;
    if (rc) {
        delete t;
        return rc;
    }
    if (I.index.status == RIO_ERR_UNSUPPORTED || I.data.status == RIO_ERR_UNSUPPORTED) {
        delete t;
        return RIO_ERR_UNSUPPORTED;
    }
    *out = t;
    return RIO_OK;
}

extern "C" int rio_sst_entry(const rio_sst* t, uint64_t i, const uint8_t** key, uint64_t* key_len,
                             const uint8_t** value, uint64_t* value_len, int* is_nil, uint64_t* value_offset,
                             uint64_t* checksum, uint64_t* crc) {
    if (!t || i >= t->info.n_entries) return RIO_ERR_ARG;
    if (key) *key = t->index.data() + t->key_off[i];
    if (key_len) *key_len = t->key_len[i];
    if (value_offset) *value_offset = t->value_off[i];
    if (checksum) *checksum = t->checksum[i];
    if (crc) *crc = t->crc[i];
    if (i >= t->info.data.n_records) {
        if (value) *value = nullptr;
        if (value_len) *value_len = 0;
        if (is_nil) *is_nil = 0;
        return t->info.data.status == RIO_OK ? RIO_EOF : t->info.data.status;
    }
    if (t->data_flags[i] & (RIO_FLAG_CORRUPT | RIO_FLAG_EOF)) {  // the scan's ReadNext error for this value
        if (value) *value = nullptr;
        if (value_len) *value_len = 0;
        if (is_nil) *is_nil = 0;
        return (t->data_flags[i] & RIO_FLAG_EOF) ? RIO_EOF_CODEC : RIO_ERR_DECOMPRESS;
    }
    if (t->v0) {  // DataEntry.value of data record i
        const uint64_t b = t->view[2 * i], e = t->view[2 * i + 1];
        const bool nil = b == RIO_VALUE_NIL || b == RIO_VALUE_BAD;
        if (value) *value = nil ? nullptr : t->data.data() + b;
        if (value_len) *value_len = nil ? 0 : e - b;
        if (is_nil) *is_nil = b == RIO_VALUE_NIL ? 1 : 0;
        return b == RIO_VALUE_BAD ? RIO_ERR_PROTO : RIO_OK;
    }
    const bool nil = (t->data_flags[i] & RIO_FLAG_NIL) != 0;
    if (value) *value = nil ? nullptr : t->data.data() + t->data_off[i];
    if (value_len) *value_len = t->data_off[i + 1] - t->data_off[i];
    if (is_nil) *is_nil = nil ? 1 : 0;
    return RIO_OK;
}

extern "C" void rio_sst_free(rio_sst* t) { delete t; }

// ------------------------------------------------------------------------------------------
// DiskKeyIndex lookups (k_index_search in rio_kernels.hip)
// ------------------------------------------------------------------------------------------
extern "C" int rio_device_index_search(rio_ctx* ctx, const uint8_t* d_file, uint64_t len, uint64_t seek_len,
                                       const uint8_t* d_keys, const uint64_t* d_key_off, uint64_t n,
                                       rio_index_hit* d_hits, void* stream) {
    if (!ctx || !d_file || (n && (!d_keys || !d_key_off || !d_hits))) return RIO_ERR_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    const uint32_t* perm = nullptr;
    if (n >= 4096 && n < 0x7FFFFFFFull) {  // big batches: visit the queries in key order (rio_sort.hip)
        const size_t tb = std::max<size_t>(key_sort_tmp_bytes(n), 256);
        HIP_TRY(ctx->q_pfx.ensure(n * 8));
        HIP_TRY(ctx->q_pfx_out.ensure(n * 8));
        HIP_TRY(ctx->q_idx.ensure(n * 4));
        HIP_TRY(ctx->q_perm.ensure(n * 4));
        HIP_TRY(ctx->q_tmp.ensure(tb));
        HIP_TRY(launch_key_sort(d_keys, d_key_off, n, ctx->q_pfx.as<uint64_t>(), ctx->q_pfx_out.as<uint64_t>(),
                                ctx->q_idx.as<uint32_t>(), ctx->q_perm.as<uint32_t>(), ctx->q_tmp.p, ctx->q_tmp.cap, s));
        perm = ctx->q_perm.as<uint32_t>();
    }
    HIP_TRY(launch_index_search(d_file, len, seek_len ? seek_len : 4096, d_keys, d_key_off, n, perm, d_hits, s));
    return RIO_OK;
}

struct rio_index {
    rio_ctx* ctx = nullptr;
    uint64_t len = 0;
    DevBuf file, keys, key_off, hits;
    // a compressed index.rio: its decoded records and SeekNext map (k_index_search_view)
    bool view = false;
    uint64_t n = 0, K = 0;
    DevBuf v_out, v_off, v_rec, v_flags, v_P, v_R;
};

// The view of a compressed index (DiskKeyIndex over rProto.NewMMapProtoReaderWithPath, which decompresses
// every record it reads, sstables/disk_key_index.go:173): the FileReader sequence of records (rio_frame +
// rio_decode on the index's context) and the SeekNext map over the file (build_seek_map), all resident.
static int index_build_view(rio_index* x, const uint8_t* file, uint64_t len) {
    rio_ctx* ctx = x->ctx;
    std::lock_guard<std::mutex> cg(ctx->mu);  // reader handles sharing the context take it around device use
    rio_file_info fi{};
    int rc = rio_frame(ctx, file, len, &fi);
    if (rc) return rc;
    if (fi.status == RIO_ERR_VERSION || fi.status == RIO_ERR_COMPRESSION_TYPE || fi.status == RIO_ERR_UNSUPPORTED ||
        fi.status == RIO_ERR_SHORT_FILE_HEADER)
        return RIO_OK;  // no view: the kernel reports the header's status per query
    const uint64_t n = fi.n_records, nb = fi.total_out_bytes;
    std::vector<uint8_t> out(nb + 1), flags(n + 1);
    std::vector<uint64_t> off(n + 1), rec(n + 1);
    rc = rio_decode(ctx, out.data(), nb, off.data(), rec.data(), flags.data(), n, &fi);
    if (rc) return rc;
    const uint64_t m = std::min<uint64_t>(fi.n_records, n);
    HIP_TRY(x->v_out.ensure(nb + 16));
    HIP_TRY(x->v_off.ensure((m + 1) * 8));
    HIP_TRY(x->v_rec.ensure((m + 1) * 8));
    HIP_TRY(x->v_flags.ensure(m + 8));
    if (nb) HIP_TRY(hipMemcpyAsync(x->v_out.p, out.data(), nb, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(x->v_off.p, off.data(), (m + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
    if (m) {
        HIP_TRY(hipMemcpyAsync(x->v_rec.p, rec.data(), m * 8, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(hipMemcpyAsync(x->v_flags.p, flags.data(), m, hipMemcpyHostToDevice, ctx->stream));
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    std::vector<uint64_t> P, R;
    if (build_seek_map(x->file.as<uint8_t>(), len, x->v_rec.as<uint64_t>(), x->v_flags.as<uint8_t>(), m, P, R,
                       ctx->stream))
        return RIO_ERR_HIP;
    HIP_TRY(x->v_P.ensure(P.size() * 8 + 8));
    HIP_TRY(x->v_R.ensure(R.size() * 8 + 8));
    if (!P.empty()) {
        HIP_TRY(hipMemcpyAsync(x->v_P.p, P.data(), P.size() * 8, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(hipMemcpyAsync(x->v_R.p, R.data(), R.size() * 8, hipMemcpyHostToDevice, ctx->stream));
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    x->n = m;
    x->K = P.size();
    x->view = true;
    return RIO_OK;
}

extern "C" int rio_index_open(rio_ctx* ctx, const uint8_t* file, uint64_t len, rio_index** out) {
    if (!ctx || !out || (!file && len)) return RIO_ERR_ARG;
    *out = nullptr;
    HIP_TRY(hipSetDevice(ctx->device));
    auto* x = new rio_index();
    x->ctx = ctx;
    x->len = len;
    int rc = x->file.ensure(len + RIO_DEVICE_PAD) ? RIO_ERR_HIP : RIO_OK;
    if (!rc) rc = h2d_staged(ctx, x->file.p, file, len);
    if (!rc && hipMemsetAsync(x->file.as<uint8_t>() + len, 0, RIO_DEVICE_PAD, ctx->stream) != hipSuccess) rc = RIO_ERR_HIP;
    if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = RIO_ERR_HIP;
    if (!rc && len >= RIO_FILE_HEADER_BYTES) {
        const uint32_t v = file[0] | (uint32_t)file[1] << 8 | (uint32_t)file[2] << 16 | (uint32_t)file[3] << 24;
        const uint32_t c = file[4] | (uint32_t)file[5] << 8 | (uint32_t)file[6] << 16 | (uint32_t)file[7] << 24;
        if (v >= RIO_VERSION1 && v <= RIO_VERSION4 && c != RIO_COMP_NONE && c <= RIO_COMP_LZW) rc = index_build_view(x, file, len);
    }
    if (rc) {
        for (DevBuf* b : {&x->file, &x->v_out, &x->v_off, &x->v_rec, &x->v_flags, &x->v_P, &x->v_R}) b->release();
        delete x;
        return rc;
    }
    *out = x;
    return RIO_OK;
}

extern "C" int rio_index_search(rio_index* x, const uint8_t* keys, const uint64_t* key_off, uint64_t n,
                                rio_index_hit* hits) {
    if (!x || (n && (!key_off || !hits))) return RIO_ERR_ARG;
    if (n == 0) return RIO_OK;
    rio_ctx* ctx = x->ctx;
    HIP_TRY(hipSetDevice(ctx->device));
    const uint64_t kb = key_off[n];
    if (kb && !keys) return RIO_ERR_ARG;
    HIP_TRY(x->keys.ensure(kb + 16));
    HIP_TRY(x->key_off.ensure((n + 1) * 8));
    HIP_TRY(x->hits.ensure(n * sizeof(rio_index_hit)));
    int rc = kb ? h2d_staged(ctx, x->keys.p, keys, kb) : RIO_OK;
    if (!rc) rc = h2d_staged(ctx, x->key_off.p, reinterpret_cast<const uint8_t*>(key_off), (n + 1) * 8);
    if (rc) return rc;
    if (x->view) {
        HIP_TRY(launch_index_search_view(x->v_out.as<uint8_t>(), x->v_off.as<uint64_t>(), x->v_flags.as<uint8_t>(), x->n,
                                         x->v_P.as<uint64_t>(), x->K, x->v_R.as<uint64_t>(), x->len, x->keys.as<uint8_t>(),
                                         x->key_off.as<uint64_t>(), n, nullptr, x->hits.as<rio_index_hit>(), ctx->stream));
    } else {
        rc = rio_device_index_search(ctx, x->file.as<uint8_t>(), x->len, 4096, x->keys.as<uint8_t>(),
                                     x->key_off.as<uint64_t>(), n, x->hits.as<rio_index_hit>(), nullptr);
        if (rc) return rc;
    }
    return d2h_staged(ctx, reinterpret_cast<uint8_t*>(hits), x->hits.p, n * sizeof(rio_index_hit));
}

extern "C" void rio_index_free(rio_index* x) {
    if (!x) return;
    hipSetDevice(x->ctx->device);
    hipStreamSynchronize(x->ctx->stream);
    for (DevBuf* b : {&x->file, &x->keys, &x->key_off, &x->hits, &x->v_out, &x->v_off, &x->v_rec, &x->v_flags, &x->v_P,
                      &x->v_R})
        b->release();
    delete x;
}

// ------------------------------------------------------------------------------------------
// recordio v4 encoding (rio_encode.hip)
// ------------------------------------------------------------------------------------------
extern "C" uint64_t rio_encode_bound(uint64_t n, uint64_t total_bytes, uint32_t compression) {
    const uint64_t payload = compression == RIO_COMP_SNAPPY ? 32 * n + total_bytes + total_bytes / 6 : total_bytes;
    return RIO_FILE_HEADER_BYTES + RIO_RECORD_HEADER_V4_MAX * n + payload + 64;
}

extern "C" int rio_device_encode(rio_ctx* ctx, const uint8_t* d_records, const uint64_t* d_rec_off,
                                 const uint8_t* d_flags, uint64_t n, uint64_t total_bytes, uint32_t compression,
                                 uint8_t* d_out, uint64_t out_cap, uint64_t* d_out_rec_off, uint64_t* d_out_len,
                                 void* stream) {
    if (!ctx || !d_rec_off || !d_out || !d_out_len || (n && (!d_records || !d_out_rec_off))) return RIO_ERR_ARG;
    if (compression != RIO_COMP_NONE && compression != RIO_COMP_SNAPPY) return RIO_ERR_UNSUPPORTED;
    HIP_TRY(hipSetDevice(ctx->device));
    const size_t cub = std::max<size_t>(enc_cub_bytes(n), 256);
    HIP_TRY(ctx->enc_scr.ensure(enc_scratch_bytes(n, total_bytes, compression)));
    HIP_TRY(ctx->enc_scr_off.ensure((n + 1) * 8));
    HIP_TRY(ctx->enc_clen.ensure(n * 8 + 8));
    // per-lane global hash tables only when some record can exceed the LDS kernel's 1 KiB
    if (compression == RIO_COMP_SNAPPY) HIP_TRY(ctx->enc_tab.ensure(enc_table_bytes()));
    HIP_TRY(ctx->enc_hdr.ensure(n * 64 + 64));
    HIP_TRY(ctx->enc_size.ensure((n + 1) * 8));
    HIP_TRY(ctx->enc_tmp.ensure((n + 1) * 8));
    HIP_TRY(ctx->enc_cub.ensure(cub));
    EncParams P{};
    P.rec = d_records;
    P.rec_off = d_rec_off;
    P.flags = d_flags;
    P.n = n;
    P.compression = compression;
    P.scratch = ctx->enc_scr.as<uint8_t>();
    P.scr_off = ctx->enc_scr_off.as<uint64_t>();
    P.clen = ctx->enc_clen.as<uint64_t>();
    P.gtab = ctx->enc_tab.as<uint16_t>();
    P.hdr = ctx->enc_hdr.as<uint8_t>();
    P.size = ctx->enc_size.as<uint64_t>();
    P.tmp = ctx->enc_tmp.as<uint64_t>();
    P.out = d_out;
    P.out_cap = out_cap;
    P.out_rec_off = d_out_rec_off;
    P.out_len = d_out_len;
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    HIP_TRY(launch_encode(P, ctx->enc_cub.p, ctx->enc_cub.cap, s));
    return RIO_OK;
}

extern "C" int rio_encode_file(rio_ctx* ctx, const uint8_t* records, const uint64_t* rec_off, const uint8_t* flags,
                               uint64_t n, uint32_t compression, uint8_t* out, uint64_t out_cap, uint64_t* out_rec_off,
                               uint64_t* out_len) {
    if (!ctx || !rec_off || !out_len || (n && !out_rec_off)) return RIO_ERR_ARG;
    HIP_TRY(hipSetDevice(ctx->device));
    const uint64_t total = rec_off[n] - rec_off[0];
    if (total && !records) return RIO_ERR_ARG;
    const uint64_t bound = rio_encode_bound(n, total, compression);
    HIP_TRY(ctx->enc_rec.ensure(total + RIO_DEVICE_PAD));
    HIP_TRY(ctx->enc_rec_off.ensure((n + 1) * 8));
    HIP_TRY(ctx->enc_flags.ensure(n + 8));
    HIP_TRY(ctx->enc_out.ensure(bound));
    HIP_TRY(ctx->enc_out_off.ensure(n * 8 + 8));
    HIP_TRY(ctx->enc_len.ensure(8));
    int rc = total ? h2d_staged(ctx, ctx->enc_rec.p, records + rec_off[0], total) : RIO_OK;
    // offsets relative to the first record
    std::vector<uint64_t> rel(n + 1);
    for (uint64_t i = 0; i <= n; i++) rel[i] = rec_off[i] - rec_off[0];
    if (!rc) rc = h2d_staged(ctx, ctx->enc_rec_off.p, reinterpret_cast<const uint8_t*>(rel.data()), (n + 1) * 8);
    if (!rc && flags && n) rc = h2d_staged(ctx, ctx->enc_flags.p, flags, n);
    if (rc) return rc;
    rc = rio_device_encode(ctx, ctx->enc_rec.as<uint8_t>(), ctx->enc_rec_off.as<uint64_t>(),
                           flags ? ctx->enc_flags.as<uint8_t>() : nullptr, n, total, compression,
                           ctx->enc_out.as<uint8_t>(), bound, ctx->enc_out_off.as<uint64_t>(),
                           ctx->enc_len.as<uint64_t>(), nullptr);
    if (rc) return rc;
    uint64_t len = 0;
    rc = d2h_staged(ctx, reinterpret_cast<uint8_t*>(&len), ctx->enc_len.p, 8);
    if (rc) return rc;
    *out_len = len;
    if (len > out_cap || !out) return RIO_ERR_CAPACITY;
    rc = d2h_staged(ctx, out, ctx->enc_out.p, len);
    if (!rc && n) rc = d2h_staged(ctx, reinterpret_cast<uint8_t*>(out_rec_off), ctx->enc_out_off.p, n * 8);
    return rc;
}
