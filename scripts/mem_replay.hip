// mem_replay.hip — the vector-memory schedule of k_snappy_pipe on C2, replayed without the decode, to find what
// the address path (TA / TCP / TD) costs the decoder and what a cooperative input prefetch would save.
// Model of one lane = one 1 KiB record, 136 steps (C2: 134 pieces per record), 8 waves per CU as in the
// decoder (80 KiB of LDS per 4-wave workgroup), three vector-memory operations per step in the decoder's order:
//   store   cooperative flush: owners 16 (j % 4) .. + 15, each quad stores one owner's next 64-B block
//           when the owner has one complete (output grows 1024 / 136 bytes per step);
//   far     16 B at a 4-aligned position 232..1000 bytes below the lane's output position, 16 per record
//           (C2's far pieces; 11 % of 136 steps), from a hash of (record, step);
//   input   the lane's next 16-B input chunk whenever its parse position (560 B per record) needs it,
//           4 chunks ahead (the decoder's 64-B input ring).
// Loads are consumed 3 steps after issue (4 rotating slots, as the decoder's vmcnt schedule). V VALU per
// step (v_alignbyte chains) stand in for the decode. Modes switch one stream to out-of-range offsets, or
// the input to a quad-cooperative prefetch (4 lanes load 64 contiguous bytes of one owner's record; each
// owner is served every 4th step).
// Round 6: the step count per record (kSteps) and LDS dword reads / writes per step (kR / kW, per-lane columns of
// the decoder's image layout: conflict-free) are template parameters, so candidate step shapes are priced before
// they are built: "cand" rows (main) give each candidate's (steps, VALU, VMEM streams, LDS ops).
// Standalone: hipcc --offload-arch=gfx950 -O3 scripts/mem_replay.hip -o scripts/mem_replay && scripts/mem_replay
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr uint32_t kRecs = 1u << 20;
constexpr uint32_t kInStride = 576;  // compressed record + header
constexpr uint32_t kInLen = 560;
constexpr uint32_t kOutLen = 1024;
constexpr uint32_t kOob = 0xFFFFFFC0u;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

enum { kAll = 0, kNoStore = 1, kNoFar = 2, kNoIn = 3, kCoopIn = 4, kNone = 5, kNoFarCoopIn = 6, kMerged = 7, kMasked = 8 };

__device__ __forceinline__ uint32_t hsh(uint32_t a, uint32_t b) {
    uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u;
    h ^= h >> 15;
    h *= 0xC2B2AE3Du;
    return h ^ (h >> 13);
}

template <int kMode, int kV, int kSteps = 136, int kR = 0, int kW = 0>
__global__ void __launch_bounds__(256) k_replay(const uint8_t* in, uint8_t* out, uint32_t* res, uint32_t* next) {
    extern __shared__ uint32_t lds[];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t nwaves = gridDim.x * 4;
    // 32-bit offsets fit: 1M x 576 < 2^30, 1M x 1024 = 2^30
    const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, kRecs * kInStride, 0x00020000);
    const __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc((void*)out, (short)0, kRecs * kOutLen, 0x00020000);
    uint32_t x = lane, x1 = lane + 1, x2 = lane + 2, x3 = lane + 3;
    v4u acc = {0, 0, 0, 0};
    uint32_t chunk = wave;
    const uint32_t nchunks = kRecs / 64;
    while (chunk < nchunks) {
        const uint32_t r = chunk * 64 + lane;
        const uint32_t ib = r * kInStride, ob = r * kOutLen;
        uint32_t cn = 4;       // next input chunk to load (4 primed)
        uint32_t fl[4] = {0, 0, 0, 0};  // blocks flushed by owner group g (uniform: every owner grows alike)
        v4u f0 = {0, 0, 0, 0}, f1 = f0, f2 = f0, f3 = f0, i0 = f0, i1 = f0, i2 = f0, i3 = f0;
        auto step = [&](uint32_t j, v4u& fs, v4u& is) __attribute__((always_inline)) {
            // consume the slot's loads issued 4 steps ago (the decoder lands them after 3)
            acc ^= fs;
            acc ^= is;
            const uint32_t d = j * kOutLen / kSteps;  // output position
            // 1. flush store
            {
                const uint32_t g = j & 3, o = 16 * g + (lane >> 2);
                const uint32_t ready = d / 64;
                uint32_t f = g == 0 ? fl[0] : g == 1 ? fl[1] : g == 2 ? fl[2] : fl[3];
                const bool go = ready > f && kMode != kNoStore && kMode != kNone;
                const uint32_t off = go ? (chunk * 64 + o) * kOutLen + 64 * f + 16 * (lane & 3) : kOob;
                const v4u w = {j, lane, r, 7};
                if (kMode == kMasked) {
                    if (go) __builtin_amdgcn_raw_buffer_store_b128(w, rout, off, 0, 2);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b128(w, rout, off, 0, 2);
                }
                f += ready > f ? 1 : 0;
                if (g == 0) fl[0] = f; else if (g == 1) fl[1] = f; else if (g == 2) fl[2] = f; else fl[3] = f;
            }
            // 2. far load
            {
                const uint32_t h = hsh(r, j);
                const uint32_t back = 232 + (h >> 8) % 768;
                const bool far = (h & 1023) < 16u * 1024u / kSteps && d >= back + 16 && kMode != kNoFar && kMode != kNone && kMode != kNoFarCoopIn;
                if (kMode == kMerged) {
                    // one load per step: the far piece when there is one, else the input chunk
                    const uint32_t need = 4 + (j * kInLen / kSteps) / 16;
                    const bool gin = !far && cn < need && cn * 16 < kInLen;
                    const uint8_t* a = far ? out + ob + ((d - back) & ~3u) : gin ? in + ib + 16 * cn : out + (size_t)wave * 64;
                    fs = *reinterpret_cast<const v4u*>(a);
                    cn += gin ? 1 : 0;
                } else if (kMode == kMasked) {
                    if (far) fs = __builtin_amdgcn_raw_buffer_load_b128(rout, ob + ((d - back) & ~3u), 0, 0);
                } else {
                    fs = __builtin_amdgcn_raw_buffer_load_b128(rout, far ? ob + ((d - back) & ~3u) : kOob, 0, 0);
                }
            }
            // 3. input prefetch
            {
                const uint32_t need = 4 + (j * kInLen / kSteps) / 16;  // chunks the ring must hold
                if (kMode == kCoopIn || kMode == kNoFarCoopIn) {
                    // owner group g's records, one 64-B block per turn when the owner's ring has room
                    const uint32_t g = j & 3, o = 16 * g + (lane >> 2);
                    const uint32_t blk = need / 4;  // block the owner needs next (uniform model)
                    const bool go = (need & 3) == 0 && blk * 64 < kInLen;
                    const uint32_t off = go ? (chunk * 64 + o) * kInStride + 64 * blk + 16 * (lane & 3) : kOob;
                    is = __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, 0);
                } else if (kMode == kMerged) {
                } else if (kMode == kMasked) {
                    const bool go = cn < need && cn * 16 < kInLen;
                    if (go) is = __builtin_amdgcn_raw_buffer_load_b128(rin, ib + 16 * cn, 0, 0);
                    cn += go ? 1 : 0;
                } else {
                    const bool go = cn < need && cn * 16 < kInLen && kMode != kNoIn && kMode != kNone;
                    is = __builtin_amdgcn_raw_buffer_load_b128(rin, go ? ib + 16 * cn : kOob, 0, 0);
                    cn += go ? 1 : 0;
                }
            }
            // LDS: kR dword reads and kW dword writes of this lane's own column (row stride 1 KiB, as the decoder's
            // images), rows from the step index; the reads feed the VALU chains so they are not dropped
            {
                const uint32_t col = (threadIdx.x >> 6) * 64 + lane;
#pragma unroll
                for (int k = 0; k < kR; k++) x1 ^= lds[(((j * 7 + k * 5 + x3) & 63) << 8) | col];
#pragma unroll
                for (int k = 0; k < kW; k++) lds[(((j * 3 + k) & 63) << 8) | col] = x2 + k;
            }
#pragma unroll
            for (int k = 0; k < kV / 4; k++) {
                asm volatile("v_alignbyte_b32 %0, %0, %0, 1" : "+v"(x));
                asm volatile("v_alignbyte_b32 %0, %0, %0, 1" : "+v"(x1));
                asm volatile("v_alignbyte_b32 %0, %0, %0, 1" : "+v"(x2));
                asm volatile("v_alignbyte_b32 %0, %0, %0, 1" : "+v"(x3));
            }
        };
        for (uint32_t j = 0; j < kSteps; j += 4) {
            step(j, f0, i0);
            step(j + 1, f1, i1);
            step(j + 2, f2, i2);
            step(j + 3, f3, i3);
        }
        acc ^= f0 ^ f1 ^ f2 ^ f3 ^ i0 ^ i1 ^ i2 ^ i3;
        uint32_t nx = 0;
        if (lane == 0) nx = atomicAdd(next, 1u);
        chunk = nwaves + __shfl(nx, 0);
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w ^ x ^ x1 ^ x2 ^ x3) == 0x12345678u) res[0] = 1;
}

template <int kMode, int kV, int kSteps = 136, int kR = 0, int kW = 0>
static void run(const char* name, const uint8_t* in, uint8_t* out, uint32_t* res, uint32_t* next) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_replay<kMode, kV, kSteps, kR, kW>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024));
    float best = 1e9;
    for (int it = 0; it < 4; it++) {
        CK(hipMemset(next, 0, 4));
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((k_replay<kMode, kV, kSteps, kR, kW>), dim3(512), dim3(256), 80 * 1024, 0, in, out, res, next);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it > 0 && ms < best) best = ms;
    }
    printf("replay %-34s S=%3d V=%3d R=%2d W=%2d: %7.3f ms\n", name, kSteps, kV, kR, kW, best);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

template <int kV>
static void row(const uint8_t* in, uint8_t* out, uint32_t* res, uint32_t* next) {
    run<kAll, kV>("all three streams", in, out, res, next);
    run<kNoStore, kV>("no flush stores", in, out, res, next);
    run<kNoFar, kV>("no far loads", in, out, res, next);
    run<kNoIn, kV>("no input loads", in, out, res, next);
    run<kCoopIn, kV>("input quad-cooperative", in, out, res, next);
    run<kNoFarCoopIn, kV>("coop input, no far", in, out, res, next);
    run<kNone, kV>("every lane out of range", in, out, res, next);
    run<kMerged, kV>("far + input as one load", in, out, res, next);
    run<kMasked, kV>("idle lanes exec-masked", in, out, res, next);
}

// round 6 candidates (steps per record from scripts/lane_sim-style counts on C2, VALU / LDS per step from hipcc -S of
// each step shape): current decoder, the merged far + input load, two-piece steps (a second element in the
// same 16-byte destination window), both
static void candidates(const uint8_t* in, uint8_t* out, uint32_t* res, uint32_t* next) {
    run<kAll, 160, 136, 18, 4>("cand current (3 VMEM)", in, out, res, next);
    run<kMerged, 166, 136, 18, 4>("cand merged load (2 VMEM)", in, out, res, next);
    run<kAll, 160, 136, 0, 0>("cand current, no LDS", in, out, res, next);
    run<kAll, 128, 136, 18, 4>("cand current at 128 VALU", in, out, res, next);
    run<kMerged, 128, 136, 18, 4>("cand merged at 128 VALU", in, out, res, next);
    run<kAll, 230, 96, 24, 4>("cand two-piece shared window", in, out, res, next);
    run<kMerged, 236, 96, 24, 4>("cand two-piece + merged", in, out, res, next);
    run<kAll, 260, 86, 28, 8>("cand two-piece separate windows", in, out, res, next);
    run<kMerged, 200, 96, 24, 4>("cand two-piece + merged at 200", in, out, res, next);
}

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    uint8_t *in, *out;
    uint32_t *res, *next;
    CK(hipMalloc(&in, (size_t)kRecs * kInStride + 4096));
    CK(hipMalloc(&out, (size_t)kRecs * kOutLen + 4096));
    CK(hipMalloc(&res, 64));
    CK(hipMalloc(&next, 64));
    CK(hipMemset(in, 3, (size_t)kRecs * kInStride));
    CK(hipMemset(out, 0, (size_t)kRecs * kOutLen));
    if (argc > 1) {  // "cand": the round-6 candidate rows only
        for (int rep = 0; rep < 2; rep++) candidates(in, out, res, next);
        printf("done\n");
        return 0;
    }
    for (int rep = 0; rep < 2; rep++) {
        row<0>(in, out, res, next);
        row<128>(in, out, res, next);
        row<172>(in, out, res, next);
        row<256>(in, out, res, next);
    }
    printf("done\n");
    return 0;
}
