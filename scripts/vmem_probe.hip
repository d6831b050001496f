// vmem_probe.hip — cost of one 16-byte-per-lane vector-memory instruction on MI355X by how many lanes
// are active and how many cache lines they touch (the Snappy lane decoder's loads and stores are of
// this kind: a few lanes with real work, the rest idle). Data is L2-resident (a small buffer), 12
// waves per CU each keep 8 independent instructions in flight; the figure is CU-cycles per
// wave-instruction (kernel time x 256 CUs x clock / instructions).
// hipcc --offload-arch=gfx950 -O3 scripts/vmem_probe.hip -o scripts/vmem_probe && scripts/vmem_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr uint32_t kLines = 1u << 14;  // 2 MiB of 128-byte lines
constexpr int kIters = 512, kUnroll = 8;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    return x;
}

// pattern: 0 all lanes distinct lines; 1 16 active distinct, 48 to one sink line; 2 16 active
// distinct, 48 exec-masked; 3 buffer, 16 active distinct, 48 out of range; 4 all lanes one line;
// 5 16 lines x 4 lanes (64 contiguous bytes); 6 8 lines x 8 lanes (128 contiguous bytes);
// 7 buffer, all out of range; 8 buffer all lanes distinct
template <int kPat, bool kStore>
__global__ void __launch_bounds__(256) k_probe(uint4* buf, uint4* out, uint32_t salt) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, kLines * 128, 0x00020000);
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    v4 acc = {0, 0, 0, 0};
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int u = 0; u < kUnroll; u++) {
            const uint32_t h = mix(wave * 7919u + (uint32_t)it * 131u + (uint32_t)u * 17u + salt);
            uint32_t line, sub = 0;
            bool active = true;
            if (kPat == 0 || kPat == 8) {
                line = h + lane * 97u;
            } else if (kPat == 1 || kPat == 2 || kPat == 3) {
                active = (lane & 3) == (h & 3);
                line = h + lane * 97u;
                if (kPat == 1 && !active) line = wave;  // the wave's sink line
            } else if (kPat == 4) {
                line = h;
            } else if (kPat == 5) {
                line = h + (lane >> 2) * 97u;
                sub = lane & 3;
            } else if (kPat == 6) {
                line = h + (lane >> 3) * 97u;
                sub = lane & 7;
            } else {
                line = h;
                active = false;
            }
            const uint32_t idx = (line % kLines) * 8 + sub;  // uint4 index
            if (kStore) {
                const v4 v = {h, lane, (uint32_t)it, 7};
                if (kPat == 2) {
                    if (active) *reinterpret_cast<v4*>(buf + idx) = v;
                } else if (kPat == 3 || kPat == 7 || kPat == 8) {
                    __builtin_amdgcn_raw_buffer_store_b128(v, r, active ? idx * 16 : 0x80000000u, 0, 0);
                } else {
                    *reinterpret_cast<v4*>(buf + idx) = v;
                }
            } else {
                v4 v = {0, 0, 0, 0};
                if (kPat == 2) {
                    if (active) v = *reinterpret_cast<const v4*>(buf + idx);
                } else if (kPat == 3 || kPat == 7 || kPat == 8) {
                    v = __builtin_bit_cast(v4, __builtin_amdgcn_raw_buffer_load_b128(r, active ? idx * 16 : 0x80000000u, 0, 0));
                } else {
                    v = *reinterpret_cast<const v4*>(buf + idx);
                }
                acc ^= v;
            }
        }
    }
    if (!kStore && (acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = make_uint4(acc.x, acc.y, acc.z, acc.w);
}

template <int kPat, bool kStore>
static void run(const char* name, uint4* buf, uint4* out, int grid) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_probe<kPat, kStore>), dim3(grid), dim3(256), 0, 0, buf, out, 1u);
    (void)hipEventRecord(e0);
    const int reps = 5;
    for (int i = 0; i < reps; i++) hipLaunchKernelGGL((k_probe<kPat, kStore>), dim3(grid), dim3(256), 0, 0, buf, out, 2u + i);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double instrs = (double)grid * 4 * kIters * kUnroll * reps;
    const double cyc = ms * 1e-3 * 2.1e9 * 256 / instrs;
    printf("%-6s %-44s %8.3f ms  %6.1f CU-cycles per wave-instruction\n", kStore ? "store" : "load", name, ms / reps, cyc);
}

int main() {
    uint4 *buf, *out;
    (void)hipMalloc(&buf, (size_t)kLines * 128);
    (void)hipMalloc(&out, 64);
    (void)hipMemset(buf, 1, (size_t)kLines * 128);
    const int grid = 256 * 3;  // 12 waves per CU
#define RUN(P, S, N) run<P, S>(N, buf, out, grid)
    RUN(0, false, "64 lanes, 64 distinct lines");
    RUN(1, false, "16 active distinct + 48 on one sink line");
    RUN(2, false, "16 active distinct, 48 exec-masked");
    RUN(3, false, "buffer: 16 active distinct, 48 out of range");
    RUN(4, false, "64 lanes, one line");
    RUN(5, false, "16 lines x 4 lanes (64 B each)");
    RUN(6, false, "8 lines x 8 lanes (128 B each)");
    RUN(7, false, "buffer: all out of range");
    RUN(8, false, "buffer: 64 lanes, 64 distinct lines");
    RUN(0, true, "64 lanes, 64 distinct lines");
    RUN(1, true, "16 active distinct + 48 on one sink line");
    RUN(2, true, "16 active distinct, 48 exec-masked");
    RUN(3, true, "buffer: 16 active distinct, 48 out of range");
    RUN(5, true, "16 lines x 4 lanes (64 B each)");
    RUN(6, true, "8 lines x 8 lanes (128 B each)");
    RUN(7, true, "buffer: all out of range");
    return 0;
}
