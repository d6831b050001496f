// mem_probe.hip — throughput of the global access shapes available to a lane-per-record decoder
// (one 1 KiB record per lane): 16 B per lane per instruction in 64 different records (lane
// streams), 4 lanes x 16 B = 64 contiguous bytes of 16 records (quad streams), and 1 KiB
// contiguous per wave-instruction (coalesced). Loads and stores. Standalone:
// hipcc --offload-arch=gfx950 -O3 scripts/mem_probe.hip -o scripts/mem_probe && scripts/mem_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr uint64_t kRec = 1024;
constexpr uint64_t kRecs = 1u << 20;  // 1 GiB

// shape 0: lane streams, 1: quad streams, 2: coalesced, 3: pair streams (2 lanes x 16 B = 32 contiguous
// bytes of 32 records per instruction), 4: octet streams (8 lanes x 16 B = 128 B of 8 records)
template <int kShape, bool kStore>
__global__ void __launch_bounds__(256) k_mem(uint4* buf, uint4* sink) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    uint4 acc = make_uint4(0, 0, 0, 0);
    // each wave handles batches of 64 consecutive records
    for (uint64_t b = wave; b < kRecs / 64; b += waves) {
        const uint64_t r0 = b * 64;
        for (uint32_t j = 0; j < kRec / 16; j++) {
            uint64_t idx;  // uint4 index
            if (kShape == 0) {
                idx = (r0 + lane) * (kRec / 16) + j;  // record r0+lane, chunk j
            } else if (kShape == 1) {
                const uint32_t rec = (j & 3) * 16 + (lane >> 2), ch = (j >> 2) * 4 + (lane & 3);
                idx = (r0 + rec) * (kRec / 16) + ch;  // 16 records x 64 B per instruction
            } else if (kShape == 3) {
                const uint32_t rec = (j & 1) * 32 + (lane >> 1), ch = (j >> 1) * 2 + (lane & 1);
                idx = (r0 + rec) * (kRec / 16) + ch;  // 32 records x 32 B per instruction
            } else if (kShape == 4) {
                const uint32_t rec = (j & 7) * 8 + (lane >> 3), ch = (j >> 3) * 8 + (lane & 7);
                idx = (r0 + rec) * (kRec / 16) + ch;  // 8 records x 128 B per instruction
            } else {
                idx = r0 * (kRec / 16) + (uint64_t)j * 64 + lane;  // 1 KiB contiguous
            }
            if (kStore) {
                buf[idx] = make_uint4(j, lane, (uint32_t)b, 7);
            } else {
                const uint4 v = buf[idx];
                acc.x ^= v.x;
                acc.y += v.y;
                acc.z ^= v.z;
                acc.w += v.w;
            }
        }
    }
    if (!kStore && (acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) sink[0] = acc;
}

template <int kShape, bool kStore>
static void run(const char* name, uint4* buf, uint4* sink) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int grid : {512, 1024, 2048}) {
        hipLaunchKernelGGL((k_mem<kShape, kStore>), dim3(grid), dim3(256), 0, 0, buf, sink);  // warm
        (void)hipEventRecord(e0);
        for (int i = 0; i < 5; i++) hipLaunchKernelGGL((k_mem<kShape, kStore>), dim3(grid), dim3(256), 0, 0, buf, sink);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s grid %4d: %7.1f GB/s (%.3f ms)\n", name, grid, kRec * kRecs * 5 / (ms * 1e-3) / 1e9, ms / 5);
    }
}

int main() {
    uint4 *buf, *sink;
    if (hipMalloc(&buf, kRec * kRecs) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, kRec * kRecs);
    run<0, false>("load  lane streams (64 rec)", buf, sink);
    run<1, false>("load  quad streams (16 rec)", buf, sink);
    run<2, false>("load  coalesced", buf, sink);
    run<0, true>("store lane streams (64 rec)", buf, sink);
    run<1, true>("store quad streams (16 rec)", buf, sink);
    run<2, true>("store coalesced", buf, sink);
    run<3, true>("store pair streams (32 rec)", buf, sink);
    run<4, true>("store octet streams (8 rec)", buf, sink);
    run<3, false>("load  pair streams (32 rec)", buf, sink);
    return 0;
}
