// lds_probe.hip — micro-probe of CDNA4 LDS access behaviour used to pick the Snappy decoder's
// history layout: correctness and cost of byte-unaligned ds_read_b32 / ds_write_b32 and of
// ds_read_b128 / ds_read2_b64 against the aligned forms. Standalone: hipcc --offload-arch=gfx950 -O3
// scripts/lds_probe.hip -o /tmp/lds_probe && /tmp/lds_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int kLds = 32768;
constexpr int kIters = 4096;

__device__ __forceinline__ uint32_t pat(uint32_t i) { return (i * 7u + 3u + (i >> 8)) & 0xFFu; }
__device__ __forceinline__ uint32_t pat4(uint32_t a) {
    return pat(a) | pat(a + 1) << 8 | pat(a + 2) << 16 | pat(a + 3) << 24;
}

// mode 0: ds_read_b32 4-aligned          1: ds_read_b32 at any byte address
//      2: ds_read_b128 16-aligned        3: ds_read_b128 4-aligned (not 16)
//      4: ds_write_b32 at any byte address (then read back bytewise)
//      5: ds_read2_b64 8-aligned (offset1:1)
__global__ void k_probe(int mode, unsigned long long* cycles, unsigned* bad) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    for (int i = threadIdx.x; i < kLds; i += blockDim.x) lds[i] = (uint8_t)pat(i);
    __syncthreads();
    const uint32_t lane = threadIdx.x;
    uint32_t acc = 0, errs = 0;
    // each lane owns a 128-byte region (writes stay private), random offsets inside it
    const uint32_t base = lane * 128u;
    uint32_t x = lane * 2654435761u + 1;
    const long long t0 = clock64();
    for (int it = 0; it < kIters; it++) {
        x = x * 1103515245u + 12345u;
        uint32_t off = (x >> 16) % 96u;
        if (mode == 0) off &= ~3u;
        if (mode == 2) off &= ~15u;
        if (mode == 3) off = (off & ~15u) | 4u;
        if (mode == 5) off &= ~7u;
        const uint32_t addr = base + off;
        if (mode <= 1) {
            uint32_t v;
            asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
            errs += v != pat4(addr);
            acc += v;
        } else if (mode <= 3) {
            v4u v;
            asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
            errs += (v.x != pat4(addr)) + (v.y != pat4(addr + 4)) + (v.z != pat4(addr + 8)) + (v.w != pat4(addr + 12));
            acc += v.x ^ v.w;
        } else if (mode == 4) {
            const uint32_t val = pat4(addr);  // rewrite the pattern's own bytes: reads stay checkable
            asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(addr), "v"(val) : "memory");
            acc += val;
        } else {
            v4u v;
            asm volatile("ds_read2_b64 %0, %1 offset1:1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
            errs += (v.x != pat4(addr)) + (v.y != pat4(addr + 4)) + (v.z != pat4(addr + 8)) + (v.w != pat4(addr + 12));
            acc += v.x ^ v.w;
        }
    }
    const long long t1 = clock64();
    if (mode == 4) {
        __syncthreads();
        for (int i = threadIdx.x; i < kLds; i += blockDim.x) errs += lds[i] != (uint8_t)pat(i);
    }
    atomicAdd(cycles, (unsigned long long)(t1 - t0));
    atomicAdd(bad, errs);
    if (acc == 0x12345678u) bad[1] = acc;
}

int main() {
    unsigned long long* cyc;
    unsigned* bad;
    (void)hipMalloc(&cyc, 8);
    (void)hipMalloc(&bad, 8);
    const char* names[] = {"read_b32 aligned", "read_b32 byte-unaligned", "read_b128 aligned", "read_b128 4-aligned",
                           "write_b32 byte-unaligned", "read2_b64 8-aligned"};
    for (int threads : {64, 256}) {
        for (int mode = 0; mode < 6; mode++) {
            (void)hipMemset(cyc, 0, 8);
            (void)hipMemset(bad, 0, 8);
            hipLaunchKernelGGL(k_probe, dim3(1), dim3(threads), kLds, 0, mode, cyc, bad);
            unsigned long long c = 0;
            unsigned b[2] = {0, 0};
            (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            (void)hipMemcpy(b, bad, 8, hipMemcpyDeviceToHost);
            printf("threads=%3d %-26s cycles/access/lane-avg %7.1f  errors %u\n", threads, names[mode],
                   (double)c / threads / kIters, b[0]);
        }
    }
    return 0;
}
