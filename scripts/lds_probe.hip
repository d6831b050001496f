// lds_probe.hip — micro-probe of CDNA4 LDS access behaviour used to pick the Snappy decoder's
// history layout: correctness and cost of byte-unaligned ds_read / ds_write (b32 and b128) against
// the aligned forms. Standalone: hipcc --offload-arch=gfx950 -O3 scripts/lds_probe.hip -o /tmp/lds_probe
// && /tmp/lds_probe
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
//      6: ds_read_b128 at any byte address
//      7: ds_write_b128 at any byte address (pattern bytes; read back bytewise)
//      8: ds_write_b128 16-aligned
//      9: ds_write_b128 at any byte address, then ds_read_b128 at another byte address of the
//         same lane region issued right after (read-after-write ordering, no wait in between)
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
        if (mode == 2 || mode == 8) off &= ~15u;
        if (mode == 3) off = (off & ~15u) | 4u;
        if (mode == 5) off &= ~7u;
        const uint32_t addr = base + off;
        if (mode <= 1) {
            uint32_t v;
            asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
            errs += v != pat4(addr);
            acc += v;
        } else if (mode <= 3 || mode == 6) {
            v4u v;
            asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
            errs += (v.x != pat4(addr)) + (v.y != pat4(addr + 4)) + (v.z != pat4(addr + 8)) + (v.w != pat4(addr + 12));
            acc += v.x ^ v.w;
        } else if (mode == 4) {
            const uint32_t val = pat4(addr);  // rewrite the pattern's own bytes: reads stay checkable
            asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(addr), "v"(val) : "memory");
            acc += val;
        } else if (mode == 7 || mode == 8) {
            v4u val = {pat4(addr), pat4(addr + 4), pat4(addr + 8), pat4(addr + 12)};
            asm volatile("ds_write_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(addr), "v"(val) : "memory");
            acc += val.x;
        } else if (mode == 9) {
            // write a lane-tagged value at addr, read 16 bytes at addr + d (d in [-15, 15]) right after
            const uint32_t tag = (lane * 0x01010101u) ^ (uint32_t)it;
            v4u val = {tag, tag + 1, tag + 2, tag + 3};
            const uint32_t d = (x >> 8) & 15u;
            const uint32_t raddr = addr + d;
            v4u v;
            asm volatile("ds_write_b128 %1, %2\n\tds_read_b128 %0, %3\n\ts_waitcnt lgkmcnt(0)"
                         : "=v"(v) : "v"(addr), "v"(val), "v"(raddr) : "memory");
            // the bytes [d, 16) of the write must be the first 16 - d bytes read
            const uint8_t* vb = reinterpret_cast<const uint8_t*>(&v);
            const uint8_t* wb = reinterpret_cast<const uint8_t*>(&val);
            for (uint32_t k = 0; k + d < 16; k++) errs += vb[k] != wb[k + d];
            acc += v.x;
            // restore the pattern so the region stays meaningful
            v4u p = {pat4(addr), pat4(addr + 4), pat4(addr + 8), pat4(addr + 12)};
            asm volatile("ds_write_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(addr), "v"(p) : "memory");
        } else {
            v4u v;
            asm volatile("ds_read2_b64 %0, %1 offset1:1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
            errs += (v.x != pat4(addr)) + (v.y != pat4(addr + 4)) + (v.z != pat4(addr + 8)) + (v.w != pat4(addr + 12));
            acc += v.x ^ v.w;
        }
    }
    const long long t1 = clock64();
    if (mode == 4 || mode == 7 || mode == 8 || mode == 9) {
        __syncthreads();
        for (int i = threadIdx.x; i < kLds; i += blockDim.x) errs += lds[i] != (uint8_t)pat(i);
    }
    atomicAdd(cycles, (unsigned long long)(t1 - t0));
    atomicAdd(bad, errs);
    if (acc == 0x12345678u) bad[1] = acc;
}

// Throughput form: every lane of 4 waves per SIMD streams unaligned 16-byte reads/writes without
// waiting after each (counted in bulk), to price the LDS array / store path rather than latency.
// mode 0: aligned read, 1: unaligned read, 2: aligned write, 3: unaligned write,
//      4: read 4-aligned, 5: read 8-aligned, 6: write 4-aligned, 7: write 8-aligned (all b128)
//      8: b32 read byte-unaligned, 9: b32 write byte-unaligned, 10: b32 read aligned, 11: b32 write aligned,
//      12: u8 read, 13: b8 write, 14: b64 read byte-unaligned, 15: b64 write byte-unaligned,
//      16: u16 read byte-unaligned, 17: b16 write byte-unaligned
__global__ void k_tput(int mode, unsigned long long* cycles, unsigned* sink) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t t = threadIdx.x;
    const uint32_t base = (t & 63u) * 304u + (t >> 6) * 19456u;  // waves' regions overlap: timing only
    uint32_t x = t * 2654435761u + 7;
    v4u acc = {0, 0, 0, 0};
    __syncthreads();
    const long long t0 = clock64();
    for (int it = 0; it < kIters; it++) {
        x = x * 1103515245u + 12345u;
        uint32_t off = (x >> 16) % 256u;
        if (mode == 0 || mode == 2) off &= ~15u;
        if (mode == 4 || mode == 6) off &= ~3u;
        if (mode == 5 || mode == 7) off &= ~7u;
        const uint32_t addr = (base + off) % (kLds * 4 - 32);
        if (mode == 10 || mode == 11) off &= ~3u;
        const uint32_t a2 = (base + off) % (kLds * 4 - 32);
        if (mode >= 8) {
            uint32_t v = acc.x + x;
            if (mode == 8 || mode == 10) {
                asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(a2) : "memory");
            } else if (mode == 9 || mode == 11) {
                asm volatile("ds_write_b32 %0, %1" ::"v"(a2), "v"(v) : "memory");
            } else if (mode == 12) {
                asm volatile("ds_read_u8 %0, %1" : "=v"(v) : "v"(a2) : "memory");
            } else if (mode == 13) {
                asm volatile("ds_write_b8 %0, %1" ::"v"(a2), "v"(v) : "memory");
            } else if (mode == 14) {
                uint64_t w;
                asm volatile("ds_read_b64 %0, %1" : "=v"(w) : "v"(a2) : "memory");
                v = (uint32_t)w ^ (uint32_t)(w >> 32);
            } else if (mode == 15) {
                uint64_t w = ((uint64_t)v << 32) | x;
                asm volatile("ds_write_b64 %0, %1" ::"v"(a2), "v"(w) : "memory");
            } else if (mode == 16) {
                asm volatile("ds_read_u16 %0, %1" : "=v"(v) : "v"(a2) : "memory");
            } else {
                asm volatile("ds_write_b16 %0, %1" ::"v"(a2), "v"(v) : "memory");
            }
            if ((it & 15) == 15) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            acc.x += v;
        } else if (mode <= 1 || mode == 4 || mode == 5) {
            typedef v4u __attribute__((aligned(1))) v4b;
            acc += *reinterpret_cast<const v4b*>(lds + addr);
        } else {
            typedef v4u __attribute__((aligned(1))) v4b;
            *reinterpret_cast<v4b*>(lds + addr) = acc + x;
        }
    }
    __syncthreads();
    const long long t1 = clock64();
    if (t == 0) atomicAdd(cycles, (unsigned long long)(t1 - t0));
    if (acc.x == 0x12345678u) sink[0] = acc.y;
}

int main() {
    unsigned long long* cyc;
    unsigned* bad;
    (void)hipMalloc(&cyc, 8);
    (void)hipMalloc(&bad, 8);
    const char* names[] = {"read_b32 aligned", "read_b32 byte-unaligned", "read_b128 aligned", "read_b128 4-aligned",
                           "write_b32 byte-unaligned", "read2_b64 8-aligned", "read_b128 byte-unaligned",
                           "write_b128 byte-unaligned", "write_b128 aligned", "write_b128+read_b128 RAW"};
    for (int threads : {64, 256}) {
        for (int mode = 0; mode < 10; mode++) {
            (void)hipMemset(cyc, 0, 8);
            (void)hipMemset(bad, 0, 8);
            hipLaunchKernelGGL(k_probe, dim3(1), dim3(threads), kLds, 0, mode, cyc, bad);
            unsigned long long c = 0;
            unsigned b[2] = {0, 0};
            (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            (void)hipMemcpy(b, bad, 8, hipMemcpyDeviceToHost);
            printf("threads=%3d %-28s cycles/access/lane-avg %7.1f  errors %u\n", threads, names[mode],
                   (double)c / threads / kIters, b[0]);
        }
    }
    const char* tnames[] = {"tput read_b128 aligned", "tput read_b128 unaligned", "tput write_b128 aligned",
                            "tput write_b128 unaligned", "tput read_b128 4-aligned", "tput read_b128 8-aligned",
                            "tput write_b128 4-aligned", "tput write_b128 8-aligned",
                            "tput read_b32 unaligned", "tput write_b32 unaligned", "tput read_b32 aligned",
                            "tput write_b32 aligned", "tput read_u8", "tput write_b8", "tput read_b64 unaligned",
                            "tput write_b64 unaligned", "tput read_u16 unaligned", "tput write_b16 unaligned"};
    for (int mode = 0; mode < 18; mode++) {
        (void)hipMemset(cyc, 0, 8);
        // 1024 threads = 16 waves on one CU (4 per SIMD), 128 KiB LDS
        hipLaunchKernelGGL(k_tput, dim3(1), dim3(1024), kLds * 4, 0, mode, cyc, bad);
        unsigned long long c = 0;
        (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-28s CU cycles per wave-instruction %6.2f\n", tnames[mode], (double)c / (16.0 * kIters));
    }
    hipError_t e = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(e));
    return 0;
}
