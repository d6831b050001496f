// What one scattered 16-byte load costs the memory side on gfx950 (C4's far-history loads: 4..11-byte copies
// read from output written up to 64 KiB earlier, far past L2 and MALL). Every lane issues independent loads at
// random 4-byte-aligned offsets of a 2 GiB buffer, with each buffer-load cache policy (aux bits: 1 sc0, 2 nt,
// 16 sc1) and two widths; time per variant from HIP events. Run under rocprofv3 --pmc FETCH_SIZE (one pass) to
// see the bytes fetched per load for each policy: 128 per load = whole L2 lines, 64 = half lines. Then the
// default policy over spans from 16 MiB to 1 GiB: the random-request rate when the lines come from L2, the
// MALL or HBM.
//   hipcc -O3 --offload-arch=gfx950 scripts/fetch_probe.hip -o /tmp/fetch_probe && /tmp/fetch_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                             \
        }                                                                         \
    } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr uint32_t kLoads = 64;  // loads per lane

template <int kCp, int kWide>
__global__ void __launch_bounds__(256) k_fetch(const uint8_t* buf, uint32_t words, uint32_t* out) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(buf), 0, 0x7fffffff, 0x00020000);
    uint32_t x = (blockIdx.x * 256u + threadIdx.x) * 2654435761u + 12345u;
    uint32_t acc = 0;
#pragma unroll 8
    for (uint32_t k = 0; k < kLoads; k++) {
        x = x * 1664525u + 1013904223u;
        const uint32_t off = (uint32_t)(((uint64_t)x * (words - 4)) >> 32) * 4u;
        if (kWide) {
            const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kCp);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        } else {
            acc ^= __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, kCp);
        }
    }
    out[blockIdx.x * 256u + threadIdx.x] = acc;
}

template <int kCp, int kWide>
static int run(const uint8_t* buf, uint32_t words, uint32_t* out, uint32_t blocks, const char* name) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_fetch<kCp, kWide>), dim3(blocks), dim3(256), 0, 0, buf, words, out);  // warm the TLB
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((k_fetch<kCp, kWide>), dim3(blocks), dim3(256), 0, 0, buf, words, out);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double loads = (double)blocks * 256 * kLoads;
    std::printf("%-14s %8.3f ms  %6.2f G loads/s  at 128 B/load %6.2f TB/s, at 64 B/load %6.2f TB/s\n", name, ms,
                loads / ms * 1e-6, loads * 128 / ms * 1e-9, loads * 64 / ms * 1e-9);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return 0;
}

int main() {
    const size_t bytes = (size_t)2 << 30;
    uint32_t words = (uint32_t)(bytes / 4);
    const uint32_t blocks = 8192;  // 2 M lanes x 64 loads
    uint8_t* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
    CK(hipMemset(buf, 1, bytes));
    CK(hipDeviceSynchronize());
    int rc = 0;
    rc |= run<0, 1>(buf, words, out, blocks, "b128 cp0");
    rc |= run<1, 1>(buf, words, out, blocks, "b128 sc0");
    rc |= run<2, 1>(buf, words, out, blocks, "b128 nt");
    rc |= run<3, 1>(buf, words, out, blocks, "b128 sc0nt");
    rc |= run<16, 1>(buf, words, out, blocks, "b128 sc1");
    rc |= run<17, 1>(buf, words, out, blocks, "b128 sc01");
    rc |= run<19, 1>(buf, words, out, blocks, "b128 all");
    rc |= run<0, 0>(buf, words, out, blocks, "b32 cp0");
    rc |= run<17, 0>(buf, words, out, blocks, "b32 sc01");
    // the same random 16-byte loads over smaller spans: inside L2 (4 MiB per XCD), inside the 256 MiB MALL, past it
    for (const uint32_t mib : {16u, 64u, 128u, 192u, 256u, 512u, 1024u}) {
        words = mib << 18;
        char name[32];
        std::snprintf(name, sizeof name, "span %4u MiB", mib);
        rc |= run<0, 1>(buf, words, out, blocks, name);
    }
    CK(hipFree(buf));
    CK(hipFree(out));
    return rc;
}
