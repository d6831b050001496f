// issue_probe.hip — what a SIMD issues per 4-cycle slot, by instruction class and by waves per SIMD, and
// what a buffer_load_dwordx4 costs the CU by address shape (out-of-range lanes, one line, 16 lines, 64 lines).
// Questions it answers for k_snappy_pipe:
//   * can two waves of a SIMD issue two integer VALU per 4-cycle slot, or is the pipe full at one?
//   * does SALU / LDS issue of one wave overlap the other wave's VALU?
//   * does a lane whose buffer offset is out of range cost address-unit cycles?
// Standalone: hipcc --offload-arch=gfx950 -O3 scripts/issue_probe.hip -o scripts/issue_probe && scripts/issue_probe
// Timing: per-wave s_memtime deltas (shader clock) and hipEvent wall time; every loop is inline asm with a
// fixed instruction count, 8 independent chains per wave so one wave is not latency-bound.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

constexpr int kIters = 1024;

// instruction groups of 8 (one per chain)
#define G8(OP)                                                   \
    asm volatile(OP : "+v"(a0) : "v"(b), "v"(c));                \
    asm volatile(OP : "+v"(a1) : "v"(b), "v"(c));                \
    asm volatile(OP : "+v"(a2) : "v"(b), "v"(c));                \
    asm volatile(OP : "+v"(a3) : "v"(b), "v"(c));                \
    asm volatile(OP : "+v"(a4) : "v"(b), "v"(c));                \
    asm volatile(OP : "+v"(a5) : "v"(b), "v"(c));                \
    asm volatile(OP : "+v"(a6) : "v"(b), "v"(c));                \
    asm volatile(OP : "+v"(a7) : "v"(b), "v"(c));
#define G8C                                                              \
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a0) : "v"(b), "s"(msk)); \
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a1) : "v"(b), "s"(msk)); \
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a2) : "v"(b), "s"(msk)); \
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a3) : "v"(b), "s"(msk)); \
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a4) : "v"(b), "s"(msk)); \
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a5) : "v"(b), "s"(msk)); \
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a6) : "v"(b), "s"(msk)); \
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a7) : "v"(b), "s"(msk));
#define S4(OP)                                  \
    asm volatile(OP : "+s"(s0) : "s"(sb));      \
    asm volatile(OP : "+s"(s1) : "s"(sb));      \
    asm volatile(OP : "+s"(s2) : "s"(sb));      \
    asm volatile(OP : "+s"(s3) : "s"(sb));

// kinds: instruction mix of one loop body
enum Kind {
    kAdd,        // 64 v_add_u32
    kAlign,      // 64 v_alignbyte_b32
    kBfi,        // 64 v_bfi_b32
    kLshlOr,     // 64 v_lshl_or_b32
    kCnd,        // 64 v_cndmask_b32 (vcc)
    kFma,        // 64 v_fma_f32
    kPk16,       // 64 v_pk_add_u16
    kSalu,       // 64 s_add_u32
    kMix8to1,    // 64 v_alignbyte + 8 s_add_u32
    kMix4to1,    // 64 v_alignbyte + 16 s_add_u32
    kMix2to1,    // 64 v_alignbyte + 32 s_add_u32
    kLds,        // 16 ds_read_b32 (conflict-free) + wait
    kMixLds,     // 64 v_alignbyte + 8 ds_read_b32
    kStep,       // the decoder's step mix per 64 VALU: 10 SALU, 8 LDS
    kNKinds
};
static const char* kNames[kNKinds] = {"v_add_u32",      "v_alignbyte_b32", "v_bfi_b32",  "v_lshl_or_b32",
                                      "v_cndmask_b32",  "v_fma_f32",       "v_pk_add_u16", "s_mul_i32",
                                      "64valu+8salu",   "64valu+16salu",   "64valu+32salu", "16ds_read",
                                      "64valu+8ds_read", "64valu+10salu+8lds"};
// instructions per loop body: VALU, SALU, LDS
static const int kVal[kNKinds] = {64, 64, 64, 64, 64, 64, 64, 0, 64, 64, 64, 0, 64, 64};
static const int kSal[kNKinds] = {0, 0, 0, 0, 0, 0, 0, 64, 8, 16, 32, 0, 0, 10};
static const int kLdsN[kNKinds] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 16, 8, 8};

template <int K>
__global__ void __launch_bounds__(256) k_issue(uint32_t* out, unsigned long long* cyc, uint32_t seed) {
    extern __shared__ uint32_t lds[];
    const uint32_t t = threadIdx.x;
    uint32_t a0 = t, a1 = t + 1, a2 = t + 2, a3 = t + 3, a4 = t + 4, a5 = t + 5, a6 = t + 6, a7 = t + 7;
    uint32_t b = seed ^ t, c = seed + 3;
    const uint64_t msk = 0x5555555555555555ull ^ seed;
    uint32_t s0 = seed, s1 = seed + 1, s2 = seed + 2, s3 = seed + 3, sb = seed * 7;
    if (K == kFma) {
        a0 = __float_as_uint(1.0f + t);
        b = __float_as_uint(0.999f);
        c = __float_as_uint(0.5f);
    }
    lds[t] = t;
    __syncthreads();
    const uint32_t la = 4 * (t & 63);  // conflict-free: lane -> bank
    uint32_t l0 = 0, l1 = 0, l2 = 0, l3 = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; i++) {
        if (K == kAdd) { G8("v_add_u32 %0, %0, %1") G8("v_add_u32 %0, %0, %1") G8("v_add_u32 %0, %0, %1") G8("v_add_u32 %0, %0, %1") G8("v_add_u32 %0, %0, %1") G8("v_add_u32 %0, %0, %1") G8("v_add_u32 %0, %0, %1") G8("v_add_u32 %0, %0, %1") }
#define AL "v_alignbyte_b32 %0, %0, %1, %2"
        if (K == kAlign || K == kMix8to1 || K == kMix4to1 || K == kMix2to1 || K == kMixLds || K == kStep) {
            G8(AL)
            if (K == kMix8to1 || K == kMix4to1 || K == kMix2to1 || K == kStep) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s0) : "s"(sb)); }
            if (K == kMix4to1 || K == kMix2to1) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s1) : "s"(sb)); }
            if (K == kMix2to1) { S4("s_mul_i32 %0, %0, %1") }
            if (K == kMixLds || K == kStep) asm volatile("ds_read_b32 %0, %1" : "=v"(l0) : "v"(la));
            G8(AL)
            if (K == kMix8to1 || K == kMix4to1 || K == kMix2to1 || K == kStep) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s2) : "s"(sb)); }
            if (K == kMix4to1 || K == kMix2to1) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s3) : "s"(sb)); }
            if (K == kMix2to1) { S4("s_mul_i32 %0, %0, %1") }
            if (K == kMixLds || K == kStep) asm volatile("ds_read_b32 %0, %1 offset:1024" : "=v"(l1) : "v"(la));
            G8(AL)
            if (K == kMix8to1 || K == kMix4to1 || K == kMix2to1 || K == kStep) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s0) : "s"(sb)); }
            if (K == kMix4to1 || K == kMix2to1) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s1) : "s"(sb)); }
            if (K == kMix2to1) { S4("s_mul_i32 %0, %0, %1") }
            if (K == kMixLds || K == kStep) asm volatile("ds_read_b32 %0, %1 offset:2048" : "=v"(l2) : "v"(la));
            G8(AL)
            if (K == kMix8to1 || K == kMix4to1 || K == kMix2to1 || K == kStep) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s2) : "s"(sb)); }
            if (K == kMix4to1 || K == kMix2to1) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s3) : "s"(sb)); }
            if (K == kMix2to1) { S4("s_mul_i32 %0, %0, %1") }
            if (K == kMixLds || K == kStep) asm volatile("ds_read_b32 %0, %1 offset:3072" : "=v"(l3) : "v"(la));
            G8(AL)
            if (K == kMix8to1 || K == kMix4to1 || K == kMix2to1 || K == kStep) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s0) : "s"(sb)); }
            if (K == kMix4to1 || K == kMix2to1) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s1) : "s"(sb)); }
            if (K == kMix2to1) { S4("s_mul_i32 %0, %0, %1") }
            if (K == kMixLds || K == kStep) asm volatile("ds_read_b32 %0, %1 offset:4096" : "=v"(l0) : "v"(la));
            G8(AL)
            if (K == kMix8to1 || K == kMix4to1 || K == kMix2to1 || K == kStep) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s2) : "s"(sb)); }
            if (K == kMix4to1 || K == kMix2to1) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s3) : "s"(sb)); }
            if (K == kMix2to1) { S4("s_mul_i32 %0, %0, %1") }
            if (K == kMixLds || K == kStep) asm volatile("ds_read_b32 %0, %1 offset:5120" : "=v"(l1) : "v"(la));
            G8(AL)
            if (K == kMix8to1 || K == kMix4to1 || K == kMix2to1 || K == kStep) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s0) : "s"(sb)); }
            if (K == kMix4to1 || K == kMix2to1) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s1) : "s"(sb)); }
            if (K == kMix2to1) { S4("s_mul_i32 %0, %0, %1") }
            if (K == kMixLds || K == kStep) asm volatile("ds_read_b32 %0, %1 offset:6144" : "=v"(l2) : "v"(la));
            G8(AL)
            if (K == kMix8to1 || K == kMix4to1 || K == kMix2to1 || K == kStep) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s2) : "s"(sb)); }
            if (K == kMix4to1 || K == kMix2to1) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s3) : "s"(sb)); }
            if (K == kMix2to1) { S4("s_mul_i32 %0, %0, %1") }
            if (K == kStep) { asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s1) : "s"(sb)); asm volatile("s_mul_i32 %0, %0, %1" : "+s"(s3) : "s"(sb)); }
            if (K == kMixLds || K == kStep) asm volatile("ds_read_b32 %0, %1 offset:7168" : "=v"(l3) : "v"(la));
            if (K == kMixLds || K == kStep) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                a0 ^= l0 ^ l1;
                a1 ^= l2 ^ l3;
            }
        }
#undef AL
        if (K == kBfi) { G8("v_bfi_b32 %0, %1, %0, %2") G8("v_bfi_b32 %0, %1, %0, %2") G8("v_bfi_b32 %0, %1, %0, %2") G8("v_bfi_b32 %0, %1, %0, %2") G8("v_bfi_b32 %0, %1, %0, %2") G8("v_bfi_b32 %0, %1, %0, %2") G8("v_bfi_b32 %0, %1, %0, %2") G8("v_bfi_b32 %0, %1, %0, %2") }
        if (K == kLshlOr) { G8("v_lshl_or_b32 %0, %0, 3, %1") G8("v_lshl_or_b32 %0, %0, 3, %1") G8("v_lshl_or_b32 %0, %0, 3, %1") G8("v_lshl_or_b32 %0, %0, 3, %1") G8("v_lshl_or_b32 %0, %0, 3, %1") G8("v_lshl_or_b32 %0, %0, 3, %1") G8("v_lshl_or_b32 %0, %0, 3, %1") G8("v_lshl_or_b32 %0, %0, 3, %1") }
        if (K == kCnd) { G8C G8C G8C G8C G8C G8C G8C G8C }
        if (K == kFma) { G8("v_fma_f32 %0, %0, %1, %2") G8("v_fma_f32 %0, %0, %1, %2") G8("v_fma_f32 %0, %0, %1, %2") G8("v_fma_f32 %0, %0, %1, %2") G8("v_fma_f32 %0, %0, %1, %2") G8("v_fma_f32 %0, %0, %1, %2") G8("v_fma_f32 %0, %0, %1, %2") G8("v_fma_f32 %0, %0, %1, %2") }
        if (K == kPk16) { G8("v_pk_add_u16 %0, %0, %1") G8("v_pk_add_u16 %0, %0, %1") G8("v_pk_add_u16 %0, %0, %1") G8("v_pk_add_u16 %0, %0, %1") G8("v_pk_add_u16 %0, %0, %1") G8("v_pk_add_u16 %0, %0, %1") G8("v_pk_add_u16 %0, %0, %1") G8("v_pk_add_u16 %0, %0, %1") }
        if (K == kSalu) {
            S4("s_mul_i32 %0, %0, %1") S4("s_mul_i32 %0, %0, %1") S4("s_mul_i32 %0, %0, %1") S4("s_mul_i32 %0, %0, %1")
            S4("s_mul_i32 %0, %0, %1") S4("s_mul_i32 %0, %0, %1") S4("s_mul_i32 %0, %0, %1") S4("s_mul_i32 %0, %0, %1")
            S4("s_mul_i32 %0, %0, %1") S4("s_mul_i32 %0, %0, %1") S4("s_mul_i32 %0, %0, %1") S4("s_mul_i32 %0, %0, %1")
            S4("s_mul_i32 %0, %0, %1") S4("s_mul_i32 %0, %0, %1") S4("s_mul_i32 %0, %0, %1") S4("s_mul_i32 %0, %0, %1")
        }
        if (K == kLds) {
            asm volatile("ds_read_b32 %0, %1" : "=v"(l0) : "v"(la));
            asm volatile("ds_read_b32 %0, %1 offset:1024" : "=v"(l1) : "v"(la));
            asm volatile("ds_read_b32 %0, %1 offset:2048" : "=v"(l2) : "v"(la));
            asm volatile("ds_read_b32 %0, %1 offset:3072" : "=v"(l3) : "v"(la));
            asm volatile("ds_read_b32 %0, %1 offset:4096" : "=v"(a4) : "v"(la));
            asm volatile("ds_read_b32 %0, %1 offset:5120" : "=v"(a5) : "v"(la));
            asm volatile("ds_read_b32 %0, %1 offset:6144" : "=v"(a6) : "v"(la));
            asm volatile("ds_read_b32 %0, %1 offset:7168" : "=v"(a7) : "v"(la));
            asm volatile("ds_read_b32 %0, %1 offset:256" : "=v"(l0) : "v"(la));
            asm volatile("ds_read_b32 %0, %1 offset:1280" : "=v"(l1) : "v"(la));
            asm volatile("ds_read_b32 %0, %1 offset:2304" : "=v"(l2) : "v"(la));
            asm volatile("ds_read_b32 %0, %1 offset:3328" : "=v"(l3) : "v"(la));
            asm volatile("ds_read_b32 %0, %1 offset:4352" : "=v"(a4) : "v"(la));
            asm volatile("ds_read_b32 %0, %1 offset:5376" : "=v"(a5) : "v"(la));
            asm volatile("ds_read_b32 %0, %1 offset:6400" : "=v"(a6) : "v"(la));
            asm volatile("ds_read_b32 %0, %1 offset:7424" : "=v"(a7) : "v"(la));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ s0 ^ s1 ^ s2 ^ s3 ^ l0 ^ l1 ^ l2 ^ l3;
    if (r == 0x12345678u) out[0] = r;
    if ((t & 63) == 0) cyc[(blockIdx.x * blockDim.x + t) >> 6] = t1 - t0;
}

// buffer_load_dwordx4 shapes: 0 every lane out of range, 1 one 16-B word for all lanes, 2 coalesced 1 KiB,
// 3 quads: 16 x 64 contiguous bytes, 4 lanes: 64 distinct 128-B lines, 5 a quarter of the lanes in 64-line
// shape and the rest out of range, 6 a quarter of the lanes in 64-line shape, the rest masked off (exec)
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
template <int kShape, int kValuPer>
__global__ void __launch_bounds__(256) k_vmem(const uint8_t* buf, uint32_t* out, unsigned long long* cyc) {
    extern __shared__ uint32_t lds[];
    const uint32_t t = threadIdx.x, lane = t & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + t) >> 6;
    // 8 KiB per wave, reused every iteration: L1 / L2 hits, so the address path, not HBM, is measured
    const uint8_t* wb = buf + (wave % 4096) * 8192;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)wb, (short)0, 8192, 0x00020000);
    uint32_t off;
    switch (kShape) {
        case 0: off = 0xFFFFFFC0u; break;
        case 1: off = 0; break;
        case 2: off = 16 * lane; break;
        case 3: off = 64 * (lane >> 2) * 2 + 16 * (lane & 3); break;
        default: off = 128 * lane; break;
    }
    if (kShape == 5) off = (lane & 3) == 0 ? 128 * lane : 0xFFFFFFC0u;
    const bool act = kShape != 6 || (lane & 3) == 0;
    v4u acc = {0, 0, 0, 0};
    uint32_t x = t;
    lds[t] = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters / 8; i++) {
        v4u v[8];
        if (act) {
#pragma unroll
            for (int k = 0; k < 8; k++) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, off + (kShape == 2 ? 0 : 0), 16 * (k & 3), 0);
        }
#pragma unroll
        for (int k = 0; k < kValuPer; k++) asm volatile("v_alignbyte_b32 %0, %0, %0, 1" : "+v"(x));
        if (act) {
#pragma unroll
            for (int k = 0; k < 8; k++) acc ^= v[k];
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w ^ x) == 0x12345678u) out[0] = 1;
    if (lane == 0) cyc[wave] = t1 - t0;
}

struct Res {
    double ms, cyc;
};

template <typename F>
static Res time_launch(F launch, int nblocks, unsigned long long* dcyc, unsigned long long* hcyc) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch();  // warm
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const int nw = nblocks * 4;
    CK(hipMemcpy(hcyc, dcyc, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost));
    double s = 0;
    for (int i = 0; i < nw; i++) s += (double)hcyc[i];
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return {ms, s / nw};
}

template <int K>
static void issue_row(int cus, uint32_t* dout, unsigned long long* dcyc, unsigned long long* hcyc) {
    for (int w : {1, 2, 3, 4}) {
        const int nb = cus * w;
        const size_t lds_bytes = (160 * 1024) / w - 1024;
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_issue<K>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes));
        Res r = time_launch([&] { hipLaunchKernelGGL(k_issue<K>, dim3(nb), dim3(256), lds_bytes, 0, dout, dcyc, 7u); },
                            nb, dcyc, hcyc);
        const double per_wave = (double)kIters * (kVal[K] + kSal[K] + kLdsN[K]);
        // per SIMD: w waves, each per_wave instructions over cyc shader cycles (s_memtime counts shader clocks)
        const double ipq = w * per_wave / (r.cyc / 4.0);
        const double vpq = w * (double)kIters * kVal[K] / (r.cyc / 4.0);
        printf("issue %-20s waves/SIMD %d: %8.3f ms, %10.0f cyc/wave, instr/quad/SIMD %.3f, VALU/quad/SIMD %.3f\n",
               kNames[K], w, r.ms, r.cyc, ipq, vpq);
    }
}

template <int S, int V>
static void vmem_row(const char* name, int cus, const uint8_t* buf, uint32_t* dout, unsigned long long* dcyc,
                     unsigned long long* hcyc) {
    for (int w : {1, 2}) {
        const int nb = cus * w;
        const size_t lds_bytes = (160 * 1024) / w - 1024;
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_vmem<S, V>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes));
        Res r = time_launch([&] { hipLaunchKernelGGL((k_vmem<S, V>), dim3(nb), dim3(256), lds_bytes, 0, buf, dout, dcyc); },
                            nb, dcyc, hcyc);
        // loads per CU per cycle: 4 w waves per CU, kIters loads each
        const double loads_cu = 4.0 * w * kIters;
        printf("vmem %-34s valu/8ld %3d waves/SIMD %d: %8.3f ms, %9.0f cyc/wave, cyc per load-instr per CU %.2f\n", name, V, w,
               r.ms, r.cyc, r.cyc / loads_cu);
    }
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    setvbuf(stdout, nullptr, _IONBF, 0);
    printf("device %s, %d CUs, clock %d kHz\n", p.name, cus, p.clockRate);
    uint32_t* dout;
    unsigned long long* dcyc;
    uint8_t* buf;
    const int maxw = cus * 4 * 4;
    CK(hipMalloc(&dout, 64));
    CK(hipMalloc(&dcyc, sizeof(unsigned long long) * maxw));
    CK(hipMalloc(&buf, 4096ull * 8192 + 4096));
    CK(hipMemset(buf, 1, 4096ull * 8192 + 4096));
    unsigned long long* hcyc = (unsigned long long*)malloc(sizeof(unsigned long long) * maxw);
    issue_row<kAdd>(cus, dout, dcyc, hcyc);
    issue_row<kAlign>(cus, dout, dcyc, hcyc);
    issue_row<kBfi>(cus, dout, dcyc, hcyc);
    issue_row<kLshlOr>(cus, dout, dcyc, hcyc);
    issue_row<kCnd>(cus, dout, dcyc, hcyc);
    issue_row<kFma>(cus, dout, dcyc, hcyc);
    issue_row<kPk16>(cus, dout, dcyc, hcyc);
    issue_row<kSalu>(cus, dout, dcyc, hcyc);
    issue_row<kMix8to1>(cus, dout, dcyc, hcyc);
    issue_row<kMix4to1>(cus, dout, dcyc, hcyc);
    issue_row<kMix2to1>(cus, dout, dcyc, hcyc);
    issue_row<kLds>(cus, dout, dcyc, hcyc);
    issue_row<kMixLds>(cus, dout, dcyc, hcyc);
    issue_row<kStep>(cus, dout, dcyc, hcyc);
    vmem_row<0, 0>("all lanes out of range", cus, buf, dout, dcyc, hcyc);
    vmem_row<1, 0>("one 16-B word", cus, buf, dout, dcyc, hcyc);
    vmem_row<2, 0>("coalesced 1 KiB", cus, buf, dout, dcyc, hcyc);
    vmem_row<3, 0>("16 x 64 B (quads)", cus, buf, dout, dcyc, hcyc);
    vmem_row<4, 0>("64 lines (lane-private)", cus, buf, dout, dcyc, hcyc);
    vmem_row<5, 0>("16 lines live, 48 lanes out of range", cus, buf, dout, dcyc, hcyc);
    vmem_row<6, 0>("16 lines live, 48 lanes exec-masked", cus, buf, dout, dcyc, hcyc);
    vmem_row<0, 64>("all lanes out of range", cus, buf, dout, dcyc, hcyc);
    vmem_row<4, 64>("64 lines (lane-private)", cus, buf, dout, dcyc, hcyc);
    vmem_row<5, 64>("16 lines live, 48 lanes out of range", cus, buf, dout, dcyc, hcyc);
    vmem_row<6, 64>("16 lines live, 48 lanes exec-masked", cus, buf, dout, dcyc, hcyc);
    vmem_row<3, 64>("16 x 64 B (quads)", cus, buf, dout, dcyc, hcyc);
    printf("done\n");
    return 0;
}
