// op_probe.hip — VALU issue rate per instruction (and per encoding) on gfx950: which integer operations two waves
// of a SIMD issue at ~1.6 per 4-cycle slot (v_add_u32's rate) and which at ~1.1 (v_alignbyte_b32's), so that
// k_snappy_pipe's step can be steered to the fast forms. Companion of issue_probe.hip.
// Standalone: hipcc --offload-arch=gfx950 -O3 scripts/op_probe.hip -o scripts/op_probe && scripts/op_probe
// Every loop body is 64 inline-asm instructions of one kind over 8 independent chains; timing by s_memtime.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <utility>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

constexpr int kIters = 1024;

// two-source: a = op(a, b); three-source: a = op(a, b, c)
#define DEF2(ID, STR) \
    if constexpr (K == ID) { \
        _Pragma("unroll") for (int g = 0; g < 8; g++) { \
            asm volatile(STR : "+v"(a0) : "v"(b), "v"(c)); asm volatile(STR : "+v"(a1) : "v"(b), "v"(c)); \
            asm volatile(STR : "+v"(a2) : "v"(b), "v"(c)); asm volatile(STR : "+v"(a3) : "v"(b), "v"(c)); \
            asm volatile(STR : "+v"(a4) : "v"(b), "v"(c)); asm volatile(STR : "+v"(a5) : "v"(b), "v"(c)); \
            asm volatile(STR : "+v"(a6) : "v"(b), "v"(c)); asm volatile(STR : "+v"(a7) : "v"(b), "v"(c)); \
        } \
    }
// compares: write a mask (vcc or an SGPR pair), read a_i and b
#define DEFC(ID, STR) \
    if constexpr (K == ID) { \
        _Pragma("unroll") for (int g = 0; g < 8; g++) { \
            asm volatile(STR : "=s"(m0) : "v"(a0), "v"(b)); asm volatile(STR : "=s"(m1) : "v"(a1), "v"(b)); \
            asm volatile(STR : "=s"(m2) : "v"(a2), "v"(b)); asm volatile(STR : "=s"(m3) : "v"(a3), "v"(b)); \
            asm volatile(STR : "=s"(m0) : "v"(a4), "v"(b)); asm volatile(STR : "=s"(m1) : "v"(a5), "v"(b)); \
            asm volatile(STR : "=s"(m2) : "v"(a6), "v"(b)); asm volatile(STR : "=s"(m3) : "v"(a7), "v"(b)); \
        } \
    }
#define DEFCV(ID, STR) \
    if constexpr (K == ID) { \
        _Pragma("unroll") for (int g = 0; g < 64; g++) { asm volatile(STR : : "v"(a0), "v"(b) : "vcc"); } \
    }

static const char* kNames[] = {
    "v_add_u32 (VOP2)",          "v_add_u32_e64",           "v_and_b32",              "v_or_b32",
    "v_xor_b32",                 "v_lshlrev_b32",           "v_lshrrev_b32",          "v_lshrrev_b32_e64",
    "v_sub_u32",                 "v_min_u32",               "v_mul_u32_u24",          "v_cndmask_b32 (vcc)",
    "v_cndmask_b32_e64 (sgpr)",  "v_alignbyte_b32",         "v_bfi_b32",              "v_and_or_b32",
    "v_or3_b32",                 "v_add3_u32",              "v_lshl_or_b32",          "v_lshl_add_u32",
    "v_bfe_u32",                 "v_perm_b32",              "v_xad_u32",              "v_mad_u32_u24",
    "v_cmp_gt_u32 (vcc, VOPC)",  "v_cmp_gt_u32_e64 (sgpr)", "v_mov_b32 (VOP1)",       "v_ffbl_b32 (VOP1)",
    "v_pk_add_u16",              "v_add_co_u32 (vcc)",      "v_max3_u32",             "v_med3_u32",
};
constexpr int kNOps = sizeof(kNames) / sizeof(kNames[0]);

template <int K>
__global__ void __launch_bounds__(256) k_op(uint32_t* out, unsigned long long* cyc, uint32_t seed) {
    const uint32_t t = threadIdx.x;
    uint32_t a0 = t, a1 = t + 1, a2 = t + 2, a3 = t + 3, a4 = t + 4, a5 = t + 5, a6 = t + 6, a7 = t + 7;
    uint32_t b = (seed ^ t) & 15u, c = seed + 3;
    uint64_t m0 = 0, m1 = 0, m2 = 0, m3 = 0;
    if constexpr (K == 11) asm volatile("s_mov_b64 vcc, %0" : : "s"(0x5555555555555555ull ^ seed) : "vcc");
    const uint64_t msk = 0x5555555555555555ull ^ seed;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; i++) {
        DEF2(0, "v_add_u32 %0, %0, %1")
        DEF2(1, "v_add_u32_e64 %0, %0, %1")
        DEF2(2, "v_and_b32 %0, %0, %1")
        DEF2(3, "v_or_b32 %0, %0, %1")
        DEF2(4, "v_xor_b32 %0, %0, %1")
        DEF2(5, "v_lshlrev_b32 %0, %1, %0")
        DEF2(6, "v_lshrrev_b32 %0, %1, %0")
        DEF2(7, "v_lshrrev_b32_e64 %0, %1, %0")
        DEF2(8, "v_sub_u32 %0, %0, %1")
        DEF2(9, "v_min_u32 %0, %0, %1")
        DEF2(10, "v_mul_u32_u24 %0, %0, %1")
        DEF2(11, "v_cndmask_b32 %0, %0, %1, vcc")
        if constexpr (K == 12) {
#pragma unroll
            for (int g = 0; g < 8; g++) {
                asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a0) : "v"(b), "s"(msk));
                asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a1) : "v"(b), "s"(msk));
                asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a2) : "v"(b), "s"(msk));
                asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a3) : "v"(b), "s"(msk));
                asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a4) : "v"(b), "s"(msk));
                asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a5) : "v"(b), "s"(msk));
                asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a6) : "v"(b), "s"(msk));
                asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a7) : "v"(b), "s"(msk));
            }
        }
        DEF2(13, "v_alignbyte_b32 %0, %0, %1, %2")
        DEF2(14, "v_bfi_b32 %0, %1, %0, %2")
        DEF2(15, "v_and_or_b32 %0, %0, %1, %2")
        DEF2(16, "v_or3_b32 %0, %0, %1, %2")
        DEF2(17, "v_add3_u32 %0, %0, %1, %2")
        DEF2(18, "v_lshl_or_b32 %0, %0, 3, %1")
        DEF2(19, "v_lshl_add_u32 %0, %0, 3, %1")
        DEF2(20, "v_bfe_u32 %0, %0, %1, 8")
        DEF2(21, "v_perm_b32 %0, %0, %1, %2")
        DEF2(22, "v_xad_u32 %0, %0, %1, %2")
        DEF2(23, "v_mad_u32_u24 %0, %0, %1, %2")
        DEFCV(24, "v_cmp_gt_u32 vcc, %0, %1")
        DEFC(25, "v_cmp_gt_u32_e64 %0, %1, %2")
        DEF2(26, "v_mov_b32 %0, %1")
        DEF2(27, "v_ffbl_b32 %0, %0")
        DEF2(28, "v_pk_add_u16 %0, %0, %1")
        if constexpr (K == 29) {
#pragma unroll
            for (int g = 0; g < 8; g++) {
                asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a0) : "v"(b) : "vcc");
                asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a1) : "v"(b) : "vcc");
                asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a2) : "v"(b) : "vcc");
                asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a3) : "v"(b) : "vcc");
                asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a4) : "v"(b) : "vcc");
                asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a5) : "v"(b) : "vcc");
                asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a6) : "v"(b) : "vcc");
                asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a7) : "v"(b) : "vcc");
            }
        }
        DEF2(30, "v_max3_u32 %0, %0, %1, %2")
        DEF2(31, "v_med3_u32 %0, %0, %1, %2")
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(m0 ^ m1 ^ m2 ^ m3);
    if (r == 0x12345678u) out[0] = r;
    if ((t & 63) == 0) cyc[(blockIdx.x * blockDim.x + t) >> 6] = t1 - t0;
}

template <int K>
static void row(int cus, uint32_t* dout, unsigned long long* dcyc, unsigned long long* hcyc) {
    printf("%-28s", kNames[K]);
    for (int w : {1, 2, 4}) {
        const int nb = cus * w;  // 4 waves per block: w waves per SIMD
        const size_t lds = (160 * 1024) / w - 1024;  // pins w blocks per CU
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_op<K>), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(k_op<K>, dim3(nb), dim3(256), lds, 0, dout, dcyc, 7u);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(k_op<K>, dim3(nb), dim3(256), lds, 0, dout, dcyc, 7u);
        CK(hipDeviceSynchronize());
        const int nw = nb * 4;
        CK(hipMemcpy(hcyc, dcyc, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost));
        double s = 0;
        for (int i = 0; i < nw; i++) s += (double)hcyc[i];
        const double cyc = s / nw;
        printf("  w%d %.3f", w, w * 64.0 * kIters / (cyc / 4.0));
    }
    printf("   (instr per 4-cycle slot per SIMD)\n");
}

template <int... Ks>
static void rows(std::integer_sequence<int, Ks...>, int cus, uint32_t* d, unsigned long long* c, unsigned long long* h) {
    (row<Ks>(cus, d, c, h), ...);
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    setvbuf(stdout, nullptr, _IONBF, 0);
    printf("device %s, %d CUs\n", p.name, p.multiProcessorCount);
    uint32_t* dout;
    unsigned long long* dcyc;
    const int maxw = p.multiProcessorCount * 16;
    CK(hipMalloc(&dout, 64));
    CK(hipMalloc(&dcyc, sizeof(unsigned long long) * maxw));
    unsigned long long* hcyc = (unsigned long long*)malloc(sizeof(unsigned long long) * maxw);
    rows(std::make_integer_sequence<int, kNOps>{}, p.multiProcessorCount, dout, dcyc, hcyc);
    printf("done\n");
    return 0;
}
