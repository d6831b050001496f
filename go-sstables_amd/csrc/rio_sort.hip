// rio_sort.hip — ordering a batch of DiskKeyIndex queries by key before the search (k_index_search).
//
// Every lane of k_index_search runs its own binary search; lanes whose keys are close take the same
// first probes (same SeekNext offsets: broadcast loads, no divergence). The batch is therefore
// visited in the order of each key's first 8 bytes (big-endian, a radix sort of (prefix, index)
// pairs); results still land at each query's own index. Order does not change any result: each
// lookup is independent (a freshly loaded index, rio.h).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

namespace rio {

__global__ void __launch_bounds__(256) k_key_prefix(const uint8_t* keys, const uint64_t* key_off, uint64_t n,
                                                    uint64_t* pfx, uint32_t* idx) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint8_t* k = keys + key_off[i];
        const uint64_t kl = key_off[i + 1] - key_off[i];
        uint64_t p = 0;
        for (uint32_t b = 0; b < 8; b++) p = (p << 8) | (b < kl ? k[b] : 0u);
        pfx[i] = p;
        idx[i] = (uint32_t)i;
    }
}

size_t key_sort_tmp_bytes(uint64_t n) {
    size_t b = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, b, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                           (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n) != hipSuccess)
        return 0;
    return b;
}

// perm[k] = index of the k-th query in key-prefix order
hipError_t launch_key_sort(const uint8_t* keys, const uint64_t* key_off, uint64_t n, uint64_t* pfx_in, uint64_t* pfx_out,
                           uint32_t* idx_in, uint32_t* perm, void* tmp, size_t tmp_bytes, hipStream_t s) {
    const unsigned g = (unsigned)std::min<uint64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_key_prefix, dim3(g ? g : 1), dim3(256), 0, s, keys, key_off, n, pfx_in, idx_in);
    size_t tb = tmp_bytes;
    return hipcub::DeviceRadixSort::SortPairs(tmp, tb, pfx_in, pfx_out, idx_in, perm, (int)n, 0, 64, s);
}

}  // namespace rio
