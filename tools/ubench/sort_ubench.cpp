// Library baseline for the LSD radix sort: rocPRIM radix_sort_pairs (onesweep) on n
// (40-bit u64 key, u32 value) pairs, the shape of cfg 5's pair-key sort.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -x hip sort_ubench.cpp -o sort_ubench
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void gen(uint64_t *k, uint32_t *v, int64_t n, int bits) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = (uint64_t)i + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        k[i] = z & ((1ull << bits) - 1);
        v[i] = (uint32_t)i;
    }
}

__global__ void check(const uint64_t *k, int64_t n, unsigned *bad) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i + 1 < n; i += (int64_t)gridDim.x * blockDim.x)
        if (k[i] > k[i + 1]) atomicAdd(bad, 1u);
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 1000000000LL;
    const int bits = argc > 2 ? atoi(argv[2]) : 40;
    uint64_t *k0, *k1; uint32_t *v0, *v1; unsigned *bad;
    CK(hipMalloc(&k0, n * 8)); CK(hipMalloc(&k1, n * 8));
    CK(hipMalloc(&v0, n * 4)); CK(hipMalloc(&v1, n * 4)); CK(hipMalloc(&bad, 4));
    size_t tmp_bytes = 0;
    rocprim::double_buffer<uint64_t> kb(k0, k1);
    rocprim::double_buffer<uint32_t> vb(v0, v1);
    CK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, kb, vb, (size_t)n, 0, bits));
    void *tmp; CK(hipMalloc(&tmp, tmp_bytes));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int it = 0; it < 4; ++it) {
        hipLaunchKernelGGL(gen, dim3(4096), dim3(256), 0, 0, k0, v0, n, bits);
        rocprim::double_buffer<uint64_t> kk(k0, k1);
        rocprim::double_buffer<uint32_t> vv(v0, v1);
        CK(hipEventRecord(a));
        CK(rocprim::radix_sort_pairs(tmp, tmp_bytes, kk, vv, (size_t)n, 0, bits));
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        CK(hipMemset(bad, 0, 4));
        hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, kk.current(), n, bad);
        unsigned hb; CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
        printf("rocprim radix_sort_pairs n=%lld bits=%d: %.2f ms (tmp %.1f MB) unsorted=%u\n", (long long)n, bits, ms,
               tmp_bytes / 1e6, hb);
    }
    return 0;
}
