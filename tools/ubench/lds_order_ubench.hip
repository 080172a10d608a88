// Are LDS atomics with return stable by lane?  The window partition passes rank every tile's rows
// stably (rows of one digit keep their input order) so that the inverse passes can replay the
// ranking.  If ds_add_rtn_u32 serves the lanes of one instruction that hit the same word in lane
// order, a per-wave packed-u16 counter table ranks rows stably with one LDS atomic per row instead
// of a ballot match over every digit bit.
//   mode 0: every wave does NJ rounds; in round j each lane adds (1 << 16 * (d & 1)) to word d >> 1
//           of its wave's counters (d = random digit of DBITS bits) and keeps the old half-word.
// The host checks that every returned rank equals the number of earlier rows (earlier round, or
// same round and lower lane) of the same wave with the same digit, and that two runs agree.
// Then a timing of the atomic ranking against the ballot-match ranking (same tile shape).
// Dev tool only.  Build: hipcc --offload-arch=gfx950 -O3 -o lds_order_ubench lds_order_ubench.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

constexpr int BLOCK = 1024, NJ = 8, DIG = 1024;

__device__ __host__ inline uint64_t smix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// digit of row (block, wave, j, lane): skewed patterns too (dmask narrows the digit range, so
// many lanes of one instruction hit the same word)
__device__ __host__ inline uint32_t digit_of(uint64_t seed, int b, int w, int j, int lane, uint32_t dmask) {
    return (uint32_t)smix(seed ^ ((uint64_t)b << 40) ^ ((uint64_t)w << 20) ^ ((uint64_t)j << 8) ^ (uint64_t)lane) & dmask;
}

__global__ __launch_bounds__(BLOCK) void k_rank_atomic(uint64_t seed, uint32_t dmask, uint16_t *out, int reps) {
    __shared__ uint32_t wc[BLOCK / 64][DIG / 2];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t acc = 0;
    for (int rep = 0; rep < reps; ++rep) {
        for (int i = lane; i < DIG / 2; i += 64) wc[wave][i] = 0u;
        __builtin_amdgcn_s_waitcnt(0xc07f);
        uint32_t d[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) d[j] = digit_of(seed + rep, blockIdx.x, wave, j, lane, dmask);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const uint32_t sh = (d[j] & 1u) * 16u;
            const uint32_t old = atomicAdd(&wc[wave][d[j] >> 1], 1u << sh);
            const uint32_t r = (old >> sh) & 0xFFFFu;
            acc += r;
            if (rep == 0) out[(((int64_t)blockIdx.x * (BLOCK / 64) + wave) * NJ + j) * 64 + lane] = (uint16_t)r;
        }
    }
    if (acc == 0xFFFFFFFFu) out[0] = 1;
}

// the ballot-match ranking of k_window.hip (10 digit bits), same shape, for timing
__global__ __launch_bounds__(BLOCK) void k_rank_ballot(uint64_t seed, uint32_t dmask, uint16_t *out, int reps) {
    __shared__ uint16_t wc[BLOCK / 64][DIG];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t acc = 0;
    for (int rep = 0; rep < reps; ++rep) {
        uint32_t *wz = (uint32_t *)wc[wave];
        for (int i = lane; i < DIG / 2; i += 64) wz[i] = 0u;
        __builtin_amdgcn_s_waitcnt(0xc07f);
        uint32_t d[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) d[j] = digit_of(seed + rep, blockIdx.x, wave, j, lane, dmask);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            uint64_t m = ~0ull;
#pragma unroll
            for (int b = 0; b < 10; ++b) {
                const uint32_t rep2 = (uint32_t)(__builtin_amdgcn_sbfe((int32_t)d[j], b, 1));
                const uint64_t bb = __ballot(rep2 != 0u);
                m &= ~(bb ^ (((uint64_t)rep2 << 32) | rep2));
            }
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            const uint32_t old = (uint32_t)wc[wave][d[j]];
            if (below == 0) wc[wave][d[j]] = (uint16_t)(old + (uint32_t)__popcll(m));
            const uint32_t r = old + below;
            __builtin_amdgcn_s_waitcnt(0xc07f);
            acc += r;
            if (rep == 0) out[(((int64_t)blockIdx.x * (BLOCK / 64) + wave) * NJ + j) * 64 + lane] = (uint16_t)r;
        }
    }
    if (acc == 0xFFFFFFFFu) out[0] = 1;
}

int main() {
    const int blocks = 2048;
    const size_t rows = (size_t)blocks * BLOCK * NJ;
    uint16_t *d_out;
    CK(hipMalloc(&d_out, rows * 2));
    std::vector<uint16_t> h(rows), h2(rows);
    int bad_total = 0;
    for (uint32_t dmask : {1023u, 63u, 3u, 0u}) {
        for (int kind = 0; kind < 2; ++kind) {
            auto kern = kind == 0 ? k_rank_atomic : k_rank_ballot;
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(BLOCK), 0, 0, 12345ull, dmask, d_out, 1);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), d_out, rows * 2, hipMemcpyDeviceToHost));
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(BLOCK), 0, 0, 12345ull, dmask, d_out, 1);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h2.data(), d_out, rows * 2, hipMemcpyDeviceToHost));
            int64_t bad = 0, nondet = 0;
            std::vector<uint32_t> cnt(DIG);
            for (int b = 0; b < blocks; ++b)
                for (int w = 0; w < BLOCK / 64; ++w) {
                    std::fill(cnt.begin(), cnt.end(), 0u);
                    for (int j = 0; j < NJ; ++j)
                        for (int l = 0; l < 64; ++l) {
                            const uint32_t dd = digit_of(12345ull, b, w, j, l, dmask);
                            const size_t idx = (((size_t)b * (BLOCK / 64) + w) * NJ + j) * 64 + l;
                            if (h[idx] != cnt[dd]) ++bad;
                            if (h[idx] != h2[idx]) ++nondet;
                            ++cnt[dd];
                        }
                }
            std::printf("%s dmask=%4u: %lld of %zu ranks differ from lane-stable order, %lld differ between runs\n",
                        kind == 0 ? "atomic" : "ballot", dmask, (long long)bad, rows, (long long)nondet);
            bad_total += bad != 0;
        }
    }
    // timing: reps rounds of ranking per launch
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int kind = 0; kind < 2; ++kind) {
        auto kern = kind == 0 ? k_rank_atomic : k_rank_ballot;
        hipLaunchKernelGGL(kern, dim3(512), dim3(BLOCK), 0, 0, 7ull, 1023u, d_out, 64);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(kern, dim3(512), dim3(BLOCK), 0, 0, 7ull, 1023u, d_out, 64);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double ranked = 512.0 * BLOCK * NJ * 64;
        std::printf("%s ranking: %.3f ms for %.3g rows = %.1f G rows/s (incl. digit hashing)\n",
                    kind == 0 ? "atomic" : "ballot", ms, ranked, ranked / ms / 1e6);
    }
    std::printf(bad_total ? "RESULT: atomic ranking NOT lane-stable\n" : "RESULT: stable\n");
    return 0;
}
