// Microbenchmark: what the memory system charges for the write pattern of a 1024-way stable
// partition pass (config 5's window pass 1: 16 B read, 8-B order key + 2-B key bits written per row)
// against aligned, chunked variants of the same bytes.  One 1024-thread workgroup per CU, 8192-row
// tiles, 16-B loads of the two input columns; the "partition" is synthetic (row s of a tile goes to
// digit s / 8, eight rows per digit per tile), so the time is the memory system's, not the ranking's.
//   W0  loads only
//   W1  per-tile runs at arbitrary alignment (the pass's pattern): 8 x 8 B + 8 x 2 B per digit run
//   W2  the same runs, 64-B aligned (8-item chunks of the 8-B stream)
//   W3  16-item chunks every other tile (128-B aligned order-key chunks, 32-B key-bit chunks)
//   W4  80-B records (8 order keys + 8 key-bit words in one contiguous record per run)
//   W5  sequential (each workgroup one contiguous output range): the write floor
//   W6  32-item chunks every fourth tile (256-B aligned order-key chunks, 64-B key-bit chunks)
// Dev tool only (not the product).
//   hipcc --offload-arch=gfx950 -O3 wpat_ubench.hip -o wpat_ubench && ./wpat_ubench [rows] [reps]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

typedef long long v2i64 __attribute__((ext_vector_type(2)));
constexpr int kBlock = 1024, TILE = 8192;

__global__ void k_fill(int64_t *a, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        a[i] = (int64_t)(i * 0x9E3779B97F4A7C15ull);
}

template <int W, int DIG = 1024>
__global__ __launch_bounds__(kBlock) void k_wpat(const int64_t *__restrict__ K, const int64_t *__restrict__ V,
                                                 int64_t tiles_per_wg, uint64_t *__restrict__ okey, uint16_t *__restrict__ okl,
                                                 uint8_t *__restrict__ orec, int64_t *__restrict__ sink) {
    constexpr int RUN = TILE / DIG;  // rows per digit per tile
    const int tid = threadIdx.x;
    const int64_t wg = blockIdx.x, G = gridDim.x;
    // digit d's region for this workgroup: RUN items per tile, tiles_per_wg tiles (+ 8 slack, + an
    // odd offset for W1 so runs start anywhere)
    const uint64_t per = (uint64_t)tiles_per_wg * RUN + 16;
    int64_t acc = 0;
    for (int64_t t = 0; t < tiles_per_wg; ++t) {
        const int64_t r0 = (wg * tiles_per_wg + t) * TILE;
        v2i64 k[4], v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            k[j] = __builtin_nontemporal_load((const v2i64 *)(K + r0 + j * 2048 + 2 * tid));
            v[j] = __builtin_nontemporal_load((const v2i64 *)(V + r0 + j * 2048 + 2 * tid));
        }
        if (W == 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) acc += k[j][0] ^ v[j][1];
            continue;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                // the staged tile is flushed slot by slot: consecutive lanes write consecutive slots,
                // so one store instruction covers 8 runs of 8 contiguous items (as pass 1's flush)
                const int s = (j * 2 + e) * 1024 + tid;
                const int d = s / RUN, x = s % RUN;
                const uint64_t val = (uint64_t)v[j][e];
                const uint16_t kl = (uint16_t)k[j][e];
                const uint64_t region = ((uint64_t)d * G + wg) * per;
                if (W == 1 || W == 2) {
                    const uint64_t p = region + (W == 1 ? 3 : 0) + (uint64_t)t * RUN + x;
                    __builtin_nontemporal_store(val, okey + p);
                    __builtin_nontemporal_store(kl, okl + p);
                } else if (W == 3 || W == 6) {
                    // chunks of C = 16 (W3) or 32 (W6) items: every (C / RUN)-th tile writes C-item
                    // runs for its digits (the others none) -- the same bytes in whole aligned chunks
                    constexpr int C = W == 3 ? 16 : 32, Q = C / RUN;
                    if (t % Q == Q - 1) {
#pragma unroll
                        for (int q = 0; q < Q; ++q) {
                            const int s2 = (j * 2 + e) * 1024 * Q + q * 1024 + tid;  // slot among Q tiles' worth
                            const int d2 = (s2 / C) % DIG, x2 = s2 % C;
                            const uint64_t reg2 = ((uint64_t)d2 * G + wg) * per;
                            const uint64_t p = reg2 + (uint64_t)(t / Q) * C + x2;
                            __builtin_nontemporal_store(val, okey + p);
                            __builtin_nontemporal_store(kl, okl + p);
                        }
                    }
                } else if (W == 4) {
                    uint8_t *rec = orec + (region + (uint64_t)t * RUN) * 10;
                    __builtin_nontemporal_store(val, (uint64_t *)rec + x);
                    __builtin_nontemporal_store(kl, (uint16_t *)(rec + 64) + x);
                } else {  // W5: sequential per workgroup
                    const uint64_t p = (uint64_t)wg * tiles_per_wg * TILE + (uint64_t)t * TILE + s;
                    __builtin_nontemporal_store(val, okey + p);
                    __builtin_nontemporal_store(kl, okl + p);
                }
            }
    }
    if (acc == 0x12345) sink[0] = acc;
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? std::atoll(argv[1]) : 1000000000ll;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    const int G = pr.multiProcessorCount;
    const int64_t tiles_per_wg = n / TILE / G, rows = tiles_per_wg * G * TILE;
    int64_t *K, *V, *sink;
    uint64_t *okey;
    uint16_t *okl;
    uint8_t *orec;
    const uint64_t per = (uint64_t)tiles_per_wg * 8 + 16, items = per * 1024 * G;
    CK(hipMalloc(&K, rows * 8));
    CK(hipMalloc(&V, rows * 8));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&okey, items * 8));
    CK(hipMalloc(&okl, items * 2));
    CK(hipMalloc(&orec, items * 10));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, K, rows);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, V, rows);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char *names[] = {"W0 loads only", "W1 runs, any alignment (pass 1)", "W2 runs, 64-B aligned",
                           "W3 2-tile chunks, 128-B aligned", "W4 80-B records", "W5 sequential", "W6 4-tile chunks, 256-B aligned",
                           "W7 runs of 16 (512 digits), any alignment", "W8 runs of 32 (256 digits), any alignment",
                           "W9 runs of 64 (128 digits), any alignment"};
    auto run = [&](int w) {
        auto go = [&]() {
            switch (w) {
                case 0: hipLaunchKernelGGL(k_wpat<0>, dim3(G), dim3(kBlock), 0, 0, K, V, tiles_per_wg, okey, okl, orec, sink); break;
                case 1: hipLaunchKernelGGL(k_wpat<1>, dim3(G), dim3(kBlock), 0, 0, K, V, tiles_per_wg, okey, okl, orec, sink); break;
                case 2: hipLaunchKernelGGL(k_wpat<2>, dim3(G), dim3(kBlock), 0, 0, K, V, tiles_per_wg, okey, okl, orec, sink); break;
                case 3: hipLaunchKernelGGL(k_wpat<3>, dim3(G), dim3(kBlock), 0, 0, K, V, tiles_per_wg, okey, okl, orec, sink); break;
                case 4: hipLaunchKernelGGL(k_wpat<4>, dim3(G), dim3(kBlock), 0, 0, K, V, tiles_per_wg, okey, okl, orec, sink); break;
                case 6: hipLaunchKernelGGL(k_wpat<6>, dim3(G), dim3(kBlock), 0, 0, K, V, tiles_per_wg, okey, okl, orec, sink); break;
                case 7: hipLaunchKernelGGL((k_wpat<1, 512>), dim3(G), dim3(kBlock), 0, 0, K, V, tiles_per_wg, okey, okl, orec, sink); break;
                case 8: hipLaunchKernelGGL((k_wpat<1, 256>), dim3(G), dim3(kBlock), 0, 0, K, V, tiles_per_wg, okey, okl, orec, sink); break;
                case 9: hipLaunchKernelGGL((k_wpat<1, 128>), dim3(G), dim3(kBlock), 0, 0, K, V, tiles_per_wg, okey, okl, orec, sink); break;
                default: hipLaunchKernelGGL(k_wpat<5>, dim3(G), dim3(kBlock), 0, 0, K, V, tiles_per_wg, okey, okl, orec, sink); break;
            }
        };
        go();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(a));
            go();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
        }
        const double gb = rows * (w ? 26.0 : 16.0) / 1e9;
        std::printf("%-36s %8.3f ms  %6.1f GB  %5.2f TB/s\n", names[w], best, gb, gb / best);
    };
    for (int w = 0; w < 10; ++w) run(w);
    return 0;
}
