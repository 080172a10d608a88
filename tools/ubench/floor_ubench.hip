// Microbenchmark: the traffic floor of the metric query's phase A (k_slice_partition).
// Streams the three 1e9-row fact columns (x, k, v: 24 GB) with one 1024-thread workgroup per CU
// and writes the same bytes phase A writes (10 B per selected row, half the rows): sequentially,
// or as phase A's 32-item chunks (64 B of keys + 256 B of values) spread over F slice regions per
// workgroup -- no LDS work at all, so the time is what the memory system charges for the pattern.
// Dev tool only (not the product).
//   hipcc --offload-arch=gfx950 -O3 floor_ubench.hip -o floor_ubench && ./floor_ubench [rows] [reps]
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
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
constexpr int kBlock = 1024;
constexpr int F = 153;       // slices of the bench's 1e7-key table
constexpr int CH = 32;       // items per chunk

__device__ __host__ inline uint64_t smix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ void k_gen(int64_t *x, int64_t *k, double *v, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        x[i] = (int64_t)(smix(i * 3 + 1) % 100);
        k[i] = (int64_t)(smix(i * 3 + 2) % 10000000ull);
        v[i] = (double)(smix(i * 3 + 3) >> 11) * 0x1.0p-53;
    }
}

template <int P>
struct Tile {
    v2i64 x[P], k[P], v[P];
    __device__ __forceinline__ void issue(const int64_t *X, const int64_t *K, const int64_t *V, int64_t base) {
#pragma unroll
        for (int j = 0; j < P; ++j) k[j] = __builtin_nontemporal_load((const v2i64 *)(K + base + j * 128));
#pragma unroll
        for (int j = 0; j < P; ++j) x[j] = __builtin_nontemporal_load((const v2i64 *)(X + base + j * 128));
#pragma unroll
        for (int j = 0; j < P; ++j) v[j] = __builtin_nontemporal_load((const v2i64 *)(V + base + j * 128));
    }
    __device__ __forceinline__ int64_t fold() const {
        int64_t s = 0;
#pragma unroll
        for (int j = 0; j < P; ++j) s += (x[j][0] > 49 ? k[j][0] ^ v[j][0] : 0) + (x[j][1] > 49 ? k[j][1] ^ v[j][1] : 0);
        return s;
    }
};

// MODE 0: loads only.  1: + sequential stores (each workgroup its own contiguous region).
// 2: + phase A's chunk pattern: per tile TILE/2/CH chunks, chunk c of tile t to slice (c*37+t) % F,
//    region (wg, slice) appended in whole chunks.
// AHEAD: loads of tile t+1 issued before tile t is folded (register double buffer at P pairs).
template <int P, int MODE, bool AHEAD, bool NTS, int VB = 8, int CHK = CH>
__global__ __launch_bounds__(kBlock) void k_floor(const int64_t *__restrict__ X, const int64_t *__restrict__ K,
                                                  const int64_t *__restrict__ V, int64_t n_tiles, uint16_t *__restrict__ okey,
                                                  int64_t *__restrict__ oval, uint64_t cap, int64_t *__restrict__ sink) {
    constexpr int R = 2 * P, TILE = kBlock * R, NCH = TILE / 2 / CH;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ uint32_t pos[F];
    for (int i = tid; i < F; i += kBlock) pos[i] = 0;
    __syncthreads();
    int64_t acc = 0;
    uint64_t seq = (uint64_t)blockIdx.x * cap * F;  // MODE 1: items written so far
    Tile<P> a, b;
    int64_t tile = blockIdx.x;
    auto base = [&](int64_t t) { return t * TILE + (int64_t)wave * (64 * R) + 2 * lane; };
    if (tile < n_tiles) a.issue(X, K, V, base(tile));
    int it = 0;
    for (; tile < n_tiles; tile += gridDim.x, ++it) {
        if (AHEAD) {
            if (tile + gridDim.x < n_tiles) b.issue(X, K, V, base(tile + gridDim.x));
            acc += a.fold();
        } else {
            acc += a.fold();
        }
        if (MODE == 1) {
            // TILE/2 items: keys 2 B, values 8 B, 16-B stores
            const uint64_t o = seq;
            for (int i = tid * 8; i < TILE / 2; i += kBlock * 8) {
                v4u32 w = {(uint32_t)acc, (uint32_t)i, 0u, 0u};
                if (NTS) __builtin_nontemporal_store(w, (v4u32 *)(okey + o + i));
                else *(v4u32 *)(okey + o + i) = w;
            }
            // VB bytes of value per item (8: f64; 4 / 2: narrower items), 16-B stores
            int64_t *ob = (int64_t *)((char *)oval + o * VB);
            for (int i = tid * 2; i < TILE / 2 * VB / 8; i += kBlock * 2) {
                v2i64 w = {acc, (int64_t)i};
                if (NTS) __builtin_nontemporal_store(w, (v2i64 *)(ob + i));
                else *(v2i64 *)(ob + i) = w;
            }
            seq += TILE / 2;
        } else if (MODE == 4) {
            // 32-item chunks as one contiguous 320-B record block [64 B keys | 256 B values]
            for (int c = tid / 20; c < NCH; c += kBlock / 20) {
                const int s = (int)((c * 37 + it * 11 + blockIdx.x) % F);
                const uint64_t blk = ((uint64_t)blockIdx.x * F + s) * cap + pos[s];  // items
                char *b = (char *)oval + blk * 10;
                const int q = tid % 20;  // 20 x 16 B = 320 B
                v2i64 w = {acc, (int64_t)c};
                if (NTS) __builtin_nontemporal_store(w, (v2i64 *)(b + q * 16));
                else *(v2i64 *)(b + q * 16) = w;
            }
            __syncthreads();
            for (int c = tid; c < NCH; c += kBlock) {
                const int s = (int)((c * 37 + it * 11 + blockIdx.x) % F);
                atomicAdd(&pos[s], (uint32_t)CH);
            }
            __syncthreads();
            for (int i = tid; i < F; i += kBlock)
                if (pos[i] + CH > cap) pos[i] = 0;
            __syncthreads();
        } else if (MODE == 5 || MODE == 6) {
            // MODE 5: slot (slice s, chunk j of this workgroup for s, workgroup w) = (s * JM + j) * G + w:
            //   the j-th chunks of one slice from every workgroup sit side by side, so the workgroups'
            //   concurrent writes land close together and a slice is one contiguous range for phase B.
            // MODE 6: one global chunk stream in (iteration, workgroup, chunk) order (the k_produce shape).
            const uint32_t xl = (tid & (CH / 2 - 1)) * 2;
            const uint64_t G = gridDim.x, JM = cap / CH;
            for (int c = tid / (CH / 2); c < NCH; c += kBlock / (CH / 2)) {
                const int s = (int)((c * 37 + it * 11 + blockIdx.x) % F);
                const uint64_t j = pos[s] / CH;
                const uint64_t slot = MODE == 5 ? ((uint64_t)s * JM + j) * G + blockIdx.x
                                                : (((uint64_t)it * G + blockIdx.x) * NCH + c) % (F * JM * G);
                const uint64_t o = slot * CH + xl;
                const uint32_t kw = (uint32_t)acc ^ xl;
                v2i64 w = {acc, (int64_t)c};
                *(uint32_t *)(okey + o) = kw;
                if (NTS) __builtin_nontemporal_store(w, (v2i64 *)(oval + o));
                else *(v2i64 *)(oval + o) = w;
            }
            __syncthreads();
            for (int c = tid; c < NCH; c += kBlock) {
                const int s = (int)((c * 37 + it * 11 + blockIdx.x) % F);
                atomicAdd(&pos[s], (uint32_t)CH);
            }
            __syncthreads();
            for (int i = tid; i < F; i += kBlock)
                if (pos[i] + CH > cap) pos[i] = 0;
            __syncthreads();
        } else if (MODE == 2) {
            // one chunk per quarter-wave, two items per lane: 4-B key store + 16-B value store
            constexpr int NCK = TILE / 2 / CHK;
            const uint32_t xl = (tid & (CHK / 2 - 1)) * 2;
            for (int c = tid / (CHK / 2); c < NCK; c += kBlock / (CHK / 2)) {
                const int s = (int)((c * 37 + it * 11 + blockIdx.x) % F);
                const uint64_t o = ((uint64_t)blockIdx.x * F + s) * cap + pos[s] + xl;
                const uint32_t kw = (uint32_t)acc ^ xl;
                v2i64 w = {acc, (int64_t)c};
                *(uint32_t *)(okey + o) = kw;
                if (NTS) __builtin_nontemporal_store(w, (v2i64 *)(oval + o));
                else *(v2i64 *)(oval + o) = w;
            }
            __syncthreads();
            for (int c = tid; c < NCK; c += kBlock) {
                const int s = (int)((c * 37 + it * 11 + blockIdx.x) % F);
                atomicAdd(&pos[s], (uint32_t)CHK);
            }
            __syncthreads();
            for (int i = tid; i < F; i += kBlock)
                if (pos[i] + CHK > cap) pos[i] = 0;
            __syncthreads();
        }
        if (AHEAD) a = b;
        else if (tile + gridDim.x < n_tiles) a.issue(X, K, V, base(tile + gridDim.x));
    }
    if (acc == 0x123456789) sink[blockIdx.x] = acc;
}

// pure streams for reference: write or read `n16` 16-B words, grid-stride, 16 B per lane
template <bool WRITE>
__global__ __launch_bounds__(kBlock) void k_pure(v2i64 *__restrict__ p, int64_t n16, int64_t *__restrict__ sink) {
    int64_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n16; i += (int64_t)gridDim.x * kBlock) {
        if (WRITE) {
            v2i64 w = {i, i};
            __builtin_nontemporal_store(w, p + i);
        } else {
            v2i64 w = __builtin_nontemporal_load(p + i);
            acc += w[0] ^ w[1];
        }
    }
    if (acc == 0x123456789) sink[blockIdx.x] = acc;
}

// Chunked producer / consumer through a MALL-sized ring: k_produce streams rows [r0, r0 + cr) of
// x, k, v and writes 5 B per row (cached or nt stores) into the ring; k_consume reads the ring back
// (16-B loads, cached or nt).  Alternated over chunks on one stream: what a chunked phase A / phase B
// pipeline whose exchange stays in the Infinity Cache would cost.
template <bool NTS>
__global__ __launch_bounds__(kBlock) void k_produce(const int64_t *__restrict__ X, const int64_t *__restrict__ K,
                                                    const int64_t *__restrict__ V, int64_t r0, int64_t cr,
                                                    v2i64 *__restrict__ ring, int64_t *__restrict__ sink) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int P = 4, R = 8, TILE = kBlock * R;
    int64_t acc = 0;
    const int64_t nt = cr / TILE;
    for (int64_t t = blockIdx.x; t < nt; t += gridDim.x) {
        Tile<P> a;
        a.issue(X, K, V, r0 + t * TILE + (int64_t)wave * (64 * R) + 2 * lane);
        acc += a.fold();
        // 5 B per row = TILE * 5 / 16 16-B words per tile
        v2i64 *o = ring + t * (TILE * 5 / 16);
        for (int i = tid; i < TILE * 5 / 16; i += kBlock) {
            v2i64 w = {acc, (int64_t)i};
            if (NTS) __builtin_nontemporal_store(w, o + i);
            else o[i] = w;
        }
    }
    if (acc == 0x123456789) sink[blockIdx.x] = acc;
}
template <bool NTL>
__global__ __launch_bounds__(kBlock) void k_consume(const v2i64 *__restrict__ ring, int64_t n16, int64_t *__restrict__ sink) {
    int64_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n16; i += (int64_t)gridDim.x * kBlock) {
        v2i64 w = NTL ? __builtin_nontemporal_load(ring + i) : ring[i];
        acc += w[0] ^ w[1];
    }
    if (acc == 0x123456789) sink[blockIdx.x] = acc;
}

template <class L>
static float time_it(L launch, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f, tot = 0;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        tot += ms;
    }
    return tot / reps;
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? std::atoll(argv[1]) : 1000000000ll;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    int64_t *x, *k, *v, *sink;
    CK(hipMalloc(&x, n * 8));
    CK(hipMalloc(&k, n * 8));
    CK(hipMalloc(&v, n * 8));
    CK(hipMalloc(&sink, 4096 * 8));
    hipLaunchKernelGGL(k_gen, dim3(4096), dim3(256), 0, 0, x, k, (double *)v, n);
    CK(hipDeviceSynchronize());
    // regions: every workgroup F regions of cap items (half the rows, +25 %)
    const uint64_t cap = ((uint64_t)(n / 2 / cus / F * 1.25) + 64) / CH * CH;
    uint16_t *okey;
    int64_t *oval;
    CK(hipMalloc(&okey, (size_t)cus * F * cap * 2 + 4096));
    CK(hipMalloc(&oval, (size_t)cus * F * cap * 10 + 4096));  // MODE 4 writes 10 B per item
    const double rd = 24.0 * n / 1e9, wr = 5.0 * n / 1e9;
    auto run = [&](const char *name, auto kern, int P, int mode) {
        const int64_t tile = (int64_t)kBlock * 2 * P;
        const int64_t nt = n / tile;
        float ms = time_it([&] { hipLaunchKernelGGL(kern, dim3(cus), dim3(kBlock), 0, 0, x, k, v, nt, okey, oval, cap, sink); },
                           reps);
        const double gb = rd + (mode ? wr : 0.0);
        std::printf("%-58s %8.3f ms  %7.1f GB  %6.2f TB/s (reads alone %5.2f TB/s)\n", name, ms, gb, gb / ms, rd / ms);
        std::fflush(stdout);
    };
    run("read 24 B/row, P=4, reload after fold", k_floor<4, 0, false, true>, 4, 0);
    run("read 24 B/row, P=2, loads one tile ahead", k_floor<2, 0, true, true>, 2, 0);
    run("read 24 B/row, P=4, loads one tile ahead", k_floor<4, 0, true, true>, 4, 0);
    run("+ sequential 5 B/row nt stores, P=4", k_floor<4, 1, false, true>, 4, 1);
    run("+ sequential 5 B/row nt stores, P=2 ahead", k_floor<2, 1, true, true>, 2, 1);
    run("+ sequential 5 B/row cached stores, P=2 ahead", k_floor<2, 1, true, false>, 2, 1);
    run("+ chunked slice stores (nt values), P=4", k_floor<4, 2, false, true>, 4, 1);
    run("+ chunked slice stores (nt values), P=2 ahead", k_floor<2, 2, true, true>, 2, 1);
    run("+ chunked slice stores (nt values), P=4 ahead", k_floor<4, 2, true, true>, 4, 1);
    run("+ chunked slice stores (cached values), P=2 ahead", k_floor<2, 2, true, false>, 2, 1);
    run("+ chunked slice stores, 64-item chunks, P=4", k_floor<4, 2, false, true, 8, 64>, 4, 1);
    run("+ chunks, slots interleaved by workgroup per slice, P=4", k_floor<4, 5, false, true>, 4, 1);
    run("+ chunks, slots interleaved by workgroup per slice, P=4 ahead", k_floor<4, 5, true, true>, 4, 1);
    run("+ chunks, one global chunk stream, P=4", k_floor<4, 6, false, true>, 4, 1);
    run("+ chunked slice stores (nt values) again, P=4", k_floor<4, 2, false, true>, 4, 1);
    run("+ contiguous 320-B chunk records, P=4", k_floor<4, 4, false, true>, 4, 1);
    {
        auto r2 = [&](const char *name, auto kern, double wgb) {
            const int64_t nt = n / (kBlock * 8);
            float ms = time_it([&] { hipLaunchKernelGGL(kern, dim3(cus), dim3(kBlock), 0, 0, x, k, v, nt, okey, oval, cap, sink); },
                               reps);
            std::printf("%-58s %8.3f ms  %7.1f GB  %6.2f TB/s (reads alone %5.2f TB/s)\n", name, ms, rd + wgb, (rd + wgb) / ms,
                        rd / ms);
        };
        r2("+ sequential 4 B/row (8-B items) nt stores, P=4", k_floor<4, 1, false, true, 6>, 4.0 * n / 1e9);
        r2("+ sequential 3 B/row (6-B items) nt stores, P=4", k_floor<4, 1, false, true, 4>, 3.0 * n / 1e9);
        r2("+ sequential 2 B/row (4-B items) nt stores, P=4", k_floor<4, 1, false, true, 2>, 2.0 * n / 1e9);
    }
    {
        const int64_t n16 = (int64_t)(5.0 * n / 16);
        v2i64 *buf = (v2i64 *)oval;
        for (int per : {1, 4, 8}) {
            float msw = time_it([&] { hipLaunchKernelGGL(k_pure<true>, dim3(cus * per), dim3(kBlock), 0, 0, buf, n16, sink); }, reps);
            float msr = time_it([&] { hipLaunchKernelGGL(k_pure<false>, dim3(cus * per), dim3(kBlock), 0, 0, buf, n16, sink); }, reps);
            std::printf("pure nt write 5 GB, %d WG/CU: %.3f ms = %.2f TB/s; pure nt read 5 GB: %.3f ms = %.2f TB/s\n", per, msw,
                        n16 * 16 / 1e9 / msw, msr, n16 * 16 / 1e9 / msr);
        }
    }
    if (argc > 3) {  // the chunked producer / consumer pipe (round-4 record: no gain from a MALL ring)
        v2i64 *ring = (v2i64 *)oval;
        for (int64_t cr : {(int64_t)1 << 23, (int64_t)1 << 24, (int64_t)1 << 25, (int64_t)1 << 26, (int64_t)1 << 28}) {
            const int64_t nch = n / cr, n16 = cr * 5 / 16;
            auto pipe = [&](bool nts, bool ntl) {
                for (int64_t c = 0; c < nch; ++c) {
                    if (nts) hipLaunchKernelGGL(k_produce<true>, dim3(cus), dim3(kBlock), 0, 0, x, k, v, c * cr, cr, ring, sink);
                    else hipLaunchKernelGGL(k_produce<false>, dim3(cus), dim3(kBlock), 0, 0, x, k, v, c * cr, cr, ring, sink);
                    if (ntl) hipLaunchKernelGGL(k_consume<true>, dim3(cus * 4), dim3(kBlock), 0, 0, ring, n16, sink);
                    else hipLaunchKernelGGL(k_consume<false>, dim3(cus * 4), dim3(kBlock), 0, 0, ring, n16, sink);
                }
            };
            const double ringmb = cr * 5.0 / 1e6;
            for (int mode = 0; mode < 3; ++mode) {
                const bool nts = mode == 2, ntl = mode == 2;
                float ms = time_it([&] { pipe(nts, ntl); }, reps);
                std::printf("pipe: %lld chunks of %lld rows (ring %.0f MB), %s stores / %s loads: %.3f ms\n", (long long)nch,
                            (long long)cr, ringmb, nts ? "nt" : "cached", ntl ? "nt" : "cached", ms);
                if (mode == 0) mode = 1;  // cached/cached and nt/nt
            }
            // producer alone (no consumer) for the same chunks
            float msp = time_it([&] {
                for (int64_t c = 0; c < nch; ++c)
                    hipLaunchKernelGGL(k_produce<false>, dim3(cus), dim3(kBlock), 0, 0, x, k, v, c * cr, cr, ring, sink);
            }, reps);
            std::printf("pipe: producer alone, cached stores: %.3f ms\n", msp);
        }
    }
    return 0;
}
