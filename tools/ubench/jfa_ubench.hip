// Microbenchmark: where does the time of the fused filter -> probe -> group-by
// pass go?  Decomposes k_join_agg_fast's work (stream, table lookup, LDS
// aggregation) and the two-phase partitioned alternative's phase B, each as
// its own kernel over the BASELINE metric shapes (1e9 rows, 1e7-key u16
// direct table, 1024 groups).  Dev tool only (not the product).
//   hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics jfa_ubench.hip -o jfa_ubench
//   ./jfa_ubench [rows] [dim] [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

typedef long long v2i64 __attribute__((ext_vector_type(2)));
constexpr int kBlock = 256, kPairs = 4, kR = 8, kTile = kBlock * kR;
constexpr int G = 1024;

__device__ __host__ inline uint64_t smix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_gen(int64_t *x, int64_t *k, double *v, int64_t n, int64_t dim) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        x[i] = (int64_t)(smix(i * 3 + 1) % 100);
        k[i] = (int64_t)(smix(i * 3 + 2) % (uint64_t)dim);
        v[i] = (double)(smix(i * 3 + 3) >> 11) * 0x1.0p-53;
    }
}
__global__ void k_gen_table(uint16_t *t, int64_t dim) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < dim; i += (int64_t)gridDim.x * blockDim.x)
        t[i] = (uint16_t)(smix(i ^ 0xABCDEF) % G + 1);
}
// phase-B style items: key offsets inside one slice per partition
__global__ void k_gen_items(uint32_t *ko, double *v, int64_t n, int64_t slice) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        ko[i] = (uint32_t)(smix(i * 5 + 7) % (uint64_t)slice);
        v[i] = (double)(smix(i * 5 + 9) >> 11) * 0x1.0p-53;
    }
}

__device__ __forceinline__ v2i64 ld2(const int64_t *p) { return __builtin_nontemporal_load((const v2i64 *)p); }

// LOOKUP: 0 none (gid from a multiplicative hash), 1 u16 direct table
// ATOM:   0 none (register sinks), 1 u64 count + f64 sum in LDS, 2 u32 count + f64 sum,
//         3 f64 sum only, 4 u32 count only
template <int LOOKUP, int ATOM>
__global__ __launch_bounds__(kBlock) void k_fused(const int64_t *__restrict__ x, const int64_t *__restrict__ k,
                                                  const int64_t *__restrict__ v, const uint16_t *__restrict__ t,
                                                  int64_t n_tiles, double *__restrict__ out_sum,
                                                  unsigned long long *__restrict__ out_cnt) {
    __shared__ double s_sum[G];
    __shared__ unsigned long long s_cnt64[G];
    __shared__ uint32_t s_cnt32[G];
    for (int i = threadIdx.x; i < G; i += kBlock) {
        s_sum[i] = 0;
        s_cnt64[i] = 0;
        s_cnt32[i] = 0;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double rs = 0;
    uint32_t rc = 0;
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int64_t base = tile * kTile + (int64_t)wave * (64 * kR) + 2 * lane;
        v2i64 kk[kPairs], xx[kPairs], vv[kPairs];
#pragma unroll
        for (int j = 0; j < kPairs; ++j) kk[j] = ld2(k + base + j * 128);
#pragma unroll
        for (int j = 0; j < kPairs; ++j) xx[j] = ld2(x + base + j * 128);
#pragma unroll
        for (int j = 0; j < kPairs; ++j) vv[j] = ld2(v + base + j * 128);
        uint32_t sel = 0;
#pragma unroll
        for (int r = 0; r < kR; ++r) sel |= (xx[r >> 1][r & 1] > 49 ? 1u : 0u) << r;
        uint32_t gid[kR];
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            const int64_t key = kk[r >> 1][r & 1];
            gid[r] = 0;
            if ((sel >> r) & 1) {
                if (LOOKUP) gid[r] = (uint32_t)t[key] - 1u;
                else gid[r] = ((uint32_t)key * 0x9E3779B1u) >> 22;
            }
        }
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            if (!((sel >> r) & 1)) continue;
            const double val = __builtin_bit_cast(double, vv[r >> 1][r & 1]);
            const uint32_t g = gid[r] & (G - 1);
            if (ATOM == 0) {
                rs += val;
                rc += g;
            } else {
                if (ATOM == 1) atomicAdd(&s_cnt64[g], 1ull);
                if (ATOM == 2 || ATOM == 4) atomicAdd(&s_cnt32[g], 1u);
                if (ATOM != 4) atomicAdd(&s_sum[g], val);
            }
        }
    }
    __syncthreads();
    if (ATOM == 0) {
        atomicAdd(&s_sum[threadIdx.x], rs);
        atomicAdd(&s_cnt32[threadIdx.x], rc);
        __syncthreads();
    }
    for (int i = threadIdx.x; i < G; i += kBlock) {
        unsafeAtomicAdd(&out_sum[i], s_sum[i]);
        atomicAdd(&out_cnt[i], s_cnt64[i] + s_cnt32[i]);
    }
}

// Phase-B loop: items (u32 key offset, f64 v) streamed, lookups into a slice.
template <int LOOKUP, int ATOM, int U>
__global__ __launch_bounds__(kBlock) void k_phaseb(const uint32_t *__restrict__ ko, const double *__restrict__ v,
                                                   const uint16_t *__restrict__ t, int64_t n,
                                                   double *__restrict__ out_sum, unsigned long long *__restrict__ out_cnt) {
    __shared__ double s_sum[G];
    __shared__ unsigned long long s_cnt64[G];
    __shared__ uint32_t s_cnt32[G];
    for (int i = threadIdx.x; i < G; i += kBlock) {
        s_sum[i] = 0;
        s_cnt64[i] = 0;
        s_cnt32[i] = 0;
    }
    __syncthreads();
    double rs = 0;
    uint32_t rc = 0;
    const int64_t stride = (int64_t)gridDim.x * kBlock * U;
    for (int64_t i0 = (int64_t)blockIdx.x * kBlock * U + threadIdx.x; i0 < n; i0 += stride) {
        uint32_t kk[U];
        double vv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int64_t i = i0 + (int64_t)u * kBlock;
            i = i < n ? i : n - 1;
            kk[u] = __builtin_nontemporal_load(ko + i);
            vv[u] = __builtin_nontemporal_load(v + i);
        }
        uint32_t gid[U];
#pragma unroll
        for (int u = 0; u < U; ++u) gid[u] = LOOKUP ? (uint32_t)t[kk[u]] - 1u : ((kk[u] * 0x9E3779B1u) >> 22);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i0 + (int64_t)u * kBlock >= n) continue;
            const uint32_t g = gid[u] & (G - 1);
            if (ATOM == 0) {
                rs += vv[u];
                rc += g;
            } else {
                if (ATOM == 1) atomicAdd(&s_cnt64[g], 1ull);
                if (ATOM == 2 || ATOM == 4) atomicAdd(&s_cnt32[g], 1u);
                if (ATOM != 4) atomicAdd(&s_sum[g], vv[u]);
            }
        }
    }
    __syncthreads();
    if (ATOM == 0) {
        atomicAdd(&s_sum[threadIdx.x], rs);
        atomicAdd(&s_cnt32[threadIdx.x], rc);
        __syncthreads();
    }
    for (int i = threadIdx.x; i < G; i += kBlock) {
        unsafeAtomicAdd(&out_sum[i], s_sum[i]);
        atomicAdd(&out_cnt[i], s_cnt64[i] + s_cnt32[i]);
    }
}


// Mixed-traffic roofline: read x, k, v (24 B/row) and write 10 B per 2 rows
// (v of the odd rows + 16-bit keys) fully coalesced with 16-B stores.
template <bool NTS>
__global__ __launch_bounds__(kBlock) void k_mixed(const int64_t *__restrict__ x, const int64_t *__restrict__ k,
                                                  const int64_t *__restrict__ v, int64_t n_tiles, int64_t *__restrict__ ov,
                                                  uint16_t *__restrict__ ok, int64_t ring_items = 0) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int64_t base = tile * kTile + (int64_t)wave * (64 * kR) + 2 * lane;
        v2i64 kk[kPairs], xx[kPairs], vv[kPairs];
#pragma unroll
        for (int j = 0; j < kPairs; ++j) kk[j] = ld2(k + base + j * 128);
#pragma unroll
        for (int j = 0; j < kPairs; ++j) xx[j] = ld2(x + base + j * 128);
#pragma unroll
        for (int j = 0; j < kPairs; ++j) vv[j] = ld2(v + base + j * 128);
        // 4 output items per lane: v (32 B) + keys (8 B)
        int64_t ob = (tile * kTile) / 2 + (int64_t)wave * (64 * kR / 2) + 4 * lane;
        if (ring_items) ob %= ring_items;  // writes wrap around a small ring
        v2i64 o0 = {vv[0][0] + xx[0][0], vv[1][0] + xx[1][0]}, o1 = {vv[2][0] + xx[2][0], vv[3][0] + xx[3][0]};
        if (NTS) {
            __builtin_nontemporal_store(o0, (v2i64 *)(ov + ob));
            __builtin_nontemporal_store(o1, (v2i64 *)(ov + ob + 2));
        } else {
            *(v2i64 *)(ov + ob) = o0;
            *(v2i64 *)(ov + ob + 2) = o1;
        }
        const uint64_t kw = (uint64_t)(uint16_t)kk[0][0] | ((uint64_t)(uint16_t)kk[1][0] << 16) |
                            ((uint64_t)(uint16_t)kk[2][0] << 32) | ((uint64_t)(uint16_t)kk[3][0] << 48);
        if (NTS) __builtin_nontemporal_store(kw, (uint64_t *)(ok + ob));
        else *(uint64_t *)(ok + ob) = kw;
    }
}

template <typename F>
static float time_it(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? std::atoll(argv[1]) : 1000000000ll;
    const int64_t dim = argc > 2 ? std::atoll(argv[2]) : 10000000ll;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 5;
    const int64_t n_tiles = n / kTile;
    const int64_t rows = n_tiles * kTile;
    int64_t *x, *k, *v;
    uint16_t *t, *t_small;
    double *osum;
    unsigned long long *ocnt;
    CK(hipMalloc(&x, rows * 8));
    CK(hipMalloc(&k, rows * 8));
    CK(hipMalloc(&v, rows * 8));
    CK(hipMalloc(&t, dim * 2));
    const int64_t dim_small = 1000000;
    CK(hipMalloc(&t_small, dim_small * 2));
    CK(hipMalloc(&osum, G * 8));
    CK(hipMalloc(&ocnt, G * 8));
    hipLaunchKernelGGL(k_gen, dim3(8192), dim3(256), 0, 0, x, k, (double *)v, rows, dim);
    hipLaunchKernelGGL(k_gen_table, dim3(4096), dim3(256), 0, 0, t, dim);
    hipLaunchKernelGGL(k_gen_table, dim3(4096), dim3(256), 0, 0, t_small, dim_small);
    CK(hipDeviceSynchronize());
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::printf("rows=%lld dim=%lld cus=%d\n", (long long)rows, (long long)dim, cus);
    const double bytes = 24.0 * rows;
    auto report = [&](const char *name, float ms) {
        std::printf("%-44s %8.3f ms  %7.1f GB/s (24 B/row)\n", name, ms, bytes / ms / 1e6);
        std::fflush(stdout);
    };
    {
        int64_t *ov;
        uint16_t *okk;
        CK(hipMalloc(&ov, rows / 2 * 8));
        CK(hipMalloc(&okk, rows / 2 * 2));
        for (int per_cu : {4, 8}) {
            const int grid = cus * per_cu;
            report("mixed: read 24B/row + write 5B/row (16B st)",
                   time_it([&] { hipLaunchKernelGGL((k_mixed<false>), dim3(grid), dim3(kBlock), 0, 0, x, k, v, n_tiles, ov, okk); }, reps));
            report("mixed, nontemporal stores",
                   time_it([&] { hipLaunchKernelGGL((k_mixed<true>), dim3(grid), dim3(kBlock), 0, 0, x, k, v, n_tiles, ov, okk); }, reps));
        }
        for (int64_t ring_mb : {16, 64, 128, 512}) {
            const int64_t ring = ring_mb * (1 << 20) / 8;
            char name[96];
            std::snprintf(name, sizeof name, "mixed, writes into a %lld MB ring", (long long)ring_mb);
            report(name, time_it([&] { hipLaunchKernelGGL((k_mixed<false>), dim3(cus * 8), dim3(kBlock), 0, 0, x, k, v, n_tiles, ov, okk, ring); }, reps));
            std::snprintf(name, sizeof name, "mixed NT, writes into a %lld MB ring", (long long)ring_mb);
            report(name, time_it([&] { hipLaunchKernelGGL((k_mixed<true>), dim3(cus * 8), dim3(kBlock), 0, 0, x, k, v, n_tiles, ov, okk, ring); }, reps));
        }
        CK(hipFree(ov));
        CK(hipFree(okk));
    }
    if (argc > 4) return 0;  // mixed-traffic section only
    for (int per_cu : {4, 8}) {
        const int grid = cus * per_cu;
        std::printf("-- fused, %d workgroups/CU\n", per_cu);
#define RUNF(L, A, TBL, NAME)                                                                                   \
    report(NAME, time_it([&] { hipLaunchKernelGGL((k_fused<L, A>), dim3(grid), dim3(kBlock), 0, 0, x, k, v, TBL, \
                                                   n_tiles, osum, ocnt); }, reps))
        RUNF(0, 0, t, "stream only");
        RUNF(1, 0, t, "stream + lookup 20MB");
        RUNF(0, 1, t, "stream + LDS u64cnt+f64sum");
        RUNF(0, 2, t, "stream + LDS u32cnt+f64sum");
        RUNF(0, 3, t, "stream + LDS f64sum");
        RUNF(0, 4, t, "stream + LDS u32cnt");
        RUNF(1, 1, t, "full u64cnt (20MB table)");
        RUNF(1, 2, t, "full u32cnt (20MB table)");
    }
    // small-table fused: keys % dim_small via a second key column is not
    // available; instead regenerate keys in range
    hipLaunchKernelGGL(k_gen, dim3(8192), dim3(256), 0, 0, x, k, (double *)v, rows, dim_small);
    CK(hipDeviceSynchronize());
    {
        const int grid = cus * 8;
        RUNF(1, 0, t_small, "stream + lookup 2MB");
        RUNF(1, 1, t_small, "full u64cnt (2MB table)");
    }
    // phase B: 5e8 items (u32 key offset, f64 v); slice 1.25M keys = 2.5 MB of u16
    const int64_t ni = rows / 2;
    uint32_t *ko = (uint32_t *)x;  // reuse
    double *iv = (double *)k;
    hipLaunchKernelGGL(k_gen_items, dim3(8192), dim3(256), 0, 0, ko, iv, ni, dim / 8);
    CK(hipDeviceSynchronize());
    const double bbytes = 12.0 * ni;
    auto reportb = [&](const char *name, float ms) {
        std::printf("%-44s %8.3f ms  %7.1f GB/s (12 B/item)  %.2f Gitem/s\n", name, ms, bbytes / ms / 1e6, ni / ms / 1e6);
        std::fflush(stdout);
    };
    for (int per_cu : {4, 8}) {
        const int grid = cus * per_cu;
        std::printf("-- phase B (%lld items), %d workgroups/CU\n", (long long)ni, per_cu);
#define RUNB(L, A, U, NAME)                                                                                       \
    reportb(NAME, time_it([&] { hipLaunchKernelGGL((k_phaseb<L, A, U>), dim3(grid), dim3(kBlock), 0, 0, ko, iv, t, ni, \
                                                    osum, ocnt); }, reps))
        RUNB(0, 0, 8, "B stream only");
        RUNB(1, 0, 8, "B + lookup 2.5MB slice");
        RUNB(0, 1, 8, "B + LDS u64cnt+f64sum");
        RUNB(0, 2, 8, "B + LDS u32cnt+f64sum");
        RUNB(1, 1, 8, "B full u64cnt U8");
        RUNB(1, 1, 16, "B full u64cnt U16");
        RUNB(1, 2, 16, "B full u32cnt U16");
    }
    std::printf("done\n");
    return 0;
}
