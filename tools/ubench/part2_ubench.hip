// Prototype of the LDS-slice partitioned probe for filter -> join -> group-by:
//   phase A streams (x, k, v), filters, and appends each selected row's
//   (16-bit key offset inside its table slice, v) to a per-(workgroup, slice)
//   region, staged in LDS so every region is written in contiguous runs;
//   phase B loads one table slice (2^SHIFT u16 entries) into LDS and drains
//   that slice's regions with LDS lookups and LDS aggregate states.
// Chunked variant: phase A and B alternate over fact chunks so the exchanged
// items can stay in the Infinity Cache.  Dev tool only.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <chrono>
#include <algorithm>

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
constexpr int G = 1024;
constexpr int kMaxF = 512;

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
__device__ __forceinline__ v2i64 ld2(const int64_t *p) { return __builtin_nontemporal_load((const v2i64 *)p); }

// ---- reference single pass ----
__global__ __launch_bounds__(256) void k_ref(const int64_t *x, const int64_t *k, const int64_t *v, const uint16_t *t, int64_t n,
                                             double *osum, unsigned long long *ocnt) {
    __shared__ double s_sum[G];
    __shared__ uint32_t s_cnt[G];
    for (int i = threadIdx.x; i < G; i += 256) s_sum[i] = 0, s_cnt[i] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        if (x[i] > 49) {
            uint32_t e = t[k[i]];
            if (e) {
                atomicAdd(&s_sum[e - 1], __builtin_bit_cast(double, v[i]));
                atomicAdd(&s_cnt[e - 1], 1u);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < G; i += 256) {
        unsafeAtomicAdd(&osum[i], s_sum[i]);
        atomicAdd(&ocnt[i], (unsigned long long)s_cnt[i]);
    }
}

// ---- phase A ----
template <int SHIFT, int BLOCK, int AMODE = 0>
__global__ __launch_bounds__(BLOCK) void k_pa(const int64_t *__restrict__ x, const int64_t *__restrict__ k,
                                              const int64_t *__restrict__ v, int64_t n_tiles, int64_t dim, int F,
                                              uint64_t cap, uint16_t *__restrict__ keyo, int64_t *__restrict__ vo,
                                              uint32_t *__restrict__ cnt_out, uint32_t *__restrict__ overflow) {
    constexpr int R = 8, TILE = BLOCK * R;
    __shared__ uint32_t cnt[kMaxF], lofs[kMaxF], cur[kMaxF];
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t s_total;
    __shared__ uint16_t st_key[TILE], st_b[TILE];
    __shared__ int64_t st_v[TILE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < kMaxF; i += BLOCK) cnt[i] = 0, cur[i] = 0;
    __syncthreads();
    int64_t tile = blockIdx.x;
    v2i64 kk[4], xx[4], vv[4];
    auto load = [&](int64_t t) {
        const int64_t base = t * TILE + (int64_t)wave * (64 * R) + 2 * lane;
#pragma unroll
        for (int j = 0; j < 4; ++j) kk[j] = ld2(k + base + j * 128);
#pragma unroll
        for (int j = 0; j < 4; ++j) xx[j] = ld2(x + base + j * 128);
#pragma unroll
        for (int j = 0; j < 4; ++j) vv[j] = ld2(v + base + j * 128);
    };
    if (tile < n_tiles) load(tile);
    const uint64_t region0 = (uint64_t)blockIdx.x * F;
    for (; tile < n_tiles; tile += gridDim.x) {
        uint32_t sel = 0, bk[R], rk[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t key = kk[r >> 1][r & 1];
            bk[r] = 0;
            rk[r] = 0;
            if (xx[r >> 1][r & 1] > 49 && key >= 0 && key < dim) {
                sel |= 1u << r;
                bk[r] = (uint32_t)key;
                rk[r] = atomicAdd(&cnt[(uint32_t)key >> SHIFT], 1u);
            }
        }
        __syncthreads();
        if (tid < kMaxF) {
            const uint32_t c = cnt[tid];
            uint32_t s = c;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t t2 = __shfl_up(s, d, 64);
                if (lane >= d) s += t2;
            }
            if (lane == 63) wsum[wave] = s;
            lofs[tid] = s - c;
        }
        __syncthreads();
        if (tid < kMaxF) {
            uint32_t add = 0;
            for (int w = 0; w < wave; ++w) add += wsum[w];
            lofs[tid] += add;
            if (tid == kMaxF - 1) s_total = lofs[tid] + cnt[tid];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (!((sel >> r) & 1)) continue;
            const uint32_t b = bk[r] >> SHIFT;
            const uint32_t s = lofs[b] + rk[r];
            st_key[s] = (uint16_t)(bk[r] & ((1u << SHIFT) - 1));
            st_b[s] = (uint16_t)b;
            st_v[s] = vv[r >> 1][r & 1];
        }
        if (tile + gridDim.x < n_tiles) load(tile + gridDim.x);
        __syncthreads();
        const uint32_t total = s_total;
        for (uint32_t i = tid; i < total; i += BLOCK) {
            const uint32_t b = st_b[i];
            const uint64_t dst = (uint64_t)cur[b] + (i - lofs[b]);
            if (AMODE == 1) continue;  // no global stores
            if (AMODE == 2) {          // same stores, linear per-workgroup addresses
                const uint64_t o = region0 * cap + ((uint64_t)(tile / gridDim.x) * TILE + i) % (F * cap);
                keyo[o] = st_key[i];
                vo[o] = st_v[i];
                continue;
            }
            if (dst < cap) {
                const uint64_t o = (region0 + b) * cap + dst;
                keyo[o] = st_key[i];
                vo[o] = st_v[i];
            } else {
                *overflow = 1u;
            }
        }
        __syncthreads();
        if (tid < kMaxF) {
            cur[tid] += cnt[tid];
            cnt[tid] = 0;
        }
        __syncthreads();
    }
    for (int b = tid; b < F; b += BLOCK) cnt_out[region0 + b] = cur[b] < cap ? cur[b] : (uint32_t)cap;
}


// ---- phase B, flattened over the regions of a unit ----
template <int SHIFT, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_pb2(const uint16_t *__restrict__ table, int64_t dim, int F, int nreg, int splits,
                                               uint64_t cap, const uint16_t *__restrict__ keyo,
                                               const int64_t *__restrict__ vo, const uint32_t *__restrict__ cnt_in,
                                               double *__restrict__ osum, unsigned long long *__restrict__ ocnt) {
    constexpr int S = 1 << SHIFT;
    __shared__ double s_sum[G];
    __shared__ uint32_t s_cnt[G];
    __shared__ uint32_t pref[1025];
    __shared__ uint32_t wsum[16];
    __shared__ __attribute__((aligned(16))) uint16_t tslice[S];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < G; i += BLOCK) s_sum[i] = 0, s_cnt[i] = 0;
    int cur_b = -1;
    const int units = F * splits;
    for (int u = blockIdx.x; u < units; u += gridDim.x) {
        const int b = u / splits, sp = u % splits;
        const int r0 = (int)((int64_t)sp * nreg / splits), r1 = (int)((int64_t)(sp + 1) * nreg / splits);
        const int nr = r1 - r0;  // <= BLOCK
        __syncthreads();
        if (b != cur_b) {
            const int64_t k0 = (int64_t)b * S;
            const int64_t nk = dim - k0 < S ? dim - k0 : S;
            for (int i = tid * 8; i < S; i += BLOCK * 8) {
                v4u32 w = {0, 0, 0, 0};
                if (i < nk) w = *(const v4u32 *)(table + k0 + i);
                *(v4u32 *)&tslice[i] = w;
            }
            cur_b = b;
        }
        {
            const uint32_t c = tid < nr ? cnt_in[(uint64_t)(r0 + tid) * F + b] : 0u;
            uint32_t s = c;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t t2 = __shfl_up(s, d, 64);
                if (lane >= d) s += t2;
            }
            if (lane == 63) wsum[wave] = s;
            __syncthreads();
            uint32_t add = 0;
            for (int w = 0; w < wave; ++w) add += wsum[w];
            pref[tid + 1] = s + add;
            if (tid == 0) pref[0] = 0;
        }
        __syncthreads();
        const uint32_t total = pref[nr];
        for (uint32_t base = 0; base < total; base += BLOCK * 8) {
            uint32_t kk8[8];
            int64_t vv8[8];
            uint32_t live = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t idx = base + j * BLOCK + tid;
                kk8[j] = 0;
                vv8[j] = 0;
                if (idx < total) {
                    // last region whose prefix <= idx
                    int lo = 0, hi = nr;  // pref[lo] <= idx < pref[hi]
                    while (hi - lo > 1) {
                        const int mid = (lo + hi) >> 1;
                        if (pref[mid] <= idx) lo = mid; else hi = mid;
                    }
                    const uint64_t o = ((uint64_t)(r0 + lo) * F + b) * cap + (idx - pref[lo]);
                    kk8[j] = keyo[o];
                    vv8[j] = __builtin_nontemporal_load(vo + o);
                    live |= 1u << j;
                }
            }
            uint32_t e8[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) e8[j] = ((live >> j) & 1) ? (uint32_t)tslice[kk8[j]] : 0u;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (!e8[j]) continue;
                atomicAdd(&s_sum[e8[j] - 1], __builtin_bit_cast(double, vv8[j]));
                atomicAdd(&s_cnt[e8[j] - 1], 1u);
            }
        }
    }
    __syncthreads();
    for (int i = tid; i < G; i += BLOCK) {
        unsafeAtomicAdd(&osum[i], s_sum[i]);
        atomicAdd(&ocnt[i], (unsigned long long)s_cnt[i]);
    }
}

template <int SHIFT, int BA, int BB>
static void run_chunked(int64_t *x, int64_t *k, int64_t *v, uint16_t *t, int64_t rows, int64_t dim, int cus, int reps,
                        int64_t chunk_rows, int splits, int streams, const std::vector<double> &rsum,
                        const std::vector<unsigned long long> &rcnt) {
    const int F = (int)((dim + (1 << SHIFT) - 1) >> SHIFT);
    const int gridA = cus;
    constexpr int TILE = BA * 8;
    chunk_rows = chunk_rows / TILE * TILE;
    const int64_t n_chunks = (rows + chunk_rows - 1) / chunk_rows;
    const uint64_t nreg = (uint64_t)gridA * F;
    const double avg = (double)chunk_rows / 2 / nreg;
    uint64_t cap = (uint64_t)(avg * 1.25 + 256);
    cap = (cap + 7) & ~7ull;
    const int nslot = streams;
    uint16_t *keyo[2];
    int64_t *vo[2];
    uint32_t *cnt[2], *ovf;
    double *osum;
    unsigned long long *ocnt;
    for (int sl = 0; sl < nslot; ++sl) {
        CK(hipMalloc(&keyo[sl], nreg * cap * 2 + 64));
        CK(hipMalloc(&vo[sl], nreg * cap * 8 + 64));
        CK(hipMalloc(&cnt[sl], nreg * 4));
    }
    CK(hipMalloc(&ovf, 4));
    CK(hipMalloc(&osum, G * 8));
    CK(hipMalloc(&ocnt, G * 8));
    CK(hipMemset(ovf, 0, 4));
    hipStream_t st[2];
    CK(hipStreamCreateWithFlags(&st[0], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&st[1], hipStreamNonBlocking));
    hipEvent_t evA[2], evB[2];
    for (int i = 0; i < 2; ++i) {
        CK(hipEventCreateWithFlags(&evA[i], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&evB[i], hipEventDisableTiming));
    }
    const int gridB = cus * (SHIFT == 15 ? 2 : 1);
    const int nregB = gridA;  // regions per bucket
    auto whole = [&] {
        for (int64_t c = 0; c < n_chunks; ++c) {
            const int sl = (int)(c % nslot);
            const int64_t r0 = c * chunk_rows;
            const int64_t nr = rows - r0 < chunk_rows ? rows - r0 : chunk_rows;
            hipStream_t sa = st[0], sb = st[nslot > 1 ? 1 : 0];
            if (nslot > 1 && c >= 2) CK(hipStreamWaitEvent(sa, evB[sl], 0));
            hipLaunchKernelGGL((k_pa<SHIFT, BA>), dim3(gridA), dim3(BA), 0, sa, x + r0, k + r0, v + r0, nr / TILE, dim, F,
                               cap, keyo[sl], vo[sl], cnt[sl], ovf);
            if (nslot > 1) {
                CK(hipEventRecord(evA[sl], sa));
                CK(hipStreamWaitEvent(sb, evA[sl], 0));
            }
            hipLaunchKernelGGL((k_pb2<SHIFT, BB>), dim3(gridB), dim3(BB), 0, sb, t, dim, F, nregB, splits, cap, keyo[sl],
                               vo[sl], cnt[sl], osum, ocnt);
            if (nslot > 1) CK(hipEventRecord(evB[sl], sb));
        }
    };
    auto timed = [&] {
        whole();
        CK(hipStreamSynchronize(st[0]));
        CK(hipStreamSynchronize(st[1]));
    };
    timed();
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int i = 0; i < reps; ++i) timed();
    auto t1 = std::chrono::high_resolution_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count() / reps;
    CK(hipMemset(osum, 0, G * 8));
    CK(hipMemset(ocnt, 0, G * 8));
    timed();
    std::vector<double> s(G);
    std::vector<unsigned long long> c(G);
    uint32_t of = 0;
    CK(hipMemcpy(s.data(), osum, G * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(c.data(), ocnt, G * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&of, ovf, 4, hipMemcpyDeviceToHost));
    double maxrel = 0;
    bool cnt_ok = true;
    for (int g = 0; g < G; ++g) {
        cnt_ok &= c[g] == rcnt[g];
        maxrel = std::fmax(maxrel, std::fabs(s[g] - rsum[g]) / std::fmax(1e-300, std::fabs(rsum[g])));
    }
    std::printf("chunked SHIFT=%d F=%d chunk=%lld (%lld chunks) streams=%d splits=%d | %.3f ms = %.1f GB/s alg | counts %s "
                "maxrel %.2e overflow %u\n",
                SHIFT, F, (long long)chunk_rows, (long long)n_chunks, streams, splits, ms, 24.0 * rows / ms / 1e6,
                cnt_ok ? "ok" : "BAD", maxrel, of);
    std::fflush(stdout);
    for (int sl = 0; sl < nslot; ++sl) {
        CK(hipFree(keyo[sl]));
        CK(hipFree(vo[sl]));
        CK(hipFree(cnt[sl]));
    }
    CK(hipFree(ovf));
    CK(hipFree(osum));
    CK(hipFree(ocnt));
    CK(hipStreamDestroy(st[0]));
    CK(hipStreamDestroy(st[1]));
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? std::atoll(argv[1]) : 1000000000ll;
    const int64_t dim = argc > 2 ? std::atoll(argv[2]) : 10000000ll;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 3;
    const int64_t rows = n / 8192 * 8192;
    int64_t *x, *k, *v;
    uint16_t *t;
    double *osum;
    unsigned long long *ocnt;
    CK(hipMalloc(&x, rows * 8));
    CK(hipMalloc(&k, rows * 8));
    CK(hipMalloc(&v, rows * 8));
    CK(hipMalloc(&t, dim * 2 + 64));
    CK(hipMalloc(&osum, G * 8));
    CK(hipMalloc(&ocnt, G * 8));
    hipLaunchKernelGGL(k_gen, dim3(8192), dim3(256), 0, 0, x, k, (double *)v, rows, dim);
    hipLaunchKernelGGL(k_gen_table, dim3(4096), dim3(256), 0, 0, t, dim);
    CK(hipMemset(osum, 0, G * 8));
    CK(hipMemset(ocnt, 0, G * 8));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipLaunchKernelGGL(k_ref, dim3(cus * 8), dim3(256), 0, 0, x, k, v, t, rows, osum, ocnt);
    CK(hipDeviceSynchronize());
    std::vector<double> rsum(G);
    std::vector<unsigned long long> rcnt(G);
    CK(hipMemcpy(rsum.data(), osum, G * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rcnt.data(), ocnt, G * 8, hipMemcpyDeviceToHost));
    std::printf("rows=%lld dim=%lld cus=%d\n", (long long)rows, (long long)dim, cus);
    const int64_t chunks[] = {(int64_t)rows, (int64_t)64 << 20, (int64_t)32 << 20, (int64_t)16 << 20, (int64_t)8 << 20};
    for (int64_t ch : chunks)
        for (int streams : {1, 2}) {
            if (ch >= rows && streams == 2) continue;
            run_chunked<15, 1024, 512>(x, k, v, t, rows, dim, cus, reps, ch, 2, streams, rsum, rcnt);
        }
    run_chunked<15, 1024, 512>(x, k, v, t, rows, dim, cus, reps, (int64_t)16 << 20, 4, 2, rsum, rcnt);
    run_chunked<16, 1024, 1024>(x, k, v, t, rows, dim, cus, reps, (int64_t)16 << 20, 2, 2, rsum, rcnt);
    std::printf("done\n");
    return 0;
}
