// Prototype 6 (tile / block / chunk-size sweep of prototype 3) of the LDS-slice partitioned probe (filter -> join -> group-by):
//   phase A: stream (x, k, v), filter, rank rows by table slice (key >> 16) in
//   LDS, stage the tile sorted by slice, and write every slice's items to the
//   workgroup's region for that slice only in whole, aligned 32-item chunks
//   (keys u16: 64 B, values: 256 B); the < 32 left over per slice are carried
//   in LDS to the next tile, so HBM sees whole-sector writes.
//   phase B: one workgroup per CU loads a 64 Ki-entry u16 table slice (128 KB)
//   into LDS and drains that slice's regions with LDS lookups + LDS states.
// Checked against a single-pass reference kernel.  Dev tool only.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
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

typedef long long v2i64 __attribute__((ext_vector_type(2)));
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
constexpr int G = 1024;
constexpr int SHIFT = 16, S = 1 << SHIFT;
constexpr int kMaxF = 160;

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
// Workgroup barrier that orders LDS only: global loads stay in flight (a
// plain __syncthreads() also drains vmcnt, which would wait for the prefetch).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ v2i64 ld2(const int64_t *p) { return __builtin_nontemporal_load((const v2i64 *)p); }

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
template <int BLOCK, bool EARLY, bool NTX = true, int R = 8, int CH = 32>
__global__ __launch_bounds__(BLOCK) void k_pa3(const int64_t *__restrict__ x, const int64_t *__restrict__ k,
                                               const int64_t *__restrict__ v, int64_t n_tiles, int64_t dim, int F,
                                               uint64_t cap, uint16_t *__restrict__ keyo, int64_t *__restrict__ vo,
                                               uint32_t *__restrict__ cnt_out, uint32_t *__restrict__ overflow) {
    constexpr int TILE = BLOCK * R, P = R / 2;
    constexpr int kMaxChunks = TILE / CH + kMaxF;
    __shared__ uint32_t cnt[kMaxF], lofs[kMaxF], cn[kMaxF], pos[kMaxF], mpre[kMaxF];
    __shared__ uint32_t s_M;
    __shared__ uint16_t chunk_b[kMaxChunks];
    __shared__ uint16_t st_key[TILE];
    __shared__ int64_t st_v[TILE];
    __shared__ uint16_t c_key[kMaxF * CH];
    __shared__ int64_t c_v[kMaxF * CH];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < kMaxF; i += BLOCK) cnt[i] = 0, cn[i] = 0, pos[i] = 0;
    lds_barrier();
    int64_t tile = blockIdx.x;
    v2i64 kk[P], xx[P], vv[P];
    auto load = [&](int64_t t) {
        const int64_t base = t * TILE + (int64_t)wave * (64 * R) + 2 * lane;
#pragma unroll
        for (int j = 0; j < P; ++j) kk[j] = ld2(k + base + j * 128);
#pragma unroll
        for (int j = 0; j < P; ++j) xx[j] = ld2(x + base + j * 128);
#pragma unroll
        for (int j = 0; j < P; ++j) vv[j] = ld2(v + base + j * 128);
    };
    if (tile < n_tiles) load(tile);
    const uint64_t region0 = (uint64_t)blockIdx.x * F;
    bool ovf = false;
    for (; tile < n_tiles; tile += gridDim.x) {
        uint32_t sel = 0, key32[R], rk[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int64_t key = kk[r >> 1][r & 1];
            key32[r] = 0;
            rk[r] = 0;
            if (xx[r >> 1][r & 1] > 49 && key >= 0 && key < dim) {
                sel |= 1u << r;
                key32[r] = (uint32_t)key;
                rk[r] = atomicAdd(&cnt[(uint32_t)key >> SHIFT], 1u);
            }
        }
        v2i64 vcur[P];
#pragma unroll
        for (int j = 0; j < P; ++j) vcur[j] = vv[j];
        if (EARLY && tile + gridDim.x < n_tiles) load(tile + gridDim.x);
        lds_barrier();  // (1) counts complete
        if (wave == 0) {
            // three consecutive slices per lane: exclusive scans of n (staging
            // offsets) and m (whole chunks this tile)
            uint32_t n3[3], m3[3], ns = 0, ms = 0;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const int b = lane * 3 + q;
                n3[q] = b < F ? cnt[b] : 0u;
                m3[q] = b < F ? (cn[b] + n3[q]) / CH : 0u;
                ns += n3[q];
                ms += m3[q];
            }
            uint32_t ni = ns, mi = ms;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t a = __shfl_up(ni, d, 64), c = __shfl_up(mi, d, 64);
                if (lane >= d) ni += a, mi += c;
            }
            uint32_t no = ni - ns, mo = mi - ms;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const int b = lane * 3 + q;
                if (b < kMaxF) lofs[b] = no, mpre[b] = mo;
                no += n3[q];
                mo += m3[q];
            }
            if (lane == 63) s_M = mi;
        }
        lds_barrier();  // (2) offsets ready
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (!((sel >> r) & 1)) continue;
            const uint32_t b = key32[r] >> SHIFT;
            const uint32_t s = lofs[b] + rk[r];
            st_key[s] = (uint16_t)(key32[r] & (S - 1));
            st_v[s] = vcur[r >> 1][r & 1];
        }
        if (tid < F) {
            const uint32_t m = (cn[tid] + cnt[tid]) / CH, m0 = mpre[tid];
            for (uint32_t j = 0; j < m; ++j) chunk_b[m0 + j] = (uint16_t)tid;
        }
        if (!EARLY && tile + gridDim.x < n_tiles) load(tile + gridDim.x);
        lds_barrier();  // (3) staged
        {
            const uint32_t M = s_M;
            const int h = tid >> 5, kx0 = tid & 31;
            for (uint32_t c = h; c < M; c += BLOCK / 32) {
                const uint32_t b = chunk_b[c];
                const uint32_t j = c - mpre[b];
                const uint32_t kx = j * CH + kx0, cb = cn[b];
                uint16_t kv;
                int64_t vvv;
                if (kx < cb) {
                    kv = c_key[b * CH + kx];
                    vvv = c_v[b * CH + kx];
                } else {
                    kv = st_key[lofs[b] + kx - cb];
                    vvv = st_v[lofs[b] + kx - cb];
                }
                const uint64_t dst = (uint64_t)pos[b] + kx;
                if (dst < cap) {
                    const uint64_t o = (region0 + b) * cap + dst;
                    keyo[o] = kv;
                    if (NTX) __builtin_nontemporal_store(vvv, vo + o);
                    else vo[o] = vvv;
                } else {
                    ovf = true;
                }
            }
        }
        lds_barrier();  // (4) flushed: carries may be overwritten
        for (int p = tid; p < F * CH; p += BLOCK) {
            const int b = p / CH, kx = p % CH;
            const uint32_t cb = cn[b], nb = cnt[b], T = cb + nb, L = T % CH;
            if (T < CH) {
                if (kx >= (int)cb && kx < (int)T) {
                    c_key[b * CH + kx] = st_key[lofs[b] + kx - cb];
                    c_v[b * CH + kx] = st_v[lofs[b] + kx - cb];
                }
            } else if (kx < (int)L) {
                c_key[b * CH + kx] = st_key[lofs[b] + nb - L + kx];
                c_v[b * CH + kx] = st_v[lofs[b] + nb - L + kx];
            }
        }
        lds_barrier();  // (5) carries updated
        if (tid < F) {
            const uint32_t T = cn[tid] + cnt[tid];
            pos[tid] += (T / CH) * CH;
            cn[tid] = T % CH;
            cnt[tid] = 0;
        }
        lds_barrier();  // (6)
    }
    // final partial chunks
    for (int p = tid; p < F * CH; p += BLOCK) {
        const int b = p / CH, kx = p % CH;
        if (kx < (int)cn[b]) {
            const uint64_t dst = (uint64_t)pos[b] + kx;
            if (dst < cap) {
                const uint64_t o = (region0 + b) * cap + dst;
                keyo[o] = c_key[b * CH + kx];
                vo[o] = c_v[b * CH + kx];
            } else {
                ovf = true;
            }
        }
    }
    if (ovf) *overflow = 1u;
    for (int b = tid; b < F; b += BLOCK) {
        const uint64_t n = (uint64_t)pos[b] + cn[b];
        cnt_out[region0 + b] = (uint32_t)(n < cap ? n : cap);
    }
}

// ---- phase B ----
template <int BLOCK, bool NTX = true>
__global__ __launch_bounds__(BLOCK) void k_pb3(const uint16_t *__restrict__ table, int64_t dim, int F, int nreg, int splits,
                                               uint64_t cap, const uint16_t *__restrict__ keyo,
                                               const int64_t *__restrict__ vo, const uint32_t *__restrict__ cnt_in,
                                               double *__restrict__ osum, unsigned long long *__restrict__ ocnt) {
    __shared__ double s_sum[G];
    __shared__ uint32_t s_cnt[G];
    __shared__ __attribute__((aligned(16))) uint16_t tslice[S];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int W = BLOCK / 64;
    for (int i = tid; i < G; i += BLOCK) s_sum[i] = 0, s_cnt[i] = 0;
    int cur_b = -1;
    const int units = F * splits;
    for (int u = blockIdx.x; u < units; u += gridDim.x) {
        const int b = u / splits, sp = u % splits;
        if (b != cur_b) {
            __syncthreads();
            const int64_t k0 = (int64_t)b * S;
            const int64_t nk = dim - k0 < S ? dim - k0 : S;
            for (int i = tid * 8; i < S; i += BLOCK * 8) {
                v4u32 w = {0, 0, 0, 0};
                if (i + 8 <= nk) {
                    w = *(const v4u32 *)(table + k0 + i);
                } else {
                    for (int q = 0; q < 8; ++q)
                        if (i + q < nk) w[q >> 1] |= (uint32_t)table[k0 + i + q] << ((q & 1) * 16);
                }
                *(v4u32 *)&tslice[i] = w;
            }
            cur_b = b;
            __syncthreads();
        }
        const int r0 = (int)((int64_t)sp * nreg / splits), r1 = (int)((int64_t)(sp + 1) * nreg / splits);
        for (int r = r0 + wave; r < r1; r += W) {
            const uint64_t reg = (uint64_t)r * F + b;
            const uint32_t n_r = cnt_in[reg];
            const uint16_t *kp = keyo + reg * cap;
            const int64_t *vp = vo + reg * cap;
            for (uint32_t i0 = 0; i0 < n_r; i0 += 64 * 8) {
                uint32_t kk8[8];
                int64_t vv8[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t i = i0 + j * 64 + lane;
                    const uint32_t ii = i < n_r ? i : 0;
                    if (NTX) {
                        kk8[j] = __builtin_nontemporal_load(kp + ii);
                        vv8[j] = __builtin_nontemporal_load(vp + ii);
                    } else {
                        kk8[j] = kp[ii];
                        vv8[j] = vp[ii];
                    }
                }
                uint32_t e8[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) e8[j] = (i0 + j * 64 + lane < n_r) ? (uint32_t)tslice[kk8[j]] : 0u;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (!e8[j]) continue;
                    atomicAdd(&s_sum[e8[j] - 1], __builtin_bit_cast(double, vv8[j]));
                    atomicAdd(&s_cnt[e8[j] - 1], 1u);
                }
            }
        }
    }
    __syncthreads();
    for (int i = tid; i < G; i += BLOCK) {
        unsafeAtomicAdd(&osum[i], s_sum[i]);
        atomicAdd(&ocnt[i], (unsigned long long)s_cnt[i]);
    }
}

template <typename Fn>
static float time_it(Fn f, int reps) {
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
    constexpr int BA = 1024, BB = 1024, TILE = BA * 8;
    const int64_t rows = n / TILE * TILE;
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
    std::vector<double> rsum(G), s(G);
    std::vector<unsigned long long> rcnt(G), c(G);
    CK(hipMemcpy(rsum.data(), osum, G * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rcnt.data(), ocnt, G * 8, hipMemcpyDeviceToHost));
    const int F = (int)((dim + S - 1) >> SHIFT);
    if (F > kMaxF) {
        std::printf("dim too large\n");
        return 1;
    }
    const int gridA = cus;
    const int64_t n_tiles = rows / TILE;
    const uint64_t nreg = (uint64_t)gridA * F;
    const double avg = (double)rows / 2 / nreg;
    uint64_t cap = (uint64_t)(avg * 1.25 + 256);
    cap = (cap + 31) / 32 * 32;
    uint16_t *keyo;
    int64_t *vo;
    uint32_t *cnt, *ovf;
    CK(hipMalloc(&keyo, nreg * cap * 2 + 64));
    CK(hipMalloc(&vo, nreg * cap * 8 + 64));
    CK(hipMalloc(&cnt, nreg * 4));
    CK(hipMalloc(&ovf, 4));
    CK(hipMemset(ovf, 0, 4));
    std::printf("rows=%lld dim=%lld cus=%d F=%d cap=%llu\n", (long long)rows, (long long)dim, cus, F,
                (unsigned long long)cap);
    auto runA = [&](auto kern, int block, int tile, int per_cu, const char *name) {
        const int gA = cus * per_cu;
        const int64_t nt = rows / tile;
        const uint64_t nreg2 = (uint64_t)gA * F;
        uint64_t cp = (uint64_t)((double)(nt + gA - 1) / gA * tile / 2 / F * 1.25) + 256;
        cp = (cp + 31) / 32 * 32;
        if (nreg2 * cp > nreg * cap) cp = (nreg * cap / nreg2) / 32 * 32;
        auto A = [&] { hipLaunchKernelGGL(kern, dim3(gA), dim3(block), 0, 0, x, k, v, nt, dim, F, cp, keyo, vo, cnt, ovf); };
        auto B = [&] { hipLaunchKernelGGL((k_pb3<BB>), dim3(cus), dim3(BB), 0, 0, t, dim, F, gA, 3, cp, keyo, vo, cnt, osum, ocnt); };
        const float ta = time_it(A, reps);
        const float tab = time_it([&] { A(); B(); }, reps);
        CK(hipMemset(osum, 0, G * 8));
        CK(hipMemset(ocnt, 0, G * 8));
        CK(hipMemset(ovf, 0, 4));
        A();
        B();
        CK(hipDeviceSynchronize());
        uint32_t of = 0;
        CK(hipMemcpy(s.data(), osum, G * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(c.data(), ocnt, G * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&of, ovf, 4, hipMemcpyDeviceToHost));
        double maxrel = 0;
        bool ok = true;
        for (int g = 0; g < G; ++g) {
            ok &= c[g] == rcnt[g];
            maxrel = std::fmax(maxrel, std::fabs(s[g] - rsum[g]) / std::fabs(rsum[g]));
        }
        std::printf("%-40s | A %.3f ms  A+B %.3f ms = %.1f%% of 8 TB/s | counts %s maxrel %.2e overflow %u\n", name, ta, tab,
                    24.0 * rows / tab / 1e6 / 80, ok ? "ok" : "BAD", maxrel, of);
        std::fflush(stdout);
    };
    runA(k_pa3<1024, true, true, 8, 32>, 1024, 8192, 1, "1024 thr, 8192-row tile, CH 32 (current)");
    runA(k_pa3<1024, true, true, 4, 64>, 1024, 4096, 1, "1024 thr, 4096-row tile, CH 64");
    runA(k_pa3<1024, true, true, 2, 64>, 1024, 2048, 1, "1024 thr, 2048-row tile, CH 64");
    runA(k_pa3<512, true, true, 8, 64>, 512, 4096, 1, "512 thr, 4096-row tile, CH 64");
    runA(k_pa3<1024, true, true, 4, 32>, 1024, 4096, 1, "1024 thr, 4096-row tile, CH 32");
    std::printf("done\n");
    return 0;
}
