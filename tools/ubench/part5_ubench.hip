// Prototype 5: pipelined owner-computes exchange with whole-chunk writes.
// As prototype 4, but each workgroup carries < 16 items per owner in LDS and
// writes only whole 16-item chunks (128 B of values + 32 B of keys) into the
// per-(chunk, producer, owner) regions; carries survive across chunks and are
// flushed once at the end.  2048-row tiles keep the LDS within 160 KB.
// One persistent 1024-thread workgroup per CU.  Workgroup w owns table slice w
// (range / grid keys, u16 entries resident in LDS for the whole kernel) and
// its aggregate states.  The fact table is processed in chunks; for chunk c a
// workgroup
//   A(c):   streams its tiles, filters, and appends each selected row's
//           (slice-local key, v) to region [c % 2][w][owner] (staged in LDS
//           so every owner's run is written contiguously),
//           then publishes (vmcnt(0), barrier, agent release, counter add);
//   B(c-1): waits until every workgroup published chunk c-1 and drains the
//           regions [(c-1) % 2][*][w] addressed to it: LDS lookups + LDS states.
// A(c+2) reuses buffer c % 2 only after every owner finished B(c).  Chunks are
// small enough (tens of MB of exchange) to stay in L2 / Infinity Cache, so the
// exchange costs little HBM traffic.  Dev tool only.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
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
constexpr int G = 1024;
constexpr int BLOCK = 1024, R = 2, TILE = BLOCK * R;  // 2048 rows per tile
constexpr int CH = 16;                                // items per written chunk
constexpr int MAXO = 256;                             // owners (= grid)
constexpr int MAXS = 40960;                           // keys per slice (u16 entries in LDS)

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

__device__ __forceinline__ v2i64 ld2(const int64_t *p) { return __builtin_nontemporal_load((const v2i64 *)p); }
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct Pipe {
    uint16_t *key;               // [2][grid][grid][cap]
    int64_t *val;                // [2][grid][grid][cap]
    uint32_t *count;             // [2][grid][grid]
    unsigned long long *prod;    // published A chunks (all workgroups)
    unsigned long long *cons;    // finished B chunks
    uint32_t *flag;              // bit 0 overflow, bit 1 spin timeout
    uint64_t cap;
    int64_t kmin;
    uint32_t range, S;           // keys per slice
    float invS;
};

__device__ bool spin_until(unsigned long long *ctr, unsigned long long want, uint32_t *flag) {
    for (uint32_t it = 0; it < (1u << 24); ++it) {
        if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) return true;
        __builtin_amdgcn_s_sleep(2);
    }
    atomicOr(flag, 2u);
    return false;
}

template <int TW, int BMODE>
__global__ __launch_bounds__(BLOCK) void k_pipe(const int64_t *__restrict__ x, const int64_t *__restrict__ k,
                                                const int64_t *__restrict__ v, const uint16_t *__restrict__ table,
                                                int n_chunks, Pipe p, double *osum, unsigned long long *ocnt) {
    __shared__ __attribute__((aligned(16))) uint16_t tslice[MAXS];
    __shared__ double s_sum[G];
    __shared__ uint32_t s_cnt[G];
    __shared__ uint16_t st_key[TILE];
    __shared__ int64_t st_v[TILE];
    __shared__ uint16_t c_key[MAXO * CH];
    __shared__ int64_t c_v[MAXO * CH];
    __shared__ uint32_t cnt[MAXO], lofs[MAXO], cur[MAXO], cn[MAXO], mpre[MAXO];
    __shared__ uint16_t chunk_own[TILE / CH + MAXO];
    __shared__ uint32_t s_chunks;
    __shared__ int s_abort;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int W = gridDim.x, w = blockIdx.x;
    const uint64_t cap = p.cap;
    for (int i = tid; i < G; i += BLOCK) s_sum[i] = 0, s_cnt[i] = 0;
    for (int i = tid; i < MAXO; i += BLOCK) cnt[i] = 0, cur[i] = 0, cn[i] = 0;
    if (tid == 0) s_abort = 0;
    {  // my slice: keys [w*S, min((w+1)*S, range))
        const uint32_t k0 = (uint32_t)w * p.S;
        const uint32_t nk = k0 < p.range ? std::min(p.S, p.range - k0) : 0u;
        for (uint32_t i = tid; i < p.S; i += BLOCK) tslice[i] = i < nk ? table[k0 + i] : (uint16_t)0;
    }
    __syncthreads();
    bool ovf = false;
    v2i64 kk[1], xx[1], vv[1];
    auto tile_of = [&](int c, int i) -> int64_t { return ((int64_t)c * TW + i) * W + w; };
    auto issue = [&](int64_t t) {
        const int64_t base = t * TILE + (int64_t)wave * (64 * R) + 2 * lane;
        kk[0] = ld2(k + base);
        xx[0] = ld2(x + base);
        vv[0] = ld2(v + base);
    };
    auto drain = [&](int c) {  // B(c): regions [c%2][*][w]
        if (tid == 0) {
            if (!spin_until(p.prod, (unsigned long long)W * (c + 1), p.flag)) s_abort = 1;
            if (BMODE == 0) __threadfence();  // acquire: invalidates this XCD's L2 view of the exchange
        }
        __syncthreads();
        if (s_abort) return;
        const int b = c & 1;
        for (int q = wave; q < W; q += BLOCK / 64) {
            const uint64_t reg = ((uint64_t)b * W + q) * W + w;
            const uint32_t n_r = p.count[reg];
            const uint16_t *kp = p.key + reg * cap;
            const int64_t *vp = p.val + reg * cap;
            for (uint32_t i0 = 0; i0 < n_r; i0 += 64 * 4) {
                uint32_t e[4];
                int64_t vx[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t i = i0 + j * 64 + lane;
                    const uint32_t ii = i < n_r ? i : 0u;
                    e[j] = kp[ii];
                    vx[j] = vp[ii];
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) e[j] = (i0 + j * 64 + lane < n_r) ? (uint32_t)tslice[e[j]] : 0u;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (!e[j]) continue;
                    atomicAdd(&s_sum[e[j] - 1], __builtin_bit_cast(double, vx[j]));
                    atomicAdd(&s_cnt[e[j] - 1], 1u);
                }
            }
        }
        __syncthreads();
        if (tid == 0) atomicAdd(p.cons, 1ull);
    };
    for (int c = 0; c < n_chunks; ++c) {
        const int b = c & 1;
        if (BMODE != 1 && BMODE != 3 && c >= 2) {  // buffer b was last read by B(c-2): wait for every owner
            if (tid == 0 && !spin_until(p.cons, (unsigned long long)W * (c - 1), p.flag)) s_abort = 1;
            __syncthreads();
            if (s_abort) break;
        }
        issue(tile_of(c, 0));
        for (int i = 0; i < TW; ++i) {
            uint32_t sel = 0, off[R], own[R], rk[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint64_t o = (uint64_t)kk[r >> 1][r & 1] - (uint64_t)p.kmin;
                own[r] = 0;
                off[r] = 0;
                rk[r] = 0;
                if (xx[r >> 1][r & 1] > 49 && o < p.range) {
                    uint32_t ow = (uint32_t)((float)o * p.invS);
                    if (ow * p.S > (uint32_t)o) --ow;
                    else if ((ow + 1) * p.S <= (uint32_t)o) ++ow;
                    own[r] = ow;
                    off[r] = (uint32_t)o - ow * p.S;
                    sel |= 1u << r;
                    rk[r] = atomicAdd(&cnt[ow], 1u);
                }
            }
            int64_t vc[R];
#pragma unroll
            for (int r = 0; r < R; ++r) vc[r] = vv[r >> 1][r & 1];
            if (i + 1 < TW) issue(tile_of(c, i + 1));
            lds_barrier();  // counts complete
            if (wave == 0) {  // four owners per lane: staging offsets and whole chunks per owner
                uint32_t n4[4], m4[4], ns = 0, ms = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int o = lane * 4 + q;
                    n4[q] = cnt[o];
                    m4[q] = (cn[o] + n4[q]) / CH;
                    ns += n4[q];
                    ms += m4[q];
                }
                uint32_t ni = ns, mi = ms;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t a = __shfl_up(ni, d, 64), cc = __shfl_up(mi, d, 64);
                    if (lane >= d) ni += a, mi += cc;
                }
                uint32_t no = ni - ns, mo = mi - ms;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int o = lane * 4 + q;
                    lofs[o] = no;
                    mpre[o] = mo;
                    no += n4[q];
                    mo += m4[q];
                }
                if (lane == 63) s_chunks = mi;
            }
            lds_barrier();
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (!((sel >> r) & 1)) continue;
                const uint32_t s = lofs[own[r]] + rk[r];
                st_key[s] = (uint16_t)off[r];
                st_v[s] = vc[r];
            }
            if (tid < MAXO) {
                const uint32_t m = (cn[tid] + cnt[tid]) / CH, m0 = mpre[tid];
                for (uint32_t q = 0; q < m; ++q) chunk_own[m0 + q] = (uint16_t)tid;
            }
            lds_barrier();  // staged
            {
                const uint32_t M = s_chunks;
                const uint32_t kx0 = tid & (CH - 1);
                for (uint32_t cc = tid / CH; cc < M; cc += BLOCK / CH) {
                    const uint32_t o = chunk_own[cc];
                    const uint32_t kx = (cc - mpre[o]) * CH + kx0, cb = cn[o];
                    uint16_t kv;
                    int64_t vx;
                    if (kx < cb) {
                        kv = c_key[o * CH + kx];
                        vx = c_v[o * CH + kx];
                    } else {
                        kv = st_key[lofs[o] + kx - cb];
                        vx = st_v[lofs[o] + kx - cb];
                    }
                    const uint64_t dst = (uint64_t)cur[o] + kx;
                    if (BMODE == 3) continue;
                    if (dst < cap) {
                        const uint64_t idx = (((uint64_t)b * W + w) * W + o) * cap + dst;
                        p.key[idx] = kv;
                        p.val[idx] = vx;
                    } else {
                        ovf = true;
                    }
                }
            }
            lds_barrier();  // flushed
            for (int q = tid; q < MAXO * CH; q += BLOCK) {
                const int o = q / CH, kx = q % CH;
                const uint32_t cb = cn[o], nb = cnt[o], T = cb + nb, L = T % CH;
                int src = -1;
                if (T < CH) {
                    if (kx >= (int)cb && kx < (int)T) src = (int)(lofs[o] + kx - cb);
                } else if (kx < (int)L) {
                    src = (int)(lofs[o] + nb - L + kx);
                }
                if (src >= 0) {
                    c_key[o * CH + kx] = st_key[src];
                    c_v[o * CH + kx] = st_v[src];
                }
            }
            lds_barrier();  // carries updated
            if (tid < MAXO) {
                const uint32_t T = cn[tid] + cnt[tid];
                cur[tid] += (T / CH) * CH;
                cn[tid] = T % CH;
                cnt[tid] = 0;
            }
            lds_barrier();
        }
        if (c == n_chunks - 1) {  // last chunk: the carried items go out as partial chunks
            for (int q = tid; q < MAXO * CH; q += BLOCK) {
                const int o = q / CH, kx = q % CH;
                if (kx >= (int)cn[o]) continue;
                const uint64_t dst = (uint64_t)cur[o] + kx;
                if (dst < cap) {
                    const uint64_t idx = (((uint64_t)b * W + w) * W + o) * cap + dst;
                    p.key[idx] = c_key[o * CH + kx];
                    p.val[idx] = c_v[o * CH + kx];
                } else {
                    ovf = true;
                }
            }
            __syncthreads();
            if (tid < MAXO) cur[tid] += cn[tid], cn[tid] = 0;
            __syncthreads();
        }
        if (tid < W) {
            p.count[((uint64_t)b * W + w) * W + tid] = cur[tid] < cap ? cur[tid] : (uint32_t)cap;
            cur[tid] = 0;
        }
        // publish A(c): every wave's stores done, then one agent-scope release + counter add
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (tid == 0) {
            if (BMODE == 0) __threadfence();
            atomicAdd(p.prod, 1ull);
        }
        if (BMODE != 1 && BMODE != 3 && c >= 1) drain(c - 1);
        if (s_abort) break;
    }
    if (BMODE != 1 && BMODE != 3 && !s_abort && n_chunks >= 1) drain(n_chunks - 1);
    if (ovf) atomicOr(p.flag, 1u);
    __syncthreads();
    for (int i = tid; i < G; i += BLOCK) {
        unsafeAtomicAdd(&osum[i], s_sum[i]);
        atomicAdd(&ocnt[i], (unsigned long long)s_cnt[i]);
    }
}

template <int TW, int BMODE = 0>
static void run(const int64_t *x, const int64_t *k, const int64_t *v, const uint16_t *t, int64_t rows, int64_t dim, int cus,
                int reps, const std::vector<double> &rsum, const std::vector<unsigned long long> &rcnt) {
    const int W = cus;
    const int64_t chunk_rows = (int64_t)W * TW * TILE;
    const int n_chunks = (int)(rows / chunk_rows);
    const int64_t used = (int64_t)n_chunks * chunk_rows;
    Pipe p{};
    p.S = (uint32_t)((dim + W - 1) / W);
    if (p.S > (uint32_t)MAXS) {
        std::printf("slice too large\n");
        return;
    }
    p.range = (uint32_t)dim;
    p.kmin = 0;
    p.invS = 1.0f / (float)p.S;
    p.cap = ((uint64_t)((double)TW * TILE / W * 1.25) + 64 + CH - 1) / CH * CH;
    const uint64_t nreg = 2ull * W * W;
    CK(hipMalloc(&p.key, nreg * p.cap * 2 + 64));
    CK(hipMalloc(&p.val, nreg * p.cap * 8 + 64));
    CK(hipMalloc(&p.count, nreg * 4));
    CK(hipMalloc(&p.prod, 64));
    CK(hipMalloc(&p.cons, 64));
    CK(hipMalloc(&p.flag, 64));
    double *osum;
    unsigned long long *ocnt;
    CK(hipMalloc(&osum, G * 8));
    CK(hipMalloc(&ocnt, G * 8));
    auto launch = [&] {
        CK(hipMemsetAsync(p.prod, 0, 8, 0));
        CK(hipMemsetAsync(p.cons, 0, 8, 0));
        hipLaunchKernelGGL((k_pipe<TW, BMODE>), dim3(W), dim3(BLOCK), 0, 0, x, k, v, t, n_chunks, p, osum, ocnt);
    };
    CK(hipMemset(p.flag, 0, 4));
    launch();
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    CK(hipMemset(osum, 0, G * 8));
    CK(hipMemset(ocnt, 0, G * 8));
    CK(hipMemset(p.flag, 0, 4));
    launch();
    CK(hipDeviceSynchronize());
    std::vector<double> s(G);
    std::vector<unsigned long long> c(G);
    uint32_t fl = 0;
    CK(hipMemcpy(s.data(), osum, G * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(c.data(), ocnt, G * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&fl, p.flag, 4, hipMemcpyDeviceToHost));
    double maxrel = 0;
    bool ok = used == rows;
    for (int g = 0; g < G; ++g) {
        ok &= c[g] == rcnt[g];
        maxrel = std::fmax(maxrel, std::fabs(s[g] - rsum[g]) / std::fabs(rsum[g]));
    }
    std::printf("BMODE=%d TW=%d chunk=%lld rows (%d chunks) cap=%llu | %.3f ms = %.1f GB/s alg (%.1f%% of 8 TB/s) | counts %s maxrel "
                "%.2e flag %u\n",
                BMODE, TW, (long long)chunk_rows, n_chunks, (unsigned long long)p.cap, ms, 24.0 * used / ms / 1e6,
                24.0 * used / ms / 1e6 / 80, ok ? "ok" : "BAD", maxrel, fl);
    std::fflush(stdout);
    CK(hipFree(p.key));
    CK(hipFree(p.val));
    CK(hipFree(p.count));
    CK(hipFree(p.prod));
    CK(hipFree(p.cons));
    CK(hipFree(p.flag));
    CK(hipFree(osum));
    CK(hipFree(ocnt));
}

int main(int argc, char **argv) {
    const int64_t dim = argc > 2 ? std::atoll(argv[2]) : 10000000ll;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 5;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    // a row count every chunk size divides: cus * 32 * 4096 * m
    const int64_t unit = (int64_t)cus * 128 * TILE;
    const int64_t want = argc > 1 ? std::atoll(argv[1]) : 1000000000ll;
    const int64_t rows = std::max<int64_t>(1, want / unit) * unit;
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
    hipLaunchKernelGGL(k_ref, dim3(cus * 8), dim3(256), 0, 0, x, k, v, t, rows, osum, ocnt);
    CK(hipDeviceSynchronize());
    std::vector<double> rsum(G);
    std::vector<unsigned long long> rcnt(G);
    CK(hipMemcpy(rsum.data(), osum, G * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rcnt.data(), ocnt, G * 8, hipMemcpyDeviceToHost));
    std::printf("rows=%lld dim=%lld cus=%d\n", (long long)rows, (long long)dim, cus);
    run<64, 0>(x, k, v, t, rows, dim, cus, reps, rsum, rcnt);
    run<64, 1>(x, k, v, t, rows, dim, cus, reps, rsum, rcnt);
    run<64, 3>(x, k, v, t, rows, dim, cus, reps, rsum, rcnt);
    run<32, 0>(x, k, v, t, rows, dim, cus, reps, rsum, rcnt);
    run<128, 0>(x, k, v, t, rows, dim, cus, reps, rsum, rcnt);
    std::printf("done\n");
    return 0;
}
