// Infinity Cache (MALL) residency under streaming traffic.  Dev tool only.
// Question for the metric's slice pipeline: can an exchange buffer E written by phase A be read
// back by phase B from the 256 MiB Infinity Cache, while phase A streams the fact columns?
//   read E cold (after a 4 GB flush stream)       -> HBM rate
//   read E right after writing it                 -> MALL rate if E fits
//   write E, stream X bytes (plain / nt loads), read E  -> is E still resident?
// Times are per kernel (hipEvents), median of repeats.
#include <hip/hip_runtime.h>

#include <algorithm>
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

typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void k_read(const v4u32 *p, int64_t n16, unsigned *out) {
    v4u32 acc = {0u, 0u, 0u, 0u};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
        v4u32 w = NT ? __builtin_nontemporal_load(p + i) : p[i];
        acc ^= w;
    }
    if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) out[0] = 1;  // keeps the loads
}

template <bool NT>
__global__ __launch_bounds__(256) void k_write(v4u32 *p, int64_t n16, unsigned seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
        v4u32 w = {(unsigned)i, seed, (unsigned)(i >> 32), 7u};
        if (NT) __builtin_nontemporal_store(w, p + i);
        else p[i] = w;
    }
}

static float median(std::vector<float> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char **argv) {
    const int grid = 256 * 8, block = 256;
    const size_t flush_bytes = 4ull << 30;
    char *F, *E;
    unsigned *out;
    CK(hipMalloc(&F, flush_bytes));
    CK(hipMalloc(&E, 256ull << 20));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(F, 1, flush_bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto rd = [&](const char *p, size_t bytes, bool nt) {
        if (nt) hipLaunchKernelGGL(k_read<true>, dim3(grid), dim3(block), 0, 0, (const v4u32 *)p, (int64_t)(bytes / 16), out);
        else hipLaunchKernelGGL(k_read<false>, dim3(grid), dim3(block), 0, 0, (const v4u32 *)p, (int64_t)(bytes / 16), out);
    };
    auto wr = [&](char *p, size_t bytes, bool nt) {
        if (nt) hipLaunchKernelGGL(k_write<true>, dim3(grid), dim3(block), 0, 0, (v4u32 *)p, (int64_t)(bytes / 16), 3u);
        else hipLaunchKernelGGL(k_write<false>, dim3(grid), dim3(block), 0, 0, (v4u32 *)p, (int64_t)(bytes / 16), 3u);
    };
    auto timed = [&](auto fn) {
        CK(hipEventRecord(a, 0));
        fn();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms;
    };
    const int reps = 9;
    std::printf("E_MB,case,stream_MB,read_E_us,GBps\n");
    for (size_t emb : {32, 64, 128, 192}) {
        const size_t eb = emb << 20;
        auto report = [&](const char *name, size_t smb, std::vector<float> &t) {
            const float us = median(t) * 1e3f;
            std::printf("%zu,%s,%zu,%.1f,%.0f\n", emb, name, smb, us, eb / (us * 1e-6) / 1e9);
        };
        {  // cold: flush first
            std::vector<float> t;
            for (int r = 0; r < reps; ++r) {
                rd(F, flush_bytes, false);
                t.push_back(timed([&] { rd(E, eb, false); }));
            }
            report("cold", 4096, t);
        }
        for (bool wnt : {false, true}) {  // right after writing E (plain / nt stores)
            std::vector<float> t;
            for (int r = 0; r < reps; ++r) {
                rd(F, flush_bytes, false);
                wr(E, eb, wnt);
                t.push_back(timed([&] { rd(E, eb, false); }));
            }
            report(wnt ? "after_nt_write" : "after_write", 0, t);
        }
        for (size_t smb : {64, 128, 256, 512, 1024, 2048}) {
            for (bool snt : {false, true}) {
                std::vector<float> t;
                for (int r = 0; r < reps; ++r) {
                    rd(F + (1ull << 30), flush_bytes - (1ull << 30), false);
                    wr(E, eb, false);
                    rd(F, smb << 20, snt);
                    t.push_back(timed([&] { rd(E, eb, false); }));
                }
                report(snt ? "write_ntstream_read" : "write_stream_read", smb, t);
            }
        }
    }
    // streaming rates themselves
    for (bool nt : {false, true}) {
        std::vector<float> t;
        for (int r = 0; r < reps; ++r) t.push_back(timed([&] { rd(F, flush_bytes, nt); }));
        std::printf("stream_read_4GB_%s,%.1f us,%.0f GB/s\n", nt ? "nt" : "plain", median(t) * 1e3f,
                    flush_bytes / (median(t) * 1e-3) / 1e9);
    }
    return 0;
}
