// Counter-based synthetic columns (BASELINE.md §2 "Data"): identical on the
// host (oracle/qe_oracle.c qo_generate) and the device, so parity tests and the
// CPU baseline see exactly the rows the GPU processes without shipping files.
#include "device_common.h"
#include "ops.h"

namespace qeh {

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <int KIND>
__global__ void k_generate(uint64_t seed, uint64_t col_id, int64_t row0, int64_t n, int64_t modulus, int64_t lo,
                           void *out) {
    const uint64_t base = seed ^ (col_id << 56);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t row = (uint64_t)(row0 + i);
        if (KIND == QEH_GEN_UNIFORM_MOD) {
            ((int64_t *)out)[i] = (int64_t)(splitmix64(base + row) % (uint64_t)modulus) + lo;
        } else if (KIND == QEH_GEN_UNIT_F64) {
            ((double *)out)[i] = (double)(splitmix64(base + row) >> 11) * 0x1.0p-53;
        } else if (KIND == QEH_GEN_SPARSE_KEY) {
            const uint64_t x = modulus > 0 ? splitmix64(base + row) % (uint64_t)modulus : row;
            ((int64_t *)out)[i] = (int64_t)splitmix64(x ^ (seed * 0xD6E8FEB86659FD93ull));
        } else {
            ((int64_t *)out)[i] = (int64_t)((row * 0x9E3779B1ull + col_id) % (uint64_t)modulus) + lo;
        }
    }
}

}  // namespace qeh

using namespace qeh;

extern "C" int qeh_generate(qeh_ctx *ctx, int kind, uint64_t seed, uint64_t col_id, int64_t row0, int64_t n,
                            int64_t modulus, int64_t lo, void *out_values) {
    if (!ctx || (n > 0 && !out_values)) return fail(QEH_E_INVALID, "qeh_generate: bad argument");
    if (n <= 0) return QEH_OK;
    if ((kind == QEH_GEN_UNIFORM_MOD || kind == QEH_GEN_PERMUTATION) && modulus <= 0)
        return fail(QEH_E_INVALID, "qeh_generate: modulus must be positive");
    if (kind == QEH_GEN_SPARSE_KEY && modulus < 0)
        return fail(QEH_E_INVALID, "qeh_generate: modulus must be positive");
    DeviceGuard dg(ctx->device);
    const int grid = grid_for(ctx, n, kBlock * 8, 8);
    KernelTimer kt(ctx, "generate");
    switch (kind) {
        case QEH_GEN_UNIFORM_MOD:
            hipLaunchKernelGGL(k_generate<QEH_GEN_UNIFORM_MOD>, dim3(grid), dim3(kBlock), 0, ctx->stream, seed, col_id, row0, n,
                               modulus, lo, out_values);
            break;
        case QEH_GEN_UNIT_F64:
            hipLaunchKernelGGL(k_generate<QEH_GEN_UNIT_F64>, dim3(grid), dim3(kBlock), 0, ctx->stream, seed, col_id, row0, n,
                               modulus, lo, out_values);
            break;
        case QEH_GEN_SPARSE_KEY:
            hipLaunchKernelGGL(k_generate<QEH_GEN_SPARSE_KEY>, dim3(grid), dim3(kBlock), 0, ctx->stream, seed, col_id, row0,
                               n, modulus, lo, out_values);
            break;
        case QEH_GEN_PERMUTATION:
            hipLaunchKernelGGL(k_generate<QEH_GEN_PERMUTATION>, dim3(grid), dim3(kBlock), 0, ctx->stream, seed, col_id, row0,
                               n, modulus, lo, out_values);
            break;
        default: return fail(QEH_E_INVALID, "qeh_generate: unknown kind");
    }
    QEH_HIP(hipGetLastError());
    return QEH_OK;
}
