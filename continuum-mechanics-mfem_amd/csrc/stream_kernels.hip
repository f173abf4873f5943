// stream_kernels.hip — HBM bandwidth probes measured on the box (report the roofline
// against the nominal 8 TB/s AND a STREAM-type rate measured on the same GPU).
#include <hip/hip_runtime.h>

#include "cdfem_internal.hpp"

namespace cdfem {

// read-only sweep, W-byte accesses per lane, grid-stride; the sum is written so nothing is DCE'd
template <int W>
__global__ void __launch_bounds__(256) k_stream_read(const double *__restrict__ a, int64_t n, double *out)
{
    double s = 0.0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    if constexpr (W == 16) {
        const double2 *a2 = reinterpret_cast<const double2 *>(a);
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 2; i += stride) {
            const double2 v = a2[i];
            s += v.x + v.y;
        }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) s += a[i];
    }
    if (s == 12345.678) out[0] = s;
}

__global__ void __launch_bounds__(256) k_stream_copy(const double *__restrict__ a, double *__restrict__ b,
                                                      int64_t n)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const double2 *a2 = reinterpret_cast<const double2 *>(a);
    double2 *b2 = reinterpret_cast<double2 *>(b);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 2; i += stride) b2[i] = a2[i];
}

// Per-wave private chunks (the brick kernel's qdata pattern): one 64-lane block streams its own
// contiguous kChunk bytes with 16-byte loads, U loads issued back to back.  PAD reserves 39 KB of
// LDS per block so that at most one wave runs per SIMD (the brick kernel's occupancy).
constexpr int64_t kChunkDoubles = 40960;  // 320 KiB
template <int U, bool PAD>
__global__ void __launch_bounds__(64) k_stream_chunk(const double *__restrict__ a, int64_t nchunks, double *out,
                                                     int64_t stride = kChunkDoubles)
{
    __shared__ double pad[PAD ? 4992 : 1];
    if (threadIdx.x == 64) pad[0] = 0.0;  // never true: keeps the allocation
    const int64_t b = blockIdx.x;
    if (b >= nchunks) return;
    const double2 *p = reinterpret_cast<const double2 *>(a + b * stride) + threadIdx.x;
    constexpr int iters = (int)(kChunkDoubles / 128);
    double s = 0.0;
    for (int i = 0; i < iters; i += U) {
        double2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = p[(int64_t)(i + u) * 64];
#pragma unroll
        for (int u = 0; u < U; ++u) s += v[u].x + v[u].y;
    }
    if (s == 12345.678) out[0] = s + pad[0];
}

// Same work per wave, INTERLEAVED layout: the i-th 1 KiB piece of wave b lives at (i * nchunks + b),
// so waves at the same step read adjacent kilobytes (candidate qdata layout [q][brick][...]).
template <int U>
__global__ void __launch_bounds__(64) k_stream_ileave(const double *__restrict__ a, int64_t nchunks, double *out)
{
    __shared__ double pad[4992];
    if (threadIdx.x == 64) pad[0] = 0.0;
    const int64_t b = blockIdx.x;
    if (b >= nchunks) return;
    const double2 *p = reinterpret_cast<const double2 *>(a) + b * 64 + threadIdx.x;
    constexpr int iters = (int)(kChunkDoubles / 128);
    double s = 0.0;
    for (int i = 0; i < iters; i += U) {
        double2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = p[(int64_t)(i + u) * nchunks * 64];
#pragma unroll
        for (int u = 0; u < U; ++u) s += v[u].x + v[u].y;
    }
    if (s == 12345.678) out[0] = s + pad[0];
}

// Workgroup chunks: NW waves of one workgroup stream ONE contiguous chunk of NW x 320 KiB together,
// NW KiB per step (wave w reads the w-th KiB), 81 KiB of LDS per workgroup so one workgroup runs
// per CU (one wave per SIMD at NW = 4): the qdata pattern of a kernel with four waves per brick.
template <int U, int NW>
__global__ void __launch_bounds__(64 * NW) k_stream_wgchunk(const double *__restrict__ a, int64_t nchunks, double *out)
{
    __shared__ double pad[10368];
    if (threadIdx.x == 64 * NW) pad[0] = 0.0;
    const int64_t b = blockIdx.x;
    if (b >= nchunks) return;
    const double2 *p = reinterpret_cast<const double2 *>(a + b * NW * kChunkDoubles) + threadIdx.x;
    constexpr int iters = (int)(kChunkDoubles / 128);
    double s = 0.0;
    for (int i = 0; i < iters; i += U) {
        double2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = p[(int64_t)(i + u) * 64 * NW];
#pragma unroll
        for (int u = 0; u < U; ++u) s += v[u].x + v[u].y;
    }
    if (s == 12345.678) out[0] = s + pad[0];
}

// Grid-stride 16-byte read with 64-thread blocks and 39 KB of LDS each (one wave per SIMD, 1024
// waves): the grid-stride pattern at the brick kernel's occupancy.
__global__ void __launch_bounds__(64) k_stream_read_1wave(const double *__restrict__ a, int64_t n, double *out)
{
    __shared__ double pad[4992];
    if (threadIdx.x == 64) pad[0] = 0.0;
    double s = 0.0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const double2 *a2 = reinterpret_cast<const double2 *>(a);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 2; i += stride) {
        const double2 v = a2[i];
        s += v.x + v.y;
    }
    if (s == 12345.678) out[0] = s + pad[0];
}

// ---- f64 compute-rate probes (VALU vs MFMA for the high-order contractions) ----
// VALU: 8 independent v_fma_f64 chains per lane.  MFMA: 4 independent v_mfma_f64_16x16x4_f64
// accumulators per wave (16 x 16 x 4 x 2 = 2048 flop per instruction).  ITERS loop trips; the
// results are written under an impossible condition so nothing is dead-code eliminated.
constexpr int kFp64Iters = 4096;
__global__ void __launch_bounds__(256) k_fp64_valu(double seed, double *out)
{
    double a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = seed + threadIdx.x + k;
    const double m = 1.0 + 1e-9 * seed, c = 1e-12;
    for (int i = 0; i < kFp64Iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = fma(a[k], m, c);
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += a[k];
    if (s == 12345.678) out[0] = s;
}

typedef double v4d_t __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) k_fp64_mfma(double seed, double *out)
{
    const double a = seed + (threadIdx.x & 63), b = 1.0 + 1e-9 * seed;
    v4d_t acc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = v4d_t{0.0, 0.0, 0.0, (double)k};
    for (int i = 0; i < kFp64Iters; ++i) {
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    if (s == 12345.678) out[0] = s;
}

// Mixed probe (the MFMA-vs-VALU question of the brick kernels): every wave interleaves
// 4 v_mfma_f64_16x16x4_f64 chains with NV independent v_fma_f64 chains per lane in one loop.  If the
// matrix core and the VALU run concurrently, the rate approaches the sum of the two single-pipe rates;
// if they share one f64 pipe, it stays at the single rate.
template <int NV>
__global__ void __launch_bounds__(256) k_fp64_mixed(double seed, double *out)
{
    const double a = seed + (threadIdx.x & 63), b = 1.0 + 1e-9 * seed;
    v4d_t acc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = v4d_t{0.0, 0.0, 0.0, (double)k};
    double v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = seed + threadIdx.x + k;
    const double m = 1.0 + 1e-9 * seed, c = 1e-12;
    for (int i = 0; i < kFp64Iters; ++i) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
#pragma unroll
            for (int j = k; j < NV; j += 4) v[j] = fma(v[j], m, c);
        }
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
#pragma unroll
    for (int k = 0; k < NV; ++k) s += v[k];
    if (s == 12345.678) out[0] = s;
}

hipError_t launch_fp64_probe(cdfem_ctx *c, int mode, double *out, double *flops)
{
    const dim3 grid(256 * 8), block(256);
    const double waves = (double)grid.x * (block.x / 64);
    if (mode == 0) {
        hipLaunchKernelGGL(k_fp64_valu, grid, block, 0, c->stream, 1.0, out);
        *flops = waves * 64.0 * 8.0 * 2.0 * kFp64Iters;
    } else if (mode == 1) {
        hipLaunchKernelGGL(k_fp64_mfma, grid, block, 0, c->stream, 1.0, out);
        *flops = waves * 4.0 * 2048.0 * kFp64Iters;
    } else if (mode == 2 || mode == 3 || mode == 4) {  // mixed: 16 / 32 / 64 VALU FMAs per 4 MFMAs
        const int nv = mode == 2 ? 16 : mode == 3 ? 32 : 64;
        if (mode == 2) hipLaunchKernelGGL(k_fp64_mixed<16>, grid, block, 0, c->stream, 1.0, out);
        if (mode == 3) hipLaunchKernelGGL(k_fp64_mixed<32>, grid, block, 0, c->stream, 1.0, out);
        if (mode == 4) hipLaunchKernelGGL(k_fp64_mixed<64>, grid, block, 0, c->stream, 1.0, out);
        *flops = waves * (4.0 * 2048.0 + 64.0 * 2.0 * nv) * kFp64Iters;
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_stream(cdfem_ctx *c, int mode, const double *a, double *b, int64_t n)
{
    const dim3 grid(256 * 16), block(256);
    const int64_t nch = n / kChunkDoubles;
    switch (mode) {
    case 3: hipLaunchKernelGGL((k_stream_chunk<8, true>), dim3(nch), dim3(64), 0, c->stream, a, nch, b); break;
    case 4: hipLaunchKernelGGL((k_stream_chunk<16, true>), dim3(nch), dim3(64), 0, c->stream, a, nch, b); break;
    case 5: hipLaunchKernelGGL((k_stream_chunk<8, false>), dim3(nch), dim3(64), 0, c->stream, a, nch, b); break;
    case 6: hipLaunchKernelGGL((k_stream_chunk<4, true>), dim3(nch), dim3(64), 0, c->stream, a, nch, b); break;
    case 7: hipLaunchKernelGGL((k_stream_chunk<32, true>), dim3(nch), dim3(64), 0, c->stream, a, nch, b); break;
    case 8: hipLaunchKernelGGL((k_stream_ileave<8>), dim3(nch), dim3(64), 0, c->stream, a, nch, b); break;
    case 10: case 11: case 12: case 13: {  // chunk U8, one wave per SIMD, chunks skewed by 256 B..4 KiB
        const int64_t skew[4] = {32, 64, 128, 512};
        const int64_t st = kChunkDoubles + skew[mode - 10], nc2 = n / st;
        hipLaunchKernelGGL((k_stream_chunk<8, true>), dim3(nc2), dim3(64), 0, c->stream, a, nc2, b, st);
        break;
    }
    case 9: hipLaunchKernelGGL((k_stream_ileave<4>), dim3(nch), dim3(64), 0, c->stream, a, nch, b); break;
    case 14: hipLaunchKernelGGL((k_stream_wgchunk<8, 4>), dim3(nch / 4), dim3(256), 0, c->stream, a, nch / 4, b); break;
    case 15: hipLaunchKernelGGL((k_stream_wgchunk<8, 2>), dim3(nch / 2), dim3(128), 0, c->stream, a, nch / 2, b); break;
    case 16: hipLaunchKernelGGL(k_stream_read_1wave, dim3(1024), dim3(64), 0, c->stream, a, n, b); break;
    case 17: hipLaunchKernelGGL(k_stream_read_1wave, dim3(4096), dim3(64), 0, c->stream, a, n, b); break;
    case 0: hipLaunchKernelGGL(k_stream_read<16>, grid, block, 0, c->stream, a, n, b); break;
    case 1: hipLaunchKernelGGL(k_stream_read<8>, grid, block, 0, c->stream, a, n, b); break;
    case 2: hipLaunchKernelGGL(k_stream_copy, grid, block, 0, c->stream, a, b, n); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace cdfem
