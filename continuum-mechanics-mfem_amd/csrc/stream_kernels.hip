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

hipError_t launch_stream(cdfem_ctx *c, int mode, const double *a, double *b, int64_t n)
{
    const dim3 grid(256 * 16), block(256);
    switch (mode) {
    case 0: hipLaunchKernelGGL(k_stream_read<16>, grid, block, 0, c->stream, a, n, b); break;
    case 1: hipLaunchKernelGGL(k_stream_read<8>, grid, block, 0, c->stream, a, n, b); break;
    case 2: hipLaunchKernelGGL(k_stream_copy, grid, block, 0, c->stream, a, b, n); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace cdfem
