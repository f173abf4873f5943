// pa_core.hpp — the per-element fused D + C + M partial-assembly apply (device code), shared by
// the generic element-block kernels (pa_kernels.hip) and the structured brick kernels
// (brick_kernels.hip).  One thread owns one element; sum factorization in registers.
#pragma once
#include <hip/hip_runtime.h>

#include "cdfem_internal.hpp"

namespace cdfem {

template <int D1, int Q1>
struct Tab {
    double B[Q1][D1];
    double G[Q1][D1];
};

template <int D1, int Q1>
static Tab<D1, Q1> make_tab(const Rule1D &r)
{
    Tab<D1, Q1> t;
    for (int q = 0; q < Q1; ++q)
        for (int d = 0; d < D1; ++d) {
            t.B[q][d] = r.B[q][d];
            t.G[q][d] = r.G[q][d];
        }
    return t;
}

// qdata component layout for a kinds mask: [D (sym) | C (dim) | M]
template <unsigned K, int DIM>
struct QLayout {
    static constexpr bool kD = (K & CDFEM_DIFFUSION) != 0;
    static constexpr bool kC = (K & CDFEM_CONVECTION) != 0;
    static constexpr bool kM = (K & CDFEM_MASS) != 0;
    static constexpr int nD = kD ? DIM * (DIM + 1) / 2 : 0;
    static constexpr int oC = nD;
    static constexpr int oM = oC + (kC ? DIM : 0);
    static constexpr int nc = oM + (kM ? 1 : 0);
};

// Y = A_e X for one element: X, Y lexicographic [dz][dy][dx]; q0 points at this element's
// qdata for q = 0 (component stride kLanes, point stride NC * kLanes).
template <int D1, int Q1, unsigned K>
__device__ __forceinline__ void elem_apply3d(const double (&X)[D1][D1][D1], const double *__restrict__ q0,
                                             const Tab<D1, Q1> &T, double (&Y)[D1][D1][D1])
{
    using L = QLayout<K, 3>;
    constexpr int NC = L::nc;
#pragma unroll
    for (int dz = 0; dz < D1; ++dz)
#pragma unroll
        for (int dy = 0; dy < D1; ++dy)
#pragma unroll
            for (int dx = 0; dx < D1; ++dx) Y[dz][dy][dx] = 0.0;

#pragma unroll
    for (int qz = 0; qz < Q1; ++qz) {
        // contract z
        double T0[D1][D1], Tz[D1][D1];
#pragma unroll
        for (int dy = 0; dy < D1; ++dy)
#pragma unroll
            for (int dx = 0; dx < D1; ++dx) {
                double s0 = 0.0, s1 = 0.0;
#pragma unroll
                for (int dz = 0; dz < D1; ++dz) {
                    s0 += T.B[qz][dz] * X[dz][dy][dx];
                    s1 += T.G[qz][dz] * X[dz][dy][dx];
                }
                T0[dy][dx] = s0;
                Tz[dy][dx] = s1;
            }
        double RT[D1][D1], RTz[D1][D1];
#pragma unroll
        for (int dy = 0; dy < D1; ++dy)
#pragma unroll
            for (int dx = 0; dx < D1; ++dx) { RT[dy][dx] = 0.0; RTz[dy][dx] = 0.0; }

#pragma unroll
        for (int qy = 0; qy < Q1; ++qy) {
            // contract y
            double a[D1], ay[D1], az[D1];
#pragma unroll
            for (int dx = 0; dx < D1; ++dx) {
                double s0 = 0.0, s1 = 0.0, s2 = 0.0;
#pragma unroll
                for (int dy = 0; dy < D1; ++dy) {
                    s0 += T.B[qy][dy] * T0[dy][dx];
                    s1 += T.G[qy][dy] * T0[dy][dx];
                    s2 += T.B[qy][dy] * Tz[dy][dx];
                }
                a[dx] = s0; ay[dx] = s1; az[dx] = s2;
            }
            double Rv[D1], Ry[D1], Rz[D1];
#pragma unroll
            for (int dx = 0; dx < D1; ++dx) { Rv[dx] = 0.0; Ry[dx] = 0.0; Rz[dx] = 0.0; }

#pragma unroll
            for (int qx = 0; qx < Q1; ++qx) {
                // contract x -> value and reference gradient at the point
                double u = 0.0, ux = 0.0, uy = 0.0, uz = 0.0;
#pragma unroll
                for (int dx = 0; dx < D1; ++dx) {
                    u += T.B[qx][dx] * a[dx];
                    ux += T.G[qx][dx] * a[dx];
                    uy += T.B[qx][dx] * ay[dx];
                    uz += T.B[qx][dx] * az[dx];
                }
                const int q = qx + Q1 * (qy + Q1 * qz);
                const double *qq = q0 + (size_t)q * NC * kLanes;
                double vv = 0.0, gx = 0.0, gy = 0.0, gz = 0.0;
                if constexpr (L::kD) {
                    const double d00 = qq[0 * kLanes], d01 = qq[1 * kLanes], d02 = qq[2 * kLanes];
                    const double d11 = qq[3 * kLanes], d12 = qq[4 * kLanes], d22 = qq[5 * kLanes];
                    gx = d00 * ux + d01 * uy + d02 * uz;
                    gy = d01 * ux + d11 * uy + d12 * uz;
                    gz = d02 * ux + d12 * uy + d22 * uz;
                }
                if constexpr (L::kC) {
                    vv = qq[(L::oC + 0) * kLanes] * ux + qq[(L::oC + 1) * kLanes] * uy +
                         qq[(L::oC + 2) * kLanes] * uz;
                }
                if constexpr (L::kM) vv += qq[L::oM * kLanes] * u;
                // transposed contraction in x
#pragma unroll
                for (int dx = 0; dx < D1; ++dx) {
                    if constexpr (L::kD) {
                        Rv[dx] += T.B[qx][dx] * vv + T.G[qx][dx] * gx;
                        Ry[dx] += T.B[qx][dx] * gy;
                        Rz[dx] += T.B[qx][dx] * gz;
                    } else {
                        Rv[dx] += T.B[qx][dx] * vv;
                    }
                }
            }
            // transposed contraction in y
#pragma unroll
            for (int dy = 0; dy < D1; ++dy)
#pragma unroll
                for (int dx = 0; dx < D1; ++dx) {
                    if constexpr (L::kD) {
                        RT[dy][dx] += T.B[qy][dy] * Rv[dx] + T.G[qy][dy] * Ry[dx];
                        RTz[dy][dx] += T.B[qy][dy] * Rz[dx];
                    } else {
                        RT[dy][dx] += T.B[qy][dy] * Rv[dx];
                    }
                }
        }
        // transposed contraction in z
#pragma unroll
        for (int dz = 0; dz < D1; ++dz)
#pragma unroll
            for (int dy = 0; dy < D1; ++dy)
#pragma unroll
                for (int dx = 0; dx < D1; ++dx) {
                    if constexpr (L::kD)
                        Y[dz][dy][dx] += T.B[qz][dz] * RT[dy][dx] + T.G[qz][dz] * RTz[dy][dx];
                    else
                        Y[dz][dy][dx] += T.B[qz][dz] * RT[dy][dx];
                }
    }

}

}  // namespace cdfem
