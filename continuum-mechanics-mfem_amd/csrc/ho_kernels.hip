// ho_kernels.hip — high-order (3D p = 3, 4) partial-assembly apply: ONE WAVEFRONT PER ELEMENT.
//
// BASELINE config C3 (128^3 hex, H1 order 4: D1 = 5 dofs and Q1 = 6 Gauss points per direction,
// 125 dofs and 216 points per element).  Thread-per-element (pa_kernels.hip) would need ~700 live
// doubles per thread, so here the 64 lanes of a wave share one element and every sum-factorisation
// stage spreads its outputs over the lanes, with the intermediates in LDS:
//   gather     X[dz][dy][dx]                       (125, from the element-major map)
//   stage x    BX, GX  [dz][dy][qx]                (2 x 150)
//   stage y    BB, BG, GB [dz][qy][qx]             (3 x 180)
//   stage z    u, ux, uy, uz at (qz,qy,qx) and, in the same lane, the quadrature-point operator
//              v0 = C.grad u + M u,  (vx,vy,vz) = D grad u   with the lane's qdata prefetched into
//              registers at kernel entry (10 x 4 coalesced 512-byte loads per lane in flight while
//              the gather and the first stages run)
//   stage z^T  W0, Wx, Wy [dz][qy][qx]             (3 x 180)
//   stage y^T  ZB, ZG [dz][dy][qx]                 (2 x 150)
//   stage x^T  Y[dz][dy][dx] -> E-vector (element-major, coalesced), summed by k_e2l.
// qdata layout (element-major, cdfem_ctx::qlay = 1): qd[(e * NC + c) * NQ + q], so a component of
// 64 consecutive points is one 512-byte wave load.  LDS: (4 NQ + 3 D1 Q1^2) doubles per wave
// (11.2 KB at p = 4), 4 waves (elements) per 256-thread block.
//
// MFMA is not used: on gfx950 the f64 MFMA rate equals the f64 vector FMA rate
// (MI355X_MICROARCH.md), and these contractions (6x5 by 5xN) fill at most 6/16 x 5/8 of a
// 16x16x4 f64 tile, so the VALU path is the faster one; the kernel is bounded by the qdata stream
// (HBM): 8 * 10 * 216 bytes per element against ~38 kflop.
#include <hip/hip_runtime.h>

#include "cdfem_internal.hpp"
#include "pa_core.hpp"

namespace cdfem {

template <int D1, int Q1, unsigned K, bool CON>
__global__ void __launch_bounds__(256)
k_apply3d_wpe(const int32_t *__restrict__ map, const double *__restrict__ x, const double *__restrict__ qd,
              double *__restrict__ Ye, const Tab<D1, Q1> T, const int ne, const KrylovState *__restrict__ st)
{
    if (st != nullptr && st->done) return;
    using L = QLayout<K, 3>;
    constexpr int ND = D1 * D1 * D1, NQ = Q1 * Q1 * Q1, NC = L::nc;
    constexpr int S1 = D1 * D1 * Q1;  // stage x / y^T outputs per field
    constexpr int S2 = D1 * Q1 * Q1;  // stage y / z^T outputs per field
    constexpr int NA = 4 * NQ, NB = 3 * S2;
    static_assert(NB >= ND && NA >= 2 * S1, "LDS buffer sizes");
    constexpr int QI = (NQ + 63) / 64;
    __shared__ double sB[Q1 * D1], sG[Q1 * D1];
    __shared__ double bufA[4][NA];
    __shared__ double bufB[4][NB];

    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int e = blockIdx.x * 4 + w;
    const bool valid = e < ne;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int q = 0; q < Q1; ++q)
#pragma unroll
            for (int d = 0; d < D1; ++d) {
                sB[q * D1 + d] = T.B[q][d];
                sG[q * D1 + d] = T.G[q][d];
            }
    }
    double *A = bufA[w], *Bf = bufB[w];

    // qdata of this lane's points, in flight from here on
    double qv[QI][NC];
#pragma unroll
    for (int i = 0; i < QI; ++i) {
        const int q = lane + 64 * i;
#pragma unroll
        for (int c = 0; c < NC; ++c)
            qv[i][c] = (valid && q < NQ) ? qd[((size_t)e * NC + c) * NQ + q] : 0.0;  // (non-temporal measured 3 % slower)
    }
    // gather
    if (valid) {
        for (int l = lane; l < ND; l += 64) {
            const int g = map[(size_t)e * ND + l];
            double v;
            if constexpr (CON) v = g < 0 ? 0.0 : x[g];
            else v = x[g < 0 ? -g - 1 : g];
            Bf[l] = v;
        }
    }
    __syncthreads();
    // stage x
    for (int o = lane; o < S1; o += 64) {
        const int qx = o % Q1, r = o / Q1;
        double bx = 0.0, gx = 0.0;
#pragma unroll
        for (int dx = 0; dx < D1; ++dx) {
            const double xv = Bf[r * D1 + dx];
            bx += sB[qx * D1 + dx] * xv;
            gx += sG[qx * D1 + dx] * xv;
        }
        A[o] = bx;
        A[S1 + o] = gx;
    }
    __syncthreads();
    // stage y
    for (int o = lane; o < S2; o += 64) {
        const int qx = o % Q1, qy = (o / Q1) % Q1, dz = o / (Q1 * Q1);
        double bb = 0.0, bg = 0.0, gb = 0.0;
#pragma unroll
        for (int dy = 0; dy < D1; ++dy) {
            const int i = (dz * D1 + dy) * Q1 + qx;
            const double bxv = A[i], gxv = A[S1 + i];
            const double by = sB[qy * D1 + dy], gy = sG[qy * D1 + dy];
            bb += by * bxv;
            bg += by * gxv;
            gb += gy * bxv;
        }
        Bf[o] = bb;
        Bf[S2 + o] = bg;
        Bf[2 * S2 + o] = gb;
    }
    __syncthreads();
    // stage z + quadrature-point operator (lane owns points lane + 64 i, as in the prefetch)
#pragma unroll
    for (int i = 0; i < QI; ++i) {
        const int o = lane + 64 * i;
        if (o < NQ) {
            const int qxy = o % (Q1 * Q1), qz = o / (Q1 * Q1);
            double u = 0.0, ux = 0.0, uy = 0.0, uz = 0.0;
#pragma unroll
            for (int dz = 0; dz < D1; ++dz) {
                const int j = dz * Q1 * Q1 + qxy;
                const double bz = sB[qz * D1 + dz], gz = sG[qz * D1 + dz];
                const double bb = Bf[j];
                u += bz * bb;
                uz += gz * bb;
                ux += bz * Bf[S2 + j];
                uy += bz * Bf[2 * S2 + j];
            }
            double v0 = 0.0, vx = 0.0, vy = 0.0, vz = 0.0;
            if constexpr (L::kD) {
                const double d00 = qv[i][0], d01 = qv[i][1], d02 = qv[i][2];
                const double d11 = qv[i][3], d12 = qv[i][4], d22 = qv[i][5];
                vx = d00 * ux + d01 * uy + d02 * uz;
                vy = d01 * ux + d11 * uy + d12 * uz;
                vz = d02 * ux + d12 * uy + d22 * uz;
            }
            if constexpr (L::kC) v0 += qv[i][L::oC] * ux + qv[i][L::oC + 1] * uy + qv[i][L::oC + 2] * uz;
            if constexpr (L::kM) v0 += qv[i][L::oM] * u;
            A[o] = v0;
            A[NQ + o] = vx;
            A[2 * NQ + o] = vy;
            A[3 * NQ + o] = vz;
        }
    }
    __syncthreads();
    // stage z^T
    for (int o = lane; o < S2; o += 64) {
        const int qxy = o % (Q1 * Q1), dz = o / (Q1 * Q1);
        double w0 = 0.0, wx = 0.0, wy = 0.0;
#pragma unroll
        for (int qz = 0; qz < Q1; ++qz) {
            const int j = qz * Q1 * Q1 + qxy;
            const double bz = sB[qz * D1 + dz], gz = sG[qz * D1 + dz];
            w0 += bz * A[j] + gz * A[3 * NQ + j];
            wx += bz * A[NQ + j];
            wy += bz * A[2 * NQ + j];
        }
        Bf[o] = w0;
        Bf[S2 + o] = wx;
        Bf[2 * S2 + o] = wy;
    }
    __syncthreads();
    // stage y^T
    for (int o = lane; o < S1; o += 64) {
        const int qx = o % Q1, dy = (o / Q1) % D1, dz = o / (Q1 * D1);
        double zb = 0.0, zg = 0.0;
#pragma unroll
        for (int qy = 0; qy < Q1; ++qy) {
            const int j = (dz * Q1 + qy) * Q1 + qx;
            const double by = sB[qy * D1 + dy], gy = sG[qy * D1 + dy];
            zb += by * Bf[j] + gy * Bf[2 * S2 + j];
            zg += by * Bf[S2 + j];
        }
        A[o] = zb;
        A[S1 + o] = zg;
    }
    __syncthreads();
    // stage x^T -> E-vector
    if (valid) {
        for (int o = lane; o < ND; o += 64) {
            const int dx = o % D1, r = o / D1;
            double y = 0.0;
#pragma unroll
            for (int qx = 0; qx < Q1; ++qx) {
                const int j = r * Q1 + qx;
                y += sB[qx * D1 + dx] * A[j] + sG[qx * D1 + dx] * A[S1 + j];
            }
            Ye[(size_t)e * ND + o] = y;
        }
    }
}

template <int D1, int Q1, unsigned K>
static hipError_t wpe_kinds(cdfem_ctx *c, const double *x, double *Ye, bool con, const KrylovState *st)
{
    const Tab<D1, Q1> T = make_tab<D1, Q1>(c->rule_op);
    const dim3 grid((unsigned)((c->ne + 3) / 4)), block(256);
    if (con)
        hipLaunchKernelGGL((k_apply3d_wpe<D1, Q1, K, true>), grid, block, 0, c->stream, c->d_map, x, c->d_qd, Ye, T,
                           c->ne, st);
    else
        hipLaunchKernelGGL((k_apply3d_wpe<D1, Q1, K, false>), grid, block, 0, c->stream, c->d_map, x, c->d_qd, Ye,
                           T, c->ne, st);
    return hipGetLastError();
}

template <int D1, int Q1>
static hipError_t wpe_dq(cdfem_ctx *c, const double *x, double *Ye, bool con, const KrylovState *st)
{
    switch (c->kinds) {
    case 1: return wpe_kinds<D1, Q1, 1>(c, x, Ye, con, st);
    case 2: return wpe_kinds<D1, Q1, 2>(c, x, Ye, con, st);
    case 3: return wpe_kinds<D1, Q1, 3>(c, x, Ye, con, st);
    case 4: return wpe_kinds<D1, Q1, 4>(c, x, Ye, con, st);
    case 5: return wpe_kinds<D1, Q1, 5>(c, x, Ye, con, st);
    case 6: return wpe_kinds<D1, Q1, 6>(c, x, Ye, con, st);
    case 7: return wpe_kinds<D1, Q1, 7>(c, x, Ye, con, st);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_apply_wpe(cdfem_ctx *c, const double *x, double *Ye, bool con, const KrylovState *st)
{
    const int q1 = c->rule_op.q1;
    if (c->p == 3 && q1 == 5) return wpe_dq<4, 5>(c, x, Ye, con, st);
    if (c->p == 4 && q1 == 6) return wpe_dq<5, 6>(c, x, Ye, con, st);
    return hipErrorInvalidValue;
}

}  // namespace cdfem
