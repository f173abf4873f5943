// pa_kernels.hip — partial-assembly kernels for H1 tensor elements on gfx950.
//
// Replaces MFEM's DiffusionIntegrator / ConvectionIntegrator / MassIntegrator AssemblePA +
// AddMultPA (called from a.Assemble() and Operator::Mult in linear_convection_diffusion_2D.cpp:
// 335-339, 364-370) with ONE fused operator: per quadrature point
//     v     = M u + C . grad_ref(u)            (mass + convection, test with phi)
//     vgrad = D grad_ref(u)                    (diffusion, test with grad phi)
// where D = W kappa adj(J)adj(J)^T/detJ, C = W alpha adj(J) c, M = W s detJ (qdata, HBM-resident).
//
// Apply kernel mapping (MI355X-first): one THREAD per element, one wavefront per
// 64-element block.  The 1D contractions (sum factorization, x/y/z) run in registers with
// compile-time-unrolled loops, so there is no LDS traffic, no barrier, and every qdata load of a
// wavefront is 512 contiguous bytes.  The element loop is a pure stream over qdata (10 doubles
// per quadrature point at p=2 = 94% of the bytes), which is what bounds the kernel (HBM roofline).
#include <hip/hip_runtime.h>

#include "cdfem_internal.hpp"
#include "pa_core.hpp"

namespace cdfem {

// ------------------------------------------------------------------------------------------------
// 3D apply: Ye = A_e x_e for every element (thread per element)
// ------------------------------------------------------------------------------------------------
template <int D1, int Q1, unsigned K, bool CON>
__global__ void __launch_bounds__(256)
k_apply3d(const int32_t *__restrict__ map, const double *__restrict__ x,
          const double *__restrict__ qd, double *__restrict__ Ye, const Tab<D1, Q1> T,
          const int nblk, const KrylovState *__restrict__ st)
{
    if (st != nullptr && st->done) return;
    using L = QLayout<K, 3>;
    constexpr int ND = D1 * D1 * D1;
    constexpr int NQ = Q1 * Q1 * Q1;
    constexpr int NC = L::nc;
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (b >= nblk) return;

    // L->E gather (fused): 64 lanes read 256 contiguous bytes of map per local dof
    const int32_t *mp = map + (size_t)b * ND * kLanes + lane;
    double X[D1][D1][D1];
#pragma unroll
    for (int dz = 0; dz < D1; ++dz)
#pragma unroll
        for (int dy = 0; dy < D1; ++dy)
#pragma unroll
            for (int dx = 0; dx < D1; ++dx) {
                const int g = mp[(dx + D1 * (dy + D1 * dz)) * kLanes];
                if constexpr (CON) {
                    const double v = x[g < 0 ? 0 : g];
                    X[dz][dy][dx] = g < 0 ? 0.0 : v;
                } else {
                    X[dz][dy][dx] = x[g < 0 ? -g - 1 : g];
                }
            }

    double Y[D1][D1][D1];
    const double *q0 = qd + (size_t)b * NQ * NC * kLanes;
    elem_apply3d<D1, Q1, K>([&](int dz, int dy, int dx) { return X[dz][dy][dx]; }, q0, lane, T, Y);

    double *yp = Ye + (size_t)b * ND * kLanes + lane;
#pragma unroll
    for (int dz = 0; dz < D1; ++dz)
#pragma unroll
        for (int dy = 0; dy < D1; ++dy)
#pragma unroll
            for (int dx = 0; dx < D1; ++dx) yp[(dx + D1 * (dy + D1 * dz)) * kLanes] = Y[dz][dy][dx];
}

// ------------------------------------------------------------------------------------------------
// 2D apply (quads), same mapping
// ------------------------------------------------------------------------------------------------
template <int D1, int Q1, unsigned K, bool CON>
__global__ void __launch_bounds__(256)
k_apply2d(const int32_t *__restrict__ map, const double *__restrict__ x,
          const double *__restrict__ qd, double *__restrict__ Ye, const Tab<D1, Q1> T,
          const int nblk, const KrylovState *__restrict__ st)
{
    if (st != nullptr && st->done) return;
    using L = QLayout<K, 2>;
    constexpr int ND = D1 * D1;
    constexpr int NQ = Q1 * Q1;
    constexpr int NC = L::nc;
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (b >= nblk) return;

    const int32_t *mp = map + (size_t)b * ND * kLanes + lane;
    double X[D1][D1];
#pragma unroll
    for (int dy = 0; dy < D1; ++dy)
#pragma unroll
        for (int dx = 0; dx < D1; ++dx) {
            const int g = mp[(dx + D1 * dy) * kLanes];
            if constexpr (CON) {
                const double v = x[g < 0 ? 0 : g];
                X[dy][dx] = g < 0 ? 0.0 : v;
            } else {
                X[dy][dx] = x[g < 0 ? -g - 1 : g];
            }
        }
    double Y[D1][D1];
#pragma unroll
    for (int dy = 0; dy < D1; ++dy)
#pragma unroll
        for (int dx = 0; dx < D1; ++dx) Y[dy][dx] = 0.0;

    const double *q0 = qd + (size_t)b * NQ * NC * kLanes;
#pragma unroll
    for (int qy = 0; qy < Q1; ++qy) {
        double a[D1], ay[D1];
#pragma unroll
        for (int dx = 0; dx < D1; ++dx) {
            double s0 = 0.0, s1 = 0.0;
#pragma unroll
            for (int dy = 0; dy < D1; ++dy) {
                s0 += T.B[qy][dy] * X[dy][dx];
                s1 += T.G[qy][dy] * X[dy][dx];
            }
            a[dx] = s0; ay[dx] = s1;
        }
        double Rv[D1], Ry[D1];
#pragma unroll
        for (int dx = 0; dx < D1; ++dx) { Rv[dx] = 0.0; Ry[dx] = 0.0; }
#pragma unroll
        for (int qx = 0; qx < Q1; ++qx) {
            double u = 0.0, ux = 0.0, uy = 0.0;
#pragma unroll
            for (int dx = 0; dx < D1; ++dx) {
                u += T.B[qx][dx] * a[dx];
                ux += T.G[qx][dx] * a[dx];
                uy += T.B[qx][dx] * ay[dx];
            }
            const int q = qx + Q1 * qy;
            double qv[NC];
            load_qp<NC, true>(q0 + (size_t)q * NC * kLanes, lane, qv);
            double vv = 0.0, gx = 0.0, gy = 0.0;
            if constexpr (L::kD) {
                gx = qv[0] * ux + qv[1] * uy;
                gy = qv[1] * ux + qv[2] * uy;
            }
            if constexpr (L::kC) vv = qv[L::oC] * ux + qv[L::oC + 1] * uy;
            if constexpr (L::kM) vv += qv[L::oM] * u;
#pragma unroll
            for (int dx = 0; dx < D1; ++dx) {
                if constexpr (L::kD) {
                    Rv[dx] += T.B[qx][dx] * vv + T.G[qx][dx] * gx;
                    Ry[dx] += T.B[qx][dx] * gy;
                } else {
                    Rv[dx] += T.B[qx][dx] * vv;
                }
            }
        }
#pragma unroll
        for (int dy = 0; dy < D1; ++dy)
#pragma unroll
            for (int dx = 0; dx < D1; ++dx) {
                if constexpr (L::kD)
                    Y[dy][dx] += T.B[qy][dy] * Rv[dx] + T.G[qy][dy] * Ry[dx];
                else
                    Y[dy][dx] += T.B[qy][dy] * Rv[dx];
            }
    }
    double *yp = Ye + (size_t)b * ND * kLanes + lane;
#pragma unroll
    for (int dy = 0; dy < D1; ++dy)
#pragma unroll
        for (int dx = 0; dx < D1; ++dx) yp[(dx + D1 * dy) * kLanes] = Y[dy][dx];
}

// ------------------------------------------------------------------------------------------------
// geometry helpers (multilinear map, lexicographic vertices)
// ------------------------------------------------------------------------------------------------
template <int DIM>
__device__ inline void q1_map(const double *__restrict__ V, const double xi[3], double x[3],
                              double J[3][3])
{
    constexpr int NV = 1 << DIM;
    for (int i = 0; i < DIM; ++i) {
        x[i] = 0.0;
        for (int k = 0; k < DIM; ++k) J[i][k] = 0.0;
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        double f[3], df[3];
#pragma unroll
        for (int k = 0; k < DIM; ++k) {
            const int bit = (v >> k) & 1;
            f[k] = bit ? xi[k] : 1.0 - xi[k];
            df[k] = bit ? 1.0 : -1.0;
        }
        double N = 1.0;
#pragma unroll
        for (int k = 0; k < DIM; ++k) N *= f[k];
#pragma unroll
        for (int k = 0; k < DIM; ++k) {
            double dN = df[k];
#pragma unroll
            for (int m = 0; m < DIM; ++m)
                if (m != k) dN *= f[m];
#pragma unroll
            for (int i = 0; i < DIM; ++i) J[i][k] += V[v * DIM + i] * dN;
        }
#pragma unroll
        for (int i = 0; i < DIM; ++i) x[i] += V[v * DIM + i] * N;
    }
}

template <int DIM>
__device__ inline double adjugate(const double J[3][3], double A[3][3])
{
    if constexpr (DIM == 2) {
        A[0][0] = J[1][1]; A[0][1] = -J[0][1];
        A[1][0] = -J[1][0]; A[1][1] = J[0][0];
        return J[0][0] * J[1][1] - J[0][1] * J[1][0];
    } else {
        A[0][0] = J[1][1] * J[2][2] - J[1][2] * J[2][1];
        A[0][1] = J[0][2] * J[2][1] - J[0][1] * J[2][2];
        A[0][2] = J[0][1] * J[1][2] - J[0][2] * J[1][1];
        A[1][0] = J[1][2] * J[2][0] - J[1][0] * J[2][2];
        A[1][1] = J[0][0] * J[2][2] - J[0][2] * J[2][0];
        A[1][2] = J[0][2] * J[1][0] - J[0][0] * J[1][2];
        A[2][0] = J[1][0] * J[2][1] - J[1][1] * J[2][0];
        A[2][1] = J[0][1] * J[2][0] - J[0][0] * J[2][1];
        A[2][2] = J[0][0] * J[1][1] - J[0][1] * J[1][0];
        return J[0][0] * A[0][0] + J[0][1] * A[1][0] + J[0][2] * A[2][0];
    }
}

__device__ inline void qpoint(int q, int q1, int dim, const Rule1D &r, double xi[3], double &W)
{
    const int qx = q % q1, qy = (q / q1) % q1, qz = q / (q1 * q1);
    xi[0] = r.pts[qx];
    xi[1] = r.pts[qy];
    xi[2] = dim == 3 ? r.pts[qz] : 0.0;
    W = r.wts[qx] * r.wts[qy] * (dim == 3 ? r.wts[qz] : 1.0);
}

// qdata setup: thread per (element-block, q, lane); coalesced writes of the [b][q][c][lane] layout
template <int DIM>
__global__ void __launch_bounds__(256)
k_setup_qdata(const double *__restrict__ verts, const int32_t *__restrict__ perm, int ne, int nblk, int qlay,
              const Rule1D r, unsigned kinds,
              int nc, double kappa, const double *__restrict__ kappa_q, const double *__restrict__ kmat_q,
              double alpha, double c0, double c1, double c2, const double *__restrict__ conv_q, double mass,
              const double *__restrict__ mass_q, double *__restrict__ qd)
{
    const int q1 = r.q1;
    const int nq = DIM == 3 ? q1 * q1 * q1 : q1 * q1;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)nblk * nq * kLanes) return;
    const int lane = (int)(t % kLanes);
    const int q = (int)((t / kLanes) % nq);
    const int b = (int)(t / ((int64_t)kLanes * nq));
    const int e = perm[(size_t)b * kLanes + lane];
    double *out = qd + ((size_t)b * nq + q) * nc * kLanes;
    // component k of this point: block layout (qd_offset) or element-major [e][k][q]
    auto put = [&](int k, double v) {
        if (qlay == 1) qd[qd_ho_index(e, k, q, nc, q1)] = v;
        else out[qd_offset(k, lane, nc)] = v;
    };
    if (e < 0 || e >= ne) {
        if (qlay == 0)
            for (int k = 0; k < nc; ++k) out[qd_offset(k, lane, nc)] = 0.0;
        return;
    }
    double xi[3], W;
    qpoint(q, q1, DIM, r, xi, W);
    double x[3], J[3][3], A[3][3];
    q1_map<DIM>(verts + (size_t)e * (1 << DIM) * DIM, xi, x, J);
    const double det = adjugate<DIM>(J, A);
    const size_t eq = (size_t)e * nq + q;
    int o = 0;
    if (kinds & CDFEM_DIFFUSION) {
        const double kap = kappa_q ? kappa_q[eq] : kappa;
        if (kmat_q) {  // MatrixCoefficient: D = W adj(J) K adj(J)^T / det J, K = kap I + K_q (symmetric)
            constexpr int NS = DIM * (DIM + 1) / 2;
            double K[3][3];
            for (int k = 0, m = 0; k < DIM; ++k)
                for (int l = k; l < DIM; ++l, ++m) K[k][l] = K[l][k] = kmat_q[eq * NS + m] + (k == l ? kap : 0.0);
            const double s = W / det;
            for (int i = 0; i < DIM; ++i)
                for (int j = i; j < DIM; ++j) {
                    double acc = 0.0;
                    for (int k = 0; k < DIM; ++k) {
                        double t = 0.0;
                        for (int l = 0; l < DIM; ++l) t += K[k][l] * A[j][l];
                        acc += A[i][k] * t;
                    }
                    put(o++, s * acc);
                }
        } else {
            const double s = W * kap / det;
            for (int i = 0; i < DIM; ++i)
                for (int j = i; j < DIM; ++j) {
                    double acc = 0.0;
                    for (int k = 0; k < DIM; ++k) acc += A[i][k] * A[j][k];
                    put(o++, s * acc);
                }
        }
    }
    if (kinds & CDFEM_CONVECTION) {
        double cv[3] = {c0, c1, c2};
        if (conv_q)
            for (int k = 0; k < DIM; ++k) cv[k] = conv_q[eq * DIM + k];
        for (int i = 0; i < DIM; ++i) {
            double acc = 0.0;
            for (int k = 0; k < DIM; ++k) acc += A[i][k] * cv[k];
            put(o++, W * alpha * acc);
        }
    }
    if ((kinds & CDFEM_MASS) && !(kinds & kMassFromD)) {  // derived from D otherwise (QLayout::kMD)
        const double s = mass_q ? mass_q[eq] : mass;
        put(o++, W * s * det);
    }
}

// physical coordinates of rule points: xyz[(e*nq + q)*dim + k]
template <int DIM>
__global__ void k_quad_points(const double *__restrict__ verts, int ne, const Rule1D r,
                              double *__restrict__ xyz)
{
    const int q1 = r.q1;
    const int nq = DIM == 3 ? q1 * q1 * q1 : q1 * q1;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)ne * nq) return;
    const int e = (int)(t / nq), q = (int)(t % nq);
    double xi[3], W, x[3], J[3][3];
    qpoint(q, q1, DIM, r, xi, W);
    q1_map<DIM>(verts + (size_t)e * (1 << DIM) * DIM, xi, x, J);
    for (int k = 0; k < DIM; ++k) xyz[t * DIM + k] = x[k];
}

// phi_l and reference gradient of local dof l at point q
__device__ inline void basis_at(int l, int q, int dim, const Rule1D &r, double &phi, double g[3])
{
    const int d1 = r.d1, q1 = r.q1;
    const int lx = l % d1, ly = (l / d1) % d1, lz = l / (d1 * d1);
    const int qx = q % q1, qy = (q / q1) % q1, qz = q / (q1 * q1);
    const double bx = r.B[qx][lx], gx = r.G[qx][lx], by = r.B[qy][ly], gy = r.G[qy][ly];
    if (dim == 2) {
        phi = bx * by; g[0] = gx * by; g[1] = bx * gy; g[2] = 0.0;
    } else {
        const double bz = r.B[qz][lz], gz = r.G[qz][lz];
        phi = bx * by * bz; g[0] = gx * by * bz; g[1] = bx * gy * bz; g[2] = bx * by * gz;
    }
}

// PA diagonal, element part: thread per (block, l, lane), Ye layout [b][l][lane]; element-major
// (qlay 1): thread per (e, l), Ye at ho_eidx(e, l)
template <int DIM>
__global__ void __launch_bounds__(256)
k_diag_elem(const double *__restrict__ qd, const int32_t *__restrict__ perm, int ne, int nblk, int nd, int qlay,
            const HoLayout ho, const Rule1D r, unsigned kinds, int nc, double *__restrict__ Ye)
{
    const int q1 = r.q1;
    const int nq = DIM == 3 ? q1 * q1 * q1 : q1 * q1;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)nblk * nd * kLanes) return;
    // element blocks: lane = element; element-major (qlay 1): consecutive threads share an
    // element (l fastest), so every qdata read of a wave is one broadcast address
    const int lane = qlay == 1 ? 0 : (int)(t % kLanes);
    const int l = qlay == 1 ? (int)(t % nd) : (int)((t / kLanes) % nd);
    const int b = qlay == 1 ? 0 : (int)(t / ((int64_t)kLanes * nd));
    const int oC = (kinds & CDFEM_DIFFUSION) ? DIM * (DIM + 1) / 2 : 0;
    const int oM = oC + ((kinds & CDFEM_CONVECTION) ? DIM : 0);
    const int e = qlay == 1 ? (int)(t / nd) : perm[(size_t)b * kLanes + lane];
    if (qlay == 1 && e >= ne) return;
    double acc = 0.0;
    for (int q = 0; q < nq; ++q) {
        const double *qb = qd + ((size_t)b * nq + q) * nc * kLanes;
        auto qq = [&](int k) {
            return qlay == 1 ? qd[qd_ho_index(e, k, q, nc, q1)] : qb[qd_offset(k, lane, nc)];
        };
        double phi, g[3];
        basis_at(l, q, DIM, r, phi, g);
        if (kinds & CDFEM_DIFFUSION) {
            if (DIM == 3) {
                const double d00 = qq(0), d01 = qq(1), d02 = qq(2);
                const double d11 = qq(3), d12 = qq(4), d22 = qq(5);
                acc += g[0] * (d00 * g[0] + d01 * g[1] + d02 * g[2]) +
                       g[1] * (d01 * g[0] + d11 * g[1] + d12 * g[2]) +
                       g[2] * (d02 * g[0] + d12 * g[1] + d22 * g[2]);
            } else {
                const double d00 = qq(0), d01 = qq(1), d11 = qq(2);
                acc += g[0] * (d00 * g[0] + d01 * g[1]) + g[1] * (d01 * g[0] + d11 * g[1]);
            }
        }
        if (kinds & CDFEM_CONVECTION) {
            double cg = 0.0;
            for (int k = 0; k < DIM; ++k) cg += qq(oC + k) * g[k];
            acc += phi * cg;
        }
        if (kinds & CDFEM_MASS) {
            double m;
            if (kinds & kMassFromD) {  // M = s det(D) / (W^2 kappa^3)
                const int qx = q % q1, qy = (q / q1) % q1, qz = q / (q1 * q1);
                const double W = r.wts[qx] * r.wts[qy] * r.wts[qz];
                m = r.mscale * det_sym3(qq(0), qq(1), qq(2), qq(3), qq(4), qq(5)) / (W * W);
            } else {
                m = qq(oM);
            }
            acc += m * phi * phi;
        }
    }
    if (qlay == 1) Ye[ho_eidx(ho, (uint32_t)e, l)] = acc;
    else Ye[t] = acc;  // t == (b*nd + l)*64 + lane
}

// PA diagonal, sum-factorised (MFEM's PA AssembleDiagonal): thread per (element, i1[, i2]) computing
// the D1 entries along the last axis.  Every term of the operator is a component c of the qdata
// times a product of 1D factors, one per axis: F_d(q, i) = u_d(q, i) v_d(q, i) with u, v = G when the
// term differentiates along d, else B, so
//   diag(i) = sum_terms mult * sum_{q_last} F_last * (... sum_{q1} F_1 * qd_c(q)).
// Terms: diffusion c = (a, b) with a <= b (off-diagonal twice), convection c = oC + k with (k, none),
// mass (none, none).  ~D1^(dim-1) threads read each element's qdata once (wave broadcast) and do
// 10 Q1^dim FMAs each, against D1^dim Q1^dim (30 flops) for the per-entry form.
// D1T / Q1T > 0: compile-time sizes (the loops unroll and each qdata row is loaded before its sums);
// 0: the rule's run-time sizes
template <int DIM, int D1T, int Q1T>
__global__ void __launch_bounds__(256)
k_diag_sf(const double *__restrict__ qd, const int32_t *__restrict__ perm, int ne, int nblk, int nd, int qlay,
          const HoLayout ho, const Rule1D r, unsigned kinds, int nc, double *__restrict__ Ye)
{
    const int d1 = D1T > 0 ? D1T : r.d1, q1 = Q1T > 0 ? Q1T : r.q1;
    const int nq = DIM == 3 ? q1 * q1 * q1 : q1 * q1;
    const int nt = DIM == 3 ? d1 * d1 : d1;  // threads per element
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t npos = qlay == 1 ? (int64_t)ne : (int64_t)nblk * kLanes;
    if (t >= npos * nt) return;
    const int64_t pos = t / nt;
    const int it = (int)(t - pos * nt);
    const int i1 = it % d1, i2 = DIM == 3 ? it / d1 : 0;
    const int b = qlay == 1 ? 0 : (int)(pos / kLanes), lane = qlay == 1 ? 0 : (int)(pos % kLanes);
    const int e = qlay == 1 ? (int)pos : perm[pos];
    auto out = [&](int i3, double v) {
        const int l = DIM == 3 ? i1 + d1 * (i2 + d1 * i3) : i1 + d1 * i3;
        if (qlay == 1) Ye[ho_eidx(ho, (uint32_t)e, l)] = v;
        else Ye[((size_t)b * nd + l) * kLanes + lane] = v;
    };
    if (e < 0 || e >= ne) {
        for (int i3 = 0; i3 < d1; ++i3) out(i3, 0.0);
        return;
    }
    // qdata of component c at (qx, qy, qz) = base_c + qz * sz + (qx + q1 qy) * sxy (cheap strides)
    const size_t plane = qd_ho_plane(nc, q1);
    auto cbase = [&](int c, size_t &sxy, size_t &sz) -> const double * {
        if (qlay == 1) {
            const int qq2 = q1 * q1;
            const bool pair = c < (nc & ~1);
            sxy = pair ? 2 : 1;
            sz = DIM == 3 ? plane : 0;
            return qd + (size_t)e * q1 * plane + (pair ? (size_t)(c >> 1) * qq2 * 2 + (c & 1) : (size_t)(nc & ~1) * qq2);
        }
        sxy = (size_t)nc * kLanes;
        sz = (size_t)q1 * q1 * nc * kLanes;
        return qd + (size_t)b * nq * nc * kLanes + qd_offset(c, lane, nc);
    };
    // this thread's 1D factors along the first axes (i1, i2 fixed)
    double B1[kMaxQ1], G1[kMaxQ1], B2[kMaxQ1], G2[kMaxQ1];
    for (int q = 0; q < q1; ++q) {
        B1[q] = r.B[q][i1];
        G1[q] = r.G[q][i1];
        B2[q] = r.B[q][i2];
        G2[q] = r.G[q][i2];
    }
    // term list: component, derivative axes a, b (-1 = none), multiplicity
    int tc[10], ta[10], tb[10];
    double tm[10];
    int nterm = 0;
    if (kinds & CDFEM_DIFFUSION) {
        int c = 0;
        for (int a = 0; a < DIM; ++a)
            for (int bb = a; bb < DIM; ++bb, ++c) {
                tc[nterm] = c; ta[nterm] = a; tb[nterm] = bb; tm[nterm] = a == bb ? 1.0 : 2.0; ++nterm;
            }
    }
    const int oC = (kinds & CDFEM_DIFFUSION) ? DIM * (DIM + 1) / 2 : 0;
    const int oM = oC + ((kinds & CDFEM_CONVECTION) ? DIM : 0);
    if (kinds & CDFEM_CONVECTION)
        for (int k = 0; k < DIM; ++k) {
            tc[nterm] = oC + k; ta[nterm] = k; tb[nterm] = -1; tm[nterm] = 1.0; ++nterm;
        }
    const bool mass_from_d = DIM == 3 && (kinds & kMassFromD) && (kinds & CDFEM_MASS) && (kinds & CDFEM_DIFFUSION);
    if (kinds & CDFEM_MASS) {  // component -1: the mass weight derived from D (QLayout::kMD)
        tc[nterm] = mass_from_d ? -1 : oM; ta[nterm] = -1; tb[nterm] = -1; tm[nterm] = 1.0; ++nterm;
    }
    const double *dbase[6] = {};
    size_t dsxy = 0, dsz = 0;
    if (mass_from_d)
        for (int k = 0; k < 6; ++k) dbase[k] = cbase(k, dsxy, dsz);
    double acc[kMaxD1];
    for (int i3 = 0; i3 < d1; ++i3) acc[i3] = 0.0;
    const int last = DIM - 1;
    for (int s = 0; s < nterm; ++s) {
        const int a = ta[s], bb = tb[s];
        size_t sxy = 0, sz = 0;
        const bool derived = tc[s] < 0;
        const double *qc = derived ? nullptr : cbase(tc[s], sxy, sz);
        double f1[kMaxQ1], f2[kMaxQ1];
        for (int q = 0; q < q1; ++q) {
            f1[q] = (a == 0 ? G1[q] : B1[q]) * (bb == 0 ? G1[q] : B1[q]);
            f2[q] = (a == 1 ? G2[q] : B2[q]) * (bb == 1 ? G2[q] : B2[q]);
        }
#pragma unroll
        for (int qz = 0; qz < (Q1T > 0 ? Q1T : kMaxQ1); ++qz) {  // the last axis' quadrature index
            if (Q1T == 0 && qz >= q1) break;
            double szs = 0.0;
            if (DIM == 3) {
                const double *qp = derived ? nullptr : qc + qz * sz;
#pragma unroll
                for (int qy = 0; qy < (Q1T > 0 ? Q1T : kMaxQ1); ++qy) {
                    if (Q1T == 0 && qy >= q1) break;
                    double v[Q1T > 0 ? Q1T : kMaxQ1];
#pragma unroll
                    for (int qx = 0; qx < (Q1T > 0 ? Q1T : kMaxQ1); ++qx)
                        if (Q1T > 0 || qx < q1) {
                            if (derived) {
                                const size_t o = qz * dsz + (size_t)(qx + q1 * qy) * dsxy;
                                const double w = r.wts[qx] * r.wts[qy] * r.wts[qz];
                                v[qx] = r.mscale *
                                        det_sym3(dbase[0][o], dbase[1][o], dbase[2][o], dbase[3][o], dbase[4][o], dbase[5][o]) /
                                        (w * w);
                            } else {
                                v[qx] = qp[(size_t)(qx + q1 * qy) * sxy];
                            }
                        }
                    double sx = 0.0;
#pragma unroll
                    for (int qx = 0; qx < (Q1T > 0 ? Q1T : kMaxQ1); ++qx)
                        if (Q1T > 0 || qx < q1) sx += f1[qx] * v[qx];
                    szs += f2[qy] * sx;
                }
            } else {
#pragma unroll
                for (int qx = 0; qx < (Q1T > 0 ? Q1T : kMaxQ1); ++qx)
                    if (Q1T > 0 || qx < q1) szs += f1[qx] * qc[(size_t)(qx + q1 * qz) * sxy];
            }
            szs *= tm[s];
            for (int i3 = 0; i3 < d1; ++i3) {
                const double u = a == last ? r.G[qz][i3] : r.B[qz][i3];
                const double v = bb == last ? r.G[qz][i3] : r.B[qz][i3];
                acc[i3] += u * v * szs;
            }
        }
    }
    for (int i3 = 0; i3 < d1; ++i3) out(i3, acc[i3]);
}

// linear form, element part: be_l = sum_q W detJ f_q phi_l; thread per (block, l, lane)
template <int DIM>
__global__ void __launch_bounds__(256)
k_lf_elem(const double *__restrict__ verts, const int32_t *__restrict__ perm, int ne, int nblk, int nd, int qlay,
          const HoLayout ho, const Rule1D r,
          const double *__restrict__ fq, double *__restrict__ Ye)
{
    const int q1 = r.q1;
    const int nq = DIM == 3 ? q1 * q1 * q1 : q1 * q1;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)nblk * nd * kLanes) return;
    // element-major (qlay 1): thread per (e, l), l fastest (as k_diag_elem)
    const int lane = qlay == 1 ? 0 : (int)(t % kLanes);
    const int l = qlay == 1 ? (int)(t % nd) : (int)((t / kLanes) % nd);
    const int b = qlay == 1 ? 0 : (int)(t / ((int64_t)kLanes * nd));
    const int e = qlay == 1 ? (int)(t / nd) : perm[(size_t)b * kLanes + lane];
    double acc = 0.0;
    if (e >= 0 && e < ne) {
        for (int q = 0; q < nq; ++q) {
            double xi[3], W, x[3], J[3][3], A[3][3], phi, g[3];
            qpoint(q, q1, DIM, r, xi, W);
            q1_map<DIM>(verts + (size_t)e * (1 << DIM) * DIM, xi, x, J);
            const double det = adjugate<DIM>(J, A);
            basis_at(l, q, DIM, r, phi, g);
            acc += W * det * fq[(size_t)e * nq + q] * phi;
        }
    }
    if (qlay == 1) {
        if (e >= 0 && e < ne) Ye[ho_eidx(ho, (uint32_t)e, l)] = acc;
    } else {
        Ye[t] = acc;
    }
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
static inline unsigned grid_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

hipError_t launch_setup_qdata(cdfem_ctx *c, const double *d_kappa_q, const double *d_kmat_q, double kappa, double alpha,
                              const double *conv, const double *d_conv_q, const double *d_mass_q,
                              double mass)
{
    const int q1 = c->rule_op.q1;
    const int nq = c->dim == 3 ? q1 * q1 * q1 : q1 * q1;
    const int64_t n = (int64_t)c->nblk * nq * kLanes;
    const double c0 = conv ? conv[0] : 0.0, c1 = conv ? conv[1] : 0.0;
    const double c2 = (conv && c->dim == 3) ? conv[2] : 0.0;
    if (c->dim == 3)
        hipLaunchKernelGGL(k_setup_qdata<3>, dim3(grid_for(n, 256)), dim3(256), 0, c->stream,
                           c->d_verts, c->d_perm, c->ne, c->nblk, c->qlay, c->rule_op, c->kinds, c->ncomp, kappa,
                           d_kappa_q, d_kmat_q, alpha, c0, c1, c2, d_conv_q, mass, d_mass_q, c->d_qd);
    else
        hipLaunchKernelGGL(k_setup_qdata<2>, dim3(grid_for(n, 256)), dim3(256), 0, c->stream,
                           c->d_verts, c->d_perm, c->ne, c->nblk, c->qlay, c->rule_op, c->kinds, c->ncomp, kappa,
                           d_kappa_q, d_kmat_q, alpha, c0, c1, c2, d_conv_q, mass, d_mass_q, c->d_qd);
    return hipGetLastError();
}

hipError_t launch_quad_points(cdfem_ctx *c, const Rule1D &r, double *xyz)
{
    const int nq = c->dim == 3 ? r.q1 * r.q1 * r.q1 : r.q1 * r.q1;
    const int64_t n = (int64_t)c->ne * nq;
    if (c->dim == 3)
        hipLaunchKernelGGL(k_quad_points<3>, dim3(grid_for(n, 256)), dim3(256), 0, c->stream,
                           c->d_verts, c->ne, r, xyz);
    else
        hipLaunchKernelGGL(k_quad_points<2>, dim3(grid_for(n, 256)), dim3(256), 0, c->stream,
                           c->d_verts, c->ne, r, xyz);
    return hipGetLastError();
}

hipError_t launch_diag_elem(cdfem_ctx *c, double *Ye)
{
    if (c->diag_sf) {  // sum-factorised (default)
        const int d1 = c->rule_op.d1, q1 = c->rule_op.q1;
        const int64_t npos = c->qlay == 1 ? (int64_t)c->ne : (int64_t)c->nblk * kLanes;
        const int64_t n = npos * (c->dim == 3 ? d1 * d1 : d1);
        const dim3 g(grid_for(n, 256)), bs(256);
#define CDFEM_DSF(DIM_, D1_, Q1_)                                                                        \
    hipLaunchKernelGGL((k_diag_sf<DIM_, D1_, Q1_>), g, bs, 0, c->stream, c->d_qd, c->d_perm, c->ne, c->nblk, \
                       c->nd, c->qlay, ho_layout(c), c->rule_op, c->kinds, c->ncomp, Ye)
        const bool three = c->dim == 3;
        if (d1 == q1 - 1 && d1 >= 2 && d1 <= 5) {  // the Gauss n = p + 2 rules of the operators
            if (three) {
                if (d1 == 2) CDFEM_DSF(3, 2, 3);
                else if (d1 == 3) CDFEM_DSF(3, 3, 4);
                else if (d1 == 4) CDFEM_DSF(3, 4, 5);
                else CDFEM_DSF(3, 5, 6);
            } else {
                if (d1 == 2) CDFEM_DSF(2, 2, 3);
                else if (d1 == 3) CDFEM_DSF(2, 3, 4);
                else if (d1 == 4) CDFEM_DSF(2, 4, 5);
                else CDFEM_DSF(2, 5, 6);
            }
        } else if (three) {
            CDFEM_DSF(3, 0, 0);
        } else {
            CDFEM_DSF(2, 0, 0);
        }
#undef CDFEM_DSF
        return hipGetLastError();
    }
    const int64_t n = (int64_t)c->nblk * c->nd * kLanes;
    if (c->dim == 3)
        hipLaunchKernelGGL(k_diag_elem<3>, dim3(grid_for(n, 256)), dim3(256), 0, c->stream,
                           c->d_qd, c->d_perm, c->ne, c->nblk, c->nd, c->qlay, ho_layout(c), c->rule_op, c->kinds, c->ncomp, Ye);
    else
        hipLaunchKernelGGL(k_diag_elem<2>, dim3(grid_for(n, 256)), dim3(256), 0, c->stream,
                           c->d_qd, c->d_perm, c->ne, c->nblk, c->nd, c->qlay, ho_layout(c), c->rule_op, c->kinds, c->ncomp, Ye);
    return hipGetLastError();
}

hipError_t launch_lf_elem(cdfem_ctx *c, const double *d_fq, double *Ye)
{
    const int64_t n = (int64_t)c->nblk * c->nd * kLanes;
    if (c->dim == 3)
        hipLaunchKernelGGL(k_lf_elem<3>, dim3(grid_for(n, 256)), dim3(256), 0, c->stream,
                           c->d_verts, c->d_perm, c->ne, c->nblk, c->nd, c->qlay, ho_layout(c), c->rule_lf, d_fq, Ye);
    else
        hipLaunchKernelGGL(k_lf_elem<2>, dim3(grid_for(n, 256)), dim3(256), 0, c->stream,
                           c->d_verts, c->d_perm, c->ne, c->nblk, c->nd, c->qlay, ho_layout(c), c->rule_lf, d_fq, Ye);
    return hipGetLastError();
}

template <int DIM, int D1, int Q1, unsigned K>
static hipError_t apply_kinds(cdfem_ctx *c, const double *x, double *Ye, bool con,
                              const KrylovState *st)
{
    const Tab<D1, Q1> T = make_tab<D1, Q1>(c->rule_op);
    const dim3 grid(grid_for(c->nblk, 4)), block(256);
    if constexpr (DIM == 3) {
        if (con)
            hipLaunchKernelGGL((k_apply3d<D1, Q1, K, true>), grid, block, 0, c->stream, c->d_map, x,
                               c->d_qd, Ye, T, c->nblk, st);
        else
            hipLaunchKernelGGL((k_apply3d<D1, Q1, K, false>), grid, block, 0, c->stream, c->d_map,
                               x, c->d_qd, Ye, T, c->nblk, st);
    } else {
        if (con)
            hipLaunchKernelGGL((k_apply2d<D1, Q1, K, true>), grid, block, 0, c->stream, c->d_map, x,
                               c->d_qd, Ye, T, c->nblk, st);
        else
            hipLaunchKernelGGL((k_apply2d<D1, Q1, K, false>), grid, block, 0, c->stream, c->d_map,
                               x, c->d_qd, Ye, T, c->nblk, st);
    }
    return hipGetLastError();
}

template <int DIM, int D1, int Q1>
static hipError_t apply_dq(cdfem_ctx *c, const double *x, double *Ye, bool con, const KrylovState *st)
{
    switch (c->kinds) {
    case 1: return apply_kinds<DIM, D1, Q1, 1>(c, x, Ye, con, st);
    case 2: return apply_kinds<DIM, D1, Q1, 2>(c, x, Ye, con, st);
    case 3: return apply_kinds<DIM, D1, Q1, 3>(c, x, Ye, con, st);
    case 4: return apply_kinds<DIM, D1, Q1, 4>(c, x, Ye, con, st);
    case 5: return apply_kinds<DIM, D1, Q1, 5>(c, x, Ye, con, st);
    case 6: return apply_kinds<DIM, D1, Q1, 6>(c, x, Ye, con, st);
    case 7: return apply_kinds<DIM, D1, Q1, 7>(c, x, Ye, con, st);
    case 5 | kMassFromD: return apply_kinds<DIM, D1, Q1, 5 | kMassFromD>(c, x, Ye, con, st);
    case 7 | kMassFromD: return apply_kinds<DIM, D1, Q1, 7 | kMassFromD>(c, x, Ye, con, st);
    default: return hipErrorInvalidValue;
    }
}

bool apply_supported(int dim, int p)
{
    if (dim == 3) return p >= 1 && p <= 4;  // p = 3, 4: wave per element (ho_kernels.hip)
    if (dim == 2) return p >= 1 && p <= 4;
    return false;
}

// the kernel-side CG loop passes its state so a finished solve turns queued launches into no-ops
hipError_t launch_apply_st(cdfem_ctx *c, const double *x, double *Ye, bool con, const KrylovState *st)
{
    const int q1 = c->rule_op.q1;
    if (c->dim == 3) {
        if (c->p == 1 && q1 == 3) return apply_dq<3, 2, 3>(c, x, Ye, con, st);
        if (c->p == 2 && q1 == 4) return apply_dq<3, 3, 4>(c, x, Ye, con, st);
        if (c->p >= 3) return launch_apply_wpe(c, x, Ye, con, st);
    } else {
        if (c->p == 1 && q1 == 2) return apply_dq<2, 2, 2>(c, x, Ye, con, st);
        if (c->p == 2 && q1 == 3) return apply_dq<2, 3, 3>(c, x, Ye, con, st);
        if (c->p == 3 && q1 == 4) return apply_dq<2, 4, 4>(c, x, Ye, con, st);
        if (c->p == 4 && q1 == 5) return apply_dq<2, 5, 5>(c, x, Ye, con, st);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_apply(cdfem_ctx *c, const double *x, double *Ye, bool constrained)
{
    return launch_apply_st(c, x, Ye, constrained, nullptr);
}

}  // namespace cdfem
