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
    double w[Q1];  // 1D rule weights (the affine-geometry apply forms W_q = (w_x w_y) w_z)
    // the rule's 1D element matrices (the Kronecker form of the affine operator, elem_apply3d_kron):
    // M1[i][j] = sum_q w_q B_qi B_qj, K1 = sum_q w_q G_qi G_qj, C1[i][j] = sum_q w_q B_qi G_qj
    // (test value i, trial derivative j; its transpose is the test-derivative / trial-value factor)
    double M1[D1][D1];
    double K1[D1][D1];
    double C1[D1][D1];
};

// Symmetry of the 1D matrices: the rule's points and weights and the GLL nodes are symmetric about
// the centre, so B[Q-1-q][D-1-i] = B[q][i] and G[Q-1-q][D-1-i] = -G[q][i]; M and K are then symmetric
// and centro-symmetric, C is centro-antisymmetric (C[D-1-i][D-1-j] = -C[i][j], its centre entry 0).
// make_tab averages each orbit into its canonical entry and the Kronecker core reads only those, so
// only the distinct values (4 + 4 + 4 at p = 2) occupy scalar registers.
__host__ __device__ constexpr int sym_can(int D, int i, int j)
{
    const int a = i * D + j, b = j * D + i, c = (D - 1 - i) * D + (D - 1 - j), d = (D - 1 - j) * D + (D - 1 - i);
    const int m1 = a < b ? a : b, m2 = c < d ? c : d;
    return m1 < m2 ? m1 : m2;
}
__host__ __device__ constexpr int anti_can(int D, int i, int j)
{
    const int a = i * D + j, c = (D - 1 - i) * D + (D - 1 - j);
    return a < c ? a : c;
}
__host__ __device__ constexpr int anti_sign(int D, int i, int j)
{
    const int a = i * D + j, c = (D - 1 - i) * D + (D - 1 - j);
    return a == c ? 0 : (a < c ? 1 : -1);
}

template <int D1, int Q1>
static Tab<D1, Q1> make_tab(const Rule1D &r)
{
    Tab<D1, Q1> t;
    for (int q = 0; q < Q1; ++q)
        for (int d = 0; d < D1; ++d) {
            t.B[q][d] = r.B[q][d];
            t.G[q][d] = r.G[q][d];
        }
    for (int q = 0; q < Q1; ++q) t.w[q] = r.wts[q];
    for (int i = 0; i < D1; ++i)
        for (int j = 0; j < D1; ++j) {
            double m = 0.0, k = 0.0, c = 0.0;
            for (int q = 0; q < Q1; ++q) {
                m += r.wts[q] * r.B[q][i] * r.B[q][j];
                k += r.wts[q] * r.G[q][i] * r.G[q][j];
                c += r.wts[q] * r.B[q][i] * r.G[q][j];
            }
            t.M1[i][j] = m;
            t.K1[i][j] = k;
            t.C1[i][j] = c;
        }
    // the orbit averages (the canonical entries the Kronecker core reads)
    Tab<D1, Q1> u = t;
    for (int i = 0; i < D1; ++i)
        for (int j = 0; j < D1; ++j) {
            const int a = D1 - 1 - i, b = D1 - 1 - j;
            u.M1[i][j] = 0.25 * ((t.M1[i][j] + t.M1[j][i]) + (t.M1[a][b] + t.M1[b][a]));
            u.K1[i][j] = 0.25 * ((t.K1[i][j] + t.K1[j][i]) + (t.K1[a][b] + t.K1[b][a]));
            u.C1[i][j] = 0.5 * (t.C1[i][j] - t.C1[a][b]);
        }
    return u;
}

// the canonical entries of the 1D matrices (compile-time indices after unrolling)
template <int D1, int Q1>
__device__ __forceinline__ double tM(const Tab<D1, Q1> &T, int i, int j)
{
    const int k = sym_can(D1, i, j);
    return T.M1[k / D1][k % D1];
}
template <int D1, int Q1>
__device__ __forceinline__ double tK(const Tab<D1, Q1> &T, int i, int j)
{
    const int k = sym_can(D1, i, j);
    return T.K1[k / D1][k % D1];
}
// acc + C[i][j] x (the centre entry is structurally zero and adds nothing)
template <int D1, int Q1>
__device__ __forceinline__ double tCacc(const Tab<D1, Q1> &T, int i, int j, double x, double acc)
{
    const int s = anti_sign(D1, i, j), k = anti_can(D1, i, j);
    if (s == 0) return acc;
    return s > 0 ? acc + T.C1[k / D1][k % D1] * x : acc - T.C1[k / D1][k % D1] * x;
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

// qdata layout inside one quadrature point's block of NC*64 doubles: components 2p, 2p+1 are
// interleaved per lane ([pair][lane][2]) so a wave reads them with ONE 16-byte load per lane
// (dwordx4: 6.45 TB/s on MI355X vs 5.90 TB/s for 8-byte loads); an odd last component follows as
// [lane].  qd_offset() is the single definition used by setup, apply and diagonal kernels.
__host__ __device__ constexpr int qd_offset(int c, int lane, int nc)
{
    return (c < (nc & ~1)) ? ((c >> 1) * kLanes + lane) * 2 + (c & 1) : (nc & ~1) * kLanes + lane;
}

typedef double v2d_t __attribute__((ext_vector_type(2)));

// NT: non-temporal (streaming) loads — qdata is read once per Mult, so it must not displace the
// L-vectors that neighbouring elements / bricks re-read from L2.  Measured on k_brick_cg (64^3,
// p = 2): 283 -> 245 us per launch, and the following CG update 42.7 -> 35.5 us (its vectors
// are still cached; tools/ab.py, round 1).
template <int NC, bool NT = false>
__device__ __forceinline__ void load_qp(const double *__restrict__ qp, int lane, double (&v)[NC])
{
#pragma unroll
    for (int p = 0; p < NC / 2; ++p) {
        if constexpr (NT) {
            const v2d_t w = __builtin_nontemporal_load(reinterpret_cast<const v2d_t *>(qp + p * 2 * kLanes) + lane);
            v[2 * p] = w.x;
            v[2 * p + 1] = w.y;
        } else {
            const double2 w = reinterpret_cast<const double2 *>(qp + p * 2 * kLanes)[lane];
            v[2 * p] = w.x;
            v[2 * p + 1] = w.y;
        }
    }
    if constexpr (NC & 1) {
        if constexpr (NT) v[NC - 1] = __builtin_nontemporal_load(qp + (NC - 1) * kLanes + lane);
        else v[NC - 1] = qp[(NC - 1) * kLanes + lane];
    }
}

// Y = A_e X for one element: X, Y lexicographic [dz][dy][dx]; q0 points at this element's
// block's qdata (q = 0, lane 0; point stride NC * kLanes), lane = element.  X is read through the
// loader xl(dz, dy, dx) once per quadrature plane, so a caller holding X in LDS keeps only one
// plane's worth of it live in registers.  QZU = unroll factor of the quadrature-plane loop
// (Q1: straight-line code, the compiler hoists qdata loads across planes; 1: one plane's loads
// in flight, ~250 VGPRs at p = 2, two waves per SIMD).
// AFF (affine elements, constant coefficients): q0 points at the block's per-element factors
// [NC][kLanes] instead, and the point data is formed as W_q * G_k, the same product the setup
// stores (k_setup_qdata, aff), so both forms apply the same operator bit for bit.
template <int D1, int Q1, unsigned K, typename XL, int QZU = Q1, bool AFF = false>
__device__ __forceinline__ void elem_apply3d(const XL &xl, const double *__restrict__ q0, int lane,
                                             const Tab<D1, Q1> &T, double (&Y)[D1][D1][D1])
{
    using L = QLayout<K, 3>;
    constexpr int NC = L::nc;
    double ga[NC];
    if constexpr (AFF) {
#pragma unroll
        for (int k = 0; k < NC; ++k) ga[k] = q0[k * kLanes + lane];
    }
#pragma unroll
    for (int dz = 0; dz < D1; ++dz)
#pragma unroll
        for (int dy = 0; dy < D1; ++dy)
#pragma unroll
            for (int dx = 0; dx < D1; ++dx) Y[dz][dy][dx] = 0.0;

#pragma unroll QZU
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
                    const double xv = xl(dz, dy, dx);
                    s0 += T.B[qz][dz] * xv;
                    s1 += T.G[qz][dz] * xv;
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
                double qv[NC];
                if constexpr (AFF) {
                    const double W = T.w[qx] * T.w[qy] * T.w[qz];
#pragma unroll
                    for (int k = 0; k < NC; ++k) qv[k] = W * ga[k];
                } else {
                    const int q = qx + Q1 * (qy + Q1 * qz);
                    load_qp<NC, true>(q0 + (size_t)q * NC * kLanes, lane, qv);
                }
                double vv = 0.0, gx = 0.0, gy = 0.0, gz = 0.0;
                if constexpr (L::kD) {
                    gx = qv[0] * ux + qv[1] * uy + qv[2] * uz;
                    gy = qv[1] * ux + qv[3] * uy + qv[4] * uz;
                    gz = qv[2] * ux + qv[4] * uy + qv[5] * uz;
                }
                if constexpr (L::kC) vv = qv[L::oC] * ux + qv[L::oC + 1] * uy + qv[L::oC + 2] * uz;
                if constexpr (L::kM) vv += qv[L::oM] * u;
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

// Y = A_e X for one affine element with constant coefficients in its Kronecker form.  With the
// Jacobian constant on the element the point data factor as W_q g_k (g = the 10 per-element factors
// k_setup_qdata keeps, pa_affine), and the tensor rule's W_q = w_x w_y w_z separates, so every term
// of the quadrature sum is a Kronecker product of the rule's 1D matrices (Tab::M1, K1, C1):
//     term                 (z, y, x) factors           coefficient
//     mass                 (M, M, M)                    s detJ
//     D_aa                 K in axis a, M elsewhere     D_aa
//     D_ab (a != b)        Ct in a, C in b, M else      D_ab (both orderings)
//     convection c_b       C in axis b, M elsewhere     c_b
// (C: trial derivative, test value; Ct = C^T: test derivative, trial value; K both; M neither).
// A_e = sum_t g_t Fz (x) Fy (x) Fx is the same operator as the quadrature form to rounding (an
// algebraic identity for any tensor rule, not an exactness argument).  Evaluated per input z plane
// jz: x stage (M, K, C, Ct on the plane's rows), the per-element combinations, y stage into the four
// z groups (M, K, C, Ct), z stage into Y.  At p = 2: 1.73 K FMA-class operations per element against
// 4.3 K for the quadrature form (elem_apply3d<..., AFF>), 45 + 27 live doubles.
// The two halves of the Kronecker form, shared by the thread-per-element core (kron_core) and the
// high-order tile kernel (ho_kernels.hip k_apply3d_ktile).
// x stage of one input row X[jz][jy][*] for output column ix: the five x-applied quantities
//   v[0] = (M X)_ix, v[1] = (C X)_ix, v[2] = u1 = s M + D_xx K + c_x C, v[3] = u3 = D_xy Ct + c_y M,
//   v[4] = u5 = D_xz Ct + c_z M   (applied along x)
template <unsigned K>
__device__ __forceinline__ void kron_xcombine(const double (&g)[QLayout<K, 3>::nc], double m, double k, double c,
                                              double ct, double (&v)[5]);
template <int D1, int Q1, unsigned K>
__device__ __forceinline__ void kron_xrow(const Tab<D1, Q1> &T, const double (&g)[QLayout<K, 3>::nc],
                                          const double (&X)[D1], int ix, double (&v)[5])
{
    using L = QLayout<K, 3>;
    constexpr bool kD = L::kD, kG = L::kD || L::kC;
    double m = 0.0, k = 0.0, c = 0.0, ct = 0.0;
#pragma unroll
    for (int jx = 0; jx < D1; ++jx) {
        m += tM(T, ix, jx) * X[jx];
        if constexpr (kD) {
            k += tK(T, ix, jx) * X[jx];
            ct = tCacc(T, jx, ix, X[jx], ct);
        }
        if constexpr (kG) c = tCacc(T, ix, jx, X[jx], c);
    }
    kron_xcombine<K>(g, m, k, c, ct, v);
}

// the per-element combinations of one x-applied row: m, k, c, ct = (M X), (K X), (C X), (Ct X)
template <unsigned K>
__device__ __forceinline__ void kron_xcombine(const double (&g)[QLayout<K, 3>::nc], double m, double k, double c,
                                              double ct, double (&v)[5])
{
    using L = QLayout<K, 3>;
    constexpr bool kD = L::kD, kC = L::kC, kM = L::kM;
    v[0] = m;
    v[1] = c;
    double a = 0.0;
    if constexpr (kM) a = g[L::oM] * m;
    if constexpr (kD) a += g[0] * k;
    if constexpr (kC) a += g[L::oC] * c;
    v[2] = a;
    v[3] = v[4] = 0.0;
    if constexpr (kD && kC) {
        v[3] = g[1] * ct + g[L::oC + 1] * m;
        v[4] = g[2] * ct + g[L::oC + 2] * m;
    } else if constexpr (kD) {
        v[3] = g[1] * ct;
        v[4] = g[2] * ct;
    } else if constexpr (kC) {
        v[3] = g[L::oC + 1] * m;
        v[4] = g[L::oC + 2] * m;
    }
}

// y stage of one output column (the x-stage quantities col(q, jy) of kron_xrow, q = 0..4, for every
// input row jy of plane jz) into the four z groups P = (pm, pk, pc, pct) of output row iy
template <int D1, int Q1, unsigned K, typename COL>
__device__ __forceinline__ void kron_y(const Tab<D1, Q1> &T, const double (&g)[QLayout<K, 3>::nc], const COL &col,
                                       int iy, double (&P)[4])
{
    using L = QLayout<K, 3>;
    constexpr bool kD = L::kD, kG = L::kD || L::kC;
    double pm = 0.0, pk = 0.0, pc = 0.0, pct = 0.0;
    {
        double s1 = 0.0;
#pragma unroll
        for (int jy = 0; jy < D1; ++jy) s1 += tM(T, iy, jy) * col(2, jy);
        pm = s1;
    }
    if constexpr (kG) {
        double s3 = 0.0, s5 = 0.0;
#pragma unroll
        for (int jy = 0; jy < D1; ++jy) {
            s3 = tCacc(T, iy, jy, col(3, jy), s3);
            s5 += tM(T, iy, jy) * col(4, jy);
        }
        pm += s3;
        pc = s5;
    }
    if constexpr (kD) {
        double kym = 0.0, ctyc = 0.0, mym = 0.0, ctym = 0.0, myc = 0.0, cym = 0.0;
#pragma unroll
        for (int jy = 0; jy < D1; ++jy) {
            const double xm = col(0, jy), xc = col(1, jy);
            kym += tK(T, iy, jy) * xm;
            ctyc = tCacc(T, jy, iy, xc, ctyc);
            mym += tM(T, iy, jy) * xm;
            ctym = tCacc(T, jy, iy, xm, ctym);
            myc += tM(T, iy, jy) * xc;
            cym = tCacc(T, iy, jy, xm, cym);
        }
        pm += g[3] * kym;
        pm += g[1] * ctyc;
        pk = g[5] * mym;
        pc += g[4] * ctym;
        pct = g[2] * myc + g[4] * cym;
    }
    P[0] = pm;
    P[1] = pk;
    P[2] = pc;
    P[3] = pct;
}

// z stage of input plane jz: Yz[iz] += the four groups P of one output (iy, ix) along z
template <int D1, int Q1, unsigned K>
__device__ __forceinline__ void kron_z(const Tab<D1, Q1> &T, const double (&P)[4], int jz, double (&Yz)[D1])
{
    using L = QLayout<K, 3>;
    constexpr bool kD = L::kD, kG = L::kD || L::kC;
    const double pm = P[0], pk = P[1], pc = P[2], pct = P[3];
#pragma unroll
    for (int iz = 0; iz < D1; ++iz) {
        double y = Yz[iz];
        y += tM(T, iz, jz) * pm;
        if constexpr (kD) {
            y += tK(T, iz, jz) * pk;
            y = tCacc(T, jz, iz, pct, y);
        }
        if constexpr (kG) y = tCacc(T, iz, jz, pc, y);
        Yz[iz] = y;
    }
}

template <int D1, int Q1, unsigned K, typename COL>
__device__ __forceinline__ void kron_yz(const Tab<D1, Q1> &T, const double (&g)[QLayout<K, 3>::nc], const COL &col,
                                        int iy, int jz, double (&Yz)[D1])
{
    double P[4];
    kron_y<D1, Q1, K>(T, g, col, iy, P);
    kron_z<D1, Q1, K>(T, P, jz, Yz);
}

// g: the element's factors (QLayout<K, 3> order), loaded by the caller (kron_load_g)
template <int D1, int Q1, unsigned K, typename XL>
__device__ __forceinline__ void kron_core(const XL &xl, const double (&g)[QLayout<K, 3>::nc], const Tab<D1, Q1> &T,
                                          double (&Y)[D1][D1][D1])
{
#pragma unroll
    for (int dz = 0; dz < D1; ++dz)
#pragma unroll
        for (int dy = 0; dy < D1; ++dy)
#pragma unroll
            for (int dx = 0; dx < D1; ++dx) Y[dz][dy][dx] = 0.0;
#pragma unroll
    for (int jz = 0; jz < D1; ++jz) {
        double X[D1][D1];
#pragma unroll
        for (int jy = 0; jy < D1; ++jy)
#pragma unroll
            for (int jx = 0; jx < D1; ++jx) X[jy][jx] = xl(jz, jy, jx);
        // one output column ix at a time (x stage of that column for every row jy, then the y and z
        // stages of the column), so only one column's intermediates are live
#pragma unroll
        for (int ix = 0; ix < D1; ++ix) {
            double v[D1][5];
#pragma unroll
            for (int jy = 0; jy < D1; ++jy) kron_xrow<D1, Q1, K>(T, g, X[jy], ix, v[jy]);
            auto col = [&](int q, int jy) { return v[jy][q]; };
#pragma unroll
            for (int iy = 0; iy < D1; ++iy) {
                double Yz[D1];
#pragma unroll
                for (int iz = 0; iz < D1; ++iz) Yz[iz] = Y[iz][iy][ix];
                kron_yz<D1, Q1, K>(T, g, col, iy, jz, Yz);
#pragma unroll
                for (int iz = 0; iz < D1; ++iz) Y[iz][iy][ix] = Yz[iz];
            }
        }
    }
}

// the factors of element `lane` of the block whose factors start at q0 ([NC][kLanes])
template <unsigned K>
__device__ __forceinline__ void kron_load_g(const double *__restrict__ q0, int lane, double (&g)[QLayout<K, 3>::nc])
{
#pragma unroll
    for (int k = 0; k < QLayout<K, 3>::nc; ++k) g[k] = q0[k * kLanes + lane];
}

template <int D1, int Q1, unsigned K, typename XL>
__device__ __forceinline__ void elem_apply3d_kron(const XL &xl, const double *__restrict__ q0, int lane,
                                                  const Tab<D1, Q1> &T, double (&Y)[D1][D1][D1])
{
    double g[QLayout<K, 3>::nc];
    kron_load_g<K>(q0, lane, g);
    kron_core<D1, Q1, K>(xl, g, T, Y);
}

// the element core of the apply kernels by affine form: AF 0 per-point stream, 1 point data formed
// from the affine factors (elem_apply3d<..., AFF>), 2 the Kronecker form of the same factors
template <int D1, int Q1, unsigned K, int AF, typename XL>
__device__ __forceinline__ void elem_apply3d_af(const XL &xl, const double *__restrict__ q0, int lane,
                                                const Tab<D1, Q1> &T, double (&Y)[D1][D1][D1])
{
    if constexpr (AF == 2) elem_apply3d_kron<D1, Q1, K>(xl, q0, lane, T, Y);
    else elem_apply3d<D1, Q1, K, XL, Q1, AF == 1>(xl, q0, lane, T, Y);
}

typedef double v4d_t __attribute__((ext_vector_type(4)));

// One block-wide GEMM on the matrix cores: out(row, col) = sum_k a(row, k) b(k, col) for
// row < ROWS (the block's elements stacked), k < 4 KS, col < 16, as v_mfma_f64_16x16x4_f64 tiles of
// 16 rows; the NW waves of the block (4 by default) take row tiles round-robin.  a() and b() return 0 outside
// the operator; o(row, col, v) stores (and drops padding columns).  Lane maps (MI355X f64 MFMA):
// A[l & 15][k = l >> 4], B[k = l >> 4][l & 15], D[(l >> 4) + 4 r][l & 15].
template <int ROWS, int KS, typename FA, typename FB, typename FO, int NW = 4>
__device__ __forceinline__ void block_mfma(const FA &a, const FB &b, const FO &o)
{
    constexpr int NTL = (ROWS + 15) / 16;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, kq = lane >> 4, col = lane & 15;
    double bop[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) bop[ks] = b(ks * 4 + kq, col);
    for (int tt = wv; tt < NTL; tt += NW) {  // (NW: the block's waves)
        const int rho = tt * 16 + col;
        v4d_t acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const double av = rho < ROWS ? a(rho, ks * 4 + kq) : 0.0;
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bop[ks], acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = tt * 16 + kq + 4 * r;
            if (row < ROWS) o(row, col, acc[r]);
        }
    }
}

// exact unsigned division by a run-time divisor: n / d == (n * m) >> k for n < 2^31
struct FastDiv {
    uint64_t m;
    uint32_t k, d;
};
inline FastDiv make_fastdiv(uint32_t d)
{
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    const uint32_t k = 32 + l;
    const uint64_t m = ((1ull << k) + d - 1) / d;
    return FastDiv{m, k, d};
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv &f)
{
    return (uint32_t)(((uint64_t)n * f.m) >> f.k);
}

// E-vector index of (element e, local dof l) on the high-order layout (qlay = 1, 3D p >= 3).
// Generic meshes: element-major [e][l].  Structured boxes (pencil != 0, cdfem_mesh_set_structured):
// [ez][dz][ey][dy][ex][dx], so every x-row of the dof lattice is ONE contiguous run of the
// E-vector (its element-boundary dofs are adjacent pairs) and k_e2l_box reads it coalesced.
struct HoLayout {
    uint32_t pencil, nx, ny, d1;
    FastDiv fnx, fny;
};
__device__ __forceinline__ size_t ho_eidx(const HoLayout &h, uint32_t e, int l)
{
    const int d1 = (int)h.d1;
    if (!h.pencil) return (size_t)e * (d1 * d1 * d1) + l;
    const uint32_t r = fdiv(e, h.fnx), ex = e - r * h.nx;
    const uint32_t ez = fdiv(r, h.fny), ey = r - ez * h.ny;
    const int dx = l % d1, dy = (l / d1) % d1, dz = l / (d1 * d1);
    return ((((size_t)ez * d1 + dz) * h.ny + ey) * d1 + dy) * ((size_t)h.nx * d1) + (size_t)ex * d1 + dx;
}
inline HoLayout ho_layout(const cdfem_ctx *c)
{
    HoLayout h{};
    h.pencil = c->epencil ? 1u : 0u;
    h.d1 = (uint32_t)c->d1;
    h.nx = (uint32_t)(c->epencil ? c->sx : 1);
    h.ny = (uint32_t)(c->epencil ? c->sy : 1);
    h.fnx = make_fastdiv(h.nx);
    h.fny = make_fastdiv(h.ny);
    return h;
}

}  // namespace cdfem
