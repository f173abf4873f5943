/*
 * cdfem_oracle.c — CPU ORACLE (TEST INFRASTRUCTURE ONLY).
 *
 * This file is the checker, never the product.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product path (continuum-mechanics-mfem_amd/)
 * never links, loads or calls it.
 *
 * What it restates: the reference's hot path, i.e. what the convection-diffusion drivers do
 * through MFEM's *legacy full assembly* on the CPU (Device("cpu"), no SetAssemblyLevel):
 *
 *   a.AddDomainIntegrator(new DiffusionIntegrator(kappa));        linear_convection_diffusion_2D.cpp:336
 *   a.AddDomainIntegrator(new ConvectionIntegrator(c, alpha));     :337  (alpha: linear_convection_diffusion_1D.cpp:396)
 *   a.AddDomainIntegrator(new MassIntegrator(s));                  :338
 *   a.Assemble();                                                  :339  -> element matrices -> CSR
 *   b.AddDomainIntegrator(new DomainLFIntegrator(f)); b.Assemble() :341-343
 *   u.ProjectBdrCoefficient(exact, ess_bdr)                        :345-347 (nodal interpolation)
 *   a.FormLinearSystem(ess, u, b, A, X, B)                         :349-351 (row+col elimination, diag 1)
 *   PetscLinearSolver (KSPGMRES + PCJACOBI, restart 30, left PC)   :364-375, Input/petsc.opts:2-6
 *   CGSolver semantics (MFEM)                                      mesh_recession_handler.cpp:270-276
 *   u.ComputeL2Error(exact, irs), order max(2, 2p+3)               :383-390
 *
 * MFEM, hypre and PETSc are not vendored in /root/reference and not installed,
 * so the library-internal semantics below are restated from their documented public behaviour
 * and marked [MFEM-ext] / [PETSc-ext]:
 *   - H1_FECollection(p): Gauss-Lobatto nodal Lagrange basis on [0,1]^d, tensor product.     [MFEM-ext]
 *   - default rules (affine/multilinear tensor elements, Gauss-Legendre, n = order/2 + 1):
 *       Diffusion  order = 2p + dim - 1                                                     [MFEM-ext]
 *       Convection order = OrderGrad + p + OrderW = (dim-1) + (p-1) + p + (dim-1)           [MFEM-ext]
 *         (older MFEM uses Trans.Order() = 1 instead of OrderW: the same n for p=1 2D, p=2,4 3D)
 *       Mass       order = 2p + OrderW = 2p + dim - 1                                       [MFEM-ext]
 *       DomainLF   order = 2p                                                               [MFEM-ext]
 *     -> Diffusion/Convection/Mass share n = p + 1 ... p + 2 points: p=1 quad n=2, p=2 hex n=4,
 *        p=4 hex n=6 (computed, not assumed, by orc_rule_npts()).
 *   - element matrix convention elmat(i,j) = a(phi_j, phi_i): row = test function.           [MFEM-ext]
 *
 * PARITY PINNING.  The reference holds no golden vectors, no recorded outputs and no tests for this
 * path, and MFEM cannot be built here.  This oracle is therefore pinned by the
 * reference's own verification method — manufactured solutions (linear_convection_diffusion_2D.cpp:159-215,
 * diffusion_mms.cpp:136-178) — turned into asserted known answers in tests/test_oracle.py:
 * exact reproduction of polynomial solutions in the FE space, O(h^{p+1}) L2 convergence, and
 * algebraic identities (mass = volume, K*1 = 0, C*1 = 0, symmetry).  Bit-level parity with an
 * actual MFEM run is UNPINNED (no MFEM in this image).
 */
#define _GNU_SOURCE
#include <sched.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_API __attribute__((visibility("default")))
#define ORC_PI 3.14159265358979323846

/* ------------------------------------------------------------------------------------------ */
/* 1D rules and basis                                                                          */
/* ------------------------------------------------------------------------------------------ */

/* Legendre P_n(t) and P_n'(t) on [-1,1] by the three-term recurrence. */
static void legendre(int n, double t, double *P, double *dP)
{
    double p0 = 1.0, p1 = t;
    if (n == 0) { *P = 1.0; *dP = 0.0; return; }
    for (int k = 2; k <= n; k++) {
        double pk = ((2.0 * k - 1.0) * t * p1 - (k - 1.0) * p0) / k;
        p0 = p1; p1 = pk;
    }
    *P = p1;
    *dP = (fabs(1.0 - t * t) > 0.0) ? n * (p0 - t * p1) / (1.0 - t * t) : 0.0;
}

/* n-point Gauss-Legendre rule on [0,1], nodes ascending, weights sum to 1. */
ORC_API void orc_gauss_legendre(int n, double *x, double *w)
{
    for (int i = 0; i < n; i++) {
        double t = cos(ORC_PI * (i + 0.75) / (n + 0.5)); /* descending guess */
        for (int it = 0; it < 100; it++) {
            double P, dP;
            legendre(n, t, &P, &dP);
            double dt = P / dP;
            t -= dt;
            if (fabs(dt) < 1e-17) break;
        }
        double P, dP;
        legendre(n, t, &P, &dP);
        /* map t in [-1,1] (descending in i) to ascending [0,1] */
        x[i] = 0.5 * (1.0 - t);
        w[i] = 1.0 / ((1.0 - t * t) * dP * dP);
    }
}

/* p+1 Gauss-Lobatto nodes on [0,1]: endpoints and the roots of P_p'. [MFEM-ext BasisType::GaussLobatto] */
ORC_API void orc_gll_nodes(int p, double *x)
{
    x[0] = 0.0;
    x[p] = 1.0;
    for (int i = 1; i < p; i++) {
        double t = -cos(ORC_PI * i / p); /* Chebyshev-Gauss-Lobatto guess, ascending */
        for (int it = 0; it < 100; it++) {
            /* f = P_p'(t), f' = P_p''(t) = (2t P_p' - p(p+1) P_p) / (1 - t^2) */
            double P, dP;
            legendre(p, t, &P, &dP);
            double d2P = (2.0 * t * dP - p * (p + 1.0) * P) / (1.0 - t * t);
            double dt = dP / d2P;
            t -= dt;
            if (fabs(dt) < 1e-17) break;
        }
        x[i] = 0.5 * (t + 1.0);
    }
    /* enforce exact symmetry, as the nodal set is symmetric about 1/2 */
    for (int i = 0; i <= p / 2; i++) {
        double a = 0.5 * (x[i] + (1.0 - x[p - i]));
        x[i] = a;
        x[p - i] = 1.0 - a;
    }
}

/* Lagrange basis through nodes[0..p] and its derivative at xi. */
ORC_API void orc_lagrange(int p, const double *nodes, double xi, double *phi, double *dphi)
{
    for (int j = 0; j <= p; j++) {
        double v = 1.0, d = 0.0;
        for (int k = 0; k <= p; k++) {
            if (k == j) continue;
            double den = nodes[j] - nodes[k];
            double f = (xi - nodes[k]) / den;
            d = d * f + v / den;
            v *= f;
        }
        phi[j] = v;
        if (dphi) dphi[j] = d;
    }
}

/* Number of 1D Gauss-Legendre points of MFEM's default rule for each integrator on a tensor
 * (quad/hex) element with a multilinear (Q1) geometry.  which: 0 diffusion, 1 convection,
 * 2 mass, 3 domain LF, 4 L2 error (driver's max(2,2p+3): linear_convection_diffusion_2D.cpp:383). */
ORC_API int orc_rule_npts(int which, int dim, int p)
{
    int order_w = dim - 1;          /* Q1: OrderW = k*dim - 1, k=1          [MFEM-ext] */
    int order;
    switch (which) {
    case 0: order = p + p + dim - 1; break;                 /* DiffusionIntegrator::GetRule  */
    case 1: order = ((dim - 1) + (p - 1)) + p + order_w; break; /* ConvectionIntegrator::GetRule */
    case 2: order = p + p + order_w; break;                 /* MassIntegrator::GetRule       */
    case 3: order = 2 * p; break;                           /* DomainLFIntegrator oa=2, ob=0 */
    case 4: order = (2 * p + 3 > 2) ? 2 * p + 3 : 2; break; /* driver's error rule           */
    default: return -1;
    }
    return order / 2 + 1;           /* IntRules.Get(Geometry::SQUARE/CUBE, order): GL n=order/2+1 */
}

/* ------------------------------------------------------------------------------------------ */
/* Structured meshes                                                                           */
/* ------------------------------------------------------------------------------------------ */

/* Deterministic hash in [-1,1) used to perturb interior vertices (non-affine test meshes). */
static double hash_unit(uint64_t a)
{
    a ^= a >> 33; a *= 0xff51afd7ed558ccdULL; a ^= a >> 33; a *= 0xc4ceb9fe1a85ec53ULL; a ^= a >> 33;
    return (double)(a >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

/*
 * Box [0,1]^dim split into nx*ny(*nz) quads/hexes, element e = ix + nx*(iy + ny*iz).
 * Element vertices in lexicographic local order v = a + 2b (+ 4c), a along x.
 * H1 order p dofs numbered globally lexicographic on the (p*nx+1) x (p*ny+1) (x (p*nz+1)) lattice
 * of *reference* GLL positions; local element dof l = dx + (p+1)(dy + (p+1) dz).
 * perturb > 0 moves interior vertices by perturb*h*hash (a non-affine multilinear mesh).
 * Boundary attribute convention follows Mesh/unit_square.geo:18-21 (1 bottom, 2 right, 3 top,
 * 4 left); the hot path marks all boundaries essential (linear_convection_diffusion_2D.cpp:319-322).
 * Outputs (caller-allocated): verts[NE*nv*dim], dofmap[NE*(p+1)^dim], bdr[NL] (1 on boundary).
 */
ORC_API void orc_mesh_box(int dim, int nx, int ny, int nz, int p, double perturb,
                          double *verts, int *dofmap, int *bdr)
{
    if (dim == 2) nz = 1;
    const int vx = nx + 1, vy = ny + 1;
    const int nv = (dim == 3) ? 8 : 4;
    const int d1 = p + 1;
    const int nd = (dim == 3) ? d1 * d1 * d1 : d1 * d1;
    const int Lx = p * nx + 1, Ly = p * ny + 1, Lz = (dim == 3) ? p * nz + 1 : 1;
    const double hx = 1.0 / nx, hy = 1.0 / ny, hz = 1.0 / nz;
    const int ne = nx * ny * nz;
    for (int e = 0; e < ne; e++) {
        int ix = e % nx, iy = (e / nx) % ny, iz = e / (nx * ny);
        for (int v = 0; v < nv; v++) {
            int a = v & 1, b = (v >> 1) & 1, c = (v >> 2) & 1;
            int gx = ix + a, gy = iy + b, gz = iz + c;
            double X[3] = {gx * hx, gy * hy, gz * hz};
            int interior = gx > 0 && gx < nx && gy > 0 && gy < ny && (dim == 2 || (gz > 0 && gz < nz));
            if (perturb > 0.0 && interior) {
                uint64_t id = (uint64_t)gx + (uint64_t)vx * ((uint64_t)gy + (uint64_t)vy * gz);
                X[0] += perturb * hx * hash_unit(3 * id + 0);
                X[1] += perturb * hy * hash_unit(3 * id + 1);
                if (dim == 3) X[2] += perturb * hz * hash_unit(3 * id + 2);
            }
            for (int k = 0; k < dim; k++) verts[((size_t)e * nv + v) * dim + k] = X[k];
        }
        for (int l = 0; l < nd; l++) {
            int dx = l % d1, dy = (l / d1) % d1, dz = l / (d1 * d1);
            int gx = p * ix + dx, gy = p * iy + dy, gz = p * iz + dz;
            dofmap[(size_t)e * nd + l] = gx + Lx * (gy + Ly * gz);
        }
    }
    const int64_t nl = (int64_t)Lx * Ly * Lz;
    for (int64_t i = 0; i < nl; i++) {
        int gx = (int)(i % Lx), gy = (int)((i / Lx) % Ly), gz = (int)(i / ((int64_t)Lx * Ly));
        int on = gx == 0 || gx == Lx - 1 || gy == 0 || gy == Ly - 1;
        if (dim == 3) on = on || gz == 0 || gz == Lz - 1;
        bdr[i] = on;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* Geometry: multilinear map from the element vertices                                          */
/* ------------------------------------------------------------------------------------------ */

/* x(xi) and J = dx/dxi at reference point xi for a Q1 element. */
static void q1_map(int dim, const double *V, const double *xi, double *x, double J[3][3])
{
    const int nv = (dim == 3) ? 8 : 4;
    for (int i = 0; i < dim; i++) {
        x[i] = 0.0;
        for (int k = 0; k < dim; k++) J[i][k] = 0.0;
    }
    for (int v = 0; v < nv; v++) {
        int bit[3] = {v & 1, (v >> 1) & 1, (v >> 2) & 1};
        double f[3], df[3];
        for (int k = 0; k < dim; k++) {
            f[k] = bit[k] ? xi[k] : 1.0 - xi[k];
            df[k] = bit[k] ? 1.0 : -1.0;
        }
        double N = 1.0;
        for (int k = 0; k < dim; k++) N *= f[k];
        for (int k = 0; k < dim; k++) {
            double dN = df[k];
            for (int m = 0; m < dim; m++) if (m != k) dN *= f[m];
            for (int i = 0; i < dim; i++) J[i][k] += V[v * dim + i] * dN;
        }
        for (int i = 0; i < dim; i++) x[i] += V[v * dim + i] * N;
    }
}

/* det(J) and adj(J) = det(J) J^{-1}. */
static double adjugate(int dim, double J[3][3], double A[3][3])
{
    if (dim == 2) {
        A[0][0] = J[1][1]; A[0][1] = -J[0][1];
        A[1][0] = -J[1][0]; A[1][1] = J[0][0];
        return J[0][0] * J[1][1] - J[0][1] * J[1][0];
    }
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

/* Tensor tables for order p at n Gauss points: B[q*(p+1)+d], G[...], pts, wts. */
static void tables(int p, int n, double *B, double *G, double *pts, double *wts)
{
    double nodes[16];
    orc_gll_nodes(p, nodes);
    orc_gauss_legendre(n, pts, wts);
    for (int q = 0; q < n; q++) orc_lagrange(p, nodes, pts[q], B + q * (p + 1), G + q * (p + 1));
}

/* Basis values and reference gradients of the nd tensor functions at tensor point (qx,qy,qz). */
static void tensor_basis(int dim, int p, const double *B, const double *G, const int *qi,
                         double *phi, double (*gphi)[3])
{
    const int d1 = p + 1;
    const int nd = (dim == 3) ? d1 * d1 * d1 : d1 * d1;
    for (int l = 0; l < nd; l++) {
        int ix = l % d1, iy = (l / d1) % d1, iz = l / (d1 * d1);
        double bx = B[qi[0] * d1 + ix], gx = G[qi[0] * d1 + ix];
        double by = B[qi[1] * d1 + iy], gy = G[qi[1] * d1 + iy];
        if (dim == 2) {
            phi[l] = bx * by;
            gphi[l][0] = gx * by; gphi[l][1] = bx * gy; gphi[l][2] = 0.0;
        } else {
            double bz = B[qi[2] * d1 + iz], gz = G[qi[2] * d1 + iz];
            phi[l] = bx * by * bz;
            gphi[l][0] = gx * by * bz; gphi[l][1] = bx * gy * bz; gphi[l][2] = bx * by * gz;
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* Full assembly (the reference's legacy FA path)                                              */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    int64_t n;        /* rows */
    int64_t nnz;
    int64_t *rp;      /* row pointer n+1 */
    int32_t *col;     /* sorted within row */
    double *val;
} orc_csr;

/* Coefficients of a(u,v) = kappa (grad u, grad v) + alpha (c . grad u, v) + s (u, v). */
typedef struct {
    double kappa, alpha, s, c[3];
    int use_diff, use_conv, use_mass;
    /* per-quadrature-point values of ONE element (NULL: the constants above), point order of the
     * element rule: Coefficient kappa_q, symmetric MatrixCoefficient K_q (xx,xy,yy / xx,xy,xz,yy,yz,zz;
     * K = kappa I + K_q, diffusion_mms_ale.cpp:474-496), VectorCoefficient c_q, Coefficient s_q */
    const double *kq, *kmq, *cq, *sq;
} orc_coef;

/* D = W adj(J) K adj(J)^T / det J, Cv = W alpha adj(J) c, M = W s det J at point q  [MFEM-ext PA qdata] */
static void point_coef(int dim, const orc_coef *cf, int q, double W, double detJ, double A[3][3],
                       double D[3][3], double Cv[3], double *M)
{
    const int ns = dim * (dim + 1) / 2;
    if (cf->use_diff) {
        const double kap = cf->kq ? cf->kq[q] : cf->kappa;
        double K[3][3] = {{0}};
        for (int k = 0, m = 0; k < dim; k++)
            for (int l = k; l < dim; l++, m++) {
                const double v = (cf->kmq ? cf->kmq[(size_t)q * ns + m] : 0.0) + (k == l ? kap : 0.0);
                K[k][l] = K[l][k] = v;
            }
        for (int i = 0; i < dim; i++)
            for (int j = 0; j < dim; j++) {
                double acc = 0.0;
                for (int k = 0; k < dim; k++)
                    for (int l = 0; l < dim; l++) acc += A[i][k] * K[k][l] * A[j][l];
                D[i][j] = W * acc / detJ;
            }
    }
    if (cf->use_conv)
        for (int i = 0; i < dim; i++) {
            double acc = 0.0;
            for (int k = 0; k < dim; k++) acc += A[i][k] * (cf->cq ? cf->cq[(size_t)q * dim + k] : cf->c[k]);
            Cv[i] = W * cf->alpha * acc;
        }
    if (cf->use_mass) *M = W * (cf->sq ? cf->sq[q] : cf->s) * detJ;
}

/* the coefficient set of element e (per-point arrays offset by e * nq) */
static orc_coef coef_of(const orc_coef *cf, int dim, int64_t e, int nq)
{
    orc_coef r = *cf;
    const size_t o = (size_t)e * nq;
    if (cf->kq) r.kq = cf->kq + o;
    if (cf->kmq) r.kmq = cf->kmq + o * (dim * (dim + 1) / 2);
    if (cf->cq) r.cq = cf->cq + o * dim;
    if (cf->sq) r.sq = cf->sq + o;
    return r;
}

/* Element matrix (row = test, col = trial), nd x nd, for element with vertices V. */
static void element_matrix(int dim, int p, const double *V, const orc_coef *cf, int nq,
                           const double *B, const double *G, const double *pts, const double *wts,
                           double *Ae)
{
    const int d1 = p + 1;
    const int nd = (dim == 3) ? d1 * d1 * d1 : d1 * d1;
    double phi[125], gphi[125][3];
    memset(Ae, 0, sizeof(double) * nd * nd);
    const int nqz = (dim == 3) ? nq : 1;
    for (int qz = 0; qz < nqz; qz++)
    for (int qy = 0; qy < nq; qy++)
    for (int qx = 0; qx < nq; qx++) {
        int qi[3] = {qx, qy, qz};
        double xi[3] = {pts[qx], pts[qy], (dim == 3) ? pts[qz] : 0.0};
        double W = wts[qx] * wts[qy] * ((dim == 3) ? wts[qz] : 1.0);
        double x[3], J[3][3], A[3][3];
        q1_map(dim, V, xi, x, J);
        double detJ = adjugate(dim, J, A);
        /* D = W kappa adj adj^T / detJ ; Cv = W alpha adj c ; M = W s detJ   [MFEM-ext PA qdata] */
        double D[3][3] = {{0}}, Cv[3] = {0}, M = 0.0;
        point_coef(dim, cf, qx + nq * (qy + nq * qz), W, detJ, A, D, Cv, &M);
        tensor_basis(dim, p, B, G, qi, phi, gphi);
        for (int j = 0; j < nd; j++) {
            double Dg[3] = {0, 0, 0};
            for (int a = 0; a < dim; a++)
                for (int b = 0; b < dim; b++) Dg[a] += D[a][b] * gphi[j][b];
            double cg = 0.0;
            for (int a = 0; a < dim; a++) cg += Cv[a] * gphi[j][a];
            double rest = cg + M * phi[j];
            for (int i = 0; i < nd; i++) {
                double v = phi[i] * rest;
                for (int a = 0; a < dim; a++) v += gphi[i][a] * Dg[a];
                Ae[i * nd + j] += v;
            }
        }
    }
}

/* CSR of sum_e A_e from element matrices Ae[e][i][j] (row = test dof, col = trial dof) and the
 * element dof map (ParBilinearForm::Assemble + Finalize, SpMat form).  Columns sorted per row;
 * each entry accumulates its contributions in ascending (element, local row, local col) order. */
static orc_csr *csr_from_elements(int nd, int ne, const int *dofmap, int64_t nl, const double *Ae)
{
    /* dof -> (element, local) transpose, element order ascending (deterministic accumulation) */
    int64_t *cnt = (int64_t *)calloc(nl + 1, sizeof(int64_t));
    for (int64_t k = 0; k < (int64_t)ne * nd; k++) cnt[dofmap[k] + 1]++;
    int64_t maxcnt = 0;
    for (int64_t i = 0; i < nl; i++) {
        if (cnt[i + 1] > maxcnt) maxcnt = cnt[i + 1];
        cnt[i + 1] += cnt[i];
    }
    int64_t *fill = (int64_t *)malloc(sizeof(int64_t) * nl);
    memcpy(fill, cnt, sizeof(int64_t) * nl);
    int64_t *el = (int64_t *)malloc(sizeof(int64_t) * (size_t)ne * nd);
    for (int64_t k = 0; k < (int64_t)ne * nd; k++) el[fill[dofmap[k]]++] = k; /* k = e*nd + l */
    free(fill);

    orc_csr *A = (orc_csr *)calloc(1, sizeof(orc_csr));
    A->n = nl;
    A->rp = (int64_t *)calloc(nl + 1, sizeof(int64_t));
    const int64_t maxc = maxcnt * nd;
    /* pass 1: row lengths */
    #pragma omp parallel
    {
        int *buf = (int *)malloc(sizeof(int) * (maxc + 1));
        #pragma omp for schedule(dynamic, 256)
        for (int64_t i = 0; i < nl; i++) {
            int m = 0;
            for (int64_t k = cnt[i]; k < cnt[i + 1]; k++) {
                int64_t e = el[k] / nd;
                for (int l = 0; l < nd; l++) buf[m++] = dofmap[e * nd + l];
            }
            for (int a = 1; a < m; a++) {  /* insertion sort + unique */
                int v = buf[a], b = a - 1;
                while (b >= 0 && buf[b] > v) { buf[b + 1] = buf[b]; b--; }
                buf[b + 1] = v;
            }
            int u = 0;
            for (int a = 0; a < m; a++) if (a == 0 || buf[a] != buf[a - 1]) u++;
            A->rp[i + 1] = u;
        }
        free(buf);
    }
    for (int64_t i = 0; i < nl; i++) A->rp[i + 1] += A->rp[i];
    A->nnz = A->rp[nl];
    A->col = (int32_t *)malloc(sizeof(int32_t) * A->nnz);
    A->val = (double *)calloc(A->nnz, sizeof(double));
    /* pass 2: columns and values */
    #pragma omp parallel
    {
        int *buf = (int *)malloc(sizeof(int) * (maxc + 1));
        #pragma omp for schedule(dynamic, 256)
        for (int64_t i = 0; i < nl; i++) {
            int m = 0;
            for (int64_t k = cnt[i]; k < cnt[i + 1]; k++) {
                int64_t e = el[k] / nd;
                for (int l = 0; l < nd; l++) buf[m++] = dofmap[e * nd + l];
            }
            for (int a = 1; a < m; a++) {
                int v = buf[a], b = a - 1;
                while (b >= 0 && buf[b] > v) { buf[b + 1] = buf[b]; b--; }
                buf[b + 1] = v;
            }
            int64_t base = A->rp[i], u = 0;
            for (int a = 0; a < m; a++) if (a == 0 || buf[a] != buf[a - 1]) A->col[base + u++] = buf[a];
            for (int64_t k = cnt[i]; k < cnt[i + 1]; k++) {
                int64_t e = el[k] / nd;
                int li = (int)(el[k] % nd);
                const double *row = Ae + (size_t)e * nd * nd + (size_t)li * nd;
                for (int l = 0; l < nd; l++) {
                    int cj = dofmap[e * nd + l];
                    int64_t lo = base, hi = base + u - 1;
                    while (lo < hi) {
                        int64_t mid = (lo + hi) >> 1;
                        if (A->col[mid] < cj) lo = mid + 1; else hi = mid;
                    }
                    A->val[lo] += row[l];
                }
            }
        }
        free(buf);
    }
    free(cnt); free(el);
    return A;
}

/* Build the CSR matrix sum_e A_e for tensor (quad/hex) elements. */
/* the same with per-quadrature-point coefficients (NULL arrays: the constants); point order per
 * element: lexicographic tensor points (qx fastest) of the operator rule, as cdfem_quadrature_points */
ORC_API orc_csr *orc_fa_assemble_q(int dim, int p, int ne, const double *verts, const int *dofmap,
                                   int64_t nl, double kappa, const double *kq, const double *kmq, double alpha,
                                   const double *c, const double *cq, double s, const double *sq, int kinds)
{
    const int d1 = p + 1;
    const int nd = (dim == 3) ? d1 * d1 * d1 : d1 * d1;
    const int nv = (dim == 3) ? 8 : 4;
    orc_coef cf = {kappa, alpha, s, {c ? c[0] : 0, c ? c[1] : 0, (c && dim == 3) ? c[2] : 0},
                   (kinds & 1) != 0, (kinds & 2) != 0, (kinds & 4) != 0, kq, kmq, cq, sq};
    /* one shared rule: Diffusion/Convection/Mass coincide on Q1 tensor elements (checked) */
    int nq = orc_rule_npts(0, dim, p);
    if (orc_rule_npts(1, dim, p) != nq || orc_rule_npts(2, dim, p) != nq) return NULL;
    double B[64], G[64], pts[8], wts[8];
    tables(p, nq, B, G, pts, wts);

    double *Ae = (double *)malloc(sizeof(double) * (size_t)ne * nd * nd);
    const int nqe = (dim == 3) ? nq * nq * nq : nq * nq;
    #pragma omp parallel for schedule(static)
    for (int e = 0; e < ne; e++) {
        const orc_coef ce = coef_of(&cf, dim, e, nqe);
        element_matrix(dim, p, verts + (size_t)e * nv * dim, &ce, nq, B, G, pts, wts,
                       Ae + (size_t)e * nd * nd);
    }
    orc_csr *A = csr_from_elements(nd, ne, dofmap, nl, Ae);
    free(Ae);
    return A;
}

ORC_API orc_csr *orc_fa_assemble(int dim, int p, int ne, const double *verts, const int *dofmap,
                                 int64_t nl, double kappa, double alpha, double s, const double *c,
                                 int kinds)
{
    return orc_fa_assemble_q(dim, p, ne, verts, dofmap, nl, kappa, NULL, NULL, alpha, c, NULL, s, NULL, kinds);
}

ORC_API void orc_csr_free(orc_csr *A)
{
    if (!A) return;
    free(A->rp); free(A->col); free(A->val); free(A);
}
ORC_API int64_t orc_csr_n(const orc_csr *A) { return A->n; }
ORC_API int64_t orc_csr_nnz(const orc_csr *A) { return A->nnz; }
ORC_API void orc_csr_export(const orc_csr *A, int64_t *rp, int32_t *col, double *val)
{
    memcpy(rp, A->rp, sizeof(int64_t) * (A->n + 1));
    memcpy(col, A->col, sizeof(int32_t) * A->nnz);
    memcpy(val, A->val, sizeof(double) * A->nnz);
}

/* a CSR from arrays (columns sorted within each row), for matrices the tests build themselves */
ORC_API orc_csr *orc_csr_import(int64_t n, const int64_t *rp, const int32_t *col, const double *val)
{
    orc_csr *A = (orc_csr *)calloc(1, sizeof(orc_csr));
    A->n = n;
    A->nnz = rp[n];
    A->rp = (int64_t *)malloc(sizeof(int64_t) * (n + 1));
    A->col = (int32_t *)malloc(sizeof(int32_t) * (A->nnz ? A->nnz : 1));
    A->val = (double *)malloc(sizeof(double) * (A->nnz ? A->nnz : 1));
    memcpy(A->rp, rp, sizeof(int64_t) * (n + 1));
    memcpy(A->col, col, sizeof(int32_t) * A->nnz);
    memcpy(A->val, val, sizeof(double) * A->nnz);
    return A;
}

ORC_API void orc_csr_spmv(const orc_csr *A, const double *x, double *y)
{
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < A->n; i++) {
        double acc = 0.0;
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; k++) acc += A->val[k] * x[A->col[k]];
        y[i] = acc;
    }
}

/*
 * FormLinearSystem (FA, single rank so P = I):  eliminate essential rows AND columns, diagonal 1,
 *   B = b - A_e X,  B[ess] = X[ess]                                 [MFEM-ext, DIAG_ONE policy]
 * Returns a new matrix; A is not modified.  ess_marker[i] != 0 marks essential dof i.
 */
ORC_API orc_csr *orc_form_linear_system(const orc_csr *A, const int *ess_marker, const double *X,
                                        const double *b, double *B)
{
    orc_csr *Ac = (orc_csr *)calloc(1, sizeof(orc_csr));
    Ac->n = A->n; Ac->nnz = A->nnz;
    Ac->rp = (int64_t *)malloc(sizeof(int64_t) * (A->n + 1));
    Ac->col = (int32_t *)malloc(sizeof(int32_t) * A->nnz);
    Ac->val = (double *)malloc(sizeof(double) * A->nnz);
    memcpy(Ac->rp, A->rp, sizeof(int64_t) * (A->n + 1));
    memcpy(Ac->col, A->col, sizeof(int32_t) * A->nnz);
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < A->n; i++) {
        if (ess_marker[i]) {
            for (int64_t k = A->rp[i]; k < A->rp[i + 1]; k++)
                Ac->val[k] = (A->col[k] == i) ? 1.0 : 0.0;
            B[i] = X[i];
        } else {
            double bi = b[i];
            for (int64_t k = A->rp[i]; k < A->rp[i + 1]; k++) {
                int j = A->col[k];
                if (ess_marker[j]) { bi -= A->val[k] * X[j]; Ac->val[k] = 0.0; }
                else Ac->val[k] = A->val[k];
            }
            B[i] = bi;
        }
    }
    return Ac;
}

ORC_API void orc_csr_diag(const orc_csr *A, double *d)
{
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < A->n; i++) {
        d[i] = 0.0;
        for (int64_t k = A->rp[i]; k < A->rp[i + 1]; k++) if (A->col[k] == i) d[i] = A->val[k];
    }
}

/* ------------------------------------------------------------------------------------------ */
/* Krylov solvers                                                                              */
/* ------------------------------------------------------------------------------------------ */

static double dot(int64_t n, const double *a, const double *b)
{
    double s = 0.0;
    #pragma omp parallel for reduction(+ : s) schedule(static)
    for (int64_t i = 0; i < n; i++) s += a[i] * b[i];
    return s;
}

/*
 * MFEM CGSolver::Mult semantics (iterative_mode = false), optional Jacobi preconditioner
 * z = dinv .* r (OperatorJacobiSmoother / HypreDiagScale).  Convergence when
 * (r, z) <= max(nom0 * rel_tol^2, abs_tol^2).  Pinned by use: mesh_recession_handler.cpp:270-276.
 * An indefinite preconditioner stops the solve unconverged, as CGSolver does [MFEM-ext]: nom0 < 0
 * at iteration 0, betanom < 0 at iteration i (tested before the convergence test).
 * Returns 1 if converged; *iters = final_iter, *final_norm = sqrt(|betanom|).
 */
typedef void (*orc_op_fn)(const void *op, const double *x, double *y);
static void csr_op(const void *op, const double *x, double *y) { orc_csr_spmv((const orc_csr *)op, x, y); }

static int cg_core(orc_op_fn apply, const void *op, int64_t n, const double *dinv, const double *b, double *x,
                   double rel_tol, double abs_tol, int max_iter, int *iters, double *final_norm);

ORC_API int orc_cg(const orc_csr *A, const double *dinv, const double *b, double *x, double rel_tol,
                   double abs_tol, int max_iter, int *iters, double *final_norm)
{
    return cg_core(csr_op, A, A->n, dinv, b, x, rel_tol, abs_tol, max_iter, iters, final_norm);
}

/* the CGSolver loop on any operator y = op(x) */
static int cg_core(orc_op_fn apply, const void *op, int64_t n, const double *dinv, const double *b, double *x,
                   double rel_tol, double abs_tol, int max_iter, int *iters, double *final_norm)
{
    double *r = (double *)malloc(sizeof(double) * n), *d = (double *)malloc(sizeof(double) * n);
    double *z = (double *)malloc(sizeof(double) * n);
    memcpy(r, b, sizeof(double) * n);
    memset(x, 0, sizeof(double) * n);
    if (dinv) { for (int64_t i = 0; i < n; i++) z[i] = dinv[i] * r[i]; memcpy(d, z, sizeof(double) * n); }
    else memcpy(d, r, sizeof(double) * n);
    double nom = dot(n, d, r);
    const double r0 = fmax(nom * rel_tol * rel_tol, abs_tol * abs_tol);
    int converged = 0;
    double betanom = nom;
    *iters = 0;
    if (nom < 0.0) { *final_norm = sqrt(-nom); free(r); free(d); free(z); return 0; }
    if (nom <= r0) { *final_norm = sqrt(nom); free(r); free(d); free(z); return 1; }
    apply(op, d, z);
    double den = dot(n, z, d);
    if (den == 0.0) { *final_norm = sqrt(nom); free(r); free(d); free(z); return 0; }
    int final_iter = max_iter;
    for (int i = 1;;) {
        double alpha = nom / den;
        #pragma omp parallel for schedule(static)
        for (int64_t k = 0; k < n; k++) { x[k] += alpha * d[k]; r[k] -= alpha * z[k]; }
        if (dinv) {
            #pragma omp parallel for schedule(static)
            for (int64_t k = 0; k < n; k++) z[k] = dinv[k] * r[k];
            betanom = dot(n, r, z);
        } else betanom = dot(n, r, r);
        if (betanom < 0.0) { final_iter = i; break; }
        if (betanom <= r0) { converged = 1; final_iter = i; break; }
        if (++i > max_iter) break;
        double beta = betanom / nom;
        const double *src = dinv ? z : r;
        #pragma omp parallel for schedule(static)
        for (int64_t k = 0; k < n; k++) d[k] = src[k] + beta * d[k];
        apply(op, d, z);
        den = dot(n, d, z);
        if (den == 0.0) { final_iter = i; break; }
        nom = betanom;
    }
    *iters = final_iter;
    *final_norm = sqrt(fabs(betanom));
    free(r); free(d); free(z);
    return converged;
}

/*
 * PETSc KSPGMRES semantics [PETSc-ext]: restarted GMRES(m), LEFT preconditioning (Jacobi when
 * dinv != NULL), classical Gram-Schmidt without refinement, Givens-rotation residual estimate,
 * zero initial guess, KSPConvergedDefault on the preconditioned residual norm:
 * converged when rnorm <= max(rtol * rnorm0, atol).  Input/petsc.opts:2-6.
 */
/*
 * ILU(0) [PETSc-ext]: PCILU with zero fill in the natural ordering, no pivoting and no shift (the
 * single-rank meaning of "-pc_type bjacobi -sub_pc_type ilu", Input/petsc_circle.opts:6-8).  IKJ
 * elimination restricted to the pattern of A:
 *   for i: for k < i in row i (ascending): a_ik /= a_kk;  a_ij -= a_ik a_kj for j > k in both rows
 * L (unit diagonal) and U share A's pattern.  Defining property, pinned in tests: (L U)_ij = a_ij
 * for every (i, j) in the pattern.
 */
ORC_API orc_csr *orc_ilu0(const orc_csr *A)
{
    orc_csr *F = (orc_csr *)calloc(1, sizeof(orc_csr));
    F->n = A->n;
    F->nnz = A->nnz;
    F->rp = (int64_t *)malloc(sizeof(int64_t) * (A->n + 1));
    F->col = (int32_t *)malloc(sizeof(int32_t) * A->nnz);
    F->val = (double *)malloc(sizeof(double) * A->nnz);
    memcpy(F->rp, A->rp, sizeof(int64_t) * (A->n + 1));
    memcpy(F->col, A->col, sizeof(int32_t) * A->nnz);
    memcpy(F->val, A->val, sizeof(double) * A->nnz);
    int64_t *diag = (int64_t *)malloc(sizeof(int64_t) * A->n);
    for (int64_t i = 0; i < A->n; i++) {
        diag[i] = -1;
        for (int64_t p = F->rp[i]; p < F->rp[i + 1]; p++)
            if (F->col[p] == i) diag[i] = p;
    }
    for (int64_t i = 0; i < F->n; i++) {
        for (int64_t pk = F->rp[i]; pk < F->rp[i + 1] && F->col[pk] < i; pk++) {
            const int64_t k = F->col[pk];
            const double lik = F->val[pk] / F->val[diag[k]];
            F->val[pk] = lik;
            /* a_ij -= l_ik u_kj for j > k present in row i and row k (sorted merge) */
            int64_t pi = pk + 1, pu = diag[k] + 1;
            while (pi < F->rp[i + 1] && pu < F->rp[k + 1]) {
                if (F->col[pi] < F->col[pu]) pi++;
                else if (F->col[pi] > F->col[pu]) pu++;
                else { F->val[pi] -= lik * F->val[pu]; pi++; pu++; }
            }
        }
    }
    free(diag);
    return F;
}

/* z = (L U)^{-1} r: forward sweep with the unit lower part, backward with the upper part; each
 * row sums in ascending column order */
ORC_API void orc_ilu_solve(const orc_csr *F, const double *r, double *z)
{
    const int64_t n = F->n;
    for (int64_t i = 0; i < n; i++) {
        double v = r[i];
        for (int64_t p = F->rp[i]; p < F->rp[i + 1] && F->col[p] < i; p++) v -= F->val[p] * z[F->col[p]];
        z[i] = v;
    }
    for (int64_t i = n - 1; i >= 0; i--) {
        double v = z[i], d = 1.0;
        for (int64_t p = F->rp[i]; p < F->rp[i + 1]; p++) {
            if (F->col[p] > i) v -= F->val[p] * z[F->col[p]];
            else if (F->col[p] == i) d = F->val[p];
        }
        z[i] = v / d;
    }
}

/* left preconditioner of GMRES: Jacobi (dinv), ILU(0) (ilu) or none; v <- M^{-1} v */
static void gmres_pc(const double *dinv, const orc_csr *ilu, int64_t n, double *v, double *tmp)
{
    if (ilu) {
        memcpy(tmp, v, sizeof(double) * n);
        orc_ilu_solve(ilu, tmp, v);
    } else if (dinv) {
        for (int64_t i = 0; i < n; i++) v[i] *= dinv[i];
    }
}

static int gmres_core(const orc_csr *A, const double *dinv, const orc_csr *ilu, const double *b, double *x,
                      int m, double rtol, double atol, int max_it, int *iters, double *final_norm);

ORC_API int orc_gmres(const orc_csr *A, const double *dinv, const double *b, double *x, int m,
                      double rtol, double atol, int max_it, int *iters, double *final_norm)
{
    return gmres_core(A, dinv, NULL, b, x, m, rtol, atol, max_it, iters, final_norm);
}

ORC_API int orc_gmres_ilu(const orc_csr *A, const orc_csr *ilu, const double *b, double *x, int m,
                          double rtol, double atol, int max_it, int *iters, double *final_norm)
{
    return gmres_core(A, NULL, ilu, b, x, m, rtol, atol, max_it, iters, final_norm);
}

static int gmres_core(const orc_csr *A, const double *dinv, const orc_csr *ilu, const double *b, double *x,
                      int m, double rtol, double atol, int max_it, int *iters, double *final_norm)
{
    const int64_t n = A->n;
    double *tmp = (double *)malloc(sizeof(double) * n);
    double *V = (double *)malloc(sizeof(double) * n * (m + 1));
    double *w = (double *)malloc(sizeof(double) * n);
    double *H = (double *)calloc((size_t)(m + 1) * m, sizeof(double));
    double *cs = (double *)malloc(sizeof(double) * m), *sn = (double *)malloc(sizeof(double) * m);
    double *g = (double *)malloc(sizeof(double) * (m + 1)), *y = (double *)malloc(sizeof(double) * m);
    memset(x, 0, sizeof(double) * n);
    int its = 0, converged = 0, first = 1;
    double ttol = 0.0, res = 0.0;
    for (;;) {
        /* preconditioned initial residual of this cycle: V0 = M^{-1}(b - A x) */
        orc_csr_spmv(A, x, w);
        for (int64_t i = 0; i < n; i++) V[i] = b[i] - w[i];
        gmres_pc(dinv, ilu, n, V, tmp);
        double beta = sqrt(dot(n, V, V));
        res = beta;
        if (first) { ttol = fmax(rtol * beta, atol); first = 0; }
        if (beta <= ttol || beta == 0.0) { converged = 1; break; }
        if (its >= max_it) break;
        for (int64_t i = 0; i < n; i++) V[i] /= beta;
        for (int i = 0; i <= m; i++) g[i] = 0.0;
        g[0] = beta;
        int j, kk = 0;
        for (j = 0; j < m && its < max_it; j++) {
            its++;
            double *vj = V + (size_t)j * n, *vn = V + (size_t)(j + 1) * n;
            orc_csr_spmv(A, vj, w);
            gmres_pc(dinv, ilu, n, w, tmp);
            /* classical Gram-Schmidt: all projections from the same w */
            for (int i = 0; i <= j; i++) H[i * m + j] = dot(n, w, V + (size_t)i * n);
            for (int i = 0; i <= j; i++) {
                const double h = H[i * m + j], *vi = V + (size_t)i * n;
                for (int64_t k = 0; k < n; k++) w[k] -= h * vi[k];
            }
            double hn = sqrt(dot(n, w, w));
            H[(j + 1) * m + j] = hn;
            for (int i = 0; i < j; i++) {
                double a = H[i * m + j], c2 = H[(i + 1) * m + j];
                H[i * m + j] = cs[i] * a + sn[i] * c2;
                H[(i + 1) * m + j] = -sn[i] * a + cs[i] * c2;
            }
            double a = H[j * m + j], c2 = H[(j + 1) * m + j];
            double rr = sqrt(a * a + c2 * c2);
            cs[j] = (rr == 0.0) ? 1.0 : a / rr;
            sn[j] = (rr == 0.0) ? 0.0 : c2 / rr;
            H[j * m + j] = rr;
            H[(j + 1) * m + j] = 0.0;
            g[j + 1] = -sn[j] * g[j];
            g[j] = cs[j] * g[j];
            res = fabs(g[j + 1]);
            kk = j + 1;
            if (hn == 0.0) break;                      /* happy breakdown */
            for (int64_t k = 0; k < n; k++) vn[k] = w[k] / hn;
            if (res <= ttol) break;
        }
        /* x += V_k y_k with H_k y_k = g_k (upper triangular) */
        for (int i = kk - 1; i >= 0; i--) {
            double acc = g[i];
            for (int l = i + 1; l < kk; l++) acc -= H[i * m + l] * y[l];
            y[i] = acc / H[i * m + i];
        }
        for (int i = 0; i < kk; i++) {
            const double *vi = V + (size_t)i * n;
            for (int64_t k = 0; k < n; k++) x[k] += y[i] * vi[k];
        }
        if (res <= ttol) { converged = 1; break; }
        if (its >= max_it) break;
    }
    *iters = its;
    *final_norm = res;
    free(V); free(w); free(H); free(cs); free(sn); free(g); free(y); free(tmp);
    return converged;
}

/* ------------------------------------------------------------------------------------------ */
/* Manufactured solutions, RHS assembly, projection, L2 error                                  */
/* ------------------------------------------------------------------------------------------ */

/*
 * prm[0] = kind:
 *   1: u = sin(n pi x) sin(m pi y) [sin(l pi z)]; f = -kappa Lap u + alpha c.grad u + s u
 *      (linear_convection_diffusion_2D.cpp:159-215; z factor is the 3D extension)
 *   2: u = prod_d g(x_d), g(t) = sum_k a_k t^k, degree p: in the FE space -> exact Galerkin
 *   3: u = sin(t) cos(2(x-.5)^2 + 2(y-.5)^2), f = u_t - alpha Lap u   (diffusion_mms.cpp:136-178)
 *   4: u = (r^2 - 1) cos(2 pi r) on the unit disk, f = -kappa Lap u + c.grad u + s u
 *      (linear_convection_diffusion_2D_circle.cpp:140-215, including its r -> 0 limits)
 * prm: [kind, kappa, s, alpha, c0, c1, c2, n, m, l, t, p, dim]
 */
#define ORC_RAD_ALPHA (2.0 * ORC_PI)   /* kAlpha, _circle.cpp:140 */
#define ORC_RAD_SMALL 1.0e-12          /* kSmallR, _circle.cpp:141 */
static double rad_u(double r) { return (r * r - 1.0) * cos(ORC_RAD_ALPHA * r); }
static double rad_ur(double r)
{
    return 2.0 * r * cos(ORC_RAD_ALPHA * r) - ORC_RAD_ALPHA * (r * r - 1.0) * sin(ORC_RAD_ALPHA * r);
}
static double rad_urr(double r)
{
    return 2.0 * cos(ORC_RAD_ALPHA * r) - 4.0 * ORC_RAD_ALPHA * r * sin(ORC_RAD_ALPHA * r) -
           ORC_RAD_ALPHA * ORC_RAD_ALPHA * (r * r - 1.0) * cos(ORC_RAD_ALPHA * r);
}
static double rad_lap(double r)
{
    if (r > ORC_RAD_SMALL) return rad_urr(r) + rad_ur(r) / r;
    return 2.0 * (2.0 + ORC_RAD_ALPHA * ORC_RAD_ALPHA);  /* lim r->0, _circle.cpp:168-169 */
}
static void poly1d(int p, double t, double *g, double *dg, double *d2g)
{
    /* fixed, non-symmetric coefficients: a_k = (k + 1) / (k + 2) * (-1)^k + 0.25 */
    *g = 0; *dg = 0; *d2g = 0;
    for (int k = 0; k <= p; k++) {
        double a = (k + 1.0) / (k + 2.0) * ((k & 1) ? -1.0 : 1.0) + 0.25;
        *g += a * pow(t, k);
        if (k >= 1) *dg += a * k * pow(t, k - 1);
        if (k >= 2) *d2g += a * k * (k - 1) * pow(t, k - 2);
    }
}

/* kind 5: the erfc solution of c_t + c_x = c_xx / Pe on x > 0 with c(0, t) = 1, c(x, 0) = 0
 * (linear_convection_diffusion_1D.cpp:128-166; exp(a) erfc(b) through the asymptotic series past
 * b = 26, :128-144).  Pe in the kappa slot, t in the t slot; no forcing. */
static double exp_times_erfc(double a, double b)
{
    if (b > 26.0) {
        const double ib = 1.0 / b, ib2 = ib * ib;
        const double er = ib / sqrt(ORC_PI) * (1.0 - 0.5 * ib2 + 0.75 * ib2 * ib2);
        const double expo = a - b * b;
        if (expo < -745.0) return 0.0;
        if (expo > 709.0) return INFINITY;
        return exp(expo) * er;
    }
    if (a > 709.0) return INFINITY;
    return exp(a) * erfc(b);
}
static double erfc_profile(double x, double t, double pe)
{
    if (t <= 0.0) return 0.0;
    const double diff = t / pe, root = sqrt(diff);
    const double a1 = (x - t) / (2.0 * root), a2 = (x + t) / (2.0 * root);
    const double gauss = -((x - t) * (x - t)) / (4.0 * diff);
    const double c = 0.5 * erfc(a1) + sqrt(t * pe / ORC_PI) * exp(gauss) -
                     0.5 * (1.0 + pe * x + pe * t) * exp_times_erfc(pe * x, a2);
    return isfinite(c) ? c : 0.0;
}

ORC_API double orc_mms_u(const double *prm, const double *x)
{
    int kind = (int)prm[0], dim = (int)prm[12];
    if (kind == 1) {
        double u = sin(prm[7] * ORC_PI * x[0]) * sin(prm[8] * ORC_PI * x[1]);
        if (dim == 3) u *= sin(prm[9] * ORC_PI * x[2]);
        return u;
    }
    if (kind == 2) {
        double u = 1.0, g, dg, d2g;
        for (int d = 0; d < dim; d++) { poly1d((int)prm[11], x[d], &g, &dg, &d2g); u *= g; }
        return u;
    }
    if (kind == 3) {
        double dx = x[0] - 0.5, dy = x[1] - 0.5;
        return sin(prm[10]) * cos(2.0 * dx * dx + 2.0 * dy * dy);
    }
    if (kind == 4) return rad_u(sqrt(x[0] * x[0] + x[1] * x[1]));
    if (kind == 5) return erfc_profile(x[0], prm[10], prm[1]);
    return 0.0;
}

ORC_API double orc_mms_f(const double *prm, const double *x)
{
    int kind = (int)prm[0], dim = (int)prm[12];
    double kappa = prm[1], s = prm[2], alpha = prm[3];
    const double *c = prm + 4;
    if (kind == 1) {
        double k[3] = {prm[7] * ORC_PI, prm[8] * ORC_PI, prm[9] * ORC_PI};
        double sv[3], cv[3];
        for (int d = 0; d < 3; d++) { sv[d] = sin(k[d] * x[d]); cv[d] = cos(k[d] * x[d]); }
        if (dim == 2) {
            /* linear_convection_diffusion_2D.cpp:198-205 (alpha = 1 there) */
            double diff = kappa * (k[0] * k[0] + k[1] * k[1]) * sv[0] * sv[1];
            double conv = c[0] * k[0] * cv[0] * sv[1] + c[1] * k[1] * sv[0] * cv[1];
            return diff + alpha * conv + s * sv[0] * sv[1];
        }
        double u = sv[0] * sv[1] * sv[2];
        double diff = kappa * (k[0] * k[0] + k[1] * k[1] + k[2] * k[2]) * u;
        double conv = c[0] * k[0] * cv[0] * sv[1] * sv[2] + c[1] * k[1] * sv[0] * cv[1] * sv[2]
                    + c[2] * k[2] * sv[0] * sv[1] * cv[2];
        return diff + alpha * conv + s * u;
    }
    if (kind == 2) {
        double g[3], dg[3], d2g[3];
        for (int d = 0; d < dim; d++) poly1d((int)prm[11], x[d], &g[d], &dg[d], &d2g[d]);
        double u = 1, lap = 0, cg = 0;
        for (int d = 0; d < dim; d++) u *= g[d];
        for (int d = 0; d < dim; d++) {
            double t2 = d2g[d], t1 = dg[d];
            for (int e = 0; e < dim; e++) if (e != d) { t2 *= g[e]; t1 *= g[e]; }
            lap += t2; cg += c[d] * t1;
        }
        return -kappa * lap + alpha * cg + s * u;
    }
    if (kind == 3) {
        double t = prm[10], dx = x[0] - 0.5, dy = x[1] - 0.5;
        double r2 = dx * dx + dy * dy, q = 2.0 * r2;
        double ut = cos(t) * cos(q);
        double lap = sin(t) * (-16.0 * r2 * cos(q) - 8.0 * sin(q));
        return ut - alpha * lap;
    }
    if (kind == 4) {  /* _circle.cpp:191-214 (alpha = 1 there) */
        const double r = sqrt(x[0] * x[0] + x[1] * x[1]);
        double ux = 0.0, uy = 0.0;
        if (r > ORC_RAD_SMALL) {
            const double sc = rad_ur(r) / r;
            ux = sc * x[0];
            uy = sc * x[1];
        }
        return -kappa * rad_lap(r) + alpha * (c[0] * ux + c[1] * uy) + s * rad_u(r);
    }
    return 0.0;
}

/* b_i = sum_e sum_q W detJ f(x_q) phi_i(xi_q), DomainLFIntegrator default order 2p. */
ORC_API void orc_lf_assemble(int dim, int p, int ne, const double *verts, const int *dofmap,
                             int64_t nl, const double *prm, double *b)
{
    const int d1 = p + 1;
    const int nd = (dim == 3) ? d1 * d1 * d1 : d1 * d1;
    const int nv = (dim == 3) ? 8 : 4;
    const int nq = orc_rule_npts(3, dim, p);
    double B[64], G[64], pts[8], wts[8];
    tables(p, nq, B, G, pts, wts);
    double *be = (double *)malloc(sizeof(double) * (size_t)ne * nd);
    #pragma omp parallel for schedule(static)
    for (int e = 0; e < ne; e++) {
        double phi[125], gphi[125][3];
        double *out = be + (size_t)e * nd;
        for (int l = 0; l < nd; l++) out[l] = 0.0;
        const int nqz = (dim == 3) ? nq : 1;
        for (int qz = 0; qz < nqz; qz++)
        for (int qy = 0; qy < nq; qy++)
        for (int qx = 0; qx < nq; qx++) {
            int qi[3] = {qx, qy, qz};
            double xi[3] = {pts[qx], pts[qy], (dim == 3) ? pts[qz] : 0.0};
            double W = wts[qx] * wts[qy] * ((dim == 3) ? wts[qz] : 1.0);
            double x[3], J[3][3], A[3][3];
            q1_map(dim, verts + (size_t)e * nv * dim, xi, x, J);
            double detJ = adjugate(dim, J, A);
            double fw = W * detJ * orc_mms_f(prm, x);
            tensor_basis(dim, p, B, G, qi, phi, gphi);
            for (int l = 0; l < nd; l++) out[l] += fw * phi[l];
        }
    }
    memset(b, 0, sizeof(double) * nl);
    for (int64_t k = 0; k < (int64_t)ne * nd; k++) b[dofmap[k]] += be[k];
    free(be);
}

/* Physical coordinates of every L-dof (GLL node images); used for nodal projection. */
ORC_API void orc_dof_coords(int dim, int p, int ne, const double *verts, const int *dofmap,
                            double *xyz)
{
    const int d1 = p + 1;
    const int nd = (dim == 3) ? d1 * d1 * d1 : d1 * d1;
    const int nv = (dim == 3) ? 8 : 4;
    double nodes[16];
    orc_gll_nodes(p, nodes);
    #pragma omp parallel for schedule(static)
    for (int e = 0; e < ne; e++)
        for (int l = 0; l < nd; l++) {
            double xi[3] = {nodes[l % d1], nodes[(l / d1) % d1], (dim == 3) ? nodes[l / (d1 * d1)] : 0};
            double x[3], J[3][3];
            q1_map(dim, verts + (size_t)e * nv * dim, xi, x, J);
            for (int k = 0; k < dim; k++) xyz[(size_t)dofmap[(size_t)e * nd + l] * dim + k] = x[k];
        }
}

/* ||u_h - u||_{L2} with the driver's rule order max(2, 2p+3)  (linear_convection_diffusion_2D.cpp:383-390). */
ORC_API double orc_l2_error(int dim, int p, int ne, const double *verts, const int *dofmap,
                            const double *u, const double *prm, int exact_zero)
{
    const int d1 = p + 1;
    const int nd = (dim == 3) ? d1 * d1 * d1 : d1 * d1;
    const int nv = (dim == 3) ? 8 : 4;
    const int nq = orc_rule_npts(4, dim, p);
    double B[64], G[64], pts[8], wts[8];
    tables(p, nq, B, G, pts, wts);
    double err = 0.0;
    #pragma omp parallel for reduction(+ : err) schedule(static)
    for (int e = 0; e < ne; e++) {
        double phi[125], gphi[125][3];
        const int nqz = (dim == 3) ? nq : 1;
        for (int qz = 0; qz < nqz; qz++)
        for (int qy = 0; qy < nq; qy++)
        for (int qx = 0; qx < nq; qx++) {
            int qi[3] = {qx, qy, qz};
            double xi[3] = {pts[qx], pts[qy], (dim == 3) ? pts[qz] : 0.0};
            double W = wts[qx] * wts[qy] * ((dim == 3) ? wts[qz] : 1.0);
            double x[3], J[3][3], A[3][3];
            q1_map(dim, verts + (size_t)e * nv * dim, xi, x, J);
            double detJ = adjugate(dim, J, A);
            tensor_basis(dim, p, B, G, qi, phi, gphi);
            double uh = 0.0;
            for (int l = 0; l < nd; l++) uh += u[dofmap[(size_t)e * nd + l]] * phi[l];
            double ex = exact_zero ? 0.0 : orc_mms_u(prm, x);
            err += W * detJ * (uh - ex) * (uh - ex);
        }
    }
    return sqrt(err);
}

/* ------------------------------------------------------------------------------------------ */
/* CPU element-by-element apply (matrix-free, no CSR; independent of the GPU algorithm)          */
/* ------------------------------------------------------------------------------------------ */

/*
 * qdata per quadrature point (element-major, q lexicographic qx fastest), 10 (3D) / 6 (2D) comps:
 *   D (sym, row-major upper: 00 01 02 11 12 22 | 2D: 00 01 11), Cv (dim), M (1)
 *   D = W kappa adj(J) adj(J)^T / detJ, Cv = W alpha adj(J) c, M = W s detJ     [MFEM-ext PA]
 * y = A x computed element by element with the full tensor basis (no sum factorization:
 * the CPU check must not share the GPU kernel's algorithm).
 */
ORC_API void orc_ebe_mult(int dim, int p, int ne, const double *verts, const int *dofmap,
                         int64_t nl, double kappa, double alpha, double s, const double *c,
                         int kinds, const double *x, double *y)
{
    const int d1 = p + 1;
    const int nd = (dim == 3) ? d1 * d1 * d1 : d1 * d1;
    const int nv = (dim == 3) ? 8 : 4;
    const int nq = orc_rule_npts(0, dim, p);
    orc_coef cf = {kappa, alpha, s, {c ? c[0] : 0, c ? c[1] : 0, (c && dim == 3) ? c[2] : 0},
                   (kinds & 1) != 0, (kinds & 2) != 0, (kinds & 4) != 0, NULL, NULL, NULL, NULL};
    double B[64], G[64], pts[8], wts[8];
    tables(p, nq, B, G, pts, wts);
    double *ye = (double *)malloc(sizeof(double) * (size_t)ne * nd);
    #pragma omp parallel for schedule(static)
    for (int e = 0; e < ne; e++) {
        double Ae[125 * 125];
        double *out = ye + (size_t)e * nd;
        element_matrix(dim, p, verts + (size_t)e * nv * dim, &cf, nq, B, G, pts, wts, Ae);
        for (int i = 0; i < nd; i++) {
            double acc = 0.0;
            for (int j = 0; j < nd; j++) acc += Ae[i * nd + j] * x[dofmap[(size_t)e * nd + j]];
            out[i] = acc;
        }
    }
    memset(y, 0, sizeof(double) * nl);
    for (int64_t k = 0; k < (int64_t)ne * nd; k++) y[dofmap[k]] += ye[k];
    free(ye);
}

ORC_API int orc_num_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

ORC_API void orc_set_num_threads(int n)
{
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* Pin the n OpenMP threads of the next parallel regions: thread t runs on cpus[t] only (the CPU
 * baseline's timing stability on a shared host; the calling thread is pinned too, and the caller
 * restores its own mask afterwards).  Returns the number of threads pinned. */
ORC_API int orc_pin_threads(const int *cpus, int n)
{
#ifdef _OPENMP
    int pinned = 0;
    omp_set_num_threads(n);
    #pragma omp parallel num_threads(n) reduction(+ : pinned)
    {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(cpus[omp_get_thread_num()], &set);
        pinned += sched_setaffinity(0, sizeof set, &set) == 0;
    }
    return pinned;
#else
    (void)cpus;
    (void)n;
    return 0;
#endif
}

/* ------------------------------------------------------------------------------------------ */
/* Simplex elements: BASELINE config C4 (unstructured tetrahedra, FA CSR + GMRES(30)/Jacobi,     */
/* the reference's own solver path: linear_convection_diffusion_2D.cpp:339,364-375,              */
/* Input/petsc.opts:2-6).  H1 P1/P2 Lagrange (MFEM H1_FECollection on simplices: nodal, vertices  */
/* then edge midpoints), affine geometry.                                                       */
/* ------------------------------------------------------------------------------------------ */

ORC_API int orc_simplex_nd(int dim, int p)
{
    if (p == 1) return dim + 1;
    if (p == 2) return (dim + 1) * (dim + 2) / 2;
    if (p == 3 && dim == 2) return 10;
    return -1;
}

static const int kEdge3[6][2] = {{0, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 3}};
static const int kEdge2[3][2] = {{0, 1}, {0, 2}, {1, 2}};

/* P3 triangle, MFEM H1_FECollection(3, 2) (BasisType::GaussLobatto): nodes = vertices, the two
 * interior GLL points of each edge (0,1), (0,2), (1,2) along a -> b, the centroid.  The nodal
 * basis is solved in the space spanned by lambda_1^a lambda_2^b (a + b <= 3). */
static double p3_coef[10][10];  /* phi_i = sum_k p3_coef[k][i] m_k */
static int p3_ready = 0;

static void p3_mono(const double *xi, double *m, double *m1, double *m2)
{
    /* m_k = l1^a l2^b with l1 = xi_0, l2 = xi_1; derivatives w.r.t. xi_0, xi_1 */
    int k = 0;
    for (int a = 0; a <= 3; a++)
        for (int b = 0; a + b <= 3; b++, k++) {
            m[k] = pow(xi[0], a) * pow(xi[1], b);
            m1[k] = a ? a * pow(xi[0], a - 1) * pow(xi[1], b) : 0.0;
            m2[k] = b ? b * pow(xi[0], a) * pow(xi[1], b - 1) : 0.0;
        }
}

static void p3_init(void)
{
    if (p3_ready) return;
    const double g = 0.5 * (1.0 - 1.0 / sqrt(5.0));
    const double V3[3][2] = {{0, 0}, {1, 0}, {0, 1}};
    double X[10][2];
    for (int v = 0; v < 3; v++) { X[v][0] = V3[v][0]; X[v][1] = V3[v][1]; }
    for (int e = 0; e < 3; e++)
        for (int k = 0; k < 2; k++) {
            const double t = k == 0 ? g : 1.0 - g;
            for (int d = 0; d < 2; d++)
                X[3 + 2 * e + k][d] = V3[kEdge2[e][0]][d] + t * (V3[kEdge2[e][1]][d] - V3[kEdge2[e][0]][d]);
        }
    X[9][0] = X[9][1] = 1.0 / 3.0;
    /* solve V c_i = e_i for all i: V[r][k] = m_k(X_r) */
    double M[10][20];
    for (int r = 0; r < 10; r++) {
        double m[10], m1[10], m2[10];
        p3_mono(X[r], m, m1, m2);
        for (int k = 0; k < 10; k++) M[r][k] = m[k];
        for (int k = 0; k < 10; k++) M[r][10 + k] = (r == k);
    }
    for (int c = 0; c < 10; c++) {
        int pr = c;
        for (int r = c + 1; r < 10; r++) if (fabs(M[r][c]) > fabs(M[pr][c])) pr = r;
        for (int k = 0; k < 20; k++) { double t = M[c][k]; M[c][k] = M[pr][k]; M[pr][k] = t; }
        const double d = M[c][c];
        for (int k = 0; k < 20; k++) M[c][k] /= d;
        for (int r = 0; r < 10; r++) if (r != c) {
            const double f = M[r][c];
            for (int k = 0; k < 20; k++) M[r][k] -= f * M[c][k];
        }
    }
    for (int k = 0; k < 10; k++)
        for (int i = 0; i < 10; i++) p3_coef[k][i] = M[k][10 + i];
    p3_ready = 1;
}

/* Collapsed (Duffy) tensor Gauss-Legendre rule on the reference simplex (vertices 0, e_1 .. e_d),
 * n points per direction, exact for polynomial degree 2n - dim:
 *   xi_1 = u, xi_2 = (1-u) v [, xi_3 = (1-u)(1-v) w],  W = w_u w_v [w_w] (1-u)^(d-1) [(1-v)].
 * Point q = (iu * n + iv) [* n + iw]. Parity is unpinned vs MFEM's simplex rules:
 * for constant coefficients on affine elements any rule exact to degree 2p gives the same
 * matrix, and this one is exact to degree 2p + 1 with n = p + 2 in 3D. */
ORC_API int orc_simplex_rule(int dim, int n, double *xi, double *w)
{
    double x[16], wx[16];
    if (n < 1 || n > 16) return -1;
    orc_gauss_legendre(n, x, wx);
    const int nq = (dim == 3) ? n * n * n : n * n;
    for (int q = 0; q < nq; q++) {
        int iu, iv, iw = 0;
        if (dim == 3) { iu = q / (n * n); iv = (q / n) % n; iw = q % n; }
        else { iu = q / n; iv = q % n; }
        const double u = x[iu], v = x[iv];
        if (dim == 3) {
            const double t = x[iw];
            xi[q * 3 + 0] = u;
            xi[q * 3 + 1] = (1.0 - u) * v;
            xi[q * 3 + 2] = (1.0 - u) * (1.0 - v) * t;
            w[q] = wx[iu] * wx[iv] * wx[iw] * (1.0 - u) * (1.0 - u) * (1.0 - v);
        } else {
            xi[q * 2 + 0] = u;
            xi[q * 2 + 1] = (1.0 - u) * v;
            w[q] = wx[iu] * wx[iv] * (1.0 - u);
        }
    }
    return nq;
}

/* MFEM's tabulated simplex rules, IntRules.Get(TRIANGLE, order <= 9) / (TETRAHEDRON, order <= 6)
 * [MFEM-ext intrules.cpp], as generated and verified by tools/simplex_rules.py (symmetric orbits with
 * the published parameters, refined to double precision on the moment equations).  Beyond the
 * tables: the collapsed rule exact to that order.  Returns the point count. */
#include "simplex_rules.inc"

ORC_API int orc_simplex_rule_order(int dim, int order, double *xi, double *w)
{
    static const double *tri[] = {k_tri1, k_tri1, k_tri2, k_tri3, k_tri4, k_tri5, k_tri6, k_tri7, k_tri8, k_tri9};
    static const int ntri[] = {1, 1, 3, 4, 6, 7, 12, 12, 16, 19};
    static const double *tet[] = {k_tet1, k_tet1, k_tet2, k_tet3, k_tet4, k_tet5, k_tet6};
    static const int ntet[] = {1, 1, 4, 5, 11, 14, 24};
    if (order < 0) order = 0;
    const double *t = NULL;
    int n = 0;
    if (dim == 2 && order <= 9) { t = tri[order]; n = ntri[order]; }
    else if (dim == 3 && order <= 6) { t = tet[order]; n = ntet[order]; }
    else return orc_simplex_rule(dim, (order + dim) / 2 + 1, xi, w);
    for (int q = 0; q < n; q++) {
        for (int k = 0; k < dim; k++) xi[q * dim + k] = t[q * (dim + 1) + k];
        w[q] = t[q * (dim + 1) + dim];
    }
    return n;
}

/* Reference basis at xi: phi[nd], dphi[nd][dim] (d/dxi_k), barycentric lambda_0 = 1 - sum xi.
 * Local order: vertices 0..dim, then (P2) edges (0,1),(0,2),(0,3),(1,2),(1,3),(2,3) [2D: (0,1),
 * (0,2),(1,2)]. */

static void simplex_basis(int dim, int p, const double *xi, double *phi, double *dphi)
{
    if (dim == 2 && p == 3) {
        double m[10], m1[10], m2[10];
        p3_mono(xi, m, m1, m2);
        for (int i = 0; i < 10; i++) {
            double v = 0.0, gx = 0.0, gy = 0.0;
            for (int k = 0; k < 10; k++) {
                v += p3_coef[k][i] * m[k];
                gx += p3_coef[k][i] * m1[k];
                gy += p3_coef[k][i] * m2[k];
            }
            phi[i] = v;
            dphi[i * 2] = gx;
            dphi[i * 2 + 1] = gy;
        }
        return;
    }
    double lam[4], dlam[4][3];  /* d lambda_a / d xi_k */
    lam[0] = 1.0;
    for (int k = 0; k < dim; k++) lam[0] -= xi[k];
    for (int k = 0; k < dim; k++) dlam[0][k] = -1.0;
    for (int a = 1; a <= dim; a++) {
        lam[a] = xi[a - 1];
        for (int k = 0; k < dim; k++) dlam[a][k] = (k == a - 1) ? 1.0 : 0.0;
    }
    if (p == 1) {
        for (int a = 0; a <= dim; a++) {
            phi[a] = lam[a];
            for (int k = 0; k < dim; k++) dphi[a * dim + k] = dlam[a][k];
        }
        return;
    }
    for (int a = 0; a <= dim; a++) {
        phi[a] = lam[a] * (2.0 * lam[a] - 1.0);
        for (int k = 0; k < dim; k++) dphi[a * dim + k] = (4.0 * lam[a] - 1.0) * dlam[a][k];
    }
    const int ne = dim == 3 ? 6 : 3;
    for (int e = 0; e < ne; e++) {
        const int a = dim == 3 ? kEdge3[e][0] : kEdge2[e][0], b = dim == 3 ? kEdge3[e][1] : kEdge2[e][1];
        const int l = dim + 1 + e;
        phi[l] = 4.0 * lam[a] * lam[b];
        for (int k = 0; k < dim; k++) dphi[l * dim + k] = 4.0 * (lam[a] * dlam[b][k] + lam[b] * dlam[a][k]);
    }
}

/* Kuhn (Freudenthal) subdivision of the n^dim cube grid of [0,1]^dim: every cube (square) splits
 * into dim! simplices v0 = corner, v_{k+1} = v_k + e_{pi(k)} for each axis permutation pi;
 * odd permutations swap the last two vertices so every element has det J > 0.  Element order:
 * cube-major (lexicographic), then permutation in lexicographic order.  Dofs: the lattice
 * (p n + 1)^dim numbered lexicographically (P2 edge midpoints are the odd lattice points, each on
 * exactly one Kuhn edge).  perturb moves interior vertices as orc_mesh_box does.
 * Returns 0, or -1 if a perturbed element is inverted. */
static const int kPerm3[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
static const int kPerm3Odd[6] = {0, 1, 1, 0, 0, 1};
static const int kPerm2[2][2] = {{0, 1}, {1, 0}};

ORC_API void orc_mesh_kuhn_sizes(int dim, int n, int p, int *ne, int64_t *nl)
{
    const int64_t L = (int64_t)p * n + 1;
    *ne = (dim == 3) ? 6 * n * n * n : 2 * n * n;
    *nl = (dim == 3) ? L * L * L : L * L;
}

ORC_API int orc_mesh_kuhn(int dim, int n, int p, double perturb, double *verts, int *dofmap, int *bdr)
{
    const int nsub = dim == 3 ? 6 : 2, nv = dim + 1, nd = orc_simplex_nd(dim, p);
    const int64_t L = (int64_t)p * n + 1;
    const int ncube = dim == 3 ? n * n * n : n * n;
    const double h = 1.0 / n;
    int bad = 0;
    for (int cidx = 0; cidx < ncube; cidx++) {
        const int c[3] = {cidx % n, (cidx / n) % n, dim == 3 ? cidx / (n * n) : 0};
        for (int s = 0; s < nsub; s++) {
            const int e = cidx * nsub + s;
            int V[4][3] = {{0}};
            for (int k = 0; k < 3; k++) V[0][k] = c[k];
            for (int k = 0; k < dim; k++) {
                const int ax = dim == 3 ? kPerm3[s][k] : kPerm2[s][k];
                for (int m = 0; m < 3; m++) V[k + 1][m] = V[k][m] + (m == ax);
            }
            const int odd = dim == 3 ? kPerm3Odd[s] : (s == 1);
            if (odd)
                for (int m = 0; m < 3; m++) { int t = V[dim][m]; V[dim][m] = V[dim - 1][m]; V[dim - 1][m] = t; }
            double X[4][3] = {{0}};
            for (int v = 0; v < nv; v++) {
                int interior = 1;
                for (int k = 0; k < dim; k++) {
                    X[v][k] = V[v][k] * h;
                    interior = interior && V[v][k] > 0 && V[v][k] < n;
                }
                if (perturb > 0.0 && interior) {
                    uint64_t id = (uint64_t)V[v][0] + (uint64_t)(n + 1) * ((uint64_t)V[v][1] + (uint64_t)(n + 1) * V[v][2]);
                    for (int k = 0; k < dim; k++) X[v][k] += perturb * h * hash_unit(3 * id + k);
                }
                for (int k = 0; k < dim; k++) verts[((size_t)e * nv + v) * dim + k] = X[v][k];
            }
            double J[3][3] = {{0}};
            for (int k = 0; k < dim; k++)
                for (int m = 0; m < dim; m++) J[k][m] = X[m + 1][k] - X[0][k];
            double A[3][3];
            if (adjugate(dim, J, A) <= 0.0) bad = 1;
            for (int l = 0; l < nd; l++) {
                int G[3] = {0, 0, 0};
                if (l < nv) {
                    for (int m = 0; m < 3; m++) G[m] = p * V[l][m];
                } else {
                    const int ed = l - nv;
                    const int a = dim == 3 ? kEdge3[ed][0] : kEdge2[ed][0], b = dim == 3 ? kEdge3[ed][1] : kEdge2[ed][1];
                    for (int m = 0; m < 3; m++) G[m] = V[a][m] + V[b][m];  /* p = 2: midpoint */
                }
                dofmap[(size_t)e * nd + l] = (int)(G[0] + L * (G[1] + L * G[2]));
            }
        }
    }
    const int64_t nl = dim == 3 ? L * L * L : L * L;
    for (int64_t i = 0; i < nl; i++) {
        const int64_t gx = i % L, gy = (i / L) % L, gz = i / (L * L);
        int on = gx == 0 || gx == L - 1 || gy == 0 || gy == L - 1;
        if (dim == 3) on = on || gz == 0 || gz == L - 1;
        bdr[i] = on;
    }
    return bad ? -1 : 0;
}

/* Element matrix of an affine simplex (same integrand as element_matrix: D = W kappa adj adj^T /
 * det J, C = W alpha adj c, M = W s det J on reference gradients). */
static void simplex_element_matrix(int dim, int p, const double *V, const orc_coef *cf, int nq,
                                   const double *xi, const double *wq, double *Ae)
{
    const int nd = orc_simplex_nd(dim, p);
    double J[3][3] = {{0}}, A[3][3];
    for (int k = 0; k < dim; k++)
        for (int m = 0; m < dim; m++) J[k][m] = V[(m + 1) * dim + k] - V[k];
    const double detJ = adjugate(dim, J, A);
    double phi[10], dphi[30];
    for (int q = 0; q < nq; q++) {  /* accumulates into Ae */
        const double W = wq[q];
        double D[3][3] = {{0}}, Cv[3] = {0}, M = 0.0;
        point_coef(dim, cf, q, W, detJ, A, D, Cv, &M);
        simplex_basis(dim, p, xi + (size_t)q * dim, phi, dphi);
        for (int j = 0; j < nd; j++) {
            double Dg[3] = {0, 0, 0}, cg = 0.0;
            for (int a = 0; a < dim; a++) {
                for (int b = 0; b < dim; b++) Dg[a] += D[a][b] * dphi[j * dim + b];
                cg += Cv[a] * dphi[j * dim + a];
            }
            const double rest = cg + M * phi[j];
            for (int i = 0; i < nd; i++) {
                double v = phi[i] * rest;
                for (int a = 0; a < dim; a++) v += dphi[i * dim + a] * Dg[a];
                Ae[i * nd + j] += v;
            }
        }
    }
}

/* Integration orders of the simplex integrators [MFEM-ext fem/bilininteg.cpp GetRule, affine
 * simplices: Trans.OrderW() = 0, Trans.Order() = 1, Trans.OrderGrad(Pk) = p - 1]:
 *   DiffusionIntegrator   trial + test - 2          = 2p - 2  (FunctionSpace::Pk)
 *   ConvectionIntegrator  OrderGrad + Order + test  = 2p
 *   MassIntegrator        trial + test + OrderW     = 2p
 * each on MFEM's tabulated rule of that order (orc_simplex_rule_order). */
ORC_API int orc_simplex_integrator_order(int p, int kind)
{
    return kind == 1 ? (2 * p - 2 > 0 ? 2 * p - 2 : 0) : 2 * p;
}

/* FA CSR of the convection-diffusion-reaction form on P1-P3 simplices: the diffusion part on its
 * rule (order 2p - 2), convection and mass on theirs (order 2p); per-point coefficient arrays are
 * element-major in the point order of the rule of the integrator they belong to (kq, kmq: diffusion;
 * cq: convection; sq: mass). */
ORC_API orc_csr *orc_fa_assemble_simplex_q(int dim, int p, int ne, const double *verts, const int *dofmap,
                                           int64_t nl, double kappa, const double *kq, const double *kmq,
                                           double alpha, const double *c, const double *cq, double s,
                                           const double *sq, int kinds)
{
    p3_init();
    const int nd = orc_simplex_nd(dim, p);
    if (nd < 0 || (dim != 2 && dim != 3)) return NULL;
    const orc_coef cf = {kappa, alpha, s, {c ? c[0] : 0, c ? c[1] : 0, (c && dim == 3) ? c[2] : 0},
                         (kinds & 1) != 0, (kinds & 2) != 0, (kinds & 4) != 0, kq, kmq, cq, sq};
    orc_coef cd = cf, ccm = cf;  /* diffusion part / convection + mass part */
    cd.use_conv = cd.use_mass = 0;
    ccm.use_diff = 0;
    double xd[64 * 3], wd[64], xc[64 * 3], wc[64];
    const int nqd = orc_simplex_rule_order(dim, orc_simplex_integrator_order(p, 1), xd, wd);
    const int nqc = orc_simplex_rule_order(dim, orc_simplex_integrator_order(p, 4), xc, wc);
    double *Ae = (double *)calloc((size_t)ne * nd * nd, sizeof(double));
    #pragma omp parallel for schedule(static)
    for (int e = 0; e < ne; e++) {
        const double *V = verts + (size_t)e * (dim + 1) * dim;
        if (cd.use_diff) {
            const orc_coef ce = coef_of(&cd, dim, e, nqd);
            simplex_element_matrix(dim, p, V, &ce, nqd, xd, wd, Ae + (size_t)e * nd * nd);
        }
        if (ccm.use_conv || ccm.use_mass) {
            const orc_coef ce = coef_of(&ccm, dim, e, nqc);
            simplex_element_matrix(dim, p, V, &ce, nqc, xc, wc, Ae + (size_t)e * nd * nd);
        }
    }
    orc_csr *A = csr_from_elements(nd, ne, dofmap, nl, Ae);
    free(Ae);
    return A;
}

ORC_API orc_csr *orc_fa_assemble_simplex(int dim, int p, int ne, const double *verts, const int *dofmap,
                                         int64_t nl, double kappa, double alpha, double s, const double *c,
                                         int kinds)
{
    return orc_fa_assemble_simplex_q(dim, p, ne, verts, dofmap, nl, kappa, NULL, NULL, alpha, c, NULL, s, NULL,
                                     kinds);
}

/* DomainLF b_i = int f phi_i and ||u_h - u||_L2 on affine simplices with the MMS data of
 * orc_mms_f / orc_mms_u; rules: MFEM's simplex rules of order 2p (LF) and max(2, 2p + 3) (error). */
static void simplex_point(int dim, const double *V, const double *xi, double *x, double *det)
{
    double J[3][3] = {{0}}, A[3][3];
    for (int k = 0; k < dim; k++) {
        x[k] = V[k];
        for (int m = 0; m < dim; m++) {
            J[k][m] = V[(m + 1) * dim + k] - V[k];
            x[k] += J[k][m] * xi[m];
        }
    }
    if (dim == 2) x[2] = 0.0;
    *det = adjugate(dim, J, A);
}

ORC_API void orc_lf_assemble_simplex(int dim, int p, int ne, const double *verts, const int *dofmap,
                                     int64_t nl, const double *prm, double *b)
{
    p3_init();
    /* DomainLFIntegrator default order 2p on MFEM's simplex rule [MFEM-ext] */
    const int nd = orc_simplex_nd(dim, p);
    double xi[7 * 7 * 7 * 3], wq[7 * 7 * 7];
    const int nq = orc_simplex_rule_order(dim, 2 * p, xi, wq);
    double *be = (double *)malloc(sizeof(double) * (size_t)ne * nd);
    #pragma omp parallel for schedule(static)
    for (int e = 0; e < ne; e++) {
        double phi[10], dphi[30], x[3], det;
        double *out = be + (size_t)e * nd;
        for (int l = 0; l < nd; l++) out[l] = 0.0;
        for (int q = 0; q < nq; q++) {
            simplex_point(dim, verts + (size_t)e * (dim + 1) * dim, xi + (size_t)q * dim, x, &det);
            simplex_basis(dim, p, xi + (size_t)q * dim, phi, dphi);
            const double fw = wq[q] * det * orc_mms_f(prm, x);
            for (int l = 0; l < nd; l++) out[l] += fw * phi[l];
        }
    }
    memset(b, 0, sizeof(double) * nl);
    for (int64_t k = 0; k < (int64_t)ne * nd; k++) b[dofmap[k]] += be[k];
    free(be);
}

ORC_API double orc_l2_error_simplex(int dim, int p, int ne, const double *verts, const int *dofmap,
                                    const double *u, const double *prm)
{
    p3_init();
    /* the drivers' error rule IntRules.Get(g, max(2, 2p + 3)) (linear_convection_diffusion_2D.cpp:383-388) */
    const int nd = orc_simplex_nd(dim, p);
    double xi[7 * 7 * 7 * 3], wq[7 * 7 * 7];
    const int nq = orc_simplex_rule_order(dim, 2 * p + 3 > 2 ? 2 * p + 3 : 2, xi, wq);
    double err = 0.0;
    #pragma omp parallel for reduction(+ : err) schedule(static)
    for (int e = 0; e < ne; e++) {
        double phi[10], dphi[30], x[3], det;
        for (int q = 0; q < nq; q++) {
            simplex_point(dim, verts + (size_t)e * (dim + 1) * dim, xi + (size_t)q * dim, x, &det);
            simplex_basis(dim, p, xi + (size_t)q * dim, phi, dphi);
            double uh = 0.0;
            for (int l = 0; l < nd; l++) uh += u[dofmap[(size_t)e * nd + l]] * phi[l];
            const double d = uh - orc_mms_u(prm, x);
            err += wq[q] * det * d * d;
        }
    }
    return sqrt(err);
}

/* Physical coordinates of the simplex dofs (vertices, edge midpoints). */
ORC_API void orc_dof_coords_simplex(int dim, int p, int ne, const double *verts, const int *dofmap, double *xyz)
{
    const int nd = orc_simplex_nd(dim, p), nv = dim + 1;
    const double g = 0.5 * (1.0 - 1.0 / sqrt(5.0));
    for (int e = 0; e < ne; e++) {
        const double *V = verts + (size_t)e * nv * dim;
        for (int l = 0; l < nd; l++) {
            double X[3] = {0, 0, 0};
            if (l < nv) {
                for (int k = 0; k < dim; k++) X[k] = V[l * dim + k];
            } else if (p == 3 && l == nd - 1) {  /* P3 centroid */
                for (int k = 0; k < dim; k++) X[k] = (V[k] + V[dim + k] + V[2 * dim + k]) / 3.0;
            } else {
                const int ed = (l - nv) / (p - 1), kk = (l - nv) % (p - 1);
                const int a = dim == 3 ? kEdge3[ed][0] : kEdge2[ed][0], b = dim == 3 ? kEdge3[ed][1] : kEdge2[ed][1];
                const double t = p == 2 ? 0.5 : (kk == 0 ? g : 1.0 - g);
                for (int k = 0; k < dim; k++) X[k] = V[a * dim + k] + t * (V[b * dim + k] - V[a * dim + k]);
            }
            for (int k = 0; k < dim; k++) xyz[(size_t)dofmap[(size_t)e * nd + l] * dim + k] = X[k];
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* CPU partial assembly as MFEM runs it on the host: the like-for-like CPU baseline of the PA    */
/* hot path (SURVEY.md 8d "CPU PA + CG"), timed by bench.py's cpu_baseline only.                 */
/* ------------------------------------------------------------------------------------------ */

/*
 * [MFEM-ext] ParBilinearForm with AssemblyLevel::PARTIAL on a hex mesh, device "cpu":
 *   - each integrator keeps its own point data (DiffusionIntegrator::AssemblePA: the 6 symmetric
 *     components of W adj(J) K adj(J)^T / detJ; ConvectionIntegrator: W alpha adj(J) c, 3 per point;
 *     MassIntegrator: W s detJ), layout [e][comp][q] as MFEM's Reshape(Q1D^3, comps, NE);
 *   - Mult = ElementRestriction::Mult (L -> E gather), then every integrator's AddMultPA over the
 *     E-vector with sum factorisation (PADiffusionApply3D, PAConvectionApply3D, PAMassApply3D: one
 *     element loop each), then ElementRestriction::MultTranspose (E -> L through per-dof offsets);
 *   - the ConstrainedOperator of FormLinearSystem: essential inputs zeroed, y_ess = x_ess;
 *   - CGSolver (cg_core) with OperatorJacobiSmoother (the caller passes 1 / diag, ess -> 1).
 * Stages written after MFEM's generic (non-shared-memory) 3D kernels: x, y, z contractions to the
 * points, the point operator, and the transposed contractions, all in per-element scratch.
 * Call sites: linear_convection_diffusion_2D.cpp:335-374 (forms, solver); the PA level is the
 * north star's (BASELINE.json); mesh_recession_handler.cpp:270-276 (CGSolver semantics).
 */
typedef struct {
    int p, d1, nq, ne, nd, q3;
    int64_t nl;
    int use_diff, use_conv, use_mass;
    double B[64], G[64];            /* [q][d] */
    double *qd_d, *qd_c, *qd_m;     /* [e][6][q3], [e][3][q3], [e][q3] */
    int *dofmap;                    /* [e][nd] (copy) */
    int64_t *off;                   /* E->L: offsets [nl + 1] into idx (element-major E-vector index) */
    int64_t *idx;
    double *xe, *ye;                /* E-vectors [e][nd] */
    const int *ess;                 /* ess marker for the constrained operator (borrowed during a solve) */
    double *xz;                     /* scratch: x with ess zeroed */
} orc_pa;

ORC_API orc_pa *orc_pa_setup(int p, int ne, const double *verts, const int *dofmap, int64_t nl, double kappa,
                             double alpha, double s, const double *c, int kinds)
{
    const int d1 = p + 1, nq = orc_rule_npts(0, 3, p), nd = d1 * d1 * d1, q3 = nq * nq * nq;
    if (d1 > 8 || nq > 8) return NULL;
    orc_pa *pa = (orc_pa *)calloc(1, sizeof(orc_pa));
    pa->p = p; pa->d1 = d1; pa->nq = nq; pa->ne = ne; pa->nd = nd; pa->q3 = q3; pa->nl = nl;
    pa->use_diff = (kinds & 1) != 0; pa->use_conv = (kinds & 2) != 0; pa->use_mass = (kinds & 4) != 0;
    double pts[8], wts[8];
    tables(p, nq, pa->B, pa->G, pts, wts);
    orc_coef cf = {kappa, alpha, s, {c ? c[0] : 0, c ? c[1] : 0, c ? c[2] : 0},
                   pa->use_diff, pa->use_conv, pa->use_mass, NULL, NULL, NULL, NULL};
    if (pa->use_diff) pa->qd_d = (double *)malloc(sizeof(double) * (size_t)ne * 6 * q3);
    if (pa->use_conv) pa->qd_c = (double *)malloc(sizeof(double) * (size_t)ne * 3 * q3);
    if (pa->use_mass) pa->qd_m = (double *)malloc(sizeof(double) * (size_t)ne * q3);
    #pragma omp parallel for schedule(static)
    for (int e = 0; e < ne; e++) {
        const double *V = verts + (size_t)e * 8 * 3;
        for (int qz = 0; qz < nq; qz++)
        for (int qy = 0; qy < nq; qy++)
        for (int qx = 0; qx < nq; qx++) {
            const int q = qx + nq * (qy + nq * qz);
            double xi[3] = {pts[qx], pts[qy], pts[qz]}, xx[3], J[3][3], A[3][3];
            q1_map(3, V, xi, xx, J);
            const double detJ = adjugate(3, J, A);
            double D[3][3] = {{0}}, Cv[3] = {0}, M = 0.0;
            point_coef(3, &cf, q, wts[qx] * wts[qy] * wts[qz], detJ, A, D, Cv, &M);
            if (pa->use_diff) {
                double *o = pa->qd_d + (size_t)e * 6 * q3 + q;
                o[0 * q3] = D[0][0]; o[1 * q3] = D[0][1]; o[2 * q3] = D[0][2];
                o[3 * q3] = D[1][1]; o[4 * q3] = D[1][2]; o[5 * q3] = D[2][2];
            }
            if (pa->use_conv)
                for (int k = 0; k < 3; k++) pa->qd_c[(size_t)e * 3 * q3 + k * q3 + q] = Cv[k];
            if (pa->use_mass) pa->qd_m[(size_t)e * q3 + q] = M;
        }
    }
    pa->dofmap = (int *)malloc(sizeof(int) * (size_t)ne * nd);
    memcpy(pa->dofmap, dofmap, sizeof(int) * (size_t)ne * nd);
    /* ElementRestriction's transpose: for every L-dof its E-vector entries in ascending order */
    pa->off = (int64_t *)calloc((size_t)nl + 1, sizeof(int64_t));
    pa->idx = (int64_t *)malloc(sizeof(int64_t) * (size_t)ne * nd);
    for (int64_t k = 0; k < (int64_t)ne * nd; k++) pa->off[dofmap[k] + 1]++;
    for (int64_t i = 0; i < nl; i++) pa->off[i + 1] += pa->off[i];
    int64_t *fill = (int64_t *)malloc(sizeof(int64_t) * (size_t)nl);
    memcpy(fill, pa->off, sizeof(int64_t) * (size_t)nl);
    for (int64_t k = 0; k < (int64_t)ne * nd; k++) pa->idx[fill[dofmap[k]]++] = k;
    free(fill);
    pa->xe = (double *)malloc(sizeof(double) * (size_t)ne * nd);
    pa->ye = (double *)malloc(sizeof(double) * (size_t)ne * nd);
    pa->xz = (double *)malloc(sizeof(double) * (size_t)nl);
    return pa;
}

ORC_API void orc_pa_free(orc_pa *pa)
{
    if (!pa) return;
    free(pa->qd_d); free(pa->qd_c); free(pa->qd_m); free(pa->dofmap); free(pa->off); free(pa->idx);
    free(pa->xe); free(pa->ye); free(pa->xz); free(pa);
}

/* value (and reference gradient) of one element's E-vector at its Q1^3 points: u[q], g[q][3] */
static void pa_interp(const orc_pa *pa, const double *X, double *u, double (*g)[3], int grad)
{
    const int D = pa->d1, Q = pa->nq;
    const double *B = pa->B, *G = pa->G;
    double tx[8][8][8][2];  /* [dz][dy][qx]: B x, G x along x */
    for (int dz = 0; dz < D; dz++)
        for (int dy = 0; dy < D; dy++)
            for (int qx = 0; qx < Q; qx++) {
                double a = 0.0, b = 0.0;
                for (int dx = 0; dx < D; dx++) {
                    const double v = X[dx + D * (dy + D * dz)];
                    a += B[qx * D + dx] * v;
                    b += G[qx * D + dx] * v;
                }
                tx[dz][dy][qx][0] = a; tx[dz][dy][qx][1] = b;
            }
    double ty[8][8][8][3];  /* [dz][qy][qx]: (Bx By), (Gx By), (Bx Gy) */
    for (int dz = 0; dz < D; dz++)
        for (int qy = 0; qy < Q; qy++)
            for (int qx = 0; qx < Q; qx++) {
                double a = 0.0, b = 0.0, c = 0.0;
                for (int dy = 0; dy < D; dy++) {
                    a += B[qy * D + dy] * tx[dz][dy][qx][0];
                    b += B[qy * D + dy] * tx[dz][dy][qx][1];
                    c += G[qy * D + dy] * tx[dz][dy][qx][0];
                }
                ty[dz][qy][qx][0] = a; ty[dz][qy][qx][1] = b; ty[dz][qy][qx][2] = c;
            }
    for (int qz = 0; qz < Q; qz++)
        for (int qy = 0; qy < Q; qy++)
            for (int qx = 0; qx < Q; qx++) {
                double a = 0.0, gx = 0.0, gy = 0.0, gz = 0.0;
                for (int dz = 0; dz < D; dz++) {
                    const double bz = B[qz * D + dz], dzv = G[qz * D + dz];
                    a += bz * ty[dz][qy][qx][0];
                    gx += bz * ty[dz][qy][qx][1];
                    gy += bz * ty[dz][qy][qx][2];
                    gz += dzv * ty[dz][qy][qx][0];
                }
                const int q = qx + Q * (qy + Q * qz);
                u[q] = a;
                if (grad) { g[q][0] = gx; g[q][1] = gy; g[q][2] = gz; }
            }
}

/* Y += sum_q (phi v[q] + grad phi . w[q]) over one element (w NULL: values only) */
static void pa_test(const orc_pa *pa, const double *v, double (*w)[3], double *Y)
{
    const int D = pa->d1, Q = pa->nq;
    const double *B = pa->B, *G = pa->G;
    double sz[8][8][8][3];  /* [dz][qy][qx]: Bz (v, wx, wy) + Gz wz */
    for (int dz = 0; dz < D; dz++)
        for (int qy = 0; qy < Q; qy++)
            for (int qx = 0; qx < Q; qx++) {
                double a = 0.0, b = 0.0, c = 0.0;
                for (int qz = 0; qz < Q; qz++) {
                    const int q = qx + Q * (qy + Q * qz);
                    const double bz = B[qz * D + dz], gz = G[qz * D + dz];
                    a += bz * v[q] + (w ? gz * w[q][2] : 0.0);
                    if (w) { b += bz * w[q][0]; c += bz * w[q][1]; }
                }
                sz[dz][qy][qx][0] = a; sz[dz][qy][qx][1] = b; sz[dz][qy][qx][2] = c;
            }
    double sy[8][8][8][2];  /* [dz][dy][qx]: By (a, b) + Gy c, i.e. the x-test value and x-test gradient parts */
    for (int dz = 0; dz < D; dz++)
        for (int dy = 0; dy < D; dy++)
            for (int qx = 0; qx < Q; qx++) {
                double a = 0.0, b = 0.0;
                for (int qy = 0; qy < Q; qy++) {
                    const double by = B[qy * D + dy], gy = G[qy * D + dy];
                    a += by * sz[dz][qy][qx][0] + (w ? gy * sz[dz][qy][qx][2] : 0.0);
                    if (w) b += by * sz[dz][qy][qx][1];
                }
                sy[dz][dy][qx][0] = a; sy[dz][dy][qx][1] = b;
            }
    for (int dz = 0; dz < D; dz++)
        for (int dy = 0; dy < D; dy++)
            for (int dx = 0; dx < D; dx++) {
                double a = 0.0;
                for (int qx = 0; qx < Q; qx++)
                    a += B[qx * D + dx] * sy[dz][dy][qx][0] + (w ? G[qx * D + dx] * sy[dz][dy][qx][1] : 0.0);
                Y[dx + D * (dy + D * dz)] += a;
            }
}

/* y = A x on L-vectors (constrained: inputs on ess zeroed, y_ess = x_ess) */
static void pa_apply(const orc_pa *pa, const double *x, double *y, int constrained)
{
    const int ne = pa->ne, nd = pa->nd, q3 = pa->q3;
    const double *xs = x;
    if (constrained) {
        #pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < pa->nl; i++) pa->xz[i] = pa->ess[i] ? 0.0 : x[i];
        xs = pa->xz;
    }
    /* ElementRestriction::Mult */
    #pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < (int64_t)ne * nd; k++) { pa->xe[k] = xs[pa->dofmap[k]]; pa->ye[k] = 0.0; }
    /* AddMultPA of each integrator: one element loop each */
    if (pa->use_diff) {
        #pragma omp parallel for schedule(static)
        for (int e = 0; e < ne; e++) {
            double u[512], g[512][3], v[512];
            pa_interp(pa, pa->xe + (size_t)e * nd, u, g, 1);
            const double *Dq = pa->qd_d + (size_t)e * 6 * q3;
            for (int q = 0; q < q3; q++) {
                const double a = g[q][0], b = g[q][1], c = g[q][2];
                const double d00 = Dq[q], d01 = Dq[q3 + q], d02 = Dq[2 * q3 + q], d11 = Dq[3 * q3 + q],
                             d12 = Dq[4 * q3 + q], d22 = Dq[5 * q3 + q];
                g[q][0] = d00 * a + d01 * b + d02 * c;
                g[q][1] = d01 * a + d11 * b + d12 * c;
                g[q][2] = d02 * a + d12 * b + d22 * c;
                v[q] = 0.0;
            }
            pa_test(pa, v, g, pa->ye + (size_t)e * nd);
        }
    }
    if (pa->use_conv) {
        #pragma omp parallel for schedule(static)
        for (int e = 0; e < ne; e++) {
            double u[512], g[512][3], v[512];
            pa_interp(pa, pa->xe + (size_t)e * nd, u, g, 1);
            const double *Cq = pa->qd_c + (size_t)e * 3 * q3;
            for (int q = 0; q < q3; q++) v[q] = Cq[q] * g[q][0] + Cq[q3 + q] * g[q][1] + Cq[2 * q3 + q] * g[q][2];
            pa_test(pa, v, NULL, pa->ye + (size_t)e * nd);
        }
    }
    if (pa->use_mass) {
        #pragma omp parallel for schedule(static)
        for (int e = 0; e < ne; e++) {
            double u[512], v[512];
            pa_interp(pa, pa->xe + (size_t)e * nd, u, NULL, 0);
            const double *Mq = pa->qd_m + (size_t)e * q3;
            for (int q = 0; q < q3; q++) v[q] = Mq[q] * u[q];
            pa_test(pa, v, NULL, pa->ye + (size_t)e * nd);
        }
    }
    /* ElementRestriction::MultTranspose (+ the constraint) */
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < pa->nl; i++) {
        double acc = 0.0;
        for (int64_t k = pa->off[i]; k < pa->off[i + 1]; k++) acc += pa->ye[pa->idx[k]];
        y[i] = (constrained && pa->ess[i]) ? x[i] : acc;
    }
}

ORC_API void orc_pa_mult(orc_pa *pa, const int *ess_marker, const double *x, double *y)
{
    pa->ess = ess_marker;
    pa_apply(pa, x, y, ess_marker != NULL);
    pa->ess = NULL;
}

/* diag_e[i] += sum_q F[q] wx[qx][ix] wy[qy][iy] wz[qz][iz] (i = ix + D (iy + D iz)): one separable term
 * of an element diagonal, contracted x, then y, then z (the shape of MFEM's PA*AssembleDiagonal kernels) */
static void pa_diag_term(int D, int Q, const double *F, const double *wx, const double *wy, const double *wz,
                         double *diag)
{
    double tx[8][8][8], ty[8][8][8];  /* [qz][qy][ix], [qz][iy][ix] */
    for (int qz = 0; qz < Q; qz++)
        for (int qy = 0; qy < Q; qy++)
            for (int ix = 0; ix < D; ix++) {
                double a = 0.0;
                for (int qx = 0; qx < Q; qx++) a += wx[qx * D + ix] * F[qx + Q * (qy + Q * qz)];
                tx[qz][qy][ix] = a;
            }
    for (int qz = 0; qz < Q; qz++)
        for (int iy = 0; iy < D; iy++)
            for (int ix = 0; ix < D; ix++) {
                double a = 0.0;
                for (int qy = 0; qy < Q; qy++) a += wy[qy * D + iy] * tx[qz][qy][ix];
                ty[qz][iy][ix] = a;
            }
    for (int iz = 0; iz < D; iz++)
        for (int iy = 0; iy < D; iy++)
            for (int ix = 0; ix < D; ix++) {
                double a = 0.0;
                for (int qz = 0; qz < Q; qz++) a += wz[qz * D + iz] * ty[qz][iy][ix];
                diag[ix + D * (iy + D * iz)] += a;
            }
}

/*
 * [MFEM-ext] BilinearForm::AssembleDiagonal at AssemblyLevel::PARTIAL: every integrator's
 * AssembleDiagonalPA on the element (PADiffusionDiagonal3D: sum_q of the symmetric point matrix against
 * the products of the 1D value / derivative tables, off-diagonal components twice; the convection and
 * mass diagonals the same way with their point data), then ElementRestriction::MultTranspose (the E->L
 * sum over every element holding the dof).  Unconstrained: the Jacobi smoother of FormLinearSystem sets
 * the essential entries to 1 itself.  The diagonal the GPU's OperatorJacobiSmoother (d_dinv) inverts.
 */
ORC_API void orc_pa_diag(orc_pa *pa, double *y)
{
    const int D = pa->d1, Q = pa->nq, nd = pa->nd, q3 = pa->q3, ne = pa->ne;
    double BB[64], BG[64], GG[64];
    for (int k = 0; k < Q * D; k++) {
        BB[k] = pa->B[k] * pa->B[k];
        BG[k] = pa->B[k] * pa->G[k];
        GG[k] = pa->G[k] * pa->G[k];
    }
    #pragma omp parallel for schedule(static)
    for (int e = 0; e < ne; e++) {
        double *de = pa->ye + (size_t)e * nd, F[512];
        for (int i = 0; i < nd; i++) de[i] = 0.0;
        if (pa->use_diff) {
            const double *Dq = pa->qd_d + (size_t)e * 6 * q3;
            /* components d00 d01 d02 d11 d12 d22: (x, y, z) weight tables and the symmetric factor */
            const double *W[6][3] = {{GG, BB, BB}, {BG, BG, BB}, {BG, BB, BG}, {BB, GG, BB}, {BB, BG, BG}, {BB, BB, GG}};
            const double f[6] = {1.0, 2.0, 2.0, 1.0, 2.0, 1.0};
            for (int k = 0; k < 6; k++) {
                for (int q = 0; q < q3; q++) F[q] = f[k] * Dq[k * q3 + q];
                pa_diag_term(D, Q, F, W[k][0], W[k][1], W[k][2], de);
            }
        }
        if (pa->use_conv) {
            const double *Cq = pa->qd_c + (size_t)e * 3 * q3;
            const double *W[3][3] = {{BG, BB, BB}, {BB, BG, BB}, {BB, BB, BG}};
            for (int k = 0; k < 3; k++) pa_diag_term(D, Q, Cq + (size_t)k * q3, W[k][0], W[k][1], W[k][2], de);
        }
        if (pa->use_mass) pa_diag_term(D, Q, pa->qd_m + (size_t)e * q3, BB, BB, BB, de);
    }
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < pa->nl; i++) {
        double acc = 0.0;
        for (int64_t k = pa->off[i]; k < pa->off[i + 1]; k++) acc += pa->ye[pa->idx[k]];
        y[i] = acc;
    }
}

static void pa_con_op(const void *op, const double *x, double *y) { pa_apply((const orc_pa *)op, x, y, 1); }

/* CGSolver on the ConstrainedOperator of the PA form (dinv: Jacobi, ess entries 1) */
ORC_API int orc_pa_cg(orc_pa *pa, const int *ess_marker, const double *dinv, const double *b, double *x,
                      double rel_tol, double abs_tol, int max_iter, int *iters, double *final_norm)
{
    pa->ess = ess_marker;
    const int r = cg_core(pa_con_op, pa, pa->nl, dinv, b, x, rel_tol, abs_tol, max_iter, iters, final_norm);
    pa->ess = NULL;
    return r;
}

/* Host memory bandwidth probe (STREAM triad a = b + s c, 24 B per index counted, best of reps) on the
 * current OpenMP threads (bench.py pins them to the CPU baseline's cores first): explains the CPU
 * baseline's spread across hosts by the bandwidth its cores actually get. */
ORC_API double orc_stream_triad(int64_t n, int reps)
{
    double *a = (double *)malloc(sizeof(double) * (size_t)n), *b = (double *)malloc(sizeof(double) * (size_t)n),
           *c = (double *)malloc(sizeof(double) * (size_t)n);
    if (!a || !b || !c) { free(a); free(b); free(c); return -1.0; }
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) { a[i] = 0.0; b[i] = 1.0; c[i] = 2.0; }
    double best = 0.0;
    for (int r = 0; r < reps; r++) {
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        const double s = 3.0 + r;
        #pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; i++) a[i] = b[i] + s * c[i];
        clock_gettime(CLOCK_MONOTONIC, &t1);
        const double dt = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
        const double gbs = 24.0 * (double)n / dt / 1e9;
        if (gbs > best) best = gbs;
    }
    volatile double sink = a[n / 2];
    (void)sink;
    free(a); free(b); free(c);
    return best;
}
