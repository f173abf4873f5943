// basis.cpp — 1D nodal bases and Gauss rules for the H1 tensor spaces (host side).
//
// H1_FECollection(order, dim) (linear_convection_diffusion_2D.cpp:311) uses MFEM's default
// BasisType::GaussLobatto: Lagrange polynomials through the p+1 Gauss-Lobatto points of [0,1].
// Integration rules are Gauss-Legendre on [0,1] with MFEM's default orders for multilinear
// tensor elements: Diffusion 2p+dim-1, Convection (dim-1)+(p-1)+p+(dim-1),
// Mass 2p+dim-1 -> one shared n = order/2+1 for the fused operator; DomainLF 2p; the driver's
// L2-error rule max(2, 2p+3) (:383).
#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <vector>

#include "cdfem_internal.hpp"

namespace cdfem {

// Shifted Legendre P_n(2s-1) and its derivative d/ds via the recurrence on [0,1].
static void shifted_legendre(int n, double s, double &P, double &dP)
{
    const double t = 2.0 * s - 1.0;
    double p0 = 1.0, p1 = t, d0 = 0.0, d1 = 2.0;
    if (n == 0) { P = 1.0; dP = 0.0; return; }
    for (int k = 2; k <= n; ++k) {
        const double pk = ((2 * k - 1) * t * p1 - (k - 1) * p0) / k;
        const double dk = ((2 * k - 1) * (2.0 * p1 + t * d1) - (k - 1) * d0) / k;
        p0 = p1; p1 = pk; d0 = d1; d1 = dk;
    }
    P = p1; dP = d1;
}

void gauss_legendre(int n, double *x, double *w)
{
    for (int i = 0; i < n; ++i) {
        // ascending initial guess on [0,1]
        double s = 0.5 * (1.0 - std::cos(M_PI * (i + 0.75) / (n + 0.5)));
        for (int it = 0; it < 64; ++it) {
            double P, dP;
            shifted_legendre(n, s, P, dP);
            const double ds = P / dP;
            s -= ds;
            if (std::fabs(ds) < 1e-17) break;
        }
        double P, dP;
        shifted_legendre(n, s, P, dP);
        x[i] = s;
        // on [0,1]: w = 1 / (s (1-s) P'(s)^2) with P' = d/ds
        w[i] = 1.0 / (s * (1.0 - s) * dP * dP);
    }
}

void gll_nodes(int p, double *x)
{
    x[0] = 0.0;
    x[p] = 1.0;
    // interior nodes: roots of dP_p/ds; Newton with the derivative from a finite recurrence
    for (int i = 1; i < p; ++i) {
        double s = 0.5 * (1.0 - std::cos(M_PI * i / p));
        for (int it = 0; it < 64; ++it) {
            double P, dP;
            shifted_legendre(p, s, P, dP);
            // Legendre ODE in s: s(1-s) P'' + (1-2s) P' + p(p+1) P = 0  (P' = d/ds)
            const double d2P = -((1.0 - 2.0 * s) * dP + p * (p + 1.0) * P) / (s * (1.0 - s));
            const double ds = dP / d2P;
            s -= ds;
            if (std::fabs(ds) < 1e-17) break;
        }
        x[i] = s;
    }
    for (int i = 0; i <= p / 2; ++i) {  // exact symmetry about 1/2
        const double a = 0.5 * (x[i] + 1.0 - x[p - i]);
        x[i] = a;
        x[p - i] = 1.0 - a;
    }
}

Rule1D make_rule(int p, int q1)
{
    if (p + 1 > kMaxD1 || q1 > kMaxQ1 || p < 1 || q1 < 1)
        throw std::runtime_error("rule size out of range");
    Rule1D r;
    r.d1 = p + 1;
    r.q1 = q1;
    double nodes[kMaxD1];
    gll_nodes(p, nodes);
    gauss_legendre(q1, r.pts, r.wts);
    for (int q = 0; q < q1; ++q) {
        const double xi = r.pts[q];
        for (int j = 0; j <= p; ++j) {
            // Lagrange basis (barycentric-free product form) and derivative
            double v = 1.0, d = 0.0;
            for (int k = 0; k <= p; ++k) {
                if (k == j) continue;
                const double den = nodes[j] - nodes[k];
                const double f = (xi - nodes[k]) / den;
                d = d * f + v / den;
                v *= f;
            }
            r.B[q][j] = v;
            r.G[q][j] = d;
        }
    }
    return r;
}

int rule_points_1d(int which, int dim, int p)
{
    int order = 0;
    switch (which) {
    case 0: {  // fused Diffusion + Convection + Mass; all three coincide (checked)
        const int od = 2 * p + dim - 1;
        const int oc = (dim - 1) + (p - 1) + p + (dim - 1);
        const int om = 2 * p + dim - 1;
        if (od / 2 != oc / 2 || od / 2 != om / 2)
            throw std::runtime_error("integrator rules do not coincide");
        order = od;
        break;
    }
    case 1: order = 2 * p; break;
    case 2: order = (2 * p + 3 > 2) ? 2 * p + 3 : 2; break;
    default: throw std::runtime_error("bad rule id");
    }
    return order / 2 + 1;
}

// ---- simplices (P1/P2 Lagrange on triangles / tetrahedra, BASELINE config C4) ----------------
// Collapsed tensor Gauss-Legendre rule on the reference simplex (0, e_1, .., e_dim), n points per
// direction: xi_1 = u, xi_2 = (1-u) v, xi_3 = (1-u)(1-v) w, weight w_u w_v w_w (1-u)^(dim-1) (1-v)
// (3D).  Exact to degree 2n - dim; n = p + 2 integrates the mass form of P2 exactly in 3D.
int simplex_rule(int dim, int n, std::vector<double> &xi, std::vector<double> &w)
{
    std::vector<double> x(n), wx(n);
    gauss_legendre(n, x.data(), wx.data());
    const int nq = dim == 3 ? n * n * n : n * n;
    xi.assign((size_t)nq * dim, 0.0);
    w.assign(nq, 0.0);
    int q = 0;
    for (int iu = 0; iu < n; ++iu)
        for (int iv = 0; iv < n; ++iv) {
            const double u = x[iu], v = x[iv];
            if (dim == 2) {
                xi[q * 2] = u;
                xi[q * 2 + 1] = (1.0 - u) * v;
                w[q] = wx[iu] * wx[iv] * (1.0 - u);
                ++q;
                continue;
            }
            for (int iw = 0; iw < n; ++iw, ++q) {
                xi[q * 3] = u;
                xi[q * 3 + 1] = (1.0 - u) * v;
                xi[q * 3 + 2] = (1.0 - u) * (1.0 - v) * x[iw];
                w[q] = wx[iu] * wx[iv] * wx[iw] * (1.0 - u) * (1.0 - u) * (1.0 - v);
            }
        }
    return nq;
}

// MFEM's tabulated simplex rules (IntRules.Get(TRIANGLE / TETRAHEDRON, order), intrules.cpp),
// generated and verified by tools/simplex_rules.py: exact to their degree in double precision.
#include "simplex_rules.inc"

int mfem_simplex_rule(int dim, int order, std::vector<double> &xi, std::vector<double> &w)
{
    static const double *tri[] = {k_tri1, k_tri1, k_tri2, k_tri3, k_tri4, k_tri5, k_tri6, k_tri7, k_tri8, k_tri9};
    static const int ntri[] = {1, 1, 3, 4, 6, 7, 12, 12, 16, 19};
    static const double *tet[] = {k_tet1, k_tet1, k_tet2, k_tet3, k_tet4, k_tet5, k_tet6};
    static const int ntet[] = {1, 1, 4, 5, 11, 14, 24};
    if (order < 0) order = 0;
    const double *t = nullptr;
    int n = 0;
    if (dim == 2 && order <= 9) {
        t = tri[order];
        n = ntri[order];
    } else if (dim == 3 && order <= 6) {
        t = tet[order];
        n = ntet[order];
    } else {
        return 0;
    }
    xi.assign((size_t)n * dim, 0.0);
    w.assign(n, 0.0);
    for (int q = 0; q < n; ++q) {
        for (int k = 0; k < dim; ++k) xi[(size_t)q * dim + k] = t[q * (dim + 1) + k];
        w[q] = t[q * (dim + 1) + dim];
    }
    return n;
}

int simplex_rule_for_order(int dim, int order, std::vector<double> &xi, std::vector<double> &w)
{
    const int n = mfem_simplex_rule(dim, order, xi, w);
    if (n > 0) return n;
    // beyond MFEM's tables here: collapsed Gauss exact to the order (n points per direction, exact
    // to degree 2n - 1 in the first direction after the Duffy factor)
    return simplex_rule(dim, (order + dim) / 2 + 1, xi, w);
}

int simplex_ndofs(int dim, int p)
{
    if (p == 1) return dim + 1;
    if (p == 2) return (dim + 1) * (dim + 2) / 2;
    if (p == 3 && dim == 2) return 10;
    return -1;
}

// P3 triangle (H1_FECollection(3, 2), GaussLobatto nodes): vertices, 2 nodes per edge at the
// interior GLL points t = (1 -+ 1/sqrt(5)) / 2 along a -> b for the edges (0,1), (0,2), (1,2),
// and the centroid.  Nodal basis = monomials x^i y^j (i + j <= 3) times the inverse Vandermonde
// matrix, formed once.
double p3_edge_t(int k) { return k == 0 ? 0.5 * (1.0 - 1.0 / std::sqrt(5.0)) : 0.5 * (1.0 + 1.0 / std::sqrt(5.0)); }

void p3_tri_nodes(double (*X)[2])
{
    const double V[3][2] = {{0, 0}, {1, 0}, {0, 1}};
    for (int v = 0; v < 3; ++v) { X[v][0] = V[v][0]; X[v][1] = V[v][1]; }
    for (int e = 0; e < 3; ++e)
        for (int k = 0; k < 2; ++k) {
            const int a = kTriEdge[e][0], b = kTriEdge[e][1];
            const double t = p3_edge_t(k);
            for (int d = 0; d < 2; ++d) X[3 + 2 * e + k][d] = V[a][d] + t * (V[b][d] - V[a][d]);
        }
    X[9][0] = X[9][1] = 1.0 / 3.0;
}

static void p3_monomials(const double *x, double *m, double *mx, double *my)
{
    int k = 0;
    for (int tot = 0; tot <= 3; ++tot)
        for (int j = 0; j <= tot; ++j, ++k) {
            const int i = tot - j;  // x^i y^j
            m[k] = std::pow(x[0], i) * std::pow(x[1], j);
            mx[k] = i > 0 ? i * std::pow(x[0], i - 1) * std::pow(x[1], j) : 0.0;
            my[k] = j > 0 ? j * std::pow(x[0], i) * std::pow(x[1], j - 1) : 0.0;
        }
}

static const std::vector<double> &p3_coeffs()
{
    static const std::vector<double> C = [] {
        double X[10][2];
        p3_tri_nodes(X);
        double A[10][20] = {};
        for (int r = 0; r < 10; ++r) {  // V[r][c] = m_c(node_r), augmented with I
            double m[10], mx[10], my[10];
            p3_monomials(X[r], m, mx, my);
            for (int c = 0; c < 10; ++c) A[r][c] = m[c];
            A[r][10 + r] = 1.0;
        }
        for (int c = 0; c < 10; ++c) {  // Gauss-Jordan, partial pivoting
            int piv = c;
            for (int r = c + 1; r < 10; ++r)
                if (std::fabs(A[r][c]) > std::fabs(A[piv][c])) piv = r;
            for (int k = 0; k < 20; ++k) std::swap(A[c][k], A[piv][k]);
            const double d = A[c][c];
            for (int k = 0; k < 20; ++k) A[c][k] /= d;
            for (int r = 0; r < 10; ++r)
                if (r != c) {
                    const double f = A[r][c];
                    for (int k = 0; k < 20; ++k) A[r][k] -= f * A[c][k];
                }
        }
        std::vector<double> out(100);  // out[c * 10 + i] = (V^-1)[c][i]: phi_i = sum_c m_c out[c][i]
        for (int c = 0; c < 10; ++c)
            for (int i = 0; i < 10; ++i) out[c * 10 + i] = A[c][10 + i];
        return out;
    }();
    return C;
}

// Local order: vertices, then edges (0,1),(0,2),(0,3),(1,2),(1,3),(2,3) [2D (0,1),(0,2),(1,2)].
const int kSimplexEdge[6][2] = {{0, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 3}};
const int kTriEdge[3][2] = {{0, 1}, {0, 2}, {1, 2}};

void simplex_basis(int dim, int p, const double *xi, double *phi, double *dphi)
{
    if (dim == 2 && p == 3) {
        const std::vector<double> &C = p3_coeffs();
        double m[10], mx[10], my[10];
        p3_monomials(xi, m, mx, my);
        for (int i = 0; i < 10; ++i) {
            double v = 0.0, gx = 0.0, gy = 0.0;
            for (int c = 0; c < 10; ++c) {
                v += m[c] * C[c * 10 + i];
                gx += mx[c] * C[c * 10 + i];
                gy += my[c] * C[c * 10 + i];
            }
            phi[i] = v;
            dphi[i * 2] = gx;
            dphi[i * 2 + 1] = gy;
        }
        return;
    }
    double lam[4], dl[4][3] = {};
    lam[0] = 1.0;
    for (int k = 0; k < dim; ++k) {
        lam[0] -= xi[k];
        dl[0][k] = -1.0;
        lam[k + 1] = xi[k];
        dl[k + 1][k] = 1.0;
    }
    for (int a = 0; a <= dim; ++a) {
        phi[a] = p == 1 ? lam[a] : lam[a] * (2.0 * lam[a] - 1.0);
        const double f = p == 1 ? 1.0 : 4.0 * lam[a] - 1.0;
        for (int k = 0; k < dim; ++k) dphi[a * dim + k] = f * dl[a][k];
    }
    if (p == 1) return;
    const int nedge = dim == 3 ? 6 : 3;
    for (int e = 0; e < nedge; ++e) {
        const int a = dim == 3 ? kSimplexEdge[e][0] : kTriEdge[e][0];
        const int b = dim == 3 ? kSimplexEdge[e][1] : kTriEdge[e][1];
        const int l = dim + 1 + e;
        phi[l] = 4.0 * lam[a] * lam[b];
        for (int k = 0; k < dim; ++k) dphi[l * dim + k] = 4.0 * (lam[a] * dl[b][k] + lam[b] * dl[a][k]);
    }
}

}  // namespace cdfem
