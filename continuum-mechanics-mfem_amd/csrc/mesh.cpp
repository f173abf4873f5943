// mesh.cpp — structured quad/hex box meshes and z-slab partitions (host side of the product).
//
// The reference reads gmsh meshes (Mesh/unit_square.msh) and refines them; BASELINE configs 2, 3
// and 5 are synthetic structured hex meshes that ship nowhere, so the product generates them:
// [0,1]^dim split into nx*ny(*nz) elements, boundary attributes as Mesh/unit_square.geo:18-21
// (all marked essential by the hot path: linear_convection_diffusion_2D.cpp:319-322).
//
// Multi-GPU element partition: rank r owns the elements with (last-axis) index in [z0, z1) — a
// slab — and numbers the dofs of its slab lexicographically (local L-vector).  Interface dofs
// (the planes at z0 > 0 and z1 < nz) are shared with the neighbouring rank; they are NOT
// essential.  This is the ParMesh / ParFiniteElementSpace element partition of the reference
// (linear_convection_diffusion_2D.cpp:300) with a slab partitioner instead of METIS.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <utility>

#include "cdfem_internal.hpp"

namespace {

// deterministic jitter in [-1, 1)
double jitter(uint64_t a)
{
    a += 0x9e3779b97f4a7c15ULL;
    a = (a ^ (a >> 30)) * 0xbf58476d1ce4e5b9ULL;
    a = (a ^ (a >> 27)) * 0x94d049bb133111ebULL;
    a ^= a >> 31;
    return (double)(a >> 11) / 4503599627370496.0 - 1.0;
}

struct Box {
    int dim, nx, ny, nz, p, z0, z1;
    int64_t Lx, Ly, Lz;       // local lattice sizes
    int ne;
};

bool make_box(int dim, int nx, int ny, int nz, int p, int z0, int z1, Box &b)
{
    if (dim != 2 && dim != 3) return false;
    if (nx < 1 || ny < 1 || p < 1) return false;
    if (dim == 2) nz = 1;
    if (nz < 1) return false;
    const int nlast = dim == 3 ? nz : ny;
    if (z1 <= 0 || z1 > nlast) z1 = nlast;
    if (z0 < 0 || z0 >= z1) return false;
    b = Box{dim, nx, ny, nz, p, z0, z1, 0, 0, 0, 0};
    b.Lx = (int64_t)p * nx + 1;
    if (dim == 3) {
        b.Ly = (int64_t)p * ny + 1;
        b.Lz = (int64_t)p * (z1 - z0) + 1;
        b.ne = nx * ny * (z1 - z0);
    } else {
        b.Ly = (int64_t)p * (z1 - z0) + 1;
        b.Lz = 1;
        b.ne = nx * (z1 - z0);
    }
    return true;
}

}  // namespace

extern "C" {

int cdfem_box_sizes(int dim, int nx, int ny, int nz, int order, int z0, int z1, int *ne,
                    int64_t *nldofs, int *n_ess)
{
    Box b;
    if (!make_box(dim, nx, ny, nz, order, z0, z1, b)) return CDFEM_ERR_ARG;
    const int nlast = dim == 3 ? b.nz : b.ny;
    int64_t ness = 0;
    const int64_t nl = b.Lx * b.Ly * b.Lz;
    for (int64_t i = 0; i < nl; ++i) {
        const int64_t gx = i % b.Lx, gy = (i / b.Lx) % b.Ly, gz = i / (b.Lx * b.Ly);
        const int64_t glast = (dim == 3 ? gz : gy) + (int64_t)order * b.z0;  // global last-axis index
        bool on = gx == 0 || gx == b.Lx - 1 || glast == 0 || glast == (int64_t)order * nlast;
        if (dim == 3) on = on || gy == 0 || gy == b.Ly - 1;
        ness += on;
    }
    if (ne) *ne = b.ne;
    if (nldofs) *nldofs = nl;
    if (n_ess) *n_ess = (int)ness;
    return CDFEM_OK;
}

int cdfem_box_mesh(int dim, int nx, int ny, int nz, int order, int z0, int z1, double perturb,
                   double *elem_verts, int32_t *elem_dofs, int32_t *ess_dofs, double *dof_xyz)
{
    Box b;
    if (!make_box(dim, nx, ny, nz, order, z0, z1, b)) return CDFEM_ERR_ARG;
    const int p = order, d1 = p + 1;
    const int nd = dim == 3 ? d1 * d1 * d1 : d1 * d1;
    const int nv = 1 << dim;
    const int nlast = dim == 3 ? b.nz : b.ny;
    const double h[3] = {1.0 / b.nx, 1.0 / b.ny, 1.0 / b.nz};
    const int64_t gvx = b.nx + 1, gvy = b.ny + 1;

    auto vertex = [&](int gx, int gy, int gz, double X[3]) {
        const int g[3] = {gx, gy, gz};
        const int n[3] = {b.nx, b.ny, b.nz};
        bool interior = true;
        for (int k = 0; k < dim; ++k) {
            X[k] = g[k] * h[k];
            interior = interior && g[k] > 0 && g[k] < n[k];
        }
        if (perturb > 0.0 && interior) {
            const uint64_t id = (uint64_t)gx + (uint64_t)gvx * ((uint64_t)gy + (uint64_t)gvy * gz);
            for (int k = 0; k < dim; ++k) X[k] += perturb * h[k] * jitter(3 * id + k);
        }
    };

    double nodes[cdfem::kMaxD1];
    cdfem::gll_nodes(p, nodes);
    for (int e = 0; e < b.ne; ++e) {
        int ix, iy, iz;
        if (dim == 3) {
            ix = e % b.nx; iy = (e / b.nx) % b.ny; iz = e / (b.nx * b.ny) + b.z0;
        } else {
            ix = e % b.nx; iy = e / b.nx + b.z0; iz = 0;
        }
        double V[8][3] = {};
        for (int v = 0; v < nv; ++v) {
            vertex(ix + (v & 1), iy + ((v >> 1) & 1), iz + ((v >> 2) & 1), V[v]);
            if (elem_verts)
                for (int k = 0; k < dim; ++k) elem_verts[((size_t)e * nv + v) * dim + k] = V[v][k];
        }
        for (int l = 0; l < nd; ++l) {
            const int dx = l % d1, dy = (l / d1) % d1, dz = l / (d1 * d1);
            int64_t lx = (int64_t)p * ix + dx, ly, lz;
            if (dim == 3) {
                ly = (int64_t)p * iy + dy;
                lz = (int64_t)p * (iz - b.z0) + dz;
            } else {
                ly = (int64_t)p * (iy - b.z0) + dy;
                lz = 0;
            }
            const int64_t gid = lx + b.Lx * (ly + b.Ly * lz);
            if (elem_dofs) elem_dofs[(size_t)e * nd + l] = (int32_t)gid;
            if (dof_xyz) {
                // multilinear image of the GLL node
                const double xi[3] = {nodes[dx], nodes[dy], dim == 3 ? nodes[dz] : 0.0};
                double X[3] = {0, 0, 0};
                for (int v = 0; v < nv; ++v) {
                    double N = 1.0;
                    for (int k = 0; k < dim; ++k) N *= ((v >> k) & 1) ? xi[k] : 1.0 - xi[k];
                    for (int k = 0; k < dim; ++k) X[k] += N * V[v][k];
                }
                for (int k = 0; k < dim; ++k) dof_xyz[gid * dim + k] = X[k];
            }
        }
    }
    if (ess_dofs) {
        const int64_t nl = b.Lx * b.Ly * b.Lz;
        int64_t m = 0;
        for (int64_t i = 0; i < nl; ++i) {
            const int64_t gx = i % b.Lx, gy = (i / b.Lx) % b.Ly, gz = i / (b.Lx * b.Ly);
            const int64_t glast = (dim == 3 ? gz : gy) + (int64_t)p * b.z0;
            bool on = gx == 0 || gx == b.Lx - 1 || glast == 0 || glast == (int64_t)p * nlast;
            if (dim == 3) on = on || gy == 0 || gy == b.Ly - 1;
            if (on) ess_dofs[m++] = (int32_t)i;
        }
    }
    return CDFEM_OK;
}

// ---- Kuhn simplex meshes (BASELINE config C4: "unstructured tet mesh ~1M elements") ----------
// [0,1]^dim cut into n^dim cubes, each split into dim! simplices along the axis permutations
// (v_{k+1} = v_k + e_pi(k)); odd permutations swap the last two vertices so det J > 0.  Element
// order: cube-major, permutations lexicographic.  H1 P1/P2 dofs = the (p n + 1)^dim lattice
// (a P2 edge midpoint is the unique odd lattice point of its edge), lexicographic.  The solver
// path treats the result as an unstructured mesh (explicit element -> dof map, CSR).
int cdfem_kuhn_sizes(int dim, int n, int order, int *ne, int64_t *nldofs, int *n_ess)
{
    if ((dim != 2 && dim != 3) || n < 1 || order < 1 || order > 2) return CDFEM_ERR_ARG;
    const int64_t L = (int64_t)order * n + 1;
    const int64_t nl = dim == 3 ? L * L * L : L * L;
    const int64_t inner = dim == 3 ? (L - 2) * (L - 2) * (L - 2) : (L - 2) * (L - 2);
    if (ne) *ne = dim == 3 ? 6 * n * n * n : 2 * n * n;
    if (nldofs) *nldofs = nl;
    if (n_ess) *n_ess = (int)(nl - inner);
    return CDFEM_OK;
}

int cdfem_kuhn_mesh(int dim, int n, int order, double perturb, double *elem_verts, int32_t *elem_dofs,
                    int32_t *ess_dofs, double *dof_xyz)
{
    static const int perm3[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
    static const int odd3[6] = {0, 1, 1, 0, 0, 1};
    static const int perm2[2][2] = {{0, 1}, {1, 0}};
    int ne;
    int64_t nl;
    if (cdfem_kuhn_sizes(dim, n, order, &ne, &nl, nullptr) != CDFEM_OK) return CDFEM_ERR_ARG;
    const int p = order, nsub = dim == 3 ? 6 : 2, nv = dim + 1, nd = cdfem::simplex_ndofs(dim, p);
    const int64_t L = (int64_t)p * n + 1;
    const int ncube = dim == 3 ? n * n * n : n * n;
    const double h = 1.0 / n;
    bool inverted = false;
    for (int ci = 0; ci < ncube; ++ci) {
        const int c[3] = {ci % n, (ci / n) % n, dim == 3 ? ci / (n * n) : 0};
        for (int s = 0; s < nsub; ++s) {
            const int e = ci * nsub + s;
            int V[4][3] = {};
            for (int k = 0; k < 3; ++k) V[0][k] = c[k];
            for (int k = 0; k < dim; ++k) {
                const int ax = dim == 3 ? perm3[s][k] : perm2[s][k];
                for (int m = 0; m < 3; ++m) V[k + 1][m] = V[k][m] + (m == ax ? 1 : 0);
            }
            if (dim == 3 ? odd3[s] : s == 1)
                for (int m = 0; m < 3; ++m) std::swap(V[dim][m], V[dim - 1][m]);
            double X[4][3] = {};
            for (int v = 0; v < nv; ++v) {
                bool interior = true;
                for (int k = 0; k < dim; ++k) {
                    X[v][k] = V[v][k] * h;
                    interior = interior && V[v][k] > 0 && V[v][k] < n;
                }
                if (perturb > 0.0 && interior) {
                    const uint64_t id = (uint64_t)V[v][0] + (uint64_t)(n + 1) * ((uint64_t)V[v][1] + (uint64_t)(n + 1) * V[v][2]);
                    for (int k = 0; k < dim; ++k) X[v][k] += perturb * h * jitter(3 * id + k);
                }
                if (elem_verts)
                    for (int k = 0; k < dim; ++k) elem_verts[((size_t)e * nv + v) * dim + k] = X[v][k];
            }
            double J[3][3] = {};
            for (int k = 0; k < dim; ++k)
                for (int m = 0; m < dim; ++m) J[k][m] = X[m + 1][k] - X[0][k];
            const double det = dim == 3 ? J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) -
                                              J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                                              J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0])
                                        : J[0][0] * J[1][1] - J[0][1] * J[1][0];
            if (!(det > 0.0)) inverted = true;
            for (int l = 0; l < nd; ++l) {
                int G[3] = {0, 0, 0};
                double Xl[3] = {0, 0, 0};
                if (l < nv) {
                    for (int m = 0; m < 3; ++m) G[m] = p * V[l][m];
                    for (int k = 0; k < dim; ++k) Xl[k] = X[l][k];
                } else {
                    const int ed = l - nv;
                    const int a = dim == 3 ? cdfem::kSimplexEdge[ed][0] : cdfem::kTriEdge[ed][0];
                    const int b = dim == 3 ? cdfem::kSimplexEdge[ed][1] : cdfem::kTriEdge[ed][1];
                    for (int m = 0; m < 3; ++m) G[m] = V[a][m] + V[b][m];
                    for (int k = 0; k < dim; ++k) Xl[k] = 0.5 * (X[a][k] + X[b][k]);
                }
                const int64_t gid = G[0] + L * (G[1] + L * G[2]);
                if (elem_dofs) elem_dofs[(size_t)e * nd + l] = (int32_t)gid;
                if (dof_xyz)
                    for (int k = 0; k < dim; ++k) dof_xyz[gid * dim + k] = Xl[k];
            }
        }
    }
    if (ess_dofs) {
        int64_t m = 0;
        for (int64_t i = 0; i < nl; ++i) {
            const int64_t gx = i % L, gy = (i / L) % L, gz = i / (L * L);
            bool on = gx == 0 || gx == L - 1 || gy == 0 || gy == L - 1;
            if (dim == 3) on = on || gz == 0 || gz == L - 1;
            if (on) ess_dofs[m++] = (int32_t)i;
        }
    }
    return inverted ? CDFEM_ERR_ARG : CDFEM_OK;
}

}  // extern "C"
