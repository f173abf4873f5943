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
#include <vector>
#include <string>
#include <sstream>
#include <map>
#include <cstdio>
#include <array>
#include <algorithm>
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

// ---- gmsh v2.2 ASCII meshes (the reference's inputs: Mesh/unit_square.msh, unit_circle.msh) ----
// replaces: make_unique<Mesh>(params.mesh_file.c_str(), 1, 1) (linear_convection_diffusion_2D.cpp:290)
// + H1_FECollection(order, dim) + ParFiniteElementSpace (:311-313) for simplex meshes.
// Domain elements: triangles (2D) or tetrahedra (3D, when present); boundary elements: lines (2D) or
// triangles (3D), physical tag = boundary attribute (1..31; a larger tag is an error, not a silently
// dropped boundary).  Numbering (MFEM's, for triangles): vertex dofs in increasing gmsh node id,
// triangles re-ordered as MFEM's Finalize does (mfem_finalize_triangle), then (order - 1) dofs per
// edge (edges in order of first appearance, dofs along the direction of increasing vertex dof), then
// P3 triangle interiors.  Tetrahedra are re-oriented to det J > 0 (MFEM's MarkTetMeshForRefinement
// vertex order is not restated).
namespace {

struct Gmsh {
    int dim = 0, order = 1, nv = 0, nd = 0;
    std::vector<int32_t> dofs;       // ne * nd
    std::vector<double> verts;       // ne * (dim + 1) * dim
    std::vector<double> xyz;         // nl * dim
    std::vector<int32_t> bmask;      // nl: bit (attr - 1) set on boundary elements of attribute attr
    int64_t nl = 0;
    int ne = 0;
};

// simplex topology: vertices (increasing gmsh node id among the nodes of domain elements), domain
// elements as vertex indices re-oriented to det J > 0, boundary elements (vertex indices) + tags
struct Topo {
    int dim = 0;
    std::vector<double> vxyz;        // nvert * dim
    std::vector<int32_t> ev;         // ne * (dim + 1)
    std::vector<int32_t> bv;         // nbe * dim
    std::vector<int32_t> battr;      // nbe
    int64_t nvert() const { return dim ? (int64_t)vxyz.size() / dim : 0; }
    int ne() const { return dim ? (int)(ev.size() / (dim + 1)) : 0; }
    int nbe() const { return (int)battr.size(); }
};

// MFEM's vertex order for a triangle read from a file: Mesh(file, generate_edges = 1, refine = 1)
// (linear_convection_diffusion_2D.cpp:290) finalizes with CheckElementOrientation(fix = true), which
// swaps vertices 0 and 1 of a clockwise triangle, and then MarkTriMeshForRefinement, which rotates
// every triangle so that its longest edge is 0-1 (Triangle::MarkEdge: squared lengths d0 = |v1-v0|^2,
// d1 = |v2-v1|^2, d2 = |v2-v0|^2; keep if d0 >= d1 and d0 >= d2, else rotate by 1 if d1 > d0 and
// d1 >= d2, else by 2).  The rotation fixes the order in which edges are first met, so it fixes the
// edge-dof numbering, which PETSc's ILU(0) (Input/petsc_circle.opts:6-8) depends on.
void mfem_finalize_triangle(const Topo &T, std::array<int32_t, 4> &v)
{
    auto P = [&](int i, int d) { return T.vxyz[(size_t)v[i] * 2 + d]; };
    const double det = (P(1, 0) - P(0, 0)) * (P(2, 1) - P(0, 1)) - (P(1, 1) - P(0, 1)) * (P(2, 0) - P(0, 0));
    if (det < 0.0) std::swap(v[0], v[1]);
    auto sq = [](double a) { return a * a; };
    const double d0 = sq(P(1, 0) - P(0, 0)) + sq(P(1, 1) - P(0, 1));
    const double d1 = sq(P(2, 0) - P(1, 0)) + sq(P(2, 1) - P(1, 1));
    const double d2 = sq(P(2, 0) - P(0, 0)) + sq(P(2, 1) - P(0, 1));
    int shift;
    if (d0 >= d1) {
        if (d0 >= d2) return;
        shift = 2;
    } else {
        shift = d1 >= d2 ? 1 : 2;
    }
    const std::array<int32_t, 4> o = v;
    if (shift == 1) { v[0] = o[1]; v[1] = o[2]; v[2] = o[0]; }
    else { v[0] = o[2]; v[1] = o[0]; v[2] = o[1]; }
}

bool parse_gmsh(const char *path, Topo &T, std::string &err)
{
    std::FILE *f = std::fopen(path, "r");
    if (!f) { err = "cannot open mesh file"; return false; }
    std::map<long, std::array<double, 3>> nodes;
    struct El { int type, tag; std::vector<long> v; };
    std::vector<El> els;
    char line[4096];
    while (std::fgets(line, sizeof line, f)) {
        if (!std::strncmp(line, "$MeshFormat", 11)) {
            double ver = 0; int ft = 0, ds = 0;
            if (!std::fgets(line, sizeof line, f) || std::sscanf(line, "%lf %d %d", &ver, &ft, &ds) != 3 ||
                ver < 2.0 || ver >= 3.0 || ft != 0) {
                err = "only gmsh 2.x ASCII meshes are supported";
                std::fclose(f);
                return false;
            }
        } else if (!std::strncmp(line, "$Nodes", 6)) {
            long n = 0;
            if (!std::fgets(line, sizeof line, f) || std::sscanf(line, "%ld", &n) != 1) break;
            for (long i = 0; i < n && std::fgets(line, sizeof line, f); ++i) {
                long id; double x, y, z;
                if (std::sscanf(line, "%ld %lf %lf %lf", &id, &x, &y, &z) == 4) nodes[id] = {x, y, z};
            }
        } else if (!std::strncmp(line, "$Elements", 9)) {
            long n = 0;
            if (!std::fgets(line, sizeof line, f) || std::sscanf(line, "%ld", &n) != 1) break;
            for (long i = 0; i < n && std::fgets(line, sizeof line, f); ++i) {
                std::istringstream ss(line);
                long id; int type, ntags;
                ss >> id >> type >> ntags;
                std::vector<long> tags(ntags);
                for (auto &t : tags) ss >> t;
                const int nn = type == 1 ? 2 : type == 2 ? 3 : type == 4 ? 4 : type == 15 ? 1 : -1;
                if (nn < 0) { err = "unsupported gmsh element type " + std::to_string(type); std::fclose(f); return false; }
                El e{type, ntags > 0 ? (int)tags[0] : 1, std::vector<long>(nn)};
                for (auto &v : e.v) ss >> v;
                els.push_back(std::move(e));
            }
        }
    }
    std::fclose(f);
    const bool has_tet = std::any_of(els.begin(), els.end(), [](const El &e) { return e.type == 4; });
    const int dim = has_tet ? 3 : 2, dtype = has_tet ? 4 : 2, btype = has_tet ? 2 : 1;
    T = Topo();
    T.dim = dim;
    std::map<long, int32_t> vid;
    for (const El &e : els)
        if (e.type == dtype)
            for (long v : e.v) vid[v] = 0;
    int32_t k = 0;
    for (auto &kv : vid) {
        auto it = nodes.find(kv.first);
        if (it == nodes.end()) { err = "element references an unknown node"; return false; }
        kv.second = k++;
        for (int d = 0; d < dim; ++d) T.vxyz.push_back(it->second[d]);
    }
    for (const El &e : els) {
        if (e.type != dtype) continue;
        std::array<int32_t, 4> v{};
        for (int i = 0; i <= dim; ++i) v[i] = vid[e.v[i]];
        if (dim == 2) mfem_finalize_triangle(T, v);
        for (int i = 0; i <= dim; ++i) T.ev.push_back(v[i]);
    }
    for (const El &e : els) {
        if (e.type != btype || e.tag < 1) continue;
        if (e.tag > 31) {
            err = "boundary physical tag " + std::to_string(e.tag) + " > 31: boundary attributes 1..31 are supported";
            return false;
        }
        bool inside = true;
        for (long n : e.v) inside = inside && vid.count(n);
        if (!inside) continue;
        for (long n : e.v) T.bv.push_back(vid[n]);
        T.battr.push_back(e.tag);
    }
    if (T.ne() == 0) { err = "mesh has no domain elements"; return false; }
    return true;
}

// H1 Lagrange space of order p on a simplex topology.  Numbering: vertex dofs = vertex index, then
// (order - 1) dofs per edge (edges in order of first appearance, dofs along the direction of
// increasing vertex dof), then P3 triangle interiors.  Elements are re-oriented to det J > 0.
const int kMfemTriEdge[3][2] = {{0, 1}, {1, 2}, {2, 0}};

bool build_space(const Topo &T, int order, Gmsh &G, std::string &err)
{
    const int dim = T.dim;
    if (order < 1 || order > (dim == 2 ? 3 : 2)) { err = "unsupported order for this mesh"; return false; }
    G = Gmsh();
    G.dim = dim; G.order = order; G.nv = dim + 1; G.nd = cdfem::simplex_ndofs(dim, order);
    const int64_t nvd = T.nvert();
    const int nedge_loc = dim == 3 ? 6 : 3, ne_dofs = order - 1;
    auto pos = [&](int32_t v, int d) { return T.vxyz[(size_t)v * dim + d]; };
    std::map<std::pair<int32_t, int32_t>, int32_t> edge;  // (lo, hi) vertex dof -> edge index
    std::vector<std::array<int32_t, 4>> tv;
    for (int e = 0; e < T.ne(); ++e) {
        std::array<int32_t, 4> v{};
        for (int i = 0; i <= dim; ++i) v[i] = T.ev[(size_t)e * (dim + 1) + i];
        for (int i = 0; i <= dim; ++i)
            if (v[i] < 0 || v[i] >= nvd) { err = "element vertex out of range"; return false; }
        double det;
        if (dim == 2) {
            det = (pos(v[1], 0) - pos(v[0], 0)) * (pos(v[2], 1) - pos(v[0], 1)) -
                  (pos(v[1], 1) - pos(v[0], 1)) * (pos(v[2], 0) - pos(v[0], 0));
            if (det < 0) std::swap(v[1], v[2]);
        } else {
            double J[3][3];
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) J[r][c] = pos(v[c + 1], r) - pos(v[0], r);
            det = J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) - J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                  J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
            if (det < 0) std::swap(v[2], v[3]);
        }
        if (det == 0.0) { err = "degenerate element"; return false; }
        tv.push_back(v);
        // edges are numbered in order of first appearance, met in MFEM's local edge order
        // (Geometry::Constants<TRIANGLE>::Edges = (0,1),(1,2),(2,0); tetrahedra (0,1),(0,2),(0,3),
        // (1,2),(1,3),(2,3)), as Mesh::GetElementToEdgeTable's DSTable does
        if (ne_dofs > 0)
            for (int ed = 0; ed < nedge_loc; ++ed) {
                const int la = dim == 3 ? cdfem::kSimplexEdge[ed][0] : kMfemTriEdge[ed][0];
                const int lb = dim == 3 ? cdfem::kSimplexEdge[ed][1] : kMfemTriEdge[ed][1];
                int32_t ga = v[la], gb = v[lb];
                if (ga > gb) std::swap(ga, gb);
                edge.emplace(std::make_pair(ga, gb), (int32_t)edge.size());
            }
    }
    G.ne = (int)tv.size();
    const int64_t nedges = (int64_t)edge.size();
    const int64_t nint = (dim == 2 && order == 3) ? G.ne : 0;
    G.nl = nvd + nedges * ne_dofs + nint;
    G.dofs.assign((size_t)G.ne * G.nd, 0);
    G.verts.assign((size_t)G.ne * G.nv * dim, 0.0);
    G.xyz.assign((size_t)G.nl * dim, 0.0);
    G.bmask.assign(G.nl, 0);
    for (int64_t v = 0; v < nvd; ++v)
        for (int d = 0; d < dim; ++d) G.xyz[(size_t)v * dim + d] = pos((int32_t)v, d);
    auto edge_t = [&](int kk) { return order == 2 ? 0.5 : cdfem::p3_edge_t(kk); };
    for (auto &kv : edge) {
        const int32_t ga = kv.first.first, gb = kv.first.second;
        for (int kk = 0; kk < ne_dofs; ++kk) {
            const int64_t g = nvd + (int64_t)kv.second * ne_dofs + kk;
            const double t = edge_t(kk);
            for (int d = 0; d < dim; ++d) G.xyz[(size_t)g * dim + d] = pos(ga, d) + t * (pos(gb, d) - pos(ga, d));
        }
    }
    for (int e = 0; e < G.ne; ++e) {
        const auto &v = tv[e];
        int32_t *ld = &G.dofs[(size_t)e * G.nd];
        for (int i = 0; i <= dim; ++i) {
            ld[i] = v[i];
            for (int d = 0; d < dim; ++d) G.verts[((size_t)e * G.nv + i) * dim + d] = pos(v[i], d);
        }
        for (int ed = 0; ed < nedge_loc && ne_dofs > 0; ++ed) {
            const int la = dim == 3 ? cdfem::kSimplexEdge[ed][0] : cdfem::kTriEdge[ed][0];
            const int lb = dim == 3 ? cdfem::kSimplexEdge[ed][1] : cdfem::kTriEdge[ed][1];
            const int32_t ga = v[la], gb = v[lb];
            const bool fwd = ga < gb;
            const int32_t id = edge[{std::min(ga, gb), std::max(ga, gb)}];
            for (int kk = 0; kk < ne_dofs; ++kk)
                ld[G.nv + ed * ne_dofs + kk] = (int32_t)(nvd + (int64_t)id * ne_dofs + (fwd ? kk : ne_dofs - 1 - kk));
        }
        if (nint) {
            const int64_t g = nvd + nedges * ne_dofs + e;
            ld[G.nd - 1] = (int32_t)g;
            for (int d = 0; d < dim; ++d) G.xyz[(size_t)g * dim + d] = (pos(v[0], d) + pos(v[1], d) + pos(v[2], d)) / 3.0;
        }
    }
    // boundary attributes: vertices and edge dofs of the boundary elements
    for (int b = 0; b < T.nbe(); ++b) {
        const int32_t bit = 1 << (T.battr[b] - 1);
        const int32_t *bv = &T.bv[(size_t)b * dim];
        for (int i = 0; i < dim; ++i) G.bmask[bv[i]] |= bit;
        for (int i = 0; i < dim && ne_dofs > 0; ++i)
            for (int j = i + 1; j < dim; ++j) {
                auto it = edge.find({std::min(bv[i], bv[j]), std::max(bv[i], bv[j])});
                if (it == edge.end()) continue;
                for (int kk = 0; kk < ne_dofs; ++kk) G.bmask[nvd + (int64_t)it->second * ne_dofs + kk] |= bit;
            }
    }
    return true;
}

bool read_gmsh(const char *path, int order, Gmsh &G, std::string &err)
{
    Topo T;
    return parse_gmsh(path, T, err) && build_space(T, order, G, err);
}

bool topo_from_args(int dim, int64_t nvert, const double *vxyz, int ne, const int32_t *elem_v, int nbe,
                    const int32_t *bdr_v, const int32_t *bdr_attr, Topo &T)
{
    if ((dim != 2 && dim != 3) || nvert < 1 || ne < 1 || !vxyz || !elem_v || nbe < 0 || (nbe > 0 && (!bdr_v || !bdr_attr)))
        return false;
    T = Topo();
    T.dim = dim;
    T.vxyz.assign(vxyz, vxyz + nvert * dim);
    T.ev.assign(elem_v, elem_v + (size_t)ne * (dim + 1));
    if (nbe > 0) {
        T.bv.assign(bdr_v, bdr_v + (size_t)nbe * dim);
        T.battr.assign(bdr_attr, bdr_attr + nbe);
    }
    for (int32_t a : T.battr)
        if (a < 1 || a > 31) return false;
    for (int32_t v : T.bv)
        if (v < 0 || v >= nvert) return false;
    return true;
}

}  // namespace

int cdfem_gmsh_sizes(const char *path, int order, int *dim, int *ne, int64_t *nldofs)
{
    if (!path) return CDFEM_ERR_ARG;
    Gmsh G;
    std::string err;
    if (!read_gmsh(path, order, G, err)) return CDFEM_ERR_ARG;
    if (dim) *dim = G.dim;
    if (ne) *ne = G.ne;
    if (nldofs) *nldofs = G.nl;
    return CDFEM_OK;
}

int cdfem_gmsh_mesh(const char *path, int order, double *elem_verts, int32_t *elem_dofs, int32_t *dof_bdr_mask,
                    double *dof_xyz)
{
    if (!path) return CDFEM_ERR_ARG;
    Gmsh G;
    std::string err;
    if (!read_gmsh(path, order, G, err)) return CDFEM_ERR_ARG;
    if (elem_verts) std::copy(G.verts.begin(), G.verts.end(), elem_verts);
    if (elem_dofs) std::copy(G.dofs.begin(), G.dofs.end(), elem_dofs);
    if (dof_bdr_mask) std::copy(G.bmask.begin(), G.bmask.end(), dof_bdr_mask);
    if (dof_xyz) std::copy(G.xyz.begin(), G.xyz.end(), dof_xyz);
    return CDFEM_OK;
}

int cdfem_gmsh_topology_sizes(const char *path, int *dim, int64_t *nvert, int *ne, int *nbe)
{
    if (!path) return CDFEM_ERR_ARG;
    Topo T;
    std::string err;
    if (!parse_gmsh(path, T, err)) return CDFEM_ERR_ARG;
    if (dim) *dim = T.dim;
    if (nvert) *nvert = T.nvert();
    if (ne) *ne = T.ne();
    if (nbe) *nbe = T.nbe();
    return CDFEM_OK;
}

int cdfem_gmsh_topology(const char *path, double *vxyz, int32_t *elem_v, int32_t *bdr_v, int32_t *bdr_attr)
{
    if (!path) return CDFEM_ERR_ARG;
    Topo T;
    std::string err;
    if (!parse_gmsh(path, T, err)) return CDFEM_ERR_ARG;
    if (vxyz) std::copy(T.vxyz.begin(), T.vxyz.end(), vxyz);
    if (elem_v) std::copy(T.ev.begin(), T.ev.end(), elem_v);
    if (bdr_v) std::copy(T.bv.begin(), T.bv.end(), bdr_v);
    if (bdr_attr) std::copy(T.battr.begin(), T.battr.end(), bdr_attr);
    return CDFEM_OK;
}

int cdfem_simplex_space_sizes(int dim, int64_t nvert, const double *vxyz, int ne, const int32_t *elem_v, int order,
                              int64_t *nldofs)
{
    Topo T;
    Gmsh G;
    std::string err;
    if (!topo_from_args(dim, nvert, vxyz, ne, elem_v, 0, nullptr, nullptr, T) || !build_space(T, order, G, err))
        return CDFEM_ERR_ARG;
    if (nldofs) *nldofs = G.nl;
    return CDFEM_OK;
}

int cdfem_simplex_space(int dim, int64_t nvert, const double *vxyz, int ne, const int32_t *elem_v, int nbe,
                        const int32_t *bdr_v, const int32_t *bdr_attr, int order, double *elem_verts,
                        int32_t *elem_dofs, int32_t *dof_bdr_mask, double *dof_xyz)
{
    Topo T;
    Gmsh G;
    std::string err;
    if (!topo_from_args(dim, nvert, vxyz, ne, elem_v, nbe, bdr_v, bdr_attr, T) || !build_space(T, order, G, err))
        return CDFEM_ERR_ARG;
    if (elem_verts) std::copy(G.verts.begin(), G.verts.end(), elem_verts);
    if (elem_dofs) std::copy(G.dofs.begin(), G.dofs.end(), elem_dofs);
    if (dof_bdr_mask) std::copy(G.bmask.begin(), G.bmask.end(), dof_bdr_mask);
    if (dof_xyz) std::copy(G.xyz.begin(), G.xyz.end(), dof_xyz);
    return CDFEM_OK;
}

// host helpers: the simplex rule and nodal basis the kernels use (for host-side functionals such as
// ComputeL2Error, linear_convection_diffusion_2D.cpp:383-392)
int cdfem_simplex_rule_order(int dim, int order, double *xi, double *w)
{
    if (dim != 2 && dim != 3) return -1;
    std::vector<double> x, ww;
    const int nq = cdfem::simplex_rule_for_order(dim, order, x, ww);
    if (xi) std::copy(x.begin(), x.end(), xi);
    if (w) std::copy(ww.begin(), ww.end(), w);
    return nq;
}

int cdfem_simplex_rule(int dim, int n, double *xi, double *w)
{
    if ((dim != 2 && dim != 3) || n < 1 || n > 16) return -CDFEM_ERR_ARG;
    std::vector<double> x, ww;
    const int nq = cdfem::simplex_rule(dim, n, x, ww);
    if (xi) std::copy(x.begin(), x.end(), xi);
    if (w) std::copy(ww.begin(), ww.end(), w);
    return nq;
}

int cdfem_simplex_basis(int dim, int order, int npts, const double *xi, double *phi, double *dphi)
{
    const int nd = cdfem::simplex_ndofs(dim, order);
    if ((dim != 2 && dim != 3) || nd < 0 || npts < 0 || !xi || !phi) return CDFEM_ERR_ARG;
    double p[10], g[30];
    for (int i = 0; i < npts; ++i) {
        cdfem::simplex_basis(dim, order, xi + (size_t)i * dim, p, g);
        std::copy(p, p + nd, phi + (size_t)i * nd);
        if (dphi) std::copy(g, g + nd * dim, dphi + (size_t)i * nd * dim);
    }
    return CDFEM_OK;
}

}  // extern "C"
