// sell_plan.cpp — row order and SELL-64 layout of the assembled (FA) operator's SpMV (host only).
//
// The reference's assembled path (HypreParMatrix -> PETSc MATAIJ, linear_convection_diffusion_2D.cpp
// :349-375) multiplies in the mesh's own dof numbering.  Here the SpMV may run on a row/column
// permutation of the same matrix, A' = P A P^T (the "space" order; the Krylov solve then runs in it,
// capi.hip cdfem_solve), and the SELL-64 slices are cut from that space in one of two layouts:
//   base order  the mesh numbering ("natural"), a geometric order (dof coordinates quantised to
//               the mean dof spacing, sorted by (z, y, x): a lattice's own order whatever the
//               numbering, and a slab order on unstructured meshes), or reverse Cuthill-McKee of the
//               CSR graph (when no coordinates are given).  A small bandwidth keeps the x gathers
//               L2-local and the 16-bit column deltas valid;
//   layout      global: rows sorted by length over the whole matrix, a row index per lane (the
//               measured best on the lattice numbering);
//               windows: the base order cut into windows of W rows, inside a window rows grouped
//               by length (descending) and stencil signature, then base position; the space order
//               IS the slice order (no row index stream, whole-line y stores, 1.00x HBM traffic),
//               W the largest candidate for which every |column' - row'| fits 16 bits.
// In the mesh order every row keeps its CSR entry order (bitwise the CSR sums).  In a permuted space
// a row's entries are summed in ascending space column, so that the j-th entries of a slice's rows
// are the same stencil neighbour (coalesced x gathers); the sums then differ from the CSR order's by
// rounding only, and the Krylov dot products run in the space order.
//
// sell_order: 0 = natural + global (the mesh order, no permutation), 1 = natural + windows,
//             2 = RCM + windows, 3 = auto (mode 0 when the mesh order is banded: 16-bit deltas and
//             bandwidth under nl / 8; else the geometric order when coordinates are given and it
//             is banded that way; else RCM + global when its bandwidth is under half the natural
//             one; when no order is banded — an unstructured mesh — Morton windows with coordinates,
//             else RCM windows, both LDS-staged, spmv_lds auto), 4 = RCM + global, 5 = geometric +
//             global, 6 = Morton + windows, 7 = Morton + global (morton_order), 8 = Morton windows
//             staged in LDS when coordinates are known, else 3 (cdfem_fa_setup's default).
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <vector>

#include "cdfem_internal.hpp"

namespace cdfem {

namespace {

template <class F>
void par_for(int64_t n, F &&f)
{
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const int64_t chunk = (n + hw - 1) / hw;
    std::vector<std::thread> th;
    for (unsigned t = 0; t < hw; ++t) {
        const int64_t lo = t * chunk, hi = std::min(n, lo + chunk);
        if (lo >= hi) break;
        th.emplace_back([&, lo, hi] { f(lo, hi); });
    }
    for (auto &x : th) x.join();
}

inline uint64_t mix64(uint64_t z)
{
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// max |pos[col] - pos[row]| over the pattern (pos = identity when empty)
int64_t bandwidth(int64_t nl, const int32_t *rowptr, const int32_t *cols, const std::vector<int32_t> &pos)
{
    std::vector<int64_t> part(16, 0);
    std::vector<std::thread> th;
    const int64_t chunk = (nl + 15) / 16;
    for (int t = 0; t < 16; ++t)
        th.emplace_back([&, t] {
            int64_t m = 0;
            for (int64_t i = t * chunk; i < std::min(nl, (t + 1) * chunk); ++i) {
                const int64_t pi = pos.empty() ? i : pos[i];
                for (int32_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
                    const int64_t pc = pos.empty() ? cols[k] : pos[cols[k]];
                    m = std::max(m, pc > pi ? pc - pi : pi - pc);
                }
            }
            part[t] = m;
        });
    for (auto &x : th) x.join();
    return *std::max_element(part.begin(), part.end());
}

// BFS levels from s over unvisited-marked rows; returns the last visited row and the depth
int64_t bfs_far(int64_t nl, const int32_t *rowptr, const int32_t *cols, int32_t s, std::vector<int32_t> &lev,
                int32_t *far_out)
{
    std::fill(lev.begin(), lev.end(), -1);
    std::vector<int32_t> q{s};
    lev[s] = 0;
    int32_t far = s;
    for (size_t h = 0; h < q.size(); ++h) {
        const int32_t u = q[h];
        if (lev[u] > lev[far] || (lev[u] == lev[far] && rowptr[u + 1] - rowptr[u] < rowptr[far + 1] - rowptr[far]))
            far = u;
        for (int32_t k = rowptr[u]; k < rowptr[u + 1]; ++k)
            if (lev[cols[k]] < 0) {
                lev[cols[k]] = lev[u] + 1;
                q.push_back(cols[k]);
            }
    }
    *far_out = far;
    (void)nl;
    return lev[far];
}

}  // namespace

// reverse Cuthill-McKee order (order[k] = row at position k): per connected component a
// pseudo-peripheral start (repeated BFS to the farthest, lowest-degree row), neighbours visited in
// ascending degree then ascending index, whole sequence reversed.  Deterministic.
std::vector<int32_t> rcm_order(int64_t nl, const int32_t *rowptr, const int32_t *cols)
{
    std::vector<int32_t> order;
    order.reserve(nl);
    std::vector<char> seen(nl, 0);
    std::vector<int32_t> lev(nl, -1), nb;
    auto deg = [&](int32_t r) { return rowptr[r + 1] - rowptr[r]; };
    for (int64_t s0 = 0; s0 < nl; ++s0) {
        if (seen[s0]) continue;
        int32_t s = (int32_t)s0, far;
        int64_t d = bfs_far(nl, rowptr, cols, s, lev, &far);
        for (int it = 0; it < 8; ++it) {  // pseudo-peripheral node
            int32_t f2;
            const int64_t d2 = bfs_far(nl, rowptr, cols, far, lev, &f2);
            if (d2 <= d) break;
            s = far;
            far = f2;
            d = d2;
        }
        const size_t h0 = order.size();
        order.push_back(s);
        seen[s] = 1;
        for (size_t h = h0; h < order.size(); ++h) {
            const int32_t u = order[h];
            nb.clear();
            for (int32_t k = rowptr[u]; k < rowptr[u + 1]; ++k)
                if (!seen[cols[k]]) {
                    seen[cols[k]] = 1;
                    nb.push_back(cols[k]);
                }
            std::sort(nb.begin(), nb.end(), [&](int32_t a, int32_t b) {
                return deg(a) != deg(b) ? deg(a) < deg(b) : a < b;
            });
            order.insert(order.end(), nb.begin(), nb.end());
        }
    }
    std::reverse(order.begin(), order.end());
    return order;
}

std::vector<double> simplex_dof_coords(int dim, int p, int ne, int nd, int64_t nl, const std::vector<double> &verts,
                                       const std::vector<int32_t> &dofs)
{
    // reference nodes (vertex 0 at the origin, vertex k at e_k), in the local dof order
    std::vector<std::array<double, 3>> ref;
    for (int v = 0; v <= dim; ++v) {
        std::array<double, 3> x{0, 0, 0};
        if (v > 0) x[v - 1] = 1.0;
        ref.push_back(x);
    }
    if (dim == 2 && p == 3) {
        double X[10][2];
        p3_tri_nodes(X);
        ref.clear();
        for (auto &r : X) ref.push_back({r[0], r[1], 0.0});
    } else if (p == 2) {
        const int ne_ = dim == 3 ? 6 : 3;
        for (int e = 0; e < ne_; ++e) {
            const int a = dim == 3 ? kSimplexEdge[e][0] : kTriEdge[e][0], b = dim == 3 ? kSimplexEdge[e][1] : kTriEdge[e][1];
            std::array<double, 3> x{0, 0, 0};
            for (int k = 0; k < 3; ++k) x[k] = 0.5 * (ref[a][k] + ref[b][k]);
            ref.push_back(x);
        }
    }
    if ((int)ref.size() != nd) throw std::runtime_error("simplex_dof_coords: unsupported element");
    std::vector<double> xyz((size_t)nl * dim, 0.0);
    for (int e = 0; e < ne; ++e) {
        const double *V = &verts[(size_t)e * (dim + 1) * dim];
        for (int l = 0; l < nd; ++l) {
            const int64_t g = dofs[(size_t)e * nd + l];
            for (int k = 0; k < dim; ++k) {
                double x = V[k];
                for (int m = 0; m < dim; ++m) x += ref[l][m] * (V[(m + 1) * dim + k] - V[k]);
                xyz[(size_t)g * dim + k] = x;
            }
        }
    }
    return xyz;
}

// geometric order: dof coordinates quantised to the mean dof spacing h = (box volume / nl)^(1/dim)
// and sorted by (z cell, y cell, x); ties by mesh index (deterministic)
std::vector<int32_t> geometric_order(int64_t nl, int dim, const double *xyz)
{
    double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
    for (int k = 0; k < dim; ++k) {
        lo[k] = hi[k] = xyz[k];
        for (int64_t i = 1; i < nl; ++i) {
            lo[k] = std::min(lo[k], xyz[i * dim + k]);
            hi[k] = std::max(hi[k], xyz[i * dim + k]);
        }
    }
    double vol = 1.0;
    for (int k = 0; k < dim; ++k) vol *= std::max(hi[k] - lo[k], 1e-300);
    const double h = std::pow(vol / (double)std::max<int64_t>(nl, 1), 1.0 / dim);
    std::vector<int64_t> cz(nl), cy(nl);
    for (int64_t i = 0; i < nl; ++i) {
        cy[i] = dim >= 2 ? std::llround((xyz[i * dim + 1] - lo[1]) / h) : 0;
        cz[i] = dim >= 3 ? std::llround((xyz[i * dim + 2] - lo[2]) / h) : 0;
    }
    std::vector<int32_t> order(nl);
    for (int64_t i = 0; i < nl; ++i) order[i] = (int32_t)i;
    std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
        if (cz[a] != cz[b]) return cz[a] < cz[b];
        if (cy[a] != cy[b]) return cy[a] < cy[b];
        const double xa = xyz[(int64_t)a * dim], xb = xyz[(int64_t)b * dim];
        return xa != xb ? xa < xb : a < b;
    });
    return order;
}

// Morton (Z-curve) order of the dof coordinates: each axis quantised to 2^21 cells of the bounding
// box, bits interleaved (x lowest), ties by mesh index.  A space-filling curve keeps every run of
// consecutive positions spatially compact on any mesh (unlike the slab order of geometric_order, whose
// bandwidth on an unstructured mesh is the long edges' reach across z cells).
std::vector<int32_t> morton_order(int64_t nl, int dim, const double *xyz)
{
    double lo[3] = {0, 0, 0}, hi[3] = {1, 1, 1};
    for (int k = 0; k < dim; ++k) {
        lo[k] = hi[k] = xyz[k];
        for (int64_t i = 1; i < nl; ++i) {
            lo[k] = std::min(lo[k], xyz[i * dim + k]);
            hi[k] = std::max(hi[k], xyz[i * dim + k]);
        }
    }
    const int bits = dim == 3 ? 21 : 31;
    const double cells = (double)((1u << bits) - 1);
    std::vector<uint64_t> key(nl);
    par_for(nl, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            uint64_t q[3] = {0, 0, 0};
            for (int k = 0; k < dim; ++k) {
                const double t = (xyz[i * dim + k] - lo[k]) / std::max(hi[k] - lo[k], 1e-300);
                q[k] = (uint64_t)std::llround(std::min(std::max(t, 0.0), 1.0) * cells);
            }
            uint64_t m = 0;
            for (int bit = bits - 1; bit >= 0; --bit)
                for (int k = dim - 1; k >= 0; --k) m = (m << 1) | ((q[k] >> bit) & 1u);
            key[i] = m;
        }
    });
    std::vector<int32_t> order(nl);
    for (int64_t i = 0; i < nl; ++i) order[i] = (int32_t)i;
    std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return key[a] != key[b] ? key[a] < key[b] : a < b; });
    return order;
}

SellPlan sell_plan(int64_t nl, const int32_t *rowptr, const int32_t *cols, int mode, int dim, const double *xyz,
                   int64_t window)
{
    SellPlan pl;
    pl.mode = mode;
    pl.base = 1;
    if (mode < 0 || mode > 8) throw std::runtime_error("sell_plan: bad mode");
    // 8 (the FA setup's default): Morton windows staged in LDS whenever the dof coordinates are known
    // (lattice or unstructured alike), else the auto mode 3
    if (mode == 8) {
        if (xyz && dim >= 1 && dim <= 3) {
            mode = 6;
            pl.auto_lds = true;
            if (window <= 0) window = kAutoLdsRows;
        } else {
            mode = 3;
        }
        pl.mode = mode;
    }
    if ((mode == 5 || mode >= 6) && !xyz) throw std::runtime_error("sell_plan: the geometric / Morton order needs dof coordinates");
    if (mode == 0 || nl == 0) return pl;
    // base order
    std::vector<int32_t> bo, bp;  // base position -> row, row -> base position (empty: identity)
    pl.bw_natural = bandwidth(nl, rowptr, cols, {});
    auto banded = [&](int64_t bw) { return bw <= 32767 && bw * 8 <= nl; };
    if ((mode == 3 || mode == 5) && xyz && dim >= 1 && dim <= 3 && !(mode == 3 && banded(pl.bw_natural))) {
        std::vector<int32_t> go = geometric_order(nl, dim, xyz), gp(nl);
        for (int64_t k = 0; k < nl; ++k) gp[go[k]] = (int32_t)k;
        pl.bw_geometric = bandwidth(nl, rowptr, cols, gp);
        if (mode == 5 || banded(pl.bw_geometric)) {
            pl.base = 3;
            pl.windowed = false;
            pl.max_delta = pl.bw_geometric;
            pl.perm = std::move(go);
            return pl;
        }
        // an unstructured mesh (no banded order exists): Morton windows, staged in LDS
        mode = 6;
        pl.auto_lds = true;
        if (window <= 0) window = kAutoLdsRows;
    }
    if (mode >= 6) {  // Morton base order: 6 + windows, 7 + global length sort (auto: an unstructured mesh)
        bo = morton_order(nl, dim, xyz);
        bp.resize(nl);
        for (int64_t k = 0; k < nl; ++k) bp[bo[k]] = (int32_t)k;
        pl.base = 4;
        pl.bw_geometric = bandwidth(nl, rowptr, cols, bp);
        if (mode == 7) {
            pl.windowed = false;
            pl.max_delta = pl.bw_geometric;
            pl.perm = std::move(bo);
            return pl;
        }
    }
    bool rcm = mode == 2 || mode == 4;
    const bool morton = mode == 6;
    // the mesh order is banded (16-bit deltas, bandwidth under nl / 8): mode 0 without the RCM pass
    if (mode == 3 && banded(pl.bw_natural)) return pl;
    if (mode >= 2 && !morton) {
        bo = rcm_order(nl, rowptr, cols);
        bp.resize(nl);
        for (int64_t k = 0; k < nl; ++k) bp[bo[k]] = (int32_t)k;
        pl.bw_rcm = bandwidth(nl, rowptr, cols, bp);
        if (mode == 3) rcm = 2 * pl.bw_rcm < pl.bw_natural;
        if (mode == 3 && rcm && !banded(pl.bw_rcm)) {
            // no coordinates and no banded order: RCM windows, staged in LDS
            mode = 2;
            pl.auto_lds = true;
            if (window <= 0) window = kAutoLdsRows;
        }
        if (!rcm) {
            bo.clear();
            bp.clear();
        }
    }
    pl.base = morton ? 4 : rcm ? 2 : 1;
    if (mode >= 3 && !morton) {  // global length sort over the base order: the space order is the base order
        pl.windowed = false;
        pl.max_delta = rcm ? pl.bw_rcm : pl.bw_natural;
        pl.perm = std::move(bo);
        return pl;
    }
    pl.windowed = true;
    auto B = [&](int64_t r) -> int64_t { return bp.empty() ? r : bp[r]; };
    auto R = [&](int64_t k) -> int32_t { return bo.empty() ? (int32_t)k : bo[k]; };
    // stencil signature: row length + order-independent hash of the base-order column offsets
    std::vector<uint64_t> sig(nl);
    par_for(nl, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; ++i) {
            uint64_t h = 0;
            for (int32_t k = rowptr[i]; k < rowptr[i + 1]; ++k) h += mix64((uint64_t)(B(cols[k]) - B(i)));
            sig[i] = h;
        }
    });
    auto len = [&](int32_t r) { return rowptr[r + 1] - rowptr[r]; };
    std::vector<int32_t> perm(nl), inv(nl);
    auto build = [&](int64_t W) {
        const int64_t nw = (nl + W - 1) / W;
        par_for(nw, [&](int64_t w0, int64_t w1) {
            std::vector<int32_t> rows, bys;
            for (int64_t w = w0; w < w1; ++w) {
                const int64_t s = w * W, e = std::min(nl, s + W);
                rows.clear();
                for (int64_t k = s; k < e; ++k) rows.push_back(R(k));
                // frequent signatures (>= one slice of rows in the window) form classes; the
                // rest (boundary rows) stay in base order inside their length group
                bys = rows;
                std::sort(bys.begin(), bys.end(), [&](int32_t a, int32_t b) { return sig[a] < sig[b]; });
                std::vector<std::pair<uint64_t, char>> cls;
                for (size_t a = 0; a < bys.size();) {
                    size_t b = a;
                    while (b < bys.size() && sig[bys[b]] == sig[bys[a]]) ++b;
                    cls.push_back({sig[bys[a]], (char)(b - a >= (size_t)kLanes)});
                    a = b;
                }
                auto frequent = [&](int32_t r) {
                    const auto it = std::lower_bound(cls.begin(), cls.end(), std::make_pair(sig[r], (char)0),
                                                     [](const auto &x, const auto &y) { return x.first < y.first; });
                    return it->second != 0;
                };
                std::vector<std::pair<char, int32_t>> key(rows.size());
                for (size_t a = 0; a < rows.size(); ++a) key[a] = {(char)(frequent(rows[a]) ? 0 : 1), rows[a]};
                std::vector<int32_t> idx(rows.size());
                for (size_t a = 0; a < idx.size(); ++a) idx[a] = (int32_t)a;
                std::sort(idx.begin(), idx.end(), [&](int32_t a, int32_t b) {
                    const int32_t ra = rows[a], rb = rows[b];
                    if (len(ra) != len(rb)) return len(ra) > len(rb);
                    if (key[a].first != key[b].first) return key[a].first < key[b].first;
                    if (key[a].first == 0 && sig[ra] != sig[rb]) return sig[ra] < sig[rb];
                    return a < b;  // base position
                });
                for (size_t a = 0; a < idx.size(); ++a) perm[s + a] = rows[idx[a]];
            }
        });
        for (int64_t k = 0; k < nl; ++k) inv[perm[k]] = (int32_t)k;
        return bandwidth(nl, rowptr, cols, inv);
    };
    // the largest window whose deltas fit 16 bits; 4096 with 32-bit columns when none does (a given
    // window: that one, the slices beyond 16 bits streaming 32-bit columns)
    int64_t chosen = 0;
    if (window > 0) {
        chosen = window;
        pl.max_delta = build(window);
    }
    for (int64_t W : {32768, 16384, 8192, 4096, 2048, 1024, 512}) {
        if (chosen) break;
        const int64_t d = build(W);
        if (d <= 32767) {
            chosen = W;
            pl.max_delta = d;
            break;
        }
    }
    if (!chosen) {
        chosen = 4096;
        pl.max_delta = build(chosen);
    }
    pl.window = chosen;
    pl.perm = std::move(perm);
    return pl;
}

// SELL-64 over the plan's space order (identity when pl.perm is empty): windowed -> slice k holds
// space rows 64k.. (no row index), global -> space rows stably sorted by length, srows per lane
void sell_build(FaPattern &P, int64_t nl, const SellPlan &pl)
{
    const std::vector<int32_t> &rowptr = P.rowptr, &cols = P.cols;
    // LDS-staged windowed layouts may give each row LPR lanes (R = 64 / LPR rows per slice, lane l
    // holding the (l / R)-th contiguous part of row l % R's entries): less padding on meshes whose row
    // lengths vary (the partial sums are combined in a fixed order by the kernel, k_sell_spmv_lds)
    const int LPR = (pl.windowed && pl.lds_rows > 0) ? std::max(1, pl.lpr) : 1;
    if (LPR != 1 && LPR != 2 && LPR != 4) throw std::runtime_error("sell_build: lanes per row must be 1, 2 or 4");
    const int R = kLanes / LPR;
    const int64_t ns = (nl + R - 1) / R;
    P.lpr = LPR;
    const std::vector<int32_t> &sp = pl.perm;  // space row -> mesh row
    std::vector<int32_t> inv;                   // mesh row -> space row
    if (!sp.empty()) {
        inv.resize(nl);
        for (int64_t k = 0; k < nl; ++k) inv[sp[k]] = (int32_t)k;
        P.perm = sp;
    }
    P.windowed = pl.windowed;
    auto mrow = [&](int64_t q) -> int32_t { return sp.empty() ? (int32_t)q : sp[q]; };
    auto rlen = [&](int64_t q) { const int32_t r = mrow(q); return rowptr[r + 1] - rowptr[r]; };
    std::vector<int32_t> order(nl);  // slice position -> space row
    for (int64_t i = 0; i < nl; ++i) order[i] = (int32_t)i;
    auto by_len = [&](int32_t a, int32_t b) { return rlen(a) > rlen(b); };
    if (!pl.windowed) std::stable_sort(order.begin(), order.end(), by_len);
    const bool permuted = pl.windowed;  // kernel row = slice position (no srows)
    P.sptr.assign(ns + 1, 0);
    if (!permuted) P.srows.assign(ns * kLanes, -1);
    int64_t stored = 0;
    for (int64_t sl = 0; sl < ns; ++sl) {
        int len = 0;  // entries per lane
        for (int l = 0; l < R && sl * R + l < nl; ++l) {
            const int32_t q = order[sl * R + l];
            if (!permuted) P.srows[sl * kLanes + l] = q;
            len = std::max(len, (rlen(q) + LPR - 1) / LPR);
        }
        stored += (int64_t)len * kLanes;
        if (stored >= ((int64_t)1 << 31)) throw std::runtime_error("SELL storage exceeds int32 indexing");
        P.sptr[sl + 1] = (int32_t)stored;
    }
    P.scols.assign(stored, 0);
    P.smap.assign(stored, -1);
    // lane's own index in the space order (the base of its column deltas): its srows entry (global
    // layout) or its slice position (windowed); padding lanes take max(row, 0) / nl - 1
    auto lane_base = [&](int64_t sl, int l) -> int64_t {
        const int64_t k = sl * R + l % R;
        if (permuted) return std::min<int64_t>(k, nl - 1);
        const int32_t r = P.srows[sl * kLanes + l];
        return r >= 0 ? r : 0;
    };
    par_for(ns, [&](int64_t s0, int64_t s1) {
        std::vector<int32_t> ent;
        for (int64_t sl = s0; sl < s1; ++sl) {
            const int len = (P.sptr[sl + 1] - P.sptr[sl]) / kLanes;
            for (int l = 0; l < kLanes; ++l) {
                const int64_t k = sl * R + l % R;
                const int part = l / R;
                const int32_t r = (k < nl && (permuted || l < R)) ? mrow(order[k]) : -1;  // mesh row
                // a row's entries in ascending space column: in a permuted space the j-th entries
                // of a slice's rows are then the same stencil neighbour (one short contiguous run
                // of x per gather); the mesh order keeps its CSR order (bitwise the CSR sums)
                ent.clear();
                if (r >= 0)
                    for (int32_t q = rowptr[r]; q < rowptr[r + 1]; ++q) ent.push_back(q);
                if (!inv.empty())
                    std::sort(ent.begin(), ent.end(), [&](int32_t a, int32_t b) { return inv[cols[a]] < inv[cols[b]]; });
                const int h = ((int)ent.size() + LPR - 1) / LPR;  // this row's entries per lane
                for (int j = 0; j < len; ++j) {
                    const int64_t t = P.sptr[sl] + (int64_t)j * kLanes + l;
                    const int e = part * h + j;
                    if (r >= 0 && j < h && e < (int)ent.size()) {
                        const int32_t c = cols[ent[e]];
                        P.scols[t] = inv.empty() ? c : inv[c];
                        P.smap[t] = ent[e];
                    } else {
                        P.scols[t] = (int32_t)lane_base(sl, l);  // padding: a valid column, value 0
                    }
                }
            }
        }
    });
    // column - lane base in 16 bits where it fits (10 instead of 12 streamed bytes per entry).  A
    // slice holding a delta beyond 16 bits (an unstructured mesh's far neighbours) keeps streaming
    // its 32-bit columns and is flagged in swide; the 16-bit stream is built when at least half of
    // the stored entries lie in slices that fit (every slice of a lattice numbering does)
    std::vector<uint8_t> wide((size_t)ns, 0);
    int64_t stored_wide = LPR > 1 ? stored : 0;  // multi-lane rows: LDS positions only, no deltas
    for (int64_t sl = 0; sl < ns && LPR > 1; ++sl) wide[sl] = 1;
    for (int64_t sl = 0; sl < ns && LPR == 1; ++sl) {
        for (int32_t t = P.sptr[sl]; t < P.sptr[sl + 1]; ++t) {
            const int64_t d = (int64_t)P.scols[t] - lane_base(sl, (t - P.sptr[sl]) % kLanes);
            if (d < -32768 || d > 32767) { wide[sl] = 1; break; }
        }
        if (wide[sl]) stored_wide += P.sptr[sl + 1] - P.sptr[sl];
    }
    if (2 * stored_wide <= stored) {
        P.sdel.assign(stored, 0);
        for (int64_t sl = 0; sl < ns; ++sl) {
            if (wide[sl]) {
                for (int32_t t = P.sptr[sl]; t < P.sptr[sl + 1]; ++t) P.nnz_wide += P.smap[t] >= 0;
                continue;
            }
            for (int32_t t = P.sptr[sl]; t < P.sptr[sl + 1]; ++t)
                P.sdel[t] = (int16_t)(P.scols[t] - lane_base(sl, (t - P.sptr[sl]) % kLanes));
        }
        if (stored_wide) P.swide = std::move(wide);
    }
    // LDS-staged windows: every window of S consecutive slices stages its distinct columns, ascending
    // (the x values it reads), and the entries address them by 16-bit window positions.  Windows
    // halve (down to one slice) until every halo fits kLdsHaloMax doubles.
    if (pl.lds_rows > 0 && permuted) {
        int64_t S = std::max<int64_t>(1, pl.lds_rows / R);  // slices per window
        for (;; S = std::max<int64_t>(1, S / 2)) {
            const int64_t nw = (ns + S - 1) / S;
            std::vector<std::vector<int32_t>> halo((size_t)nw);
            std::vector<int32_t> hmax(16, 0);
            par_for(nw, [&](int64_t w0, int64_t w1) {
                for (int64_t w = w0; w < w1; ++w) {
                    auto &h = halo[(size_t)w];
                    const int64_t s0 = w * S, s1 = std::min(ns, s0 + S);
                    h.assign(P.scols.begin() + P.sptr[s0], P.scols.begin() + P.sptr[s1]);
                    std::sort(h.begin(), h.end());
                    h.erase(std::unique(h.begin(), h.end()), h.end());
                }
            });
            int64_t big = 0;
            for (auto &h : halo) big = std::max<int64_t>(big, (int64_t)h.size());
            if (big > kLdsHaloMax && S > 1) continue;
            if (big > kLdsHaloMax) {  // one slice does not fit: no LDS layout
                if (LPR > 1) throw std::runtime_error("sell_build: a multi-lane SELL slice exceeds the LDS halo budget");
                break;
            }
            P.lds_rows = S * R;
            P.lds_max = (int32_t)big;
            P.hptr.assign((size_t)nw + 1, 0);
            for (int64_t w = 0; w < nw; ++w) P.hptr[w + 1] = P.hptr[w] + (int32_t)halo[(size_t)w].size();
            P.hidx.resize((size_t)P.hptr[nw]);
            P.sloc.resize((size_t)stored);
            par_for(nw, [&](int64_t w0, int64_t w1) {
                for (int64_t w = w0; w < w1; ++w) {
                    const auto &h = halo[(size_t)w];
                    std::copy(h.begin(), h.end(), P.hidx.begin() + P.hptr[w]);
                    const int64_t s0 = w * S, s1 = std::min(ns, s0 + S);
                    for (int32_t t = P.sptr[s0]; t < P.sptr[s1]; ++t)
                        P.sloc[t] = (uint16_t)(std::lower_bound(h.begin(), h.end(), P.scols[t]) - h.begin());
                }
            });
            break;
        }
    }
}

}  // namespace cdfem

extern "C" {

// host-only plan of the FA SpMV order (tests / tools): perm (space row -> mesh row) of nl entries,
// and info[0..6] = base (1 natural, 2 RCM, 3 geometric), window rows (0: global length sort), max
// |column - row| in the space order, natural bandwidth, RCM bandwidth (0 when not computed),
// stored SELL entries / nnz * 1e6 (padding, parts per million), geometric bandwidth (0 when not
// computed)
int cdfem_sell_plan(int64_t nl, const int32_t *rowptr, const int32_t *cols, int mode, int dim, const double *xyz,
                    int32_t *perm, int64_t *info)
{
    try {
        if (nl < 0 || (nl > 0 && (!rowptr || !cols)) || !perm || !info) return CDFEM_ERR_ARG;
        cdfem::SellPlan pl = cdfem::sell_plan(nl, rowptr, cols, mode, dim, xyz);
        cdfem::FaPattern P;
        P.rowptr.assign(rowptr, rowptr + nl + 1);
        P.cols.assign(cols, cols + rowptr[nl]);
        P.nnz = rowptr[nl];
        cdfem::sell_build(P, nl, pl);
        for (int64_t k = 0; k < nl; ++k) perm[k] = pl.perm.empty() ? (int32_t)k : pl.perm[k];
        info[0] = pl.base;
        info[1] = pl.window;
        info[2] = pl.max_delta;
        info[3] = pl.bw_natural;
        info[4] = pl.bw_rcm;
        info[5] = P.nnz ? (int64_t)((double)P.sptr.back() / (double)P.nnz * 1e6) : 0;
        info[6] = pl.bw_geometric;
        return CDFEM_OK;
    } catch (const std::exception &) {
        return CDFEM_ERR_ARG;
    }
}

}  // extern "C"
