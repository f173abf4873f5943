// partition.cpp — element partition of a conforming mesh over ranks and the rank-local H1 space
// (host only).  Replaces ParMesh(MPI_COMM_WORLD, mesh) + ParFiniteElementSpace's shared-dof groups
// (linear_convection_diffusion_2D.cpp:300,312; diffusion_mms_ale.cpp:813,826) for meshes that are
// not structured boxes (the box path uses z-slabs, cdfem_box_mesh with a z range).
//
// Partition: recursive coordinate bisection of the element centroids.  MFEM calls METIS, which is
// not available; any element partition defines the same global operator (A = sum_r P_r^T A_r P_r),
// so the solution is partition-independent up to rounding.  The bisection is deterministic (ties
// broken by element index) so every rank computes the same partition without communication.
//
// Rank-local space: the rank's elements in ascending global order; its dofs numbered with the dofs
// OWNED by a lower rank first (owner = lowest rank holding the dof), then its own, each group by
// ascending global id — so the true dofs are the suffix of the L-vector (cdfem_set_shared).  Per
// neighbour rank, the shared local dofs in ascending global id, the same order on both sides.
#include <algorithm>
#include <cstdint>
#include <numeric>
#include <vector>

#include "cdfem_internal.hpp"

namespace cdfem {

namespace {

void rcb(const std::vector<double> &cen, int dim, std::vector<int32_t> &elems, size_t lo, size_t hi, int rank0,
         int nr, int32_t *part)
{
    if (nr == 1 || hi - lo <= 1) {
        for (size_t i = lo; i < hi; ++i) part[elems[i]] = rank0;
        return;
    }
    double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
    for (size_t i = lo; i < hi; ++i)
        for (int k = 0; k < dim; ++k) {
            mn[k] = std::min(mn[k], cen[(size_t)elems[i] * dim + k]);
            mx[k] = std::max(mx[k], cen[(size_t)elems[i] * dim + k]);
        }
    int ax = 0;
    for (int k = 1; k < dim; ++k)
        if (mx[k] - mn[k] > mx[ax] - mn[ax]) ax = k;
    std::sort(elems.begin() + lo, elems.begin() + hi, [&](int32_t a, int32_t b) {
        const double ca = cen[(size_t)a * dim + ax], cb = cen[(size_t)b * dim + ax];
        return ca < cb || (ca == cb && a < b);
    });
    const int nl = nr / 2;
    const size_t cut = lo + (size_t)(((hi - lo) * (uint64_t)nl + nr / 2) / nr);
    rcb(cen, dim, elems, lo, cut, rank0, nl, part);
    rcb(cen, dim, elems, cut, hi, rank0 + nl, nr - nl, part);
}

struct LocalSpace {
    std::vector<int32_t> elems, loc_dofs, nbr_ranks, nbr_idx;
    std::vector<int64_t> l2g, nbr_off;
    int64_t n_not_owned = 0;
};

LocalSpace build_local(int ne, int nd, int64_t nl, const int32_t *elem_dofs, const int32_t *part, int rank)
{
    // (dof, rank) holder pairs, unique
    std::vector<std::pair<int32_t, int32_t>> hold;
    hold.reserve((size_t)ne * nd);
    for (int e = 0; e < ne; ++e)
        for (int l = 0; l < nd; ++l) hold.push_back({elem_dofs[(size_t)e * nd + l], part[e]});
    std::sort(hold.begin(), hold.end());
    hold.erase(std::unique(hold.begin(), hold.end()), hold.end());
    std::vector<int64_t> hoff(nl + 1, 0);
    for (auto &h : hold) hoff[h.first + 1]++;
    for (int64_t i = 0; i < nl; ++i) hoff[i + 1] += hoff[i];
    auto holds = [&](int64_t g, int r) {
        for (int64_t k = hoff[g]; k < hoff[g + 1]; ++k)
            if (hold[k].second == r) return true;
        return false;
    };
    LocalSpace L;
    for (int e = 0; e < ne; ++e)
        if (part[e] == rank) L.elems.push_back(e);
    std::vector<int64_t> notown, own;
    for (int64_t g = 0; g < nl; ++g) {
        if (hoff[g + 1] == hoff[g] || !holds(g, rank)) continue;
        (hold[hoff[g]].second < rank ? notown : own).push_back(g);  // holders sorted: first = owner
    }
    L.n_not_owned = (int64_t)notown.size();
    L.l2g = notown;
    L.l2g.insert(L.l2g.end(), own.begin(), own.end());
    std::vector<int32_t> g2l(nl, -1);
    for (size_t i = 0; i < L.l2g.size(); ++i) g2l[L.l2g[i]] = (int32_t)i;
    L.loc_dofs.resize(L.elems.size() * nd);
    for (size_t i = 0; i < L.elems.size(); ++i)
        for (int l = 0; l < nd; ++l) L.loc_dofs[i * nd + l] = g2l[elem_dofs[(size_t)L.elems[i] * nd + l]];
    // neighbours: every other holder of a local dof; lists in ascending global id
    std::vector<int64_t> sorted_g(L.l2g);
    std::sort(sorted_g.begin(), sorted_g.end());
    std::vector<std::pair<int32_t, int64_t>> pairs;  // (neighbour rank, global dof)
    for (int64_t g : sorted_g)
        for (int64_t k = hoff[g]; k < hoff[g + 1]; ++k)
            if (hold[k].second != rank) pairs.push_back({hold[k].second, g});
    std::sort(pairs.begin(), pairs.end());
    L.nbr_off.push_back(0);
    for (size_t i = 0; i < pairs.size(); ++i) {
        if (i == 0 || pairs[i].first != pairs[i - 1].first) {
            if (i > 0) L.nbr_off.push_back((int64_t)L.nbr_idx.size());
            L.nbr_ranks.push_back(pairs[i].first);
        }
        L.nbr_idx.push_back(g2l[pairs[i].second]);
    }
    if (!pairs.empty()) L.nbr_off.push_back((int64_t)L.nbr_idx.size());
    return L;
}

}  // namespace

void partition_rcb(int dim, int ne, int nv, const double *verts, int nranks, int32_t *part)
{
    std::vector<double> cen((size_t)ne * dim, 0.0);
    for (int e = 0; e < ne; ++e)
        for (int v = 0; v < nv; ++v)
            for (int k = 0; k < dim; ++k) cen[(size_t)e * dim + k] += verts[((size_t)e * nv + v) * dim + k] / nv;
    std::vector<int32_t> elems(ne);
    std::iota(elems.begin(), elems.end(), 0);
    rcb(cen, dim, elems, 0, (size_t)ne, 0, nranks, part);
}

}  // namespace cdfem

using namespace cdfem;

extern "C" {

int cdfem_partition_rcb(int dim, int ne, int nv, const double *elem_verts, int nranks, int32_t *part)
{
    if ((dim != 2 && dim != 3) || ne < 1 || nv < 1 || !elem_verts || nranks < 1 || !part) return CDFEM_ERR_ARG;
    if (nranks > ne) return CDFEM_ERR_ARG;  // every rank gets at least one element
    try {
        partition_rcb(dim, ne, nv, elem_verts, nranks, part);
    } catch (...) {
        return CDFEM_ERR_ARG;
    }
    return CDFEM_OK;
}

static int local_space(int ne, int nd, int64_t nldofs, const int32_t *elem_dofs, const int32_t *part, int rank,
                       LocalSpace &L)
{
    if (ne < 1 || nd < 1 || nldofs < 1 || !elem_dofs || !part || rank < 0) return CDFEM_ERR_ARG;
    for (int64_t k = 0; k < (int64_t)ne * nd; ++k)
        if (elem_dofs[k] < 0 || elem_dofs[k] >= nldofs) return CDFEM_ERR_ARG;
    try {
        L = build_local(ne, nd, nldofs, elem_dofs, part, rank);
    } catch (...) {
        return CDFEM_ERR_ARG;
    }
    return L.elems.empty() ? CDFEM_ERR_ARG : CDFEM_OK;
}

int cdfem_local_space_sizes(int ne, int nd, int64_t nldofs, const int32_t *elem_dofs, const int32_t *part, int rank,
                            int *ne_loc, int64_t *nl_loc, int *n_nbr, int64_t *n_shared, int64_t *n_not_owned)
{
    LocalSpace L;
    const int rc = local_space(ne, nd, nldofs, elem_dofs, part, rank, L);
    if (rc) return rc;
    if (ne_loc) *ne_loc = (int)L.elems.size();
    if (nl_loc) *nl_loc = (int64_t)L.l2g.size();
    if (n_nbr) *n_nbr = (int)L.nbr_ranks.size();
    if (n_shared) *n_shared = (int64_t)L.nbr_idx.size();
    if (n_not_owned) *n_not_owned = L.n_not_owned;
    return CDFEM_OK;
}

int cdfem_local_space(int ne, int nd, int64_t nldofs, const int32_t *elem_dofs, const int32_t *part, int rank,
                      int32_t *elems, int32_t *loc_dofs, int64_t *l2g, int32_t *nbr_ranks, int64_t *nbr_off,
                      int32_t *nbr_idx)
{
    LocalSpace L;
    const int rc = local_space(ne, nd, nldofs, elem_dofs, part, rank, L);
    if (rc) return rc;
    if (elems) std::copy(L.elems.begin(), L.elems.end(), elems);
    if (loc_dofs) std::copy(L.loc_dofs.begin(), L.loc_dofs.end(), loc_dofs);
    if (l2g) std::copy(L.l2g.begin(), L.l2g.end(), l2g);
    if (nbr_ranks) std::copy(L.nbr_ranks.begin(), L.nbr_ranks.end(), nbr_ranks);
    if (nbr_off) {
        if (L.nbr_ranks.empty()) nbr_off[0] = 0;
        else std::copy(L.nbr_off.begin(), L.nbr_off.end(), nbr_off);
    }
    if (nbr_idx) std::copy(L.nbr_idx.begin(), L.nbr_idx.end(), nbr_idx);
    return CDFEM_OK;
}

}  // extern "C"
