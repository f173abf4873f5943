// capi.hip — the C-ABI of libcdfem.so (include/cdfem.h): context, mesh/space upload, partial
// assembly, FormLinearSystem, Krylov solves, profiling.  Host-side orchestration only; all
// arithmetic on the hot path runs in the HIP kernels of pa_kernels.hip / vec_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "cdfem_internal.hpp"
#include "brick_core.hpp"

using namespace cdfem;

namespace {

struct HipError : std::runtime_error {
    explicit HipError(const std::string &m) : std::runtime_error(m) {}
};
struct ArgError : std::runtime_error {
    explicit ArgError(const std::string &m) : std::runtime_error(m) {}
};
struct StateError : std::runtime_error {
    explicit StateError(const std::string &m) : std::runtime_error(m) {}
};
struct UnsupportedError : std::runtime_error {
    explicit UnsupportedError(const std::string &m) : std::runtime_error(m) {}
};

inline void hip_check(hipError_t e, const char *what)
{
    if (e != hipSuccess) throw HipError(std::string(what) + ": " + hipGetErrorString(e));
}
#define HIPCHK(x) hip_check((x), #x)

template <typename F>
int guarded(cdfem_ctx *c, F &&f)
{
    if (!c) return CDFEM_ERR_ARG;
    try {
        c->err.clear();
        return f();
    } catch (const ArgError &e) {
        c->err = e.what();
        return CDFEM_ERR_ARG;
    } catch (const StateError &e) {
        c->err = e.what();
        return CDFEM_ERR_STATE;
    } catch (const UnsupportedError &e) {
        c->err = e.what();
        return CDFEM_ERR_UNSUPPORTED;
    } catch (const HipError &e) {
        c->err = e.what();
        return CDFEM_ERR_HIP;
    } catch (const std::bad_alloc &) {
        c->err = "host allocation failed";
        return CDFEM_ERR_HIP;
    } catch (const std::exception &e) {
        c->err = e.what();
        return CDFEM_ERR_ARG;
    }
}

template <typename T>
void dfree(T *&p)
{
    if (p) (void)hipFree((void *)p);
    p = nullptr;
}

template <typename T>
T *dalloc(size_t n)
{
    void *p = nullptr;
    if (n == 0) n = 1;
    HIPCHK(hipMalloc(&p, n * sizeof(T)));
    return static_cast<T *>(p);
}

int nq_of(const cdfem_ctx *c, const Rule1D &r) { return c->dim == 3 ? r.q1 * r.q1 * r.q1 : r.q1 * r.q1; }

// every element a parallelepiped: each vertex v (lexicographic, bit k = axis k) equals
// v0 + sum_k bit_k (v_{2^k} - v0) up to the rounding of those coordinates (32 ulp of the largest
// coordinate magnitude) plus 1e-12 of the element's longest edge.  Then the multilinear map is
// affine and its Jacobian is the edge matrix at every point (the PA setup's pa_affine form) to a
// relative 1e-12 of the element (the tolerance was 1e-13 of max(|x|, edge), which for
// small elements far from the origin admitted defects far larger than the element's own scale).
static bool mesh_is_affine(int dim, int64_t ne, const double *V)
{
    const int nv = 1 << dim;
    const double eps = std::numeric_limits<double>::epsilon();
    for (int64_t e = 0; e < ne; ++e) {
        const double *X = V + (size_t)e * nv * dim;
        double xmax = 0.0, hmax = 0.0;
        for (int v = 0; v < nv; ++v)
            for (int i = 0; i < dim; ++i) xmax = std::max(xmax, std::fabs(X[v * dim + i]));
        for (int k = 0; k < dim; ++k) {
            double h2 = 0.0;
            for (int i = 0; i < dim; ++i) {
                const double d = X[(1 << k) * dim + i] - X[i];
                h2 += d * d;
            }
            hmax = std::max(hmax, std::sqrt(h2));
        }
        const double tol = 32.0 * eps * xmax + 1e-12 * hmax;
        for (int v = 3; v < nv; ++v) {
            if ((v & (v - 1)) == 0) continue;  // the edge vertices themselves
            for (int i = 0; i < dim; ++i) {
                double p = X[i];
                for (int k = 0; k < dim; ++k)
                    if (v >> k & 1) p += X[(1 << k) * dim + i] - X[i];
                if (std::fabs(p - X[v * dim + i]) > tol) return false;
            }
        }
    }
    return true;
}

void free_mesh(cdfem_ctx *c)
{
    dfree(c->d_verts); dfree(c->d_map); dfree(c->d_e2l_off); dfree(c->d_e2l_pos);
    dfree(c->d_ess); dfree(c->d_ess_list); dfree(c->d_qd); dfree(c->d_qaff); dfree(c->d_Ye); dfree(c->d_dinv);
    for (auto &w : c->d_w) dfree(w);
    dfree(c->d_part); dfree(c->d_tpart); dfree(c->d_gm); dfree(c->d_gm_part); dfree(c->d_ktab);
    c->ktab_key = -1;  // rebuilt (and reallocated) by the next k_apply3d_ktile launch
    dfree(c->d_perm); dfree(c->d_face); dfree(c->d_ones); dfree(c->d_dalt);
    for (auto &b : c->d_if) dfree(b);
    dfree(c->d_stab); dfree(c->d_stab_lf); dfree(c->d_rowptr); dfree(c->d_cols); dfree(c->d_diagpos); dfree(c->d_coff);
    dfree(c->d_cpos); dfree(c->d_vals); dfree(c->d_vals_c); dfree(c->d_Ee);
    dfree(c->d_sptr); dfree(c->d_srows); dfree(c->d_scols); dfree(c->d_smap); dfree(c->d_sdel); dfree(c->d_svals);
    dfree(c->d_swide);
    dfree(c->d_uelem);
    c->d_sdel = nullptr;
    c->d_swide = nullptr;
    c->sell_nnz_wide = 0;
    dfree(c->d_hptr); dfree(c->d_hidx); dfree(c->d_sloc);
    c->d_hptr = c->d_hidx = nullptr;
    c->d_sloc = nullptr;
    c->lds_rows = 0;
    c->lds_max = 0;
    c->sell_lpr = 1;
    dfree(c->d_rperm); dfree(c->d_pv[0]); dfree(c->d_pv[1]); dfree(c->d_dinv_p);
    c->d_rperm = nullptr; c->d_pv[0] = c->d_pv[1] = nullptr; c->d_dinv_p = nullptr;
    dfree(c->d_svals_c);
    c->d_svals_c = nullptr;
    dfree(c->d_lfq);
    c->lfq_cap = 0;
    ilu_free(c);
    partition_free(c);
    c->nslices = c->nstored = 0;
    c->sell_windowed = false;
    c->geom = 0;
    c->fa_ready = false;
    c->nnz = 0;
    c->h_verts.clear();
    c->h_sxi_d.clear();
    c->h_sxi_cm.clear();
    c->h_sxi_lf.clear();
    c->zlo_shared = c->zhi_shared = 0;
    c->gm_cap = 0;
    c->mesh_ready = c->pa_ready = c->dinv_ready = false;
    c->structured = false;
    c->epencil = false;
    c->slab_nl_max = 0;
    c->slab_nb_max = 0;
    dfree(c->d_small);
    dfree(c->d_gsum);
    dfree(c->d_gcnt);
    c->gsum_cap = 0;
    c->den_grp = 1;
    dfree(c->d_hbpart);
    dfree(c->d_bess);
    c->hb_nblk = 0;
}

// per brick (edge E elements in x and y, EZ in z; nb* bricks per axis): 1 if a lattice dof of its patch
// (E p + 1 per axis, EZ p + 1 along z, clipped to the lattice) is essential; the brick CG kernels skip the
// essential-flag loads elsewhere
static void upload_brick_ess(cdfem_ctx *c, int E, int EZ, int nbx, int nby, int nbz)
{
    const int64_t s1 = (int64_t)E * c->p, sz1 = (int64_t)EZ * c->p, Lx = c->Lx, Ly = c->Ly, Lz = c->Lz;
    std::vector<uint8_t> has((size_t)nbx * nby * nbz, 0);
    for (int bz = 0; bz < nbz; ++bz)
        for (int by = 0; by < nby; ++by)
            for (int bx = 0; bx < nbx; ++bx) {
                uint8_t h = 0;
                for (int64_t z = bz * sz1; z <= std::min(bz * sz1 + sz1, Lz - 1) && !h; ++z)
                    for (int64_t y = by * s1; y <= std::min(by * s1 + s1, Ly - 1) && !h; ++y) {
                        const uint8_t *row = c->h_ess.data() + (size_t)(z * Ly + y) * Lx;
                        for (int64_t x = bx * s1; x <= std::min(bx * s1 + s1, Lx - 1); ++x) h |= row[x];
                    }
                has[((size_t)bz * nby + by) * nbx + bx] = h;
            }
    dfree(c->d_bess);
    c->d_bess = dalloc<uint8_t>(has.size());
    HIPCHK(hipMemcpy(c->d_bess, has.data(), has.size(), hipMemcpyHostToDevice));
}

// ---- profiling helpers ---------------------------------------------------------------------------
void prof_mark(cdfem_ctx *c, int k, bool begin)
{
    if (!c->profile || !((c->prof_mask >> k) & 1u)) return;
    ProfileSlot &s = c->prof[k];
    const size_t need = (size_t)(s.used + 1) * 2;
    while (s.ev.size() < need) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        s.ev.push_back(e);
    }
    if (begin) {
        // recorded now AND armed: a CDFEM_LAUNCH before the end mark re-records the pair tightly
        // around its own dispatch; any other launch leaves the plain event interval
        HIPCHK(hipEventRecord(s.ev[2 * s.used], c->stream));
        c->ext_ev[0] = s.ev[2 * s.used];
        c->ext_ev[1] = s.ev[2 * s.used + 1];
    } else {
        if (c->ext_ev[0]) HIPCHK(hipEventRecord(s.ev[2 * s.used + 1], c->stream));  // not consumed
        c->ext_ev[0] = c->ext_ev[1] = nullptr;
        s.used++;
    }
}

void prof_collect(cdfem_ctx *c)
{
    if (!c->profile) return;
    HIPCHK(hipStreamSynchronize(c->stream));
    for (auto &s : c->prof) {
        for (int i = 0; i < s.used; ++i) {
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, s.ev[2 * i], s.ev[2 * i + 1]));
            s.total_ms += ms;
            s.count++;
            s.each.push_back(ms);
        }
        s.used = 0;
    }
}

// (Re)build the element-block layout for a permutation perm[blk*64 + lane] = element (-1 pad):
// element map [blk][l][lane] (ess negative), E->L positions, and the device permutation.
void build_layout(cdfem_ctx *c, const std::vector<int32_t> &perm)
{
    const int nd = c->nd;
    const int64_t nl = c->nl;
    std::vector<int32_t> map((size_t)c->nblk * nd * kLanes, 0);
    std::vector<int32_t> where(c->ne, -1);
    for (size_t k = 0; k < perm.size(); ++k)
        if (perm[k] >= 0) where[perm[k]] = (int32_t)k;
    // E-vector / map index of (element, local dof): blocks of 64 lanes, or element-major
    auto eidx = [&](int e, int l) -> size_t {
        if (c->qlay == 1) return (size_t)e * nd + l;
        const int blk = where[e] / kLanes, lane = where[e] % kLanes;
        return ((size_t)blk * nd + l) * kLanes + lane;
    };
    std::vector<int32_t> cnt(nl + 1, 0);
    for (int e = 0; e < c->ne; ++e) {
        for (int l = 0; l < nd; ++l) {
            const int32_t g = c->h_dofs[(size_t)e * nd + l];
            map[eidx(e, l)] = c->h_ess[g] ? -(g + 1) : g;
            cnt[g + 1]++;
        }
    }
    for (int64_t i = 0; i < nl; ++i) cnt[i + 1] += cnt[i];
    std::vector<int32_t> pos((size_t)c->ne * nd), fill(cnt.begin(), cnt.end() - 1);
    for (int e = 0; e < c->ne; ++e) {
        for (int l = 0; l < nd; ++l) {
            const int32_t g = c->h_dofs[(size_t)e * nd + l];
            pos[fill[g]++] = (int32_t)eidx(e, l);
        }
    }
    dfree(c->d_map); dfree(c->d_e2l_off); dfree(c->d_e2l_pos); dfree(c->d_perm); dfree(c->d_Ye);
    dfree(c->d_part);
    c->d_map = dalloc<int32_t>(map.size());
    c->d_e2l_off = dalloc<int32_t>(nl + 1);
    c->d_e2l_pos = dalloc<int32_t>(pos.size());
    c->d_perm = dalloc<int32_t>(perm.size());
    c->d_Ye = dalloc<double>((size_t)c->nblk * nd * kLanes);
    c->d_part = dalloc<double>((size_t)c->red_blocks + c->nblk + 64 * 8192 + 16384);
    HIPCHK(hipMemcpyAsync(c->d_map, map.data(), map.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_e2l_off, cnt.data(), (nl + 1) * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_e2l_pos, pos.data(), pos.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_perm, perm.data(), perm.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemsetAsync(c->d_Ye, 0, (size_t)c->nblk * nd * kLanes * sizeof(double), c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
}

bool use_brick(const cdfem_ctx *c) { return c->structured && brick_supported(c->dim, c->p) && brick_fits(c); }

// the high-order brick CG (3D p = 3, 4, affine box with constant coefficients: the Kronecker tile core on
// 2^3-element blocks, brick_kernels.hip k_hobrick_cg, then the brick update); on several ranks a z-slab
// of 2^3 blocks (round 6: the plane pack and exchange of the p = 2 brick CG, rank-local den sums)
bool use_hobrick_cg(const cdfem_ctx *c)
{
    return c->ho_brick != 0 && c->structured && c->qlay == 1 && c->hb_nblk > 0 && tile_kron(c) && tile_den_ok(c) &&
           (!multi_rank(c) || (c->part_mode == 1 && c->hb_ez == kHoBrickEdge)) && !c->fa_ready && brick_fits(c);
}
bool use_brick_cg(const cdfem_ctx *c) { return use_brick(c) || use_hobrick_cg(c); }

const double *ones_vector(cdfem_ctx *c)
{
    if (!c->d_ones) {
        c->d_ones = dalloc<double>(c->nl);
        std::vector<double> one(c->nl, 1.0);
        HIPCHK(hipMemcpyAsync(c->d_ones, one.data(), c->nl * 8, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    return c->d_ones;
}

void require_mesh(cdfem_ctx *c)
{
    if (!c->mesh_ready) throw StateError("cdfem_mesh_upload has not been called");
}
void require_pa(cdfem_ctx *c)
{
    require_mesh(c);
    if (!c->pa_ready && !c->fa_ready) throw StateError("no operator: call cdfem_pa_setup or cdfem_fa_setup");
}

// a communicator of more than one rank needs a declared partition: the z-slab of a structured box
// (cdfem_set_slab) or the general shared-dof lists (cdfem_set_shared).  Without one, the exchange
// would read unset interface buffers and the ranks would take different Krylov branches.
void require_partition(cdfem_ctx *c)
{
    if (!multi_rank(c)) return;
    if (c->part_mode == 1) {
        if (!c->structured || !c->d_if[0]) throw StateError("slab partition incomplete: cdfem_set_slab after cdfem_mesh_set_structured");
        if (c->fa_ready) throw UnsupportedError("slab partitions drive partial-assembly operators; use cdfem_set_shared for assembled ones");
        return;
    }
    if (c->part_mode == 2) {
        if (use_brick(c)) throw UnsupportedError("the structured brick kernels need a slab partition (cdfem_set_slab)");
        return;
    }
    throw StateError("communicator attached (" + std::to_string(c->nranks) +
                     " ranks) but no partition declared: call cdfem_set_slab or cdfem_set_shared");
}

// operator apply into y (device pointers): Ye = A_e x, y = E->L(Ye) [+ constraint]
void op_apply(cdfem_ctx *c, const double *x, double *y, bool constrained)
{
    if (c->fa_ready) {  // assembled CSR: A, or the eliminated matrix for the constrained operator
        prof_mark(c, CDFEM_K_APPLY, true);
        HIPCHK(launch_spmv(c, constrained, x, y));
        prof_mark(c, CDFEM_K_APPLY, false);
        return;
    }
    if (use_brick(c)) {
        prof_mark(c, CDFEM_K_APPLY, true);
        HIPCHK(launch_brick_mult(c, x, y, constrained, 1));
        prof_mark(c, CDFEM_K_APPLY, false);
        prof_mark(c, CDFEM_K_E2L, true);
        HIPCHK(launch_brick_mult(c, x, y, constrained, 2));
        prof_mark(c, CDFEM_K_E2L, false);
        return;
    }
    prof_mark(c, CDFEM_K_APPLY, true);
    HIPCHK(launch_apply(c, x, c->d_Ye, constrained));
    prof_mark(c, CDFEM_K_APPLY, false);
    prof_mark(c, CDFEM_K_E2L, true);
    HIPCHK(launch_e2l(c, c->d_Ye, x, y, constrained, 0));
    prof_mark(c, CDFEM_K_E2L, false);
}

// the operator on the global (all-rank) space, rank-local L-vectors: the local apply, then the
// shared planes summed with the neighbours (MFEM P^T A P on the true dofs, then P), and for the
// constrained operator the essential rows reset to the identity (an essential dof on a shared
// plane was set by both ranks, so the sum doubled it)
void op_apply_global(cdfem_ctx *c, const double *x, double *y, bool constrained)
{
    op_apply(c, x, y, constrained);
    if (!multi_rank(c)) return;
    interface_sum(c, y);
    if (constrained) HIPCHK(launch_set_ess(c, y, x));
}

// copy-in helper: returns a device pointer holding n doubles of src (staging when on host)
const double *dev_in(cdfem_ctx *c, const double *src, int where, double *staging, size_t n)
{
    if (where == CDFEM_DEVICE) return src;
    HIPCHK(hipMemcpyAsync(staging, src, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
    return staging;
}

void dev_out(cdfem_ctx *c, double *dst, int where, const double *dsrc, size_t n)
{
    if (where == CDFEM_DEVICE) {
        if (dst != dsrc)
            HIPCHK(hipMemcpyAsync(dst, dsrc, n * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
        return;
    }
    HIPCHK(hipMemcpyAsync(dst, dsrc, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
}

void ensure_dinv(cdfem_ctx *c)
{
    if (c->dinv_ready) return;
    double *diag = c->d_w[7];
    if (c->fa_ready) {
        HIPCHK(launch_csr_diag(c, diag));
    } else {
        HIPCHK(launch_diag_elem(c, c->d_Ye));
        HIPCHK(launch_e2l(c, c->d_Ye, nullptr, diag, false, 0));
    }
    interface_sum(c, diag);  // shared planes: the full diagonal (both ranks' elements)
    HIPCHK(launch_dinv(c, diag, c->d_dinv));
    c->dinv_ready = true;
}

// the Jacobi scale in the order the running solve uses (mesh order, or the permuted SpMV order)
const double *solver_dinv(cdfem_ctx *c)
{
    ensure_dinv(c);
    if (!c->perm_space) return c->d_dinv;
    if (!c->d_dinv_p) c->d_dinv_p = dalloc<double>(c->nl);
    HIPCHK(launch_perm(c, true, c->d_dinv, c->d_dinv_p));
    return c->d_dinv_p;
}

// cg_mr_fold all-reduces partial vectors, so every rank must take it and hold as many partials as the
// others: the apply's (one per brick) and the update's (cg_den_fold_grid).  Decided by every rank of a
// multi-rank solve from the all-reduced eligibility flags and the sums of the counts and of their
// squares (equal on every rank, so every rank takes the same branch): the fold runs iff every rank is
// eligible and the counts' variance is zero.  The 5-double all-reduce runs on EVERY multi-rank brick CG
// entry, whatever the rank's local state (a cached decision let one rank skip the
// collective after an option change that left its own key unchanged while another rank's key moved).
bool mr_fold_agreed(cdfem_ctx *c)
{
    const double ok = cg_mr_fold(c) ? 1.0 : 0.0, nb = den_parts(c), ng = cg_den_fold_grid(c);
    double h[5] = {ok, nb, nb * nb, ng, ng * ng};
    if (!c->d_small) c->d_small = dalloc<double>(8);
    HIPCHK(hipMemcpyAsync(c->d_small, h, sizeof(h), hipMemcpyHostToDevice, c->stream));
    comm_allreduce(c, c->d_small, 5);
    HIPCHK(hipMemcpyAsync(h, c->d_small, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const double n = c->nranks;
    return h[0] == n && h[2] * n == h[1] * h[1] && h[4] * n == h[3] * h[3];
}

// brick-path CG (MFEM CGSolver arithmetic): per iteration k_brick_cg (direction + apply + den
// partials) -> den finalizer -> k_cg_update_faces (q assembly + x, r update + betanom partials) ->
// betanom finalizer.  The search direction alternates between two buffers.
void solve_cg_brick(cdfem_ctx *c, const cdfem_solver_params &p, const double *dB, double *dX,
                    cdfem_solver_result &res)
{
    double *x = c->d_w[2], *r = c->d_w[3], *q = c->d_w[4];
    if (!c->d_dalt) c->d_dalt = dalloc<double>(c->nl);
    const int nbrick = brick_count(c);
    if (!c->d_face) {  // (p = 3, 4: the blocks' patch buffer, first use)
        const int S = brick_patch_side(c), SZ = brick_patch_side_z(c);
        c->d_face = dalloc<double>((size_t)nbrick * S * S * SZ);
    }
    // the apply's den partials in two stages (a block per 1/256 of them, then one block) when the one
    // block finalizer would sum too many: the p = 3, 4 blocks, and one rank past the den fold's bound
    const int ndp = den_parts(c);  // the den partials the folds sum (grouped past the bounds: den_group)
    const bool two_stage = c->p >= 3 || (!multi_rank(c) && ndp > kDenFoldMaxParts);
    if (two_stage && !c->d_hbpart) c->d_hbpart = dalloc<double>(nbrick);
    c->den_out = two_stage && c->p <= 2 ? c->d_hbpart : nullptr;
    struct DenOutReset {
        cdfem_ctx *c;
        ~DenOutReset() { c->den_out = nullptr; c->den_grp = 1; }
    } den_out_reset{c};
    double *dprev = c->d_w[5], *dcur = c->d_dalt;
    const double *dinv;
    if (p.pc == CDFEM_PC_JACOBI) {
        ensure_dinv(c);
        dinv = c->d_dinv;
    } else {
        dinv = ones_vector(c);
    }
    const int check = p.check_every > 0 ? p.check_every : 16;
    const bool mr = multi_rank(c);
    double *red = c->d_state->red;  // device scalars awaiting the all-reduce
    HIPCHK(hipStreamSynchronize(c->stream));
    const auto t0 = std::chrono::steady_clock::now();
    if (mr) {
        HIPCHK(launch_cg_init_nofin(c, dB, x, r, q, dprev, dinv));
        comm_allreduce(c, red + 2, 1);
        HIPCHK(launch_init_step(c, p.rel_tol, p.abs_tol, p.max_iter));
    } else {
        HIPCHK(launch_cg_init(c, dB, x, r, q, dprev, dinv, p.rel_tol, p.abs_tol, p.max_iter));
    }
    // slab partition: the shared planes' partial sums come from the first and last brick layers
    // only, so those layers run first on a side stream, whose pack + exchange then overlap the
    // interior layers on the main stream.  Same kernels, same sums: bitwise equal
    // to the one-launch form.  Profiling keeps the one-launch form (one timed apply kernel).
    const bool overlap = mr && c->mr_overlap && !c->profile && c->p <= 2 && c->nbz >= 3;
    if (overlap && !c->stream2) {
        HIPCHK(hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking));
        for (auto &e : c->ov_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    // x-fold (set_option "cg_xfold", default): every apply after the first advances x by the previous
    // iteration's alpha d (the update kernel then streams neither x nor d); k_cg_xflush adds the
    // last update's term after the loop when the update logic stopped the solve
    const bool xfold = c->cg_xfold != 0 && pa_af(c) == 2;  // Kronecker kernel only
    double *const dbuf0 = dcur, *const dbuf1 = dprev;  // apply j writes d_j into dbuf[(j - 1) & 1]
    // betanom fold (cg_beta_fold): apply j > 0 takes the betanom step of update j - 1 (nupd updates so
    // far); the loop always ends with an apply, so every update's step runs
    // several ranks (cg_mr_fold): the den and betanom partial vectors are all-reduced and both folds
    // run as on one rank; the per-iteration kernels are then the one-rank pair plus the plane pack
    const bool mrfold = mr && mr_fold_agreed(c);
    const bool bfold = mr ? mrfold : cg_beta_fold_ok(c);
    // grouped den partials: taken when a fold sums them (several ranks: the fold; one rank: the den fold)
    const int grp = (mr ? mrfold : (!two_stage && cg_den_fold_on(c))) ? den_group(c) : 1;
    if (grp > 1 && c->gsum_cap < ndp) {
        dfree(c->d_gsum);
        dfree(c->d_gcnt);
        c->d_gsum = dalloc<double>(ndp);
        c->d_gcnt = dalloc<uint32_t>(ndp);
        HIPCHK(hipMemsetAsync(c->d_gcnt, 0, (size_t)ndp * sizeof(uint32_t), c->stream));
        c->gsum_cap = ndp;
    }
    c->den_grp = grp;
    double *const dparts = grp > 1 ? c->d_gsum : c->d_part;  // what the mr fold all-reduces (ndp of them)
    int nupd = 0;
    int napply = 0;
    auto apply = [&] {
        double *xf = (xfold && napply > 0) ? x : nullptr;
        ++napply;
        if (overlap) {
            HIPCHK(hipEventRecord(c->ov_ev[0], c->stream));
            HIPCHK(hipStreamWaitEvent(c->stream2, c->ov_ev[0], 0));
            // boundary layers on the side stream, interior layers queued on the main stream
            // before the (possibly host-blocking) exchange is issued
            HIPCHK(launch_brick_cg2_split(c, r, dinv, dprev, dcur, q, c->stream2, xf, bfold ? nupd : -1));
            HIPCHK(launch_pack_qplanes(c, q, c->stream2));
            comm_exchange(c, c->d_if[0], c->d_if[1], c->d_if[2], c->d_if[3], c->Lx * c->Ly, c->stream2);
            HIPCHK(hipEventRecord(c->ov_ev[1], c->stream2));
            HIPCHK(hipStreamWaitEvent(c->stream, c->ov_ev[1], 0));
            if (mrfold) {
                comm_allreduce(c, dparts, ndp);  // the den partials: the update sums them
            } else {
                HIPCHK(launch_fin_sum(c, nbrick, 0));
                comm_allreduce(c, red + 0, 1);  // den step: folded into the update kernel
            }
            return;
        }
        prof_mark(c, CDFEM_K_APPLY, true);
        HIPCHK(launch_brick_cg2(c, r, dinv, dprev, dcur, q, xf, bfold ? nupd : -1));
        prof_mark(c, CDFEM_K_APPLY, false);
        prof_mark(c, CDFEM_K_E2L, true);
        if (mr) {
            // neighbours' partial sums of q on the shared planes (added by the update kernel)
            HIPCHK(launch_pack_qplanes(c, q));
            comm_exchange(c, c->d_if[0], c->d_if[1], c->d_if[2], c->d_if[3], c->Lx * c->Ly);
            if (mrfold) {
                comm_allreduce(c, dparts, ndp);
            } else {
                if (c->p >= 3) HIPCHK(launch_den_local_from_partials(c, c->d_hbpart, nbrick));  // (one per block)
                else HIPCHK(launch_fin_sum(c, nbrick, 0));
                comm_allreduce(c, red + 0, 1);  // den step: folded into the update kernel
            }
        } else if (two_stage) {
            HIPCHK(launch_den_from_partials(c, c->d_hbpart, nbrick));  // (one partial per brick / block)
        } else if (!cg_den_fold_on(c)) {
            HIPCHK(launch_den_fin(c, nbrick));  // (cg_den_fold: the update kernel takes the den step)
        }
        prof_mark(c, CDFEM_K_E2L, false);
    };
    apply();
    int launched = 0;
    for (;;) {
        for (int k = 0; k < check && launched < p.max_iter; ++k, ++launched) {
            prof_mark(c, CDFEM_K_UPDATE, true);
            HIPCHK(launch_cg_update_faces(c, x, r, q, dcur, dinv,
                                          mr && c->zlo_shared ? c->d_if[1] : nullptr,
                                          mr && c->zhi_shared ? c->d_if[3] : nullptr, mr && !mrfold, xfold));
            if (mrfold) {
                comm_allreduce(c, c->d_part + c->nblk, cg_den_fold_grid(c));  // the next apply sums them
            } else if (mr) {
                comm_allreduce(c, red + 1, 1);
                HIPCHK(launch_update_step(c));
            }
            prof_mark(c, CDFEM_K_UPDATE, false);
            ++nupd;
            std::swap(dprev, dcur);
            apply();
        }
        HIPCHK(hipMemcpyAsync(c->h_state, c->d_state, sizeof(KrylovState), hipMemcpyDeviceToHost,
                              c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->h_state->done || launched >= p.max_iter) break;
    }
    if (xfold) {
        HIPCHK(launch_cg_xflush(c, x, dbuf0, dbuf1));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    const auto t1 = std::chrono::steady_clock::now();
    prof_collect(c);
    const KrylovState &s = *c->h_state;
    res.converged = s.converged;
    res.iterations = s.final_iter;
    res.initial_norm = std::sqrt(std::fabs(s.nom0));
    res.final_norm = (s.final_iter == 0) ? std::sqrt(std::fabs(s.nom0)) : std::sqrt(std::fabs(s.betanom));
    res.seconds = std::chrono::duration<double>(t1 - t0).count();
    HIPCHK(hipMemcpyAsync(dX, x, c->nl * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
}

// MFEM CGSolver on the constrained operator, device-resident
void solve_cg(cdfem_ctx *c, const cdfem_solver_params &p, const double *dB, double *dX,
              cdfem_solver_result &res)
{
    double *x = c->d_w[2], *r = c->d_w[3], *z = c->d_w[4], *d = c->d_w[5];
    const double *dinv = p.pc == CDFEM_PC_JACOBI ? solver_dinv(c) : nullptr;
    const int check = p.check_every > 0 ? p.check_every : 16;
    const bool mr = multi_rank(c);
    double *red = c->d_state->red;  // device scalars awaiting the all-reduce (multi-rank)
    // high order on a structured box, one rank: den from the apply's E-vector, E->L fused into the
    // update (ho_kernels.hip k_apply3d_tile<DEN>, vec_kernels.hip k_e2l_box<UPD>)
    const bool fused = !mr && !c->fa_ready && c->cg_fused && tile_den_ok(c) && e2l_box_ok(c) &&
                       c->nl < ((int64_t)1 << 31);  // the flat update's fast division is exact below 2^31
    if (fused && !c->d_tpart) c->d_tpart = dalloc<double>(tile_den_blocks(c, true));
    // direction fold (ho_dfold): apply j forms d_j = z + beta d_{j-1} into the other direction buffer
    const bool dfold = fused && tile_dfold_ok(c);
    if (dfold && !c->d_dalt) c->d_dalt = dalloc<double>(c->nl);
    double *dprev = d, *dcur = dfold ? c->d_dalt : d;
    HIPCHK(hipStreamSynchronize(c->stream));
    const auto t0 = std::chrono::steady_clock::now();
    if (mr) {
        HIPCHK(launch_cg_init_nofin(c, dB, x, r, z, d, dinv));
        comm_allreduce(c, red + 2, 1);
        HIPCHK(launch_init_step(c, p.rel_tol, p.abs_tol, p.max_iter));
    } else {
        HIPCHK(launch_cg_init(c, dB, x, r, z, d, dinv, p.rel_tol, p.abs_tol, p.max_iter));
    }
    // z = A d ; den = (d, z) and the MFEM den step
    auto apply = [&] {
        prof_mark(c, CDFEM_K_APPLY, true);
        if (fused) {  // Ye = A_c d and den; q stays an E-vector until the update
            if (dfold) HIPCHK(launch_apply_den_dfold(c, z, dprev, dcur, c->d_Ye, c->d_state, c->d_tpart));
            else HIPCHK(launch_apply_den(c, d, c->d_Ye, c->d_state, c->d_tpart));
            prof_mark(c, CDFEM_K_APPLY, false);
            prof_mark(c, CDFEM_K_E2L, true);
            HIPCHK(launch_den_from_partials(c, c->d_tpart, tile_den_blocks(c)));
            prof_mark(c, CDFEM_K_E2L, false);
            return;
        }
        if (c->fa_ready && !mr) {
            HIPCHK(launch_spmv_cg(c, d, z));
            prof_mark(c, CDFEM_K_APPLY, false);
            return;
        }
        if (c->fa_ready) HIPCHK(launch_spmv(c, true, d, z));
        else HIPCHK(launch_apply_st(c, d, c->d_Ye, true, c->d_state));
        prof_mark(c, CDFEM_K_APPLY, false);
        prof_mark(c, CDFEM_K_E2L, true);
        if (mr) {  // rank partition: interface sums, essential rows reset, owned den all-reduced
            if (!c->fa_ready) HIPCHK(launch_e2l(c, c->d_Ye, d, z, true, 0));
            interface_sum(c, z);
            HIPCHK(launch_set_ess(c, z, d));
            HIPCHK(launch_den_local(c, d, z));
            comm_allreduce(c, red + 0, 1);
            HIPCHK(launch_den_step(c));
        } else {
            HIPCHK(launch_e2l(c, c->d_Ye, d, z, true, 1));
        }
        prof_mark(c, CDFEM_K_E2L, false);
    };
    apply();
    int launched = 0;
    for (;;) {
        for (int k = 0; k < check && launched < p.max_iter; ++k, ++launched) {
            prof_mark(c, CDFEM_K_UPDATE, true);
            if (fused) HIPCHK(launch_e2l_cg_update(c, c->d_Ye, dcur, x, r, z, dinv));
            else HIPCHK(launch_cg_update(c, x, r, z, d, dinv));
            if (mr) {
                comm_allreduce(c, red + 1, 1);
                HIPCHK(launch_update_step(c));
            }
            prof_mark(c, CDFEM_K_UPDATE, false);
            if (dfold) {
                std::swap(dprev, dcur);
            } else {
                prof_mark(c, CDFEM_K_DIRECTION, true);
                HIPCHK(launch_cg_direction(c, z, d));
                prof_mark(c, CDFEM_K_DIRECTION, false);
            }
            apply();
        }
        HIPCHK(hipMemcpyAsync(c->h_state, c->d_state, sizeof(KrylovState), hipMemcpyDeviceToHost,
                              c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->h_state->done || launched >= p.max_iter) break;
    }
    const auto t1 = std::chrono::steady_clock::now();
    prof_collect(c);
    const KrylovState &s = *c->h_state;
    res.converged = s.converged;
    res.iterations = s.final_iter;
    res.initial_norm = std::sqrt(std::fabs(s.nom0));
    res.final_norm = (s.final_iter == 0) ? std::sqrt(std::fabs(s.nom0)) : std::sqrt(std::fabs(s.betanom));
    res.seconds = std::chrono::duration<double>(t1 - t0).count();
    HIPCHK(hipMemcpyAsync(dX, x, c->nl * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
}

// PETSc KSPGMRES(m) + left Jacobi on the constrained operator (gmres.hip).  One host sync per
// restart cycle plus a lag-one poll inside the cycle: step j + 1 is queued before the host waits
// for step j's flags, so the GPU never idles on the host; a step queued past the end of a cycle
// costs one wasted operator apply (its GMRES kernels exit at entry).
void solve_gmres(cdfem_ctx *c, const cdfem_solver_params &p, const double *dB, double *dX,
                 cdfem_solver_result &res)
{
    const int m = p.restart > 0 ? p.restart : 30;
    if (m > kGmMaxRestart) throw ArgError("restart > 64");
    const int64_t n = c->nl;
    // basis leading dimension padded to 32 doubles: every basis vector starts on a 256-byte
    // boundary, so a wave's 512-byte load of v_i covers 4 cache lines, not 5 (odd n)
    const int64_t ldv = (n + 31) / 32 * 32;
    const int nb = gmres_blocks(n);
    if (c->gm_cap < m) {
        dfree(c->d_gm);
        dfree(c->d_gm_part);
        c->d_gm = dalloc<double>((size_t)(m + 1) * ldv);
        c->d_gm_part = dalloc<double>((size_t)(m + 1) * nb);
        c->gm_cap = m;
    }
    if (!c->d_gmst) {
        HIPCHK(hipMalloc(&c->d_gmst, sizeof(GmresState)));
        // poll slots: 0 for the cycle start / end, 1 + j for inner step j (each step its own slot, so a
        // host check reads exactly the state of the step it waited for: ranks decide alike)
        HIPCHK(hipHostMalloc(&c->h_gmpoll, (kGmMaxRestart + 1) * sizeof(GmresState), hipHostMallocDefault));
        for (auto &e : c->gm_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    const double *dinv = nullptr;
    const bool ilu = p.pc == CDFEM_PC_ILU;
    if (p.pc == CDFEM_PC_JACOBI) {
        dinv = solver_dinv(c);
    } else if (ilu) {
        if (!c->fa_ready) throw UnsupportedError("ILU(0) needs an assembled operator (cdfem_fa_setup)");
        if (multi_rank(c) && c->part_mode != 2)
            throw UnsupportedError("block-Jacobi ILU(0) needs a general partition (cdfem_set_shared)");
        ilu_setup(c);
    }
    double *x = c->d_w[2], *w = c->d_w[4], *V = c->d_gm, *part = c->d_gm_part;
    GmresState *st = c->d_gmst, *poll = c->h_gmpoll;
    // the step's last scalar kernel has written poll[slot] (post_poll in gmres.hip); the event
    // marks its completion for the host.  (Measured alternatives, profiles/r03/ab_c2_gmres_poll.txt:
    // spinning on a stamp in pinned memory, 392.2 / 392.0 against 392.3 us per C2 step; polling every
    // 2 / 4 / 30 steps, 390.3 / 388.4 / 388.0 against 391.5: the host wait is not on the critical path.)
    auto post = [&](int slot) { HIPCHK(hipEventRecord(c->gm_ev[slot], c->stream)); };
    auto wait = [&](int slot) -> const GmresState & {
        HIPCHK(hipEventSynchronize(c->gm_ev[slot]));
        return poll[slot];
    };
    // one rank on the structured patch-buffer Mult: pass 1 forms A_c v_j from the patch buffer itself
    const bool gpb = c->gm_pb != 0 && !ilu && !multi_rank(c) && use_brick(c) && brick_mult_pb_on(c);
    // gm_poll k (default 4): an event and a host check every k inner steps (and at a cycle's last step)
    // instead of every step: each event costs the GPU ~5 us before the next Mult (rocprofv3 trace gaps,
    // profiles/r06/ab_gmres_poll/; C2 step 181.3-182.8 -> 178.1-178.2 us at k = 4).  Every step's last
    // scalar kernel posts the state head into its own slot poll[1 + j]; a check waits for the previous
    // check's event and reads exactly that step's slot, never a later step's (on several ranks every rank
    // must leave the loop at the same step: their collectives pair up).  Steps queued past the end of a
    // cycle exit at entry (their Mult does not check, and runs at most k - 1 times per converged cycle).

    const int pk = std::max(1, c->gm_poll);
    int nposts = 0, last_posted = -1;
    auto step_end = [&](int j, bool cycle_last) -> bool {  // true: the cycle is done, leave the step loop
        if (!cycle_last && (j + 1) % pk != 0) return false;
        post(nposts & 1);
        const int prev = last_posted;
        last_posted = j;
        ++nposts;
        if (nposts < 2 || prev < 0) return false;
        HIPCHK(hipEventSynchronize(c->gm_ev[(nposts - 2) & 1]));  // the previous check's event
        return poll[1 + prev].cycle_done != 0;                      // exactly its step's state
    };
    HIPCHK(hipStreamSynchronize(c->stream));
    const auto t0 = std::chrono::steady_clock::now();
    HIPCHK(hipMemsetAsync(x, 0, n * sizeof(double), c->stream));
    HIPCHK(launch_gm_init(c, st, m, p.max_iter));
    for (bool first = true;; first = false) {
        // v0 = M^{-1}(b - A x); x = 0 on the first cycle, so A x is skipped there
        if (!first) op_apply_global(c, x, w, true);
        if (ilu) {  // v0 = (LU)^{-1} (b - A x): the residual into w, the sweeps into ilu.z
            if (first) HIPCHK(hipMemcpyAsync(w, dB, n * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
            else HIPCHK(launch_axpby(c, 1.0, dB, -1.0, w));
            HIPCHK(ilu_apply(c));
            HIPCHK(launch_gm_residual(c, c->ilu.z, nullptr, nullptr, V, part, st, first, p.rel_tol, p.abs_tol,
                                      &poll[0]));
        } else {
            HIPCHK(launch_gm_residual(c, dB, first ? nullptr : w, dinv, V, part, st, first, p.rel_tol, p.abs_tol,
                                      &poll[0]));
        }
        post(0);
        if (wait(0).done) break;
        for (int j = 0; j < m; ++j) {
            const double *Vj = V + (int64_t)j * ldv;
            if (gpb) {  // the structured Mult's patch buffer, summed per row by pass 1 (gm_pb)
                prof_mark(c, CDFEM_K_APPLY, true);
                HIPCHK(launch_brick_mult(c, Vj, w, true, 1));
                prof_mark(c, CDFEM_K_APPLY, false);
                const GmPatchSrc src = gm_patch_src(c, Vj);
                prof_mark(c, CDFEM_K_ORTH, true);
                HIPCHK(launch_gm_orth(c, w, dinv, V, ldv, part, st, m, &poll[1 + j], &src));
                prof_mark(c, CDFEM_K_ORTH, false);
                if (step_end(j, j == m - 1)) break;
                continue;
            }
            op_apply_global(c, Vj, w, true);
            if (ilu) HIPCHK(ilu_apply(c));  // w <- (LU)^{-1} A v_j, in ilu.z
            prof_mark(c, CDFEM_K_ORTH, true);
            HIPCHK(launch_gm_orth(c, ilu ? c->ilu.z : w, dinv, V, ldv, part, st, m, &poll[1 + j]));
            prof_mark(c, CDFEM_K_ORTH, false);
            if (step_end(j, j == m - 1)) break;
        }
        nposts = 0;
        last_posted = -1;
        prof_mark(c, CDFEM_K_UPDATE, true);
        HIPCHK(launch_gm_update(c, x, V, ldv, st, &poll[0]));
        prof_mark(c, CDFEM_K_UPDATE, false);
        post(0);
        if (wait(0).done) break;
    }
    const auto t1 = std::chrono::steady_clock::now();
    prof_collect(c);
    GmresState fin{};
    HIPCHK(hipMemcpy(&fin, st, sizeof(GmresState), hipMemcpyDeviceToHost));
    res.converged = fin.converged;
    res.iterations = fin.its;
    res.initial_norm = fin.res0;
    res.final_norm = fin.res;
    res.seconds = std::chrono::duration<double>(t1 - t0).count();
    HIPCHK(hipMemcpyAsync(dX, x, n * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
}

}  // namespace

// ================================================================================================
extern "C" {

int cdfem_abi_version(void) { return CDFEM_ABI_VERSION; }

int cdfem_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int cdfem_create(int device, cdfem_ctx **out)
{
    if (!out) return CDFEM_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return CDFEM_ERR_HIP;
    if (device < 0 || device >= n) return CDFEM_ERR_ARG;
    cdfem_ctx *c = new (std::nothrow) cdfem_ctx();
    if (!c) return CDFEM_ERR_HIP;
    c->device = device;
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->d_state, sizeof(KrylovState)) != hipSuccess ||
        hipMemset(c->d_state, 0, sizeof(KrylovState)) != hipSuccess ||
        hipHostMalloc(&c->h_state, sizeof(KrylovState), hipHostMallocDefault) != hipSuccess ||
        hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) {
        cdfem_destroy(c);
        return CDFEM_ERR_HIP;
    }
    *out = c;
    return CDFEM_OK;
}

void cdfem_destroy(cdfem_ctx *c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    free_mesh(c);
    comm_destroy(c);
    if (c->d_state) (void)hipFree(c->d_state);
    if (c->h_state) (void)hipHostFree(c->h_state);
    if (c->d_gmst) (void)hipFree(c->d_gmst);
    if (c->h_gmpoll) (void)hipHostFree(c->h_gmpoll);
    for (auto e : c->gm_ev)
        if (e) (void)hipEventDestroy(e);
    for (auto &s : c->prof)
        for (auto e : s.ev) (void)hipEventDestroy(e);
    for (auto e : c->ov_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->stream2) (void)hipStreamDestroy(c->stream2);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char *cdfem_last_error(const cdfem_ctx *c) { return c ? c->err.c_str() : "null context"; }

int cdfem_synchronize(cdfem_ctx *c)
{
    return guarded(c, [&] {
        HIPCHK(hipStreamSynchronize(c->stream));
        return CDFEM_OK;
    });
}

int cdfem_alloc(cdfem_ctx *c, size_t bytes, void **dptr)
{
    return guarded(c, [&] {
        if (!dptr) throw ArgError("dptr is null");
        HIPCHK(hipMalloc(dptr, bytes ? bytes : 1));
        return CDFEM_OK;
    });
}

int cdfem_free(cdfem_ctx *c, void *dptr)
{
    return guarded(c, [&] {
        HIPCHK(hipFree(dptr));
        return CDFEM_OK;
    });
}

int cdfem_memcpy(cdfem_ctx *c, void *dst, int dw, const void *src, int sw, size_t bytes)
{
    return guarded(c, [&] {
        hipMemcpyKind k = dw == CDFEM_DEVICE ? (sw == CDFEM_DEVICE ? hipMemcpyDeviceToDevice
                                                                   : hipMemcpyHostToDevice)
                                             : (sw == CDFEM_DEVICE ? hipMemcpyDeviceToHost
                                                                   : hipMemcpyHostToHost);
        HIPCHK(hipMemcpyAsync(dst, src, bytes, k, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        return CDFEM_OK;
    });
}

int cdfem_vec_axpby(cdfem_ctx *c, int64_t n, double a, const double *x, double b, double *y)
{
    return guarded(c, [&] {
        if (n < 0) throw ArgError("n < 0");
        if (n == 0) return CDFEM_OK;
        if (!x || !y) throw ArgError("null vector");
        HIPCHK(launch_axpby_n(c, n, a, x, b, y));
        HIPCHK(hipStreamSynchronize(c->stream));
        return CDFEM_OK;
    });
}

int cdfem_mesh_upload(cdfem_ctx *c, int dim, int order, int ne, const double *elem_verts,
                      int64_t nldofs, const int32_t *elem_dofs, int n_ess, const int32_t *ess_dofs)
{
    return guarded(c, [&] {
        if (dim != 2 && dim != 3) throw ArgError("dim must be 2 or 3");
        if (order < 1 || order > kMaxD1 - 1) throw ArgError("order out of range");
        if (ne <= 0 || nldofs <= 0 || !elem_verts || !elem_dofs) throw ArgError("empty mesh");
        if (nldofs >= (int64_t)1 << 31) throw ArgError("nldofs exceeds int32 indexing");
        if (n_ess < 0 || (n_ess > 0 && !ess_dofs)) throw ArgError("bad essential list");
        HIPCHK(hipSetDevice(c->device));
        free_mesh(c);
        c->dim = dim;
        c->p = order;
        c->d1 = order + 1;
        c->nd = dim == 3 ? c->d1 * c->d1 * c->d1 : c->d1 * c->d1;
        c->nv = 1 << dim;
        c->ne = ne;
        c->nl = nldofs;
        c->nblk = (ne + kLanes - 1) / kLanes;
        c->qlay = (dim == 3 && order >= 3) ? 1 : 0;
        if ((int64_t)c->nblk * kLanes * c->nd >= (int64_t)1 << 31) throw ArgError("E-vector exceeds int32 indexing");
        c->rule_op = make_rule(order, rule_points_1d(0, dim, order));
        c->rule_lf = make_rule(order, rule_points_1d(1, dim, order));
        c->rule_err = make_rule(order, rule_points_1d(2, dim, order));

        const int nd = c->nd;
        c->h_ess.assign(nldofs, 0);
        for (int i = 0; i < n_ess; ++i) {
            if (ess_dofs[i] < 0 || ess_dofs[i] >= nldofs) throw ArgError("essential dof out of range");
            c->h_ess[ess_dofs[i]] = 1;
        }
        c->h_dofs.assign(elem_dofs, elem_dofs + (size_t)ne * nd);
        for (int32_t g : c->h_dofs)
            if (g < 0 || g >= nldofs) throw ArgError("element dof out of range");
        std::vector<int32_t> ess_list;
        for (int64_t i = 0; i < nldofs; ++i)
            if (c->h_ess[i]) ess_list.push_back((int32_t)i);
        c->n_ess = (int)ess_list.size();

        c->mesh_affine = mesh_is_affine(dim, ne, elem_verts);
        c->d_verts = dalloc<double>((size_t)ne * c->nv * dim);
        c->d_ess = dalloc<uint8_t>(nldofs);
        c->d_ess_list = dalloc<int32_t>(ess_list.size());
        c->d_dinv = dalloc<double>(nldofs);
        for (auto &w : c->d_w) w = dalloc<double>(nldofs);
        HIPCHK(hipMemcpyAsync(c->d_verts, elem_verts, (size_t)ne * c->nv * dim * sizeof(double),
                              hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(c->d_ess, c->h_ess.data(), nldofs, hipMemcpyHostToDevice, c->stream));
        if (!ess_list.empty())
            HIPCHK(hipMemcpyAsync(c->d_ess_list, ess_list.data(), ess_list.size() * 4,
                                  hipMemcpyHostToDevice, c->stream));
        // element blocks of 64 in input order (identity permutation, padded)
        std::vector<int32_t> perm((size_t)c->nblk * kLanes, -1);
        for (int e = 0; e < ne; ++e) perm[e] = e;
        build_layout(c, perm);
        c->mesh_ready = true;
        return CDFEM_OK;
    });
}

int cdfem_mesh_set_structured(cdfem_ctx *c, int nx, int ny, int nz)
{
    return guarded(c, [&] {
        if (c->mesh_ready && c->geom != 0) throw ArgError("structured bricks need a hexahedral mesh");
        require_mesh(c);
        if (c->dim != 3) throw UnsupportedError("structured fast path is 3D only");
        if (nx < 1 || ny < 1 || nz < 1 || (int64_t)nx * ny * nz != c->ne)
            throw ArgError("nx*ny*nz must equal the number of elements");
        const int p = c->p, d1 = c->d1, nd = c->nd;
        const int64_t Lx = (int64_t)p * nx + 1, Ly = (int64_t)p * ny + 1, Lz = (int64_t)p * nz + 1;
        if (Lx * Ly * Lz != c->nl) throw ArgError("dof count does not match the structured lattice");
        // the element dof map must be the lexicographic lattice numbering (cdfem_box_mesh)
        for (int e = 0; e < c->ne; ++e) {
            const int ix = e % nx, iy = (e / nx) % ny, iz = e / (nx * ny);
            for (int l = 0; l < nd; ++l) {
                const int dx = l % d1, dy = (l / d1) % d1, dz = l / (d1 * d1);
                const int64_t g = (p * ix + dx) + Lx * ((p * iy + dy) + Ly * (int64_t)(p * iz + dz));
                if (c->h_dofs[(size_t)e * nd + l] != g)
                    throw ArgError("element dof map is not the lexicographic structured numbering");
            }
        }
        c->sx = nx; c->sy = ny; c->sz = nz;
        c->Lx = Lx; c->Ly = Ly; c->Lz = Lz;
        if (c->qlay == 1) {
            // high order: lattice gather in the apply, pencil E-vector layout, lattice E->L
            // (k_e2l_box); element-major qdata and map are kept
            c->structured = true;
            c->epencil = c->nl < ((int64_t)1 << 32);
            c->hb_ez = c->ho_block_z;
            c->hb_nbx = (nx + kHoBrickEdge - 1) / kHoBrickEdge;
            c->hb_nby = (ny + kHoBrickEdge - 1) / kHoBrickEdge;
            c->hb_nbz = (nz + c->hb_ez - 1) / c->hb_ez;
            c->hb_nblk = c->hb_nbx * c->hb_nby * c->hb_nbz;
            upload_brick_ess(c, kHoBrickEdge, c->hb_ez, c->hb_nbx, c->hb_nby, c->hb_nbz);
            dfree(c->d_face);  // the high-order brick CG's patch buffer: allocated by its first solve
            return CDFEM_OK;
        }
        c->nbx = (nx + kBrick - 1) / kBrick;
        c->nby = (ny + kBrick - 1) / kBrick;
        c->nbz = (nz + kBrick - 1) / kBrick;
        c->nblk = c->nbx * c->nby * c->nbz;
        upload_brick_ess(c, kBrick, kBrick, c->nbx, c->nby, c->nbz);
        // brick permutation: block = brick (lexicographic), lane = ex + 4 (ey + 4 ez)
        std::vector<int32_t> perm((size_t)c->nblk * kLanes, -1);
        for (int b = 0; b < c->nblk; ++b) {
            const int bx = b % c->nbx, by = (b / c->nbx) % c->nby, bz = b / (c->nbx * c->nby);
            for (int t = 0; t < kLanes; ++t) {
                const int ix = kBrick * bx + (t & 3), iy = kBrick * by + ((t >> 2) & 3),
                          iz = kBrick * bz + (t >> 4);
                if (ix < nx && iy < ny && iz < nz) perm[(size_t)b * kLanes + t] = ix + nx * (iy + ny * iz);
            }
        }
        build_layout(c, perm);
        const int S = kBrick * p + 1;
        c->nface = 2 * S * S + (S - 2) * (4 * S - 4);
        dfree(c->d_face);
        // per brick: the Mult's face partials (nface) or the CG apply's whole patch output (S^3)
        c->d_face = dalloc<double>((size_t)c->nblk * std::max(c->nface, S * S * S));
        dfree(c->d_qd);
        c->structured = true;
        c->pa_ready = false;
        c->dinv_ready = false;
        return CDFEM_OK;
    });
}

int cdfem_set_slab(cdfem_ctx *c, int zlo_shared, int zhi_shared)
{
    return guarded(c, [&] {
        if (!c->structured) throw StateError("cdfem_mesh_set_structured must precede cdfem_set_slab");
        if (c->dim != 3) throw UnsupportedError("multi-rank slabs are 3D z-slabs");
        if ((zlo_shared || zhi_shared) && !c->comm) throw StateError("attach a communicator first");
        if (c->part_mode == 2) throw StateError("a general partition (cdfem_set_shared) is already declared");
        c->zlo_shared = zlo_shared != 0;
        c->zhi_shared = zhi_shared != 0;
        const int64_t n = c->Lx * c->Ly;
        c->part_mode = 1;
        c->slab_nl_max = c->nl;
        c->slab_nb_max = brick_count(c);
        if (multi_rank(c)) {  // (collective: every rank declares its slab) each rank's counts in its own slots
            const int R = c->nranks;
            std::vector<double> h((size_t)2 * R, 0.0);
            h[2 * c->rank] = (double)c->nl;
            h[2 * c->rank + 1] = (double)brick_count(c);
            double *d = dalloc<double>(h.size());
            struct Free {
                double *p;
                ~Free() { (void)hipFree(p); }
            } fr{d};
            HIPCHK(hipMemcpyAsync(d, h.data(), h.size() * 8, hipMemcpyHostToDevice, c->stream));
            comm_allreduce(c, d, 2 * R);
            HIPCHK(hipMemcpyAsync(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            for (int k = 0; k < R; ++k) {
                c->slab_nl_max = std::max<int64_t>(c->slab_nl_max, (int64_t)h[2 * k]);
                c->slab_nb_max = std::max<int64_t>(c->slab_nb_max, (int64_t)h[2 * k + 1]);
            }
        }
        c->skip_lo = c->zlo_shared ? n : 0;  // the lower plane is owned by the rank below
        for (auto &b : c->d_if) {
            dfree(b);
            b = dalloc<double>(n);
            HIPCHK(hipMemsetAsync(b, 0, n * 8, c->stream));
        }
        c->dinv_ready = false;
        return CDFEM_OK;
    });
}

int cdfem_set_shared(cdfem_ctx *c, int n_nbr, const int32_t *nbr_ranks, const int64_t *nbr_off,
                     const int32_t *nbr_idx)
{
    return guarded(c, [&] {
        require_mesh(c);
        if (!c->comm) throw StateError("attach a communicator first");
        if (c->part_mode == 1) throw StateError("a slab partition (cdfem_set_slab) is already declared");
        if (n_nbr < 0 || (n_nbr > 0 && (!nbr_ranks || !nbr_off || !nbr_idx))) throw ArgError("bad neighbour lists");
        std::vector<int32_t> ranks(nbr_ranks, nbr_ranks + n_nbr);
        std::vector<int64_t> off(nbr_off, nbr_off + n_nbr + 1);
        if (n_nbr == 0) off.assign(1, 0);
        if (off[0] != 0) throw ArgError("nbr_off[0] must be 0");
        for (int k = 0; k < n_nbr; ++k) {
            if (ranks[k] < 0 || ranks[k] >= c->nranks || ranks[k] == c->rank) throw ArgError("bad neighbour rank");
            if (k > 0 && ranks[k] <= ranks[k - 1]) throw ArgError("neighbour ranks must be strictly ascending");
            if (off[k + 1] <= off[k]) throw ArgError("every neighbour shares at least one dof");
        }
        const int64_t ntot = off[n_nbr];
        if (ntot >= ((int64_t)1 << 31)) throw ArgError("too many shared entries");
        std::vector<int32_t> idx(nbr_idx, nbr_idx + ntot);
        // holders of every shared dof (ascending rank, this rank included) and the owner
        std::vector<int32_t> first_rank(c->nl, INT32_MAX);
        std::vector<std::vector<std::pair<int32_t, int32_t>>> contrib;  // per distinct dof: (rank, src)
        std::vector<int32_t> slot(c->nl, -1), dofs;
        for (int k = 0; k < n_nbr; ++k) {
            std::vector<uint8_t> seen;
            for (int64_t j = off[k]; j < off[k + 1]; ++j) {
                const int32_t d = idx[j];
                if (d < 0 || d >= c->nl) throw ArgError("shared dof out of range");
                if (slot[d] < 0) {
                    slot[d] = (int32_t)dofs.size();
                    dofs.push_back(d);
                    contrib.push_back({{c->rank, -1}});
                }
                auto &cl = contrib[slot[d]];
                for (auto &pr : cl)
                    if (pr.first == ranks[k]) throw ArgError("a dof appears twice in one neighbour list");
                cl.push_back({ranks[k], (int32_t)j});
                first_rank[d] = std::min(first_rank[d], ranks[k]);
            }
        }
        // ownership: a dof held by a lower rank is not owned here; those dofs must be the prefix
        int64_t n_not_owned = 0;
        for (int32_t d : dofs)
            if (first_rank[d] < c->rank) ++n_not_owned;
        for (int32_t d : dofs)
            if ((first_rank[d] < c->rank) != (d < n_not_owned))
                throw ArgError("local numbering must list the dofs owned by lower ranks first (owned true dofs = suffix)");
        std::vector<int32_t> soff(1, 0), src, owner;
        for (size_t i = 0; i < dofs.size(); ++i) {
            auto cl = contrib[i];
            std::sort(cl.begin(), cl.end());
            for (auto &pr : cl) src.push_back(pr.second);
            soff.push_back((int32_t)src.size());
            owner.push_back(cl.front().first == c->rank ? -1 : cl.front().second);
        }
        partition_free(c);
        c->nbr_rank = ranks;
        c->nbr_off = off;
        c->h_sh_idx = idx;
        c->n_shd = (int32_t)dofs.size();
        c->d_sh_idx = dalloc<int32_t>(ntot);
        c->d_sh_send = dalloc<double>(ntot);
        c->d_sh_recv = dalloc<double>(ntot);
        c->d_shd = dalloc<int32_t>(dofs.size());
        c->d_shd_off = dalloc<int32_t>(soff.size());
        c->d_shd_src = dalloc<int32_t>(src.size());
        c->d_shd_owner = dalloc<int32_t>(owner.size());
        if (ntot) HIPCHK(hipMemcpyAsync(c->d_sh_idx, idx.data(), ntot * 4, hipMemcpyHostToDevice, c->stream));
        if (!dofs.empty()) {
            HIPCHK(hipMemcpyAsync(c->d_shd, dofs.data(), dofs.size() * 4, hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipMemcpyAsync(c->d_shd_src, src.data(), src.size() * 4, hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipMemcpyAsync(c->d_shd_owner, owner.data(), owner.size() * 4, hipMemcpyHostToDevice, c->stream));
        }
        HIPCHK(hipMemcpyAsync(c->d_shd_off, soff.data(), soff.size() * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        c->part_mode = 2;
        c->skip_lo = n_not_owned;
        c->dinv_ready = false;
        return CDFEM_OK;
    });
}

// every shared entry's global id against the neighbour's entry at the same position: the shared
// sums pair slot j of a neighbour list with local dof idx[j] on both sides, so the lists must agree
// entry for entry (ascending global id); a mismatch fails on both ranks of the pair
int cdfem_check_shared(cdfem_ctx *c, const int64_t *l2g)
{
    return guarded(c, [&] {
        require_mesh(c);
        if (c->part_mode != 2) throw StateError("declare the partition first (cdfem_set_shared)");
        if (!l2g) throw ArgError("l2g is null");
        const int nn = (int)c->nbr_rank.size();
        const int64_t ntot = nn ? c->nbr_off[nn] : 0;
        if (nn == 0) return CDFEM_OK;
        // 1. list lengths first: mismatched send / recv counts would hang RCCL or misread
        //    the host buffers, so both ranks of a pair compare them before any id moves
        std::vector<int64_t> off1(nn + 1);
        std::vector<double> cs(nn), cr(nn);
        for (int k = 0; k <= nn; ++k) off1[k] = k;
        for (int k = 0; k < nn; ++k) cs[k] = (double)(c->nbr_off[k + 1] - c->nbr_off[k]);
        // (the counts travel in the send / recv buffers of the shared sums when they hold nn slots,
        //  else in scratch freed on every exit path, exceptions from the exchange included)
        struct Scratch {
            double *p = nullptr;
            ~Scratch() { dfree(p); }
        } sa, sb;
        double *d_a = c->d_sh_send, *d_b = c->d_sh_recv;
        if (ntot < nn) {
            sa.p = d_a = dalloc<double>(nn);
            sb.p = d_b = dalloc<double>(nn);
        }
        HIPCHK(hipMemcpyAsync(d_a, cs.data(), nn * 8, hipMemcpyHostToDevice, c->stream));
        comm_exchange_nbr_buf(c, off1, d_a, d_b, c->stream);
        HIPCHK(hipMemcpyAsync(cr.data(), d_b, nn * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        for (int k = 0; k < nn; ++k)
            if (cr[k] != cs[k])
                throw ArgError("shared-dof list with rank " + std::to_string(c->nbr_rank[k]) + " has " +
                               std::to_string((int64_t)cs[k]) + " entries here, " + std::to_string((int64_t)cr[k]) +
                               " there");
        // 2. the ids; an out-of-range id is reported after the exchange, so every rank stays in step
        std::vector<double> send((size_t)ntot), recv((size_t)ntot);
        int64_t bad = -1;
        for (int64_t j = 0; j < ntot; ++j) {
            const int64_t g = l2g[c->h_sh_idx[j]];
            const bool ok = g >= 0 && g < ((int64_t)1 << 53);
            if (!ok && bad < 0) bad = j;
            send[j] = ok ? (double)g : -1.0;  // exact below 2^53
        }
        HIPCHK(hipMemcpyAsync(c->d_sh_send, send.data(), ntot * 8, hipMemcpyHostToDevice, c->stream));
        comm_exchange_nbr_buf(c, c->nbr_off, c->d_sh_send, c->d_sh_recv, c->stream);
        HIPCHK(hipMemcpyAsync(recv.data(), c->d_sh_recv, ntot * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (bad >= 0)
            throw ArgError("global dof id out of range: " + std::to_string(l2g[c->h_sh_idx[bad]]) +
                           " (local dof " + std::to_string(c->h_sh_idx[bad]) + ")");
        for (int k = 0; k < nn; ++k)
            for (int64_t j = c->nbr_off[k]; j < c->nbr_off[k + 1]; ++j)
                if (recv[j] != send[j])
                    throw ArgError("shared-dof list with rank " + std::to_string(c->nbr_rank[k]) + " differs at entry " +
                                   std::to_string(j - c->nbr_off[k]) + ": global id " +
                                   std::to_string((int64_t)send[j]) + " here, " + std::to_string((int64_t)recv[j]) +
                                   " there (both sides must list the shared dofs in ascending global id)");
        return CDFEM_OK;
    });
}

int cdfem_true_size(cdfem_ctx *c, int64_t *ntrue, int64_t *first_owned)
{
    return guarded(c, [&] {
        require_mesh(c);
        if (ntrue) *ntrue = c->nl - c->skip_lo;
        if (first_owned) *first_owned = c->skip_lo;
        return CDFEM_OK;
    });
}

int cdfem_prolongate(cdfem_ctx *c, const double *X, double *x, int where)
{
    return guarded(c, [&] {
        require_mesh(c);
        require_partition(c);
        if (!X || !x) throw ArgError("null vector");
        const int64_t nt = c->nl - c->skip_lo;
        double *dx = where == CDFEM_DEVICE ? x : c->d_w[1];
        HIPCHK(hipMemsetAsync(dx, 0, c->skip_lo * 8, c->stream));
        HIPCHK(hipMemcpyAsync(dx + c->skip_lo, X, nt * 8, where == CDFEM_DEVICE ? hipMemcpyDeviceToDevice
                                                                                 : hipMemcpyHostToDevice, c->stream));
        interface_copy_owner(c, dx);
        dev_out(c, x, where, dx, c->nl);
        HIPCHK(hipStreamSynchronize(c->stream));
        return CDFEM_OK;
    });
}

// simplex meshes: points of a rule (and its reference coordinates); the operator's integrators have
// rules of their own (CDFEM_RULE_DIFFUSION / CONVECTION / MASS), so CDFEM_RULE_OPERATOR is refused
static int simplex_rule_pts(const cdfem_ctx *c, int rule, const std::vector<double> **sxi)
{
    const std::vector<double> *x = nullptr;
    int nq = 0;
    switch (rule) {
    case CDFEM_RULE_DIFFUSION: x = &c->h_sxi_d; nq = c->nq_sd; break;
    case CDFEM_RULE_CONVECTION:
    case CDFEM_RULE_MASS: x = &c->h_sxi_cm; nq = c->nq_scm; break;
    case CDFEM_RULE_LINEARFORM: x = &c->h_sxi_lf; nq = c->nq_lf; break;
    case CDFEM_RULE_OPERATOR:
        throw UnsupportedError("simplex meshes: each integrator has its own rule (CDFEM_RULE_DIFFUSION, "
                               "CDFEM_RULE_CONVECTION, CDFEM_RULE_MASS)");
    default: throw UnsupportedError("simplex meshes: no such rule (the L2-error rule is host-side)");
    }
    if (sxi) *sxi = x;
    return nq;
}

int cdfem_rule_size(cdfem_ctx *c, int rule, int *nq)
{
    return guarded(c, [&] {
        require_mesh(c);
        if (!nq) throw ArgError("nq is null");
        if (c->geom != 0) {
            *nq = simplex_rule_pts(c, rule, nullptr);
            return CDFEM_OK;
        }
        const Rule1D &r = rule == CDFEM_RULE_LINEARFORM ? c->rule_lf : rule == CDFEM_RULE_ERROR ? c->rule_err
                                                                                                 : c->rule_op;
        *nq = nq_of(c, r);
        return CDFEM_OK;
    });
}

int cdfem_quadrature_points(cdfem_ctx *c, int rule, double *xyz, int where)
{
    return guarded(c, [&] {
        require_mesh(c);
        if (!xyz) throw ArgError("xyz is null");
        if (c->geom != 0) {  // affine simplices: x = v0 + J xi, evaluated on the host
            const std::vector<double> *psxi = nullptr;
            const int nq = simplex_rule_pts(c, rule, &psxi);
            const std::vector<double> &sxi = *psxi;
            const int dim = c->dim, nv = dim + 1;
            std::vector<double> out((size_t)c->ne * nq * dim);
            for (int e = 0; e < c->ne; ++e) {
                const double *V = &c->h_verts[(size_t)e * nv * dim];
                for (int q = 0; q < nq; ++q)
                    for (int k = 0; k < dim; ++k) {
                        double x = V[k];
                        for (int m = 0; m < dim; ++m) x += (V[(m + 1) * dim + k] - V[k]) * sxi[(size_t)q * dim + m];
                        out[((size_t)e * nq + q) * dim + k] = x;
                    }
            }
            if (where == CDFEM_DEVICE) {
                HIPCHK(hipMemcpyAsync(xyz, out.data(), out.size() * 8, hipMemcpyHostToDevice, c->stream));
                HIPCHK(hipStreamSynchronize(c->stream));
            } else {
                std::copy(out.begin(), out.end(), xyz);
            }
            return CDFEM_OK;
        }
        const Rule1D &r = rule == CDFEM_RULE_LINEARFORM ? c->rule_lf : rule == CDFEM_RULE_ERROR ? c->rule_err
                                                                                                 : c->rule_op;
        const size_t n = (size_t)c->ne * nq_of(c, r) * c->dim;
        double *d = where == CDFEM_DEVICE ? xyz : dalloc<double>(n);
        HIPCHK(launch_quad_points(c, r, d));
        if (where != CDFEM_DEVICE) {
            HIPCHK(hipMemcpyAsync(xyz, d, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            dfree(d);
        }
        return CDFEM_OK;
    });
}

// device copy of an optional host coefficient array (freed by the caller)
static double *upload_opt(cdfem_ctx *c, const double *h, size_t n)
{
    if (!h) return nullptr;
    double *d = dalloc<double>(n);
    HIPCHK(hipMemcpyAsync(d, h, n * 8, hipMemcpyHostToDevice, c->stream));
    return d;
}

static void check_form(const cdfem_ctx *c, const cdfem_form_coeffs *f)
{
    if (!f) throw ArgError("null form");
    if (f->kinds == 0 || f->kinds > 7) throw ArgError("kinds must be a non-empty DIFFUSION|CONVECTION|MASS mask");
    if ((f->kinds & CDFEM_CONVECTION) && !f->conv && !f->conv_q) throw ArgError("convection needs a velocity");
    (void)c;
}

static int pa_setup_form(cdfem_ctx *c, const cdfem_form_coeffs *f)
{
    return guarded(c, [&] {
        require_mesh(c);
        check_form(c, f);
        if (c->geom != 0) throw UnsupportedError("simplex meshes use full assembly: cdfem_fa_setup");
        if (!apply_supported(c->dim, c->p))
            throw UnsupportedError("no PA apply kernel built for dim=" + std::to_string(c->dim) +
                                   " order=" + std::to_string(c->p));
        const unsigned kinds = f->kinds;
        dfree(c->d_qd);
        c->kinds = kinds;
        c->ncomp = ((kinds & CDFEM_DIFFUSION) ? c->dim * (c->dim + 1) / 2 : 0) +
                   ((kinds & CDFEM_CONVECTION) ? c->dim : 0) + ((kinds & CDFEM_MASS) ? 1 : 0);
        const int nq = nq_of(c, c->rule_op);
        c->d_qd = c->qlay == 1 ? dalloc<double>((size_t)c->ne * c->rule_op.q1 * qd_ho_plane(c->ncomp, c->rule_op.q1))
                               : dalloc<double>((size_t)c->nblk * nq * c->ncomp * kLanes);
        const size_t neq = (size_t)c->ne * nq;
        dfree(c->d_qaff);
        if (c->pa_affine && c->mesh_affine && !f->kappa_q && !f->kappa_mat_q && !f->conv_q && !f->mass_q)
            c->d_qaff = dalloc<double>((size_t)c->nblk * c->ncomp * kLanes);
        double *dk = upload_opt(c, f->kappa_q, neq), *dkm = upload_opt(c, f->kappa_mat_q, neq * c->dim * (c->dim + 1) / 2);
        double *dc = upload_opt(c, f->conv_q, neq * c->dim), *dm = upload_opt(c, f->mass_q, neq);
        HIPCHK(launch_setup_qdata(c, dk, dkm, f->kappa, f->alpha, f->conv, dc, dm, f->mass));
        HIPCHK(hipStreamSynchronize(c->stream));
        dfree(dk); dfree(dkm); dfree(dc); dfree(dm);
        HIPCHK(setup_uniform_elem(c));  // pa_uniform: the common element matrix of a uniform box
        c->pa_ready = true;
        c->fa_ready = false;
        c->dinv_ready = false;
        return CDFEM_OK;
    });
}

static int fa_setup_form(cdfem_ctx *c, const cdfem_form_coeffs *f);

int cdfem_pa_setup_form(cdfem_ctx *c, const cdfem_form_coeffs *f) { return pa_setup_form(c, f); }
int cdfem_fa_setup_form(cdfem_ctx *c, const cdfem_form_coeffs *f) { return fa_setup_form(c, f); }

int cdfem_pa_setup(cdfem_ctx *c, unsigned kinds, double kappa, const double *kappa_q, double alpha,
                   const double *conv, const double *conv_q, double mass, const double *mass_q)
{
    const cdfem_form_coeffs f{kinds, kappa, kappa_q, nullptr, alpha, conv, conv_q, mass, mass_q};
    return pa_setup_form(c, &f);
}

int cdfem_fa_setup(cdfem_ctx *c, unsigned kinds, double kappa, const double *kappa_q, double alpha,
                   const double *conv, const double *conv_q, double mass, const double *mass_q)
{
    const cdfem_form_coeffs f{kinds, kappa, kappa_q, nullptr, alpha, conv, conv_q, mass, mass_q};
    return fa_setup_form(c, &f);
}

int cdfem_mesh_upload_simplex(cdfem_ctx *c, int dim, int order, int ne, const double *elem_verts,
                              int64_t nldofs, const int32_t *elem_dofs, int n_ess, const int32_t *ess_dofs)
{
    return guarded(c, [&] {
        if (dim != 2 && dim != 3) throw ArgError("dim must be 2 or 3");
        if (order < 1 || order > (dim == 2 ? 3 : 2)) throw ArgError("simplex order: 1-3 (triangles), 1-2 (tets)");
        if (ne <= 0 || nldofs <= 0 || !elem_verts || !elem_dofs) throw ArgError("empty mesh");
        if (nldofs >= (int64_t)1 << 31) throw ArgError("nldofs exceeds int32 indexing");
        if (n_ess < 0 || (n_ess > 0 && !ess_dofs)) throw ArgError("bad essential list");
        HIPCHK(hipSetDevice(c->device));
        free_mesh(c);
        c->geom = 1;
        c->dim = dim;
        c->p = order;
        c->d1 = order + 1;
        c->nd = simplex_ndofs(dim, order);
        c->nv = dim + 1;
        c->ne = ne;
        c->nl = nldofs;
        c->nblk = (ne + kLanes - 1) / kLanes;
        const int nd = c->nd;
        c->h_ess.assign(nldofs, 0);
        for (int i = 0; i < n_ess; ++i) {
            if (ess_dofs[i] < 0 || ess_dofs[i] >= nldofs) throw ArgError("essential dof out of range");
            c->h_ess[ess_dofs[i]] = 1;
        }
        c->h_dofs.assign(elem_dofs, elem_dofs + (size_t)ne * nd);
        for (int32_t g : c->h_dofs)
            if (g < 0 || g >= nldofs) throw ArgError("element dof out of range");
        c->h_verts.assign(elem_verts, elem_verts + (size_t)ne * c->nv * dim);
        std::vector<int32_t> ess_list;
        for (int64_t i = 0; i < nldofs; ++i)
            if (c->h_ess[i]) ess_list.push_back((int32_t)i);
        c->n_ess = (int)ess_list.size();
        // the integrators' rules (MFEM's GetRule on affine simplices, tabulated rules): diffusion of
        // order 2p - 2, convection and mass of order 2p; basis tables of both, diffusion first
        std::vector<double> wd, wcm, tab;
        c->nq_sd = simplex_rule_for_order(dim, std::max(2 * order - 2, 0), c->h_sxi_d, wd);
        c->nq_scm = simplex_rule_for_order(dim, 2 * order, c->h_sxi_cm, wcm);
        for (int r = 0; r < 2; ++r) {
            const std::vector<double> &xi = r == 0 ? c->h_sxi_d : c->h_sxi_cm, &w = r == 0 ? wd : wcm;
            const int nq = r == 0 ? c->nq_sd : c->nq_scm;
            const size_t o = tab.size();
            tab.resize(o + (size_t)nq * nd * (dim + 1) + nq);
            for (int q = 0; q < nq; ++q) {
                double phi[10], dphi[30];
                simplex_basis(dim, order, &xi[(size_t)q * dim], phi, dphi);
                for (int i = 0; i < nd; ++i) {
                    tab[o + (size_t)q * nd + i] = phi[i];
                    for (int k = 0; k < dim; ++k)
                        tab[o + (size_t)nq * nd + ((size_t)q * nd + i) * dim + k] = dphi[i * dim + k];
                }
                tab[o + (size_t)nq * nd * (dim + 1) + q] = w[q];
            }
        }
        // linear-form rule: DomainLFIntegrator's default order 2p, MFEM's tabulated simplex rule
        std::vector<double> wl;
        c->nq_lf = simplex_rule_for_order(dim, 2 * order, c->h_sxi_lf, wl);
        std::vector<double> tab_lf((size_t)c->nq_lf * (nd + 1));
        for (int q = 0; q < c->nq_lf; ++q) {
            double phi[10], dphi[30];
            simplex_basis(dim, order, &c->h_sxi_lf[(size_t)q * dim], phi, dphi);
            for (int i = 0; i < nd; ++i) tab_lf[(size_t)q * nd + i] = phi[i];
            tab_lf[(size_t)c->nq_lf * nd + q] = wl[q];
        }
        // E->L transpose of the element-major E-vector (linear forms)
        std::vector<int32_t> cnt(nldofs + 1, 0), pos((size_t)ne * nd);
        for (int32_t g : c->h_dofs) cnt[g + 1]++;
        for (int64_t i = 0; i < nldofs; ++i) cnt[i + 1] += cnt[i];
        {
            std::vector<int32_t> fill(cnt.begin(), cnt.end() - 1);
            for (int64_t k = 0; k < (int64_t)ne * nd; ++k) pos[fill[c->h_dofs[k]]++] = (int32_t)k;
        }
        c->d_e2l_off = dalloc<int32_t>(nldofs + 1);
        c->d_e2l_pos = dalloc<int32_t>(pos.size());
        c->d_Ye = dalloc<double>(pos.size());
        HIPCHK(hipMemcpyAsync(c->d_e2l_off, cnt.data(), (nldofs + 1) * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(c->d_e2l_pos, pos.data(), pos.size() * 4, hipMemcpyHostToDevice, c->stream));
        c->d_stab_lf = dalloc<double>(tab_lf.size());
        HIPCHK(hipMemcpyAsync(c->d_stab_lf, tab_lf.data(), tab_lf.size() * 8, hipMemcpyHostToDevice, c->stream));
        c->d_stab = dalloc<double>(tab.size());
        c->d_verts = dalloc<double>(c->h_verts.size());
        c->d_ess = dalloc<uint8_t>(nldofs);
        c->d_ess_list = dalloc<int32_t>(ess_list.size());
        c->d_dinv = dalloc<double>(nldofs);
        for (auto &v : c->d_w) v = dalloc<double>(nldofs);
        c->d_part = dalloc<double>((size_t)c->red_blocks + kSpmvMaxBlocks + 16384);
        HIPCHK(hipMemcpyAsync(c->d_stab, tab.data(), tab.size() * 8, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(c->d_verts, c->h_verts.data(), c->h_verts.size() * 8, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(c->d_ess, c->h_ess.data(), nldofs, hipMemcpyHostToDevice, c->stream));
        if (!ess_list.empty())
            HIPCHK(hipMemcpyAsync(c->d_ess_list, ess_list.data(), ess_list.size() * 4, hipMemcpyHostToDevice,
                                  c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        c->mesh_ready = true;
        return CDFEM_OK;
    });
}

static int fa_setup_form(cdfem_ctx *c, const cdfem_form_coeffs *f)
{
    return guarded(c, [&] {
        require_mesh(c);
        check_form(c, f);
        const unsigned kinds = f->kinds;
        if (c->geom != 1) throw UnsupportedError("full assembly is implemented for simplex meshes");
        if (!c->d_rowptr) {  // CSR pattern + contribution lists: once per mesh
            // a multi-rank partition keeps the mesh order (its shared-dof exchange indexes L-vectors)
            // dof coordinates for the geometric SpMV order (simplex geometry is on the host)
            std::vector<double> xyz;
            if (!multi_rank(c) && (c->sell_mode == 3 || c->sell_mode >= 5) && !c->h_verts.empty())
                xyz = simplex_dof_coords(c->dim, c->p, c->ne, c->nd, c->nl, c->h_verts, c->h_dofs);
            FaPattern P = fa_build_pattern(c->h_dofs, c->ne, c->nd, c->nl,
                                           multi_rank(c) ? 0 : c->sell_mode, c->dim,
                                           xyz.empty() ? nullptr : xyz.data(), c->sell_window, c->spmv_lds,
                                           c->spmv_lpr);
            if (P.lds_rows > 0) {
                // the LDS-staged SpMV launches one block per window (rounded up to whole XCD ranges)
                // and its CG form writes one partial per block: the grid must fit the partial slots
                // (ADVICE r03).  Windows halve below their nominal size when halos are large, so the
                // automatic choice falls back to the layout without LDS; an explicit one is refused.
                const int64_t spw = P.lds_rows / (kLanes / std::max(1, P.lpr));
                const int64_t nwin = ((int64_t)P.sptr.size() - 1 + spw - 1) / spw;
                if (8 * ((nwin + 7) / 8) > kSpmvMaxBlocks) {
                    if (c->spmv_lds >= 0)
                        throw UnsupportedError("spmv_lds " + std::to_string(c->spmv_lds) + ": " +
                                               std::to_string(nwin) + " LDS windows exceed the SpMV grid (" +
                                               std::to_string(kSpmvMaxBlocks) + " blocks); use larger windows or 0");
                    P = fa_build_pattern(c->h_dofs, c->ne, c->nd, c->nl, multi_rank(c) ? 0 : c->sell_mode,
                                         c->dim, xyz.empty() ? nullptr : xyz.data(), c->sell_window, 0, 1);
                }
            }
            c->nnz = P.nnz;
            c->d_rowptr = dalloc<int32_t>(P.rowptr.size());
            c->d_cols = dalloc<int32_t>(P.cols.size());
            c->d_diagpos = dalloc<int32_t>(P.diagpos.size());
            c->d_coff = dalloc<int32_t>(P.coff.size());
            c->d_cpos = dalloc<int32_t>(P.cpos.size());
            c->d_vals = dalloc<double>(c->nnz);
            c->d_vals_c = dalloc<double>(c->nnz);
            c->d_Ee = dalloc<double>((size_t)c->nblk * c->nd * c->nd * kLanes);
            HIPCHK(hipMemcpyAsync(c->d_rowptr, P.rowptr.data(), P.rowptr.size() * 4, hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipMemcpyAsync(c->d_cols, P.cols.data(), P.cols.size() * 4, hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipMemcpyAsync(c->d_diagpos, P.diagpos.data(), P.diagpos.size() * 4, hipMemcpyHostToDevice,
                                  c->stream));
            HIPCHK(hipMemcpyAsync(c->d_coff, P.coff.data(), P.coff.size() * 4, hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipMemcpyAsync(c->d_cpos, P.cpos.data(), P.cpos.size() * 4, hipMemcpyHostToDevice, c->stream));
            c->nslices = (int64_t)P.sptr.size() - 1;
            if ((c->nslices + 3) / 4 + 8 > kSpmvMaxBlocks) throw UnsupportedError("matrix too large for the SpMV grid");
            c->nstored = P.sptr.back();
            c->d_sptr = dalloc<int32_t>(P.sptr.size());
            c->d_srows = dalloc<int32_t>(P.srows.size());
            c->d_scols = dalloc<int32_t>(P.scols.size());
            c->d_smap = dalloc<int32_t>(P.smap.size());
            c->d_svals = dalloc<double>(c->nstored);
            c->d_svals_c = dalloc<double>(c->nstored);
            HIPCHK(hipMemcpyAsync(c->d_sptr, P.sptr.data(), P.sptr.size() * 4, hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipMemcpyAsync(c->d_srows, P.srows.data(), P.srows.size() * 4, hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipMemcpyAsync(c->d_scols, P.scols.data(), P.scols.size() * 4, hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipMemcpyAsync(c->d_smap, P.smap.data(), P.smap.size() * 4, hipMemcpyHostToDevice, c->stream));
            c->sell_windowed = P.windowed;
            if (!P.perm.empty()) {
                c->d_rperm = dalloc<int32_t>(P.perm.size());
                HIPCHK(hipMemcpyAsync(c->d_rperm, P.perm.data(), P.perm.size() * 4, hipMemcpyHostToDevice, c->stream));
                for (auto &v : c->d_pv) v = dalloc<double>(c->nl);
            }
            if (!P.sdel.empty()) {
                c->d_sdel = dalloc<int16_t>(P.sdel.size());
                HIPCHK(hipMemcpyAsync(c->d_sdel, P.sdel.data(), P.sdel.size() * 2, hipMemcpyHostToDevice, c->stream));
            }
            if (P.lds_rows > 0) {  // LDS-staged windows (sell_plan.cpp)
                c->d_hptr = dalloc<int32_t>(P.hptr.size());
                c->d_hidx = dalloc<int32_t>(std::max<size_t>(P.hidx.size(), 1));
                c->d_sloc = dalloc<uint16_t>(P.sloc.size());
                HIPCHK(hipMemcpyAsync(c->d_hptr, P.hptr.data(), P.hptr.size() * 4, hipMemcpyHostToDevice, c->stream));
                HIPCHK(hipMemcpyAsync(c->d_hidx, P.hidx.data(), P.hidx.size() * 4, hipMemcpyHostToDevice, c->stream));
                HIPCHK(hipMemcpyAsync(c->d_sloc, P.sloc.data(), P.sloc.size() * 2, hipMemcpyHostToDevice, c->stream));
                c->lds_rows = P.lds_rows;
                c->sell_lpr = P.lpr;
                c->lds_max = P.lds_max;
                c->lds_halo = (int64_t)P.hidx.size();
            }
            if (!P.swide.empty()) {  // mixed layout: the slices beyond 16 bits stream d_scols
                c->d_swide = dalloc<uint8_t>(P.swide.size());
                HIPCHK(hipMemcpyAsync(c->d_swide, P.swide.data(), P.swide.size(), hipMemcpyHostToDevice, c->stream));
                c->sell_nnz_wide = P.nnz_wide;
            }
            HIPCHK(hipStreamSynchronize(c->stream));  // P's host buffers die at scope exit
        }
        // per-point coefficients at the rule of their integrator
        const size_t nqd = (size_t)c->ne * c->nq_sd, nqc = (size_t)c->ne * c->nq_scm;
        double *dk = upload_opt(c, f->kappa_q, nqd), *dkm = upload_opt(c, f->kappa_mat_q, nqd * c->dim * (c->dim + 1) / 2);
        double *dc = upload_opt(c, f->conv_q, nqc * c->dim), *dm = upload_opt(c, f->mass_q, nqc);
        c->kinds = kinds;
        HIPCHK(launch_simplex_elem(c, dk, dkm, f->kappa, f->alpha, f->conv, dc, dm, f->mass));
        HIPCHK(launch_fa_assemble(c));
        HIPCHK(launch_sell_fill(c));
        HIPCHK(hipStreamSynchronize(c->stream));
        dfree(dk); dfree(dkm); dfree(dc); dfree(dm);
        c->fa_ready = true;
        c->pa_ready = false;
        c->dinv_ready = false;
        ilu_free(c);  // factors belong to the previous operator
        return CDFEM_OK;
    });
}

int cdfem_fa_csr(cdfem_ctx *c, int constrained, int64_t *nnz, int32_t *rowptr, int32_t *cols, double *vals)
{
    return guarded(c, [&] {
        if (!c->fa_ready) throw StateError("cdfem_fa_setup has not been called");
        if (!nnz) throw ArgError("nnz is null");
        *nnz = c->nnz;
        if (rowptr) HIPCHK(hipMemcpy(rowptr, c->d_rowptr, (c->nl + 1) * 4, hipMemcpyDeviceToHost));
        if (cols) HIPCHK(hipMemcpy(cols, c->d_cols, c->nnz * 4, hipMemcpyDeviceToHost));
        if (vals)
            HIPCHK(hipMemcpy(vals, constrained ? c->d_vals_c : c->d_vals, c->nnz * 8, hipMemcpyDeviceToHost));
        return CDFEM_OK;
    });
}

int cdfem_pa_mult(cdfem_ctx *c, const double *x, double *y, int constrained, int where)
{
    return guarded(c, [&] {
        require_pa(c);
        if (constrained != 2) require_partition(c);
        if (!x || !y) throw ArgError("null vector");
        if (constrained < 0 || constrained > 2) throw ArgError("constrained must be 0, 1 or 2 (local)");
        const double *dx = dev_in(c, x, where, c->d_w[0], c->nl);
        double *dy = where == CDFEM_DEVICE ? y : c->d_w[1];
        if (constrained == 2) op_apply(c, dx, dy, false);  // rank-local partial sums (no exchange)
        else op_apply_global(c, dx, dy, constrained != 0);  // shared dofs: neighbours' partial sums added
        dev_out(c, y, where, dy, c->nl);
        prof_collect(c);
        return CDFEM_OK;
    });
}

int cdfem_pa_diagonal(cdfem_ctx *c, double *diag, int where)
{
    return guarded(c, [&] {
        require_pa(c);
        if (!diag) throw ArgError("null vector");
        double *dd = where == CDFEM_DEVICE ? diag : c->d_w[1];
        if (c->fa_ready) {
            HIPCHK(launch_csr_diag(c, dd));
        } else {
            HIPCHK(launch_diag_elem(c, c->d_Ye));
            HIPCHK(launch_e2l(c, c->d_Ye, nullptr, dd, false, 0));
        }
        dev_out(c, diag, where, dd, c->nl);
        return CDFEM_OK;
    });
}

int cdfem_lf_assemble(cdfem_ctx *c, const double *f_q, double *b, int where)
{
    return guarded(c, [&] {
        require_mesh(c);
        if (!f_q || !b) throw ArgError("null vector");
        const size_t n = (size_t)c->ne * (c->geom != 0 ? c->nq_lf : nq_of(c, c->rule_lf));
        if (c->lfq_cap < n) {  // kept: a time loop assembles a linear form every step
            dfree(c->d_lfq);
            c->d_lfq = dalloc<double>(n);
            c->lfq_cap = n;
        }
        double *dfq = c->d_lfq;
        HIPCHK(hipMemcpyAsync(dfq, f_q, n * 8, where == CDFEM_DEVICE ? hipMemcpyDeviceToDevice
                                                                     : hipMemcpyHostToDevice, c->stream));
        double *db = where == CDFEM_DEVICE ? b : c->d_w[1];
        if (c->geom != 0) HIPCHK(launch_simplex_lf(c, dfq, c->d_Ye));
        else HIPCHK(launch_lf_elem(c, dfq, c->d_Ye));
        HIPCHK(launch_e2l(c, c->d_Ye, nullptr, db, false, 0));
        dev_out(c, b, where, db, c->nl);
        HIPCHK(hipStreamSynchronize(c->stream));
        return CDFEM_OK;
    });
}

int cdfem_form_linear_system(cdfem_ctx *c, const double *x, const double *b, double *X, double *B,
                             int where)
{
    return guarded(c, [&] {
        require_pa(c);
        require_partition(c);
        if (!x || !b || !X || !B) throw ArgError("null vector");
        const double *dx = dev_in(c, x, where, c->d_w[0], c->nl);
        const double *db = dev_in(c, b, where, c->d_w[1], c->nl);
        double *xe = c->d_w[2], *z = c->d_w[3];
        double *dB = where == CDFEM_DEVICE ? B : c->d_w[4];
        HIPCHK(launch_mask_ess(c, dx, xe));                 // x_e: essential part of x
        op_apply(c, xe, z, false);                          // z = A x_e
        if (dB != db) HIPCHK(hipMemcpyAsync(dB, db, c->nl * 8, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(launch_axpby(c, -1.0, z, 1.0, dB));          // B = b - A x_e
        interface_sum(c, dB);                               // P^T on the shared planes
        HIPCHK(launch_set_ess(c, dB, dx));                  // B[ess] = x[ess]
        dev_out(c, B, where, dB, c->nl);
        dev_out(c, X, where, dx, c->nl);
        HIPCHK(hipStreamSynchronize(c->stream));
        prof_collect(c);
        return CDFEM_OK;
    });
}

int cdfem_solve(cdfem_ctx *c, const cdfem_solver_params *p, const double *B, double *X, int where,
                cdfem_solver_result *res)
{
    return guarded(c, [&] {
        require_pa(c);
        require_partition(c);
        if (!p || !B || !X || !res) throw ArgError("null argument");
        if (p->max_iter < 0) throw ArgError("max_iter < 0");
        if (p->pc != CDFEM_PC_NONE && p->pc != CDFEM_PC_JACOBI && p->pc != CDFEM_PC_ILU)
            throw ArgError("unknown preconditioner");
        if (p->pc == CDFEM_PC_ILU && p->method != CDFEM_GMRES)
            throw UnsupportedError("ILU(0) preconditions GMRES (a nonsymmetric preconditioner for CG)");
        *res = cdfem_solver_result{};
        if (p->method != CDFEM_CG && p->method != CDFEM_GMRES) throw ArgError("unknown method");
        const double *dB = dev_in(c, B, where, c->d_w[6], c->nl);
        double *dX = where == CDFEM_DEVICE ? X : c->d_w[1];
        // permuted SpMV layout (sell_plan.cpp): the Krylov iteration runs in the SpMV's order, B in
        // and X out are permuted once per solve.  ILU(0) factors the matrix in mesh order (PETSc's
        // natural ordering), so it keeps the mesh order and permutes around each apply instead.
        const bool pspace = c->fa_ready && c->d_rperm && !multi_rank(c) && p->pc != CDFEM_PC_ILU;
        struct SpaceGuard {
            cdfem_ctx *c;
            ~SpaceGuard() { c->perm_space = false; }
        } guard{c};
        const double *dBs = dB;
        double *dXs = dX;
        if (pspace) {
            HIPCHK(launch_perm(c, true, dB, c->d_pv[0]));
            dBs = c->d_pv[0];
            dXs = c->d_pv[1];
            c->perm_space = true;
        }
        if (p->method == CDFEM_CG) {
            if (use_brick_cg(c))
                solve_cg_brick(c, *p, dBs, dXs, *res);
            else
                solve_cg(c, *p, dBs, dXs, *res);
        } else {
            solve_gmres(c, *p, dBs, dXs, *res);
        }
        if (pspace) {
            c->perm_space = false;
            HIPCHK(launch_perm(c, false, dXs, dX));
        }
        dev_out(c, X, where, dX, c->nl);
        HIPCHK(hipStreamSynchronize(c->stream));
        return res->converged ? CDFEM_OK : CDFEM_ERR_NOT_CONVERGED;
    });
}

int cdfem_stream_bench(cdfem_ctx *c, int mode, size_t bytes, int reps, double *gbps)
{
    return guarded(c, [&] {
        if (!gbps || reps < 1 || mode < 0 || mode > 17) throw ArgError("bad stream bench arguments");
        int64_t n = (int64_t)(bytes / 16) * 2;
        if (mode >= 3) n = n / 40960 * 40960;  // whole 320 KiB chunks
        double *a = dalloc<double>(n), *b = dalloc<double>(n);
        HIPCHK(hipMemsetAsync(a, 0, n * 8, c->stream));
        HIPCHK(hipMemsetAsync(b, 0, n * 8, c->stream));
        HIPCHK(launch_stream(c, mode, a, b, n));  // warm-up
        hipEvent_t e0, e1;
        HIPCHK(hipEventCreate(&e0));
        HIPCHK(hipEventCreate(&e1));
        HIPCHK(hipEventRecord(e0, c->stream));
        for (int i = 0; i < reps; ++i) HIPCHK(launch_stream(c, mode, a, b, n));
        HIPCHK(hipEventRecord(e1, c->stream));
        HIPCHK(hipEventSynchronize(e1));
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        dfree(a);
        dfree(b);
        double moved = (mode == 2 ? 2.0 : 1.0) * 8.0 * (double)n * reps;
        if (mode == 14 || mode == 15) {  // workgroup chunks: whole groups of 4 / 2 chunks
            const int64_t nw = mode == 14 ? 4 : 2;
            moved = 8.0 * 40960.0 * (double)(n / 40960 / nw * nw) * reps;
        }
        if (mode >= 10 && mode <= 13) {  // skewed chunks: whole 320 KiB chunks at a stride of 320 KiB + skew
            const int64_t skew[4] = {32, 64, 128, 512};
            moved = 8.0 * 40960.0 * (double)(n / (40960 + skew[mode - 10])) * reps;
        }
        *gbps = moved / (ms * 1e-3) / 1e9;
        return CDFEM_OK;
    });
}

int cdfem_fp64_bench(cdfem_ctx *c, int mode, int reps, double *tflops)
{
    return guarded(c, [&] {
        if (!tflops || reps < 1 || mode < 0 || mode > 4) throw ArgError("bad fp64 bench arguments");
        double *out = dalloc<double>(1), flops = 0.0;
        HIPCHK(launch_fp64_probe(c, mode, out, &flops));  // warm-up
        hipEvent_t e0, e1;
        HIPCHK(hipEventCreate(&e0));
        HIPCHK(hipEventCreate(&e1));
        HIPCHK(hipEventRecord(e0, c->stream));
        for (int i = 0; i < reps; ++i) HIPCHK(launch_fp64_probe(c, mode, out, &flops));
        HIPCHK(hipEventRecord(e1, c->stream));
        HIPCHK(hipEventSynchronize(e1));
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        dfree(out);
        *tflops = flops * reps / (ms * 1e-3) / 1e12;
        return CDFEM_OK;
    });
}

int cdfem_set_option(cdfem_ctx *c, const char *key, int value)
{
    return guarded(c, [&] {
        if (!key) throw ArgError("key is null");
        const std::string k(key);
        if (k == "brick_xcd") {
            if (value < 0 || value > 1) throw ArgError("brick_xcd must be 0 or 1");
            c->brick_xcd = value;
        } else if (k == "brick_byte_limit") {
            if (value < 0) throw ArgError("brick_byte_limit must be 0 (the default 2^31) or 1..2^31-1");
            c->brick_limit = value == 0 ? (int64_t)1 << 31 : value;
        } else if (k == "den_group") {
            if (value < 0 || value > 64 || (value & (value - 1)) != 0)
                throw ArgError("den_group must be 0 (automatic) or a power of two up to 64");
            c->den_group_opt = value;
        } else if (k == "cg_mr_fold") {
            if (value != 0 && value != 1) throw ArgError("cg_mr_fold must be 0 or 1");
            c->cg_mr_fold = value;
        } else if (k == "ho_brick_mfma") {
            if (value != 0 && value != 1) throw ArgError("ho_brick_mfma must be 0 or 1");
            c->ho_brick_mfma = value;
        } else if (k == "brick_stagger") {
            if (value < -1 || value > 511) throw ArgError("brick_stagger must be -1 (automatic), 0 (off) or 1..511");
            c->brick_stagger = value;
        } else if (k == "pa_uniform") {  // the matrix is formed by cdfem_pa_setup; 0 leaves it unused
            if (value != 0 && value != 1) throw ArgError("pa_uniform must be 0 or 1");
            c->pa_uniform = value;
        } else if (k == "brick_mfma") {
            if (value != 0 && value != 1) throw ArgError("brick_mfma must be 0 or 1");
            c->brick_mfma = value;
        } else if (k == "ho_block_z") {  // read by cdfem_mesh_set_structured
            if (value != 2 && value != 4) throw ArgError("ho_block_z must be 2 or 4");
            c->ho_block_z = value;
        } else if (k == "ho_brick") {
            if (value != 0 && value != 1) throw ArgError("ho_brick must be 0 or 1");
            c->ho_brick = value;
        } else if (k == "mr_overlap") {
            if (value < 0 || value > 1) throw ArgError("mr_overlap must be 0 or 1");
            c->mr_overlap = value;
        } else if (k == "brick_mult_pb") {
            if (value != 0 && value != 1) throw ArgError("brick_mult_pb must be 0 or 1");
            c->brick_mult_pb = value;
        } else if (k == "cg_beta_fold") {
            if (value != 0 && value != 1) throw ArgError("cg_beta_fold must be 0 or 1");
            c->cg_beta_fold = value;
        } else if (k == "cg_den_fold") {
            if (value != 0 && (value < 64 || value > 16384)) throw ArgError("cg_den_fold must be 0 or 64..16384");
            c->cg_den_fold = value;
        } else if (k == "brick_upd_pb") {
            if (value != 0 && value != 1) throw ArgError("brick_upd_pb must be 0 or 1");
            c->brick_upd_pb = value;
        } else if (k == "ho_dfold") {
            if (value != 0 && value != 1) throw ArgError("ho_dfold must be 0 or 1");
            c->ho_dfold = value;
        } else if (k == "ho_mfma") {
            if (value != 0 && value != 1 && value != 3 && value != 8 && value != 9 && value != 15)
                throw ArgError("ho_mfma must be 0, 1, 3, 8, 9 or 15");
            c->ho_mfma = value;
        } else if (k == "cg_xfold") {
            if (value != 0 && value != 1) throw ArgError("cg_xfold must be 0 or 1");
            c->cg_xfold = value;
        } else if (k == "cg_fused") {
            if (value < 0 || value > 1) throw ArgError("cg_fused must be 0 or 1");
            c->cg_fused = value;
        } else if (k == "sell_order") {  // read when the FA pattern is built (once per mesh)
            if (value < 0 || value > 8)
                throw ArgError("sell_order must be 0..8 (0 natural, 1 natural + windows, 2 RCM + windows, 3 auto, 4 RCM, 5 geometric, 6 Morton + windows, 7 Morton, 8 Morton LDS windows / auto)");
            c->sell_mode = value;
        } else if (k == "gm_poll") {
            if (value < 1 || value > 64) throw ArgError("gm_poll must be 1..64");
            c->gm_poll = value;
        } else if (k == "gm_pb") {
            if (value < 0 || value > 1) throw ArgError("gm_pb must be 0 or 1");
            c->gm_pb = value;
        } else if (k == "pa_affine") {  // read by cdfem_pa_setup
            if (value < 0 || value > 2) throw ArgError("pa_affine must be 0, 1 or 2");
            c->pa_affine = value;
        } else if (k == "spmv_lpr") {  // read when the FA pattern is built (once per mesh)
            if (value != 0 && value != 1 && value != 2 && value != 4) throw ArgError("spmv_lpr must be 0 (auto), 1, 2 or 4");
            c->spmv_lpr = value;
        } else if (k == "spmv_lds") {  // read when the FA pattern is built (once per mesh)
            if (value < -1 || (value > 0 && (value % 64 != 0 || value > 65536)))
                throw ArgError("spmv_lds must be -1 (auto), 0 (off) or rows per window, a multiple of 64 up to 65536");
            c->spmv_lds = value;
        } else if (k == "sell_window") {  // read when the FA pattern is built (once per mesh)
            if (value < 0 || (value > 0 && (value % 64 != 0 || value > (1 << 20))))
                throw ArgError("sell_window must be 0 (auto) or a multiple of 64 up to 2^20");
            c->sell_window = value;
        } else if (k == "gm_ept") {
            if (value != 0 && value != 4 && value != 5 && value != 6 && value != 8)
                throw ArgError("gm_ept must be 0 (auto), 4, 5, 6 or 8");
            c->gm_ept = value;
        } else if (k == "spmv_xcd") {
            if (value < 0 || value > 1) throw ArgError("spmv_xcd must be 0 or 1");
            c->spmv_xcd = value;
        } else if (k == "spmv_index16") {
            if (value < 0 || value > 1) throw ArgError("spmv_index16 must be 0 or 1");
            c->spmv_index16 = value;
        } else if (k == "profile_mask") {
            c->prof_mask = (unsigned)value;
        } else {
            throw ArgError("unknown option " + k);
        }
        return CDFEM_OK;
    });
}

int cdfem_profile_enable(cdfem_ctx *c, int on)
{
    return guarded(c, [&] {
        c->profile = on != 0;
        return CDFEM_OK;
    });
}

int cdfem_profile_reset(cdfem_ctx *c)
{
    return guarded(c, [&] {
        for (auto &s : c->prof) {
            s.used = 0;
            s.total_ms = 0.0;
            s.count = 0;
            s.each.clear();
        }
        return CDFEM_OK;
    });
}

int cdfem_profile_read(cdfem_ctx *c, int k, double *total_ms, int64_t *count)
{
    return guarded(c, [&] {
        if (k < 0 || k >= CDFEM_K_COUNT) throw ArgError("bad kernel id");
        if (total_ms) *total_ms = c->prof[k].total_ms;
        if (count) *count = c->prof[k].count;
        return CDFEM_OK;
    });
}

int cdfem_profile_launches(cdfem_ctx *c, int k, double *ms, int64_t cap, int64_t *count)
{
    return guarded(c, [&] {
        if (k < 0 || k >= CDFEM_K_COUNT) throw ArgError("bad kernel id");
        const auto &e = c->prof[k].each;
        const int64_t n = (int64_t)e.size();
        if (count) *count = n;
        if (ms)
            for (int64_t i = 0; i < std::min(cap, n); ++i) ms[i] = e[i];
        return CDFEM_OK;
    });
}

// name of the HIP kernel that kernel id runs as in the current configuration (rocprof's kernel
// name without its template arguments): the apply of a CG solve (the roofline kernel of the bench)
int cdfem_kernel_name(cdfem_ctx *c, int k, char *buf, size_t n)
{
    return guarded(c, [&] {
        require_pa(c);
        if (!buf || n == 0) throw ArgError("buffer is null");
        if (k != CDFEM_K_APPLY) throw UnsupportedError("kernel names: the operator apply only");
        const char *name = c->fa_ready ? (c->lds_rows > 0 ? "k_sell_spmv_lds" : "k_sell_spmv")
                           : use_brick(c) ? "k_brick_cg"
                           : use_hobrick_cg(c) ? "k_hobrick_cg"
                           : c->qlay == 1 ? (tile_kron(c) ? "k_apply3d_ktile" : "k_apply3d_tile")
                                          : "k_apply3d";
        std::snprintf(buf, n, "%s", name);
        return CDFEM_OK;
    });
}

int cdfem_kernel_flops(cdfem_ctx *c, int k, double *flops)
{
    return guarded(c, [&] {
        require_pa(c);
        if (!flops) throw ArgError("flops is null");
        if (k != CDFEM_K_APPLY || c->fa_ready || c->dim != 3)
            throw UnsupportedError("kernel flops: the 3D partial-assembly apply only");
        // sum factorization, one element (pa_core.hpp elem_apply3d): per z plane the z contraction
        // (D^3 FMA per field), per (z, y) the y contraction, per point the x contraction, the
        // point operator and the transposed x contraction, then the transposed y and z contractions.
        // Fields: value, plus the three reference derivatives when diffusion or convection is on.
        const int D = c->d1, Q = c->rule_op.q1;
        const bool kD = c->kinds & CDFEM_DIFFUSION, kC = c->kinds & CDFEM_CONVECTION, kM = c->kinds & CDFEM_MASS;
        if (c->qlay == 0 && uniform_elem(c) && use_brick(c)) {
            // the common element matrix (k_brick_cg<..., MX 2>): nd^2 MACs per element (the MFMA tiles'
            // zero padding, 56 x 1024 MACs per 64 elements against 64 x 729, is not counted)
            *flops = 2.0 * (double)c->nd * c->nd * (double)c->ne;
            return CDFEM_OK;
        }
        if ((c->qlay == 0 && pa_af(c) == 2) || (c->qlay == 1 && tile_kron(c))) {
            // Kronecker form (pa_core.hpp elem_apply3d_kron; the tile kernel k_apply3d_ktile runs the
            // same stages across threads), per input z plane: a length-n linear combination counts
            // 2n - 1 flops, an accumulation into Y 2 per term
            const bool kG = kD || kC;
            auto lc = [](int n) { return n > 0 ? 2.0 * n - 1.0 : 0.0; };
            const double x_row = lc(D) * (1 + 2 * kD + kG) + lc(kM + kD + kC) + 2 * lc(kD + kC);
            double y_pt = lc(D) + (kG ? 2 * lc(D) + 1 : 0.0);
            if (kD) y_pt += 6 * lc(D) + 2 + 2 + 1 + 2 + 3;
            const double z_pt = 2.0 * (1 + 2 * kD + kG) * D;
            *flops = (double)D * ((double)D * D * x_row + (double)D * D * (y_pt + z_pt)) * (double)c->ne;
            return CDFEM_OK;
        }
        const int g = (kD || kC) ? 1 : 0;
        double pt_fma = D * (1 + 3 * g) + D * (kD ? 4 : 1), pt_mul = 0.0;  // x contraction, transposed x
        if (kD) { pt_fma += 6; pt_mul += 3; }
        if (kC) { pt_fma += 2; pt_mul += 1; }
        if (kM) { if (kC) pt_fma += 1; else pt_mul += 1; }
        if (c->qlay == 1 ? tile_affine(c) : c->d_qaff != nullptr)
            pt_mul += c->ncomp + 2;  // point data W_q * g_k, W_q = (w_x w_y) w_z
        const double fma = Q * ((double)D * D * D * (1 + g) + Q * ((double)D * D * (1 + 2 * g) + Q * pt_fma +
                                                                   (double)D * D * (kD ? 3 : 1)) +
                                (double)D * D * D * (kD ? 2 : 1));
        const double mul = (double)Q * Q * Q * pt_mul;
        *flops = (2.0 * fma + mul) * (double)c->ne;
        return CDFEM_OK;
    });
}

int cdfem_kernel_bytes(cdfem_ctx *c, int k, double *bytes)
{
    return guarded(c, [&] {
        require_pa(c);
        if (!bytes) throw ArgError("bytes is null");
        const double nl = (double)c->nl, ne = (double)c->ne, nd = c->nd;
        if (c->fa_ready) {  // CSR SpMV: values + columns + row pointers + x + y
            if (k != CDFEM_K_APPLY) throw ArgError("FA operators report the SpMV (CDFEM_K_APPLY) only");
            // (SELL adds < 1 % padding; 16-bit column deltas when the bandwidth fits)
            // 8 B value + 2 B delta per entry (4 B column in the 32-bit slices of a mixed layout); LDS
            // windows: 8 B value + 2 B window position per entry, 4 B per staged column (the x values
            // themselves: 8 B per row, each window's halo beyond its own rows from L2)
            if (c->lds_rows > 0)
                *bytes = 10.0 * (double)c->nnz + 4.0 * (double)c->lds_halo + 4.0 * (double)(c->nslices + 1) +
                         16.0 * nl;
            else *bytes = spmv_delta(c) ? 10.0 * (double)c->nnz + 2.0 * (double)c->sell_nnz_wide + 4.0 * (nl + 1) + 16.0 * nl +
                                         (c->d_swide ? (double)c->nslices : 0.0)
                                   : 12.0 * (double)c->nnz + 4.0 * (nl + 1) + 16.0 * nl;
            return CDFEM_OK;
        }
        const double nq = nq_of(c, c->rule_op);
        if (use_hobrick_cg(c) && (k == CDFEM_K_APPLY || k == CDFEM_K_UPDATE)) {
            // the high-order brick CG: factors + gathered r, M^-1, d + ess flags + d (writer) + patch
            // outputs (+ x read and written under the x-fold); update: r, M^-1, ess, r write + patches
            const double S = brick_patch_side(c), SZ = brick_patch_side_z(c);
            const double patches = 8.0 * S * S * SZ * (double)brick_count(c);
            const bool xf = c->cg_xfold != 0;
            *bytes = k == CDFEM_K_APPLY ? 8.0 * c->ncomp * ne + 33.0 * nl + patches + (xf ? 16.0 * nl : 0.0)
                                        : (xf ? 25.0 : 49.0) * nl + patches;
            return CDFEM_OK;
        }
        if (use_brick(c)) {
            // CG-mode brick kernels (what the Krylov loop launches); see DESIGN.md section 4
            const int64_t s1 = (int64_t)kBrick * c->p;
            int64_t nface_dofs = 0;
            for (int64_t z = 0; z < c->Lz; ++z)
                for (int64_t y = 0; y < c->Ly; ++y) {
                    if (z % s1 == 0 || y % s1 == 0) { nface_dofs += c->Lx; continue; }
                    nface_dofs += (c->Lx - 1) / s1 + 1;
                }
            const double nf = (double)nface_dofs;
            const double S = kBrick * c->p + 1.0;
            const double patches = 8.0 * S * S * S * (double)c->nblk;  // the CG apply's patch outputs
            // x-fold (cg_xfold, Kronecker form): x += alpha d moves from the update into the apply
            const bool xf = c->cg_xfold != 0 && pa_af(c) == 2;
            switch (k) {
            case CDFEM_K_APPLY:   // qdata (or per-element affine factors) + gathered r, M^-1, d + ess
                                  // flags + d (each dof by its one writer brick) + patch outputs
                                  // (+ x read and written by its writer brick under the x-fold)
                // (pa_uniform: one element matrix, 14 x 64 operand doubles, instead of the factor stream)
                *bytes = (uniform_elem(c) ? 8.0 * 14 * 64 : 8.0 * c->ncomp * (c->d_qaff ? 1.0 : nq) * ne) + 24.0 * nl +
                         1.0 * nl + 8.0 * nl + patches + (xf ? 16.0 * nl : 0.0);
                return CDFEM_OK;
            case CDFEM_K_E2L:     // the Mult's row sums: the patch buffer + ess flags + y (brick_mult_pb,
                                  // Kronecker form), or face partials + x, ess, y of the face dofs
                *bytes = (c->brick_mult_pb && pa_af(c) == 2) ? patches + 9.0 * nl
                                                             : 8.0 * c->nface * (double)c->nblk + 25.0 * nf;
                return CDFEM_OK;
            case CDFEM_K_UPDATE:  // x, d, r, M^-1 read, ess, x, r write + the patch outputs (each once);
                                  // x-fold: r, M^-1, ess and r write only
                *bytes = (xf ? 25.0 : 49.0) * nl + patches;
                return CDFEM_OK;
            default: throw ArgError("kernel not launched on the brick path");
            }
        }
        // the 3D applies on affine factors read one factor set per element (the 2D apply streams)
        const double nqs = (c->qlay == 1 ? tile_affine(c) : (c->dim == 3 && c->d_qaff != nullptr)) ? 1.0 : nq;
        switch (k) {
        case CDFEM_K_APPLY:
            if (c->epencil)  // lattice gather: x + ess flags (each L-dof once) + qdata + E-vector write
                *bytes = 9.0 * nl + 8.0 * c->ncomp * nqs * ne + 8.0 * nd * ne +
                         (tile_dfold_ok(c) ? 16.0 * nl : 0.0);  // CG apply with the direction fold:
                                                                // + d_old gather, + d store
            else             // x gather (each L-dof once) + qdata stream + element map + E-vector write
                *bytes = 8.0 * nl + 8.0 * c->ncomp * nqs * ne + 4.0 * nd * ne + 8.0 * nd * ne;
            break;
        case CDFEM_K_E2L:
            if (c->epencil)  // E-vector read + ess flags + y write + x read (constraint / dot)
                *bytes = 8.0 * nd * ne + 1.0 * nl + 8.0 * nl + 8.0 * nl;
            else             // E-vector read + positions + offsets + y write + x read (constraint / dot)
                *bytes = 8.0 * nd * ne + 4.0 * nd * ne + 4.0 * nl + 8.0 * nl + 8.0 * nl;
            break;
        case CDFEM_K_UPDATE: *bytes = 8.0 * nl * 8; break;     // x,d,r,z,dinv read; x,r,z write
        case CDFEM_K_DIRECTION: *bytes = 8.0 * nl * 3; break;  // z,d read; d write
        default: throw ArgError("bad kernel id");
        }
        return CDFEM_OK;
    });
}

}  // extern "C"
