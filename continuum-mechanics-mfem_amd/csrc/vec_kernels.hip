// vec_kernels.hip — E->L summation, Krylov vector kernels and deterministic reductions.
//
// The CG loop (MFEM CGSolver::Mult semantics, as the reference pins them by use at
// mesh_recession_handler.cpp:270-276) runs entirely stream-ordered on the device: scalars live in
// a KrylovState in HBM, every reduction is a fixed-grid block reduction whose LAST arriving block
// (agent-scope release/acquire, MI355X_MICROARCH.md "Valid forms") sums the partials in index
// order, so results are bitwise reproducible run to run and independent of dispatch/XCD placement.
// Kernels queued after convergence see state->done and exit at entry, so the host polls the state
// only every `check_every` iterations.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "cdfem_internal.hpp"
#include "pa_core.hpp"
#include "reduce.hpp"

namespace cdfem {

// ------------------------------------------------------------------------------------------------
// E->L: y[i] = sum of Ye over the (element, local dof) pairs of dof i (ascending element order).
// constrained: y[ess] = x[ess] (ConstrainedOperator, DIAG_ONE).  cg_mode: also den = (x, y),
// last block: MFEM CG "den" step (alpha = betanom / den, nom = betanom).
// ------------------------------------------------------------------------------------------------
template <bool CON, bool CG>
__global__ void __launch_bounds__(kRedThreads)
k_e2l(const int32_t *__restrict__ off, const int32_t *__restrict__ pos,
      const uint8_t *__restrict__ ess, const double *__restrict__ Ye, const double *__restrict__ x,
      double *__restrict__ y, int64_t nl, double *__restrict__ part, KrylovState *__restrict__ st)
{
    __shared__ double sh[kRedThreads / 64];
    if (CG && st->done) return;
    double acc = 0.0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += stride) {
        double v;
        if (CON && ess[i]) {
            v = x[i];
        } else {
            v = 0.0;
            const int k1 = off[i + 1];
            for (int k = off[i]; k < k1; ++k) v += Ye[pos[k]];
        }
        y[i] = v;
        if (CG) acc += v * x[i];
    }
    if (!CG) return;
    store_partial(block_sum(acc, sh), part);
}

// ------------------------------------------------------------------------------------------------
// E->L on a structured box with the pencil E-vector (3D, p >= 3, ho_eidx): the (element, local
// dof) pairs of a dof follow from its lattice coordinates, so no position arrays are read, and the
// contributions to consecutive dofs of an x-row are consecutive E-vector entries (coalesced).  Per axis a
// lattice coordinate g lies in one element (interior) or two (element boundary); the pairs are
// visited z-outer / x-inner = ascending element index, the order of the generic k_e2l, so both
// give bitwise-identical sums.
// ------------------------------------------------------------------------------------------------
struct BoxE2L {
    FastDiv fLx, fLxy;
    uint32_t Lx, Ly, nx, ny, nz;
};

template <int P>
__device__ __forceinline__ int axis_pairs(uint32_t g, uint32_t n, int *el, int *lo)
{
    const int e = (int)(g / P), l = (int)(g % P);
    if (l != 0) {
        el[0] = e;
        lo[0] = l;
        return 1;
    }
    int k = 0;
    if (e > 0) {
        el[k] = e - 1;
        lo[k++] = P;
    }
    if (e < (int)n) {
        el[k] = e;
        lo[k++] = 0;
    }
    return k;
}

template <bool CON, bool CG, int P>
__global__ void __launch_bounds__(kRedThreads)
k_e2l_box(const BoxE2L bx, const uint8_t *__restrict__ ess, const double *__restrict__ Ye,
          const double *__restrict__ x, double *__restrict__ y, int64_t nl, double *__restrict__ part,
          KrylovState *__restrict__ st)
{
    // one wave per x-row (gy, gz) of the dof lattice (grid-stride over rows): the y / z element
    // pairs are uniform across the wave, lanes run along x, and the row's contributions are one
    // contiguous run of the pencil E-vector (entries gx + ex - 1 and gx + ex, ex = gx / P)
    constexpr int D1 = P + 1;
    __shared__ double sh[kRedThreads / 64];
    if (CG && st->done) return;
    double acc = 0.0;
    const int lane = threadIdx.x & 63;
    const uint32_t rows = bx.Ly * (uint32_t)(nl / ((int64_t)bx.Lx * bx.Ly));
    const uint32_t ew = bx.nx * D1;  // E-vector row length
    for (uint32_t r = blockIdx.x * (kRedThreads / 64) + (threadIdx.x >> 6); r < rows;
         r += gridDim.x * (kRedThreads / 64)) {
        const uint32_t gz = r / bx.Ly, gy = r - gz * bx.Ly;
        int ey[2], ly[2], ez[2], lz[2];
        const int nyp = axis_pairs<P>(gy, bx.ny, ey, ly);
        const int nzp = axis_pairs<P>(gz, bx.nz, ez, lz);
        int64_t erow[4];
        int ne_rows = 0;
        for (int a = 0; a < nzp; ++a)
            for (int b = 0; b < nyp; ++b)
                erow[ne_rows++] = (((int64_t)(ez[a] * D1 + lz[a]) * bx.ny + ey[b]) * D1 + ly[b]) * ew;
        for (int k = ne_rows; k < 4; ++k) erow[k] = erow[0];
        const int64_t lrow = (int64_t)r * bx.Lx;
#pragma unroll 2
        for (uint32_t gx = lane; gx < bx.Lx; gx += 64) {
            const uint32_t ex = gx / P, lx = gx - ex * P;
            const bool left = lx == 0 && ex > 0, right = lx != 0 || ex < bx.nx;
            const int64_t i = lrow + gx;
            // every load issued before the sums (clamped addresses): up to 8 E-vector entries,
            // the essential flag and x in flight together
            // (an absent neighbour reads the present entry instead: no address leaves the row)
            const int64_t cl = left ? -1 : 0, cr = right ? 0 : -1;
            double el[4], er[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const double *e0 = Ye + erow[k] + gx + ex;
                el[k] = e0[cl];
                er[k] = e0[cr];
            }
            const bool is_ess = CON && ess[i];
            const double xi = (CON || CG) ? x[i] : 0.0;
            double v = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (k < ne_rows) {
                    if (left) v += el[k];
                    if (right) v += er[k];
                }
            }
            if (is_ess) v = xi;
            y[i] = v;
            if (CG) acc += v * xi;
        }
    }
    if (!CG) return;
    store_partial(block_sum(acc, sh), part);
}

// The fused E->L + CG update (CG mode with the den already known from the apply,
// k_apply3d_tile<DEN>): the E->L sum q_i is consumed in place instead of being stored,
//   x_i += alpha d_i, r_i -= alpha q_i, z_i = M^-1 r_i, partial (r, z).
// The dofs are taken in flat lattice order: a wave covers 64 * kFlatU consecutive dofs (row-
// crossing) and every lane derives its own (gx, gy, gz) and element pairs, so no lane idles at the
// end of an x-row (one wave per 513-dof row used 8.02 of its 9 passes: 1948 -> 1837 us per update
// at C3, profiles/r03/ab_c3_e2l_flat.txt).  Pairs visited as in k_e2l_box (bitwise the same sums).
constexpr int kFlatU = 2;
template <int P>
__global__ void __launch_bounds__(kRedThreads)
k_e2l_update_flat(const BoxE2L bx, const uint8_t *__restrict__ ess, const double *__restrict__ Ye,
                  const double *__restrict__ d, double *__restrict__ z, int64_t nl, double *__restrict__ part,
                  const KrylovState *__restrict__ st, double *__restrict__ xs, double *__restrict__ res,
                  const double *__restrict__ dinv)
{
    constexpr int D1 = P + 1;
    __shared__ double sh[kRedThreads / 64];
    if (st->done) return;
    const double alpha = st->alpha;
    const uint32_t ew = bx.nx * D1, Lxy = bx.Lx * bx.Ly;
    double acc = 0.0;
    const int64_t per_block = (int64_t)kRedThreads * kFlatU;
    for (int64_t b0 = (int64_t)blockIdx.x * per_block; b0 < nl; b0 += (int64_t)gridDim.x * per_block) {
        const int64_t w0 = b0 + (int64_t)(threadIdx.x >> 6) * 64 * kFlatU + (threadIdx.x & 63);
#pragma unroll
        for (int u = 0; u < kFlatU; ++u) {
            const int64_t i0 = w0 + 64 * u;
            const bool in = i0 < nl;
            const uint32_t i = (uint32_t)(in ? i0 : nl - 1);
            const uint32_t gz = fdiv(i, bx.fLxy), rem = i - gz * Lxy;
            const uint32_t gy = fdiv(rem, bx.fLx), gx = rem - gy * bx.Lx;
            int ey[2], ly[2], ez[2], lz[2];
            const int nyp = axis_pairs<P>(gy, bx.ny, ey, ly);
            const int nzp = axis_pairs<P>(gz, bx.nz, ez, lz);
            int64_t erow[4];
            int ne_rows = 0;
            for (int a = 0; a < nzp; ++a)
                for (int b = 0; b < nyp; ++b)
                    erow[ne_rows++] = (((int64_t)(ez[a] * D1 + lz[a]) * bx.ny + ey[b]) * D1 + ly[b]) * ew;
            for (int k = ne_rows; k < 4; ++k) erow[k] = erow[0];
            const uint32_t ex = gx / P, lx = gx - ex * P;
            const bool left = lx == 0 && ex > 0, right = lx != 0 || ex < bx.nx;
            const int64_t cl = left ? -1 : 0, cr = right ? 0 : -1;
            double el[4], er[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const double *e0 = Ye + erow[k] + gx + ex;
                el[k] = e0[cl];
                er[k] = e0[cr];
            }
            const bool is_ess = ess[i];
            const double xi = d[i], si = xs[i];
            double ri = res[i];
            const double mi = dinv ? dinv[i] : 1.0;
            double v = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (k < ne_rows) {
                    if (left) v += el[k];
                    if (right) v += er[k];
                }
            }
            if (is_ess) v = xi;
            if (in) {
                __builtin_nontemporal_store(si + alpha * xi, &xs[i]);
                ri -= alpha * v;
                __builtin_nontemporal_store(ri, &res[i]);
                const double zi = mi * ri;
                __builtin_nontemporal_store(zi, &z[i]);
                acc += ri * zi;
            }
        }
    }
    store_partial(block_sum(acc, sh), part);
}

// ------------------------------------------------------------------------------------------------
// CG init: r = B, x = 0, z = M^{-1} r, d = z, nom = (d, r)
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kRedThreads)
k_cg_init(const double *__restrict__ B, double *__restrict__ x, double *__restrict__ r,
          double *__restrict__ z, double *__restrict__ d, const double *__restrict__ dinv, int64_t n,
          int64_t skip_lo, double *__restrict__ part)
{
    __shared__ double sh[kRedThreads / 64];
    double acc = 0.0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const double ri = B[i];
        const double zi = dinv ? dinv[i] * ri : ri;
        r[i] = ri;
        x[i] = 0.0;
        z[i] = zi;
        d[i] = zi;
        if (i >= skip_lo) acc += zi * ri;  // shared plane owned by the rank below
    }
    store_partial(block_sum(acc, sh), part);
}

// MFEM CGSolver initial convergence test on nom = (z, r)
__device__ inline void cg_init_logic(KrylovState *st, double nom, double rel_tol, double abs_tol,
                                     int max_iter)
{
    st->nom = st->nom0 = st->betanom = nom;
    const double r0 = fmax(nom * rel_tol * rel_tol, abs_tol * abs_tol);
    st->r0 = r0;
    st->iter = 1;
    st->max_iter = max_iter;
    st->final_iter = max_iter;
    st->converged = 0;
    st->done = 0;
    st->first_den = 1;  // next den is the initial one
    st->beta = 0.0;
    st->xflush = 0;
    if (nom < 0.0) {             // preconditioner not positive definite
        st->done = 1;
        st->final_iter = 0;
    } else if (nom <= r0) {
        st->done = 1;
        st->converged = 1;
        st->final_iter = 0;
    }
}


// one block: nom = sum of the init partials; MFEM CGSolver initial convergence test
__global__ void __launch_bounds__(1024)
k_cg_init_fin(const double *__restrict__ part, int n, double rel_tol, double abs_tol, int max_iter,
              KrylovState *__restrict__ st)
{
    __shared__ double sh[1024 / 64];
    const double nom = sum_partials(part, n, sh);
    if (threadIdx.x == 0) cg_init_logic(st, nom, rel_tol, abs_tol, max_iter);
}

// multi-rank split: rank-local sum into st->red[slot] (then all-reduce, then a *_step kernel)
__global__ void __launch_bounds__(1024)
k_fin_sum(const double *__restrict__ part, int n, int slot, KrylovState *__restrict__ st)
{
    __shared__ double sh[1024 / 64];
    if (slot != 2 && st->done) return;
    const double v = sum_partials(part, n, sh);
    if (threadIdx.x == 0) st->red[slot] = v;
}

__global__ void k_init_step(double rel_tol, double abs_tol, int max_iter, KrylovState *__restrict__ st)
{
    cg_init_logic(st, st->red[2], rel_tol, abs_tol, max_iter);
}

__global__ void k_den_step(KrylovState *__restrict__ st)
{
    if (!st->done) cg_den_step(st, st->red[0]);
}

__global__ void k_update_step(KrylovState *__restrict__ st)
{
    if (!st->done) cg_update_logic(st, st->red[1]);
}

// one block: den = sum of the partials (Mult kernels), MFEM CG den step
__global__ void __launch_bounds__(1024)
k_cg_den_fin(const double *__restrict__ part, int n, KrylovState *__restrict__ st)
{
    __shared__ double sh[1024 / 64];
    if (st->done) return;
    const double den = sum_partials(part, n, sh);
    if (threadIdx.x == 0) cg_den_step(st, den);
}

// x += alpha d, r -= alpha z, z = M^{-1} r, betanom = (r, z); last block: convergence test
template <bool STORE_Z>
__global__ void __launch_bounds__(kRedThreads)
k_cg_update(double *__restrict__ x, double *__restrict__ r, double *__restrict__ z,
            const double *__restrict__ d, const double *__restrict__ dinv, int64_t n, int64_t skip_lo,
            double *__restrict__ part, KrylovState *__restrict__ st)
{
    __shared__ double sh[kRedThreads / 64];
    if (st->done) return;
    const double alpha = st->alpha;
    double acc = 0.0;
    // 16-byte accesses: pairs (2i, 2i+1); the odd tail element is taken by thread 0 of block 0
    const int64_t n2 = n >> 1;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) {
        double2 xv = reinterpret_cast<const double2 *>(x)[i];
        const double2 dv = reinterpret_cast<const double2 *>(d)[i];
        double2 rv = reinterpret_cast<const double2 *>(r)[i];
        const double2 qv = reinterpret_cast<const double2 *>(z)[i];
        double2 mv = make_double2(1.0, 1.0);
        if (dinv) mv = reinterpret_cast<const double2 *>(dinv)[i];
        xv.x += alpha * dv.x; xv.y += alpha * dv.y;
        rv.x -= alpha * qv.x; rv.y -= alpha * qv.y;
        const double z0 = dinv ? mv.x * rv.x : rv.x, z1 = dinv ? mv.y * rv.y : rv.y;
        reinterpret_cast<double2 *>(x)[i] = xv;
        reinterpret_cast<double2 *>(r)[i] = rv;
        if (STORE_Z) reinterpret_cast<double2 *>(z)[i] = make_double2(z0, z1);
        if (2 * i >= skip_lo) acc += rv.x * z0;  // shared plane owned by the rank below
        if (2 * i + 1 >= skip_lo) acc += rv.y * z1;
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
        const int64_t i = n - 1;
        x[i] += alpha * d[i];
        const double ri = r[i] - alpha * z[i];
        r[i] = ri;
        const double zi = dinv ? dinv[i] * ri : ri;
        if (STORE_Z) z[i] = zi;
        if (i >= skip_lo) acc += ri * zi;
    }
    store_partial(block_sum(acc, sh), part);
}

// one block: betanom = sum of the update partials; MFEM CGSolver convergence test and beta
__global__ void __launch_bounds__(1024)
k_cg_update_fin(const double *__restrict__ part, int n, KrylovState *__restrict__ st)
{
    __shared__ double sh[1024 / 64];
    if (st->done) return;
    // (up to 32 loads per thread in flight: the C3 update leaves 65536 partials; same order as kB 8)
    const double betanom = sum_partials<32>(part, n, sh);
    if (threadIdx.x == 0) cg_update_logic(st, betanom);
}

// x-fold CG, after the loop: the last executed update's x += alpha_m d_m (no apply folded it)
__global__ void __launch_bounds__(kRedThreads)
k_cg_xflush(double *__restrict__ x, const double *__restrict__ d0, const double *__restrict__ d1, int64_t n,
            const KrylovState *__restrict__ st)
{
    if (!st->xflush) return;
    const double *__restrict__ d = ((st->final_iter - 1) & 1) ? d1 : d0;
    const double alpha = st->alpha;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] += alpha * d[i];
}

// d = z + beta d
__global__ void __launch_bounds__(kRedThreads)
k_cg_direction(const double *__restrict__ z, double *__restrict__ d, int64_t n,
               const KrylovState *__restrict__ st)
{
    if (st->done) return;
    const double beta = st->beta;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    // 16-byte pairs; d is streamed out (the next apply gathers it from HBM in any case)
    const int64_t n2 = n >> 1;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) {
        typedef double d2_t __attribute__((ext_vector_type(2)));
        const d2_t zv = reinterpret_cast<const d2_t *>(z)[i];
        const d2_t dv = reinterpret_cast<const d2_t *>(d)[i];
        __builtin_nontemporal_store(zv + beta * dv, reinterpret_cast<d2_t *>(d) + i);
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) d[n - 1] = z[n - 1] + beta * d[n - 1];
}

// ------------------------------------------------------------------------------------------------
// small helpers
// ------------------------------------------------------------------------------------------------
__global__ void k_set_ess(const int32_t *__restrict__ list, int n, double *__restrict__ y,
                          const double *__restrict__ x)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[list[i]] = x[list[i]];
}

__global__ void k_ess_only(const uint8_t *__restrict__ ess, const double *__restrict__ x,
                           double *__restrict__ y, int64_t n)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        y[i] = ess[i] ? x[i] : 0.0;
}

__global__ void k_axpby(double a, const double *__restrict__ x, double b, double *__restrict__ y,
                        int64_t n)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        y[i] = a * x[i] + b * y[i];
}

__global__ void k_dinv(const uint8_t *__restrict__ ess, const double *__restrict__ diag,
                       double *__restrict__ dinv, int64_t n)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        dinv[i] = ess[i] ? 1.0 : 1.0 / diag[i];
}

// deterministic dot over entries [skip_lo, n): partials, then k_dot_fin / k_fin_sum
__global__ void __launch_bounds__(kRedThreads)
k_dot(const double *__restrict__ a, const double *__restrict__ b, int64_t n, int64_t skip_lo,
      double *__restrict__ part)
{
    __shared__ double sh[kRedThreads / 64];
    double acc = 0.0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = skip_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        acc += a[i] * b[i];
    store_partial(block_sum(acc, sh), part);
}

__global__ void __launch_bounds__(1024)
k_dot_fin(const double *__restrict__ part, int n, double *__restrict__ out)
{
    __shared__ double sh[1024 / 64];
    const double s = sum_partials(part, n, sh);
    if (threadIdx.x == 0) *out = s;
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
static inline unsigned red_grid(cdfem_ctx *c, int64_t n)
{
    const int64_t need = (n + kRedThreads - 1) / kRedThreads;
    return (unsigned)(need < c->red_blocks ? (need < 1 ? 1 : need) : c->red_blocks);
}

hipError_t launch_den_fin(cdfem_ctx *c, int nparts)
{
    hipLaunchKernelGGL(k_cg_den_fin, dim3(1), dim3(1024), 0, c->stream, c->d_part, nparts, c->d_state);
    return hipGetLastError();
}

hipError_t launch_cg_xflush(cdfem_ctx *c, double *x, const double *d0, const double *d1)
{
    hipLaunchKernelGGL(k_cg_xflush, dim3(red_grid(c, c->nl)), dim3(kRedThreads), 0, c->stream, x, d0, d1, c->nl,
                       c->d_state);
    return hipGetLastError();
}

hipError_t launch_update_fin(cdfem_ctx *c, int nparts, int64_t off)
{
    hipLaunchKernelGGL(k_cg_update_fin, dim3(1), dim3(1024), 0, c->stream, c->d_part + off, nparts, c->d_state);
    return hipGetLastError();
}

static BoxE2L box_e2l(const cdfem_ctx *c)
{
    BoxE2L bx;
    bx.Lx = (uint32_t)c->Lx;
    bx.Ly = (uint32_t)c->Ly;
    bx.nx = (uint32_t)c->sx;
    bx.ny = (uint32_t)c->sy;
    bx.nz = (uint32_t)c->sz;
    bx.fLx = make_fastdiv(bx.Lx);
    bx.fLxy = make_fastdiv(bx.Lx * bx.Ly);
    return bx;
}

static dim3 box_grid(const cdfem_ctx *c) { return dim3((unsigned)std::min<int64_t>((c->Ly * c->Lz + 3) / 4, 65536)); }

bool e2l_box_ok(const cdfem_ctx *c)
{
    return c->structured && c->qlay == 1 && c->nl < ((int64_t)1 << 32) && (c->p == 3 || c->p == 4);
}

// grid partials in[0..n) -> part[0..kDenStage) (fixed ranges, fixed order), then the den step
__global__ void __launch_bounds__(kRedThreads)
k_part_reduce(const double *__restrict__ in, int64_t n, double *__restrict__ part, const KrylovState *__restrict__ st)
{
    __shared__ double sh[kRedThreads / 64];
    if (st->done) return;
    const int64_t chunk = (n + gridDim.x - 1) / gridDim.x, b0 = (int64_t)blockIdx.x * chunk;
    const int64_t b1 = b0 + chunk < n ? b0 + chunk : n;
    double v = 0.0;
    for (int64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) v += in[i];
    store_partial(block_sum(v, sh), part);
}

constexpr int kDenStage = 256;

// several ranks: the same first stage, then the rank-local sum into the state's den slot (all-reduced next)
hipError_t launch_den_local_from_partials(cdfem_ctx *c, const double *in, int64_t n)
{
    hipLaunchKernelGGL(k_part_reduce, dim3(kDenStage), dim3(kRedThreads), 0, c->stream, in, n, c->d_part,
                       (const KrylovState *)c->d_state);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_fin_sum(c, kDenStage, 0);
}

hipError_t launch_den_from_partials(cdfem_ctx *c, const double *in, int64_t n)
{
    hipLaunchKernelGGL(k_part_reduce, dim3(kDenStage), dim3(kRedThreads), 0, c->stream, in, n, c->d_part,
                       (const KrylovState *)c->d_state);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_den_fin(c, kDenStage);
}

template <int P>
static hipError_t launch_e2l_update_p(cdfem_ctx *c, const double *Ye, const double *d, double *x, double *r,
                                      double *z, const double *dinv)
{
    dim3 g;
    const dim3 b(kRedThreads);
    const int64_t per_block = (int64_t)kRedThreads * kFlatU;
    g = dim3((unsigned)std::min<int64_t>((c->nl + per_block - 1) / per_block, 65536));
    hipLaunchKernelGGL((k_e2l_update_flat<P>), g, b, 0, c->stream, box_e2l(c), c->d_ess, Ye, d, z, c->nl,
                       c->d_part, c->d_state, x, r, dinv);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_cg_update_fin, dim3(1), dim3(1024), 0, c->stream, c->d_part, (int)g.x, c->d_state);
    return hipGetLastError();
}

// fused E->L sum + CG update (single rank, den already stepped): x += alpha d, r -= alpha q,
// z = M^-1 r, betanom and the MFEM convergence test
hipError_t launch_e2l_cg_update(cdfem_ctx *c, const double *Ye, const double *d, double *x, double *r, double *z,
                                const double *dinv)
{
    if (!e2l_box_ok(c)) return hipErrorInvalidValue;
    if (c->p == 3) return launch_e2l_update_p<3>(c, Ye, d, x, r, z, dinv);
    return launch_e2l_update_p<4>(c, Ye, d, x, r, z, dinv);
}

template <int P>
static hipError_t launch_e2l_box(cdfem_ctx *c, const double *Ye, const double *x, double *y, bool con, int cg_mode)
{
    const dim3 g = box_grid(c), b(kRedThreads);
    const BoxE2L bx = box_e2l(c);
    if (cg_mode) {
        hipLaunchKernelGGL((k_e2l_box<true, true, P>), g, b, 0, c->stream, bx, c->d_ess, Ye, x, y, c->nl, c->d_part,
                           c->d_state);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        return launch_den_fin(c, (int)g.x);
    }
    if (con)
        hipLaunchKernelGGL((k_e2l_box<true, false, P>), g, b, 0, c->stream, bx, c->d_ess, Ye, x, y, c->nl, c->d_part,
                           c->d_state);
    else
        hipLaunchKernelGGL((k_e2l_box<false, false, P>), g, b, 0, c->stream, bx, c->d_ess, Ye, x, y, c->nl,
                           c->d_part, c->d_state);
    return hipGetLastError();
}

hipError_t launch_e2l(cdfem_ctx *c, const double *Ye, const double *x, double *y, bool con,
                      int cg_mode)
{
    if (e2l_box_ok(c)) return c->p == 3 ? launch_e2l_box<3>(c, Ye, x, y, con, cg_mode)
                                        : launch_e2l_box<4>(c, Ye, x, y, con, cg_mode);
    const dim3 g(red_grid(c, c->nl)), b(kRedThreads);
    if (cg_mode) {
        hipLaunchKernelGGL((k_e2l<true, true>), g, b, 0, c->stream, c->d_e2l_off, c->d_e2l_pos,
                           c->d_ess, Ye, x, y, c->nl, c->d_part, c->d_state);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        return launch_den_fin(c, (int)g.x);
    }
    else if (con)
        hipLaunchKernelGGL((k_e2l<true, false>), g, b, 0, c->stream, c->d_e2l_off, c->d_e2l_pos,
                           c->d_ess, Ye, x, y, c->nl, c->d_part, c->d_state);
    else
        hipLaunchKernelGGL((k_e2l<false, false>), g, b, 0, c->stream, c->d_e2l_off, c->d_e2l_pos,
                           c->d_ess, Ye, x, y, c->nl, c->d_part, c->d_state);
    return hipGetLastError();
}

hipError_t launch_set_ess(cdfem_ctx *c, double *y, const double *x)
{
    if (c->n_ess == 0) return hipSuccess;
    hipLaunchKernelGGL(k_set_ess, dim3((c->n_ess + 255) / 256), dim3(256), 0, c->stream,
                       c->d_ess_list, c->n_ess, y, x);
    return hipGetLastError();
}

hipError_t launch_mask_ess(cdfem_ctx *c, const double *x, double *y)
{
    hipLaunchKernelGGL(k_ess_only, dim3(red_grid(c, c->nl)), dim3(kRedThreads), 0, c->stream,
                       c->d_ess, x, y, c->nl);
    return hipGetLastError();
}

hipError_t launch_axpby(cdfem_ctx *c, double a, const double *x, double b, double *y)
{
    hipLaunchKernelGGL(k_axpby, dim3(red_grid(c, c->nl)), dim3(kRedThreads), 0, c->stream, a, x, b,
                       y, c->nl);
    return hipGetLastError();
}

hipError_t launch_axpby_n(cdfem_ctx *c, int64_t n, double a, const double *x, double b, double *y)
{
    hipLaunchKernelGGL(k_axpby, dim3(red_grid(c, n)), dim3(kRedThreads), 0, c->stream, a, x, b, y, n);
    return hipGetLastError();
}

hipError_t launch_dinv(cdfem_ctx *c, const double *diag, double *dinv)
{
    hipLaunchKernelGGL(k_dinv, dim3(red_grid(c, c->nl)), dim3(kRedThreads), 0, c->stream, c->d_ess,
                       diag, dinv, c->nl);
    return hipGetLastError();
}

hipError_t launch_cg_init(cdfem_ctx *c, const double *B, double *x, double *r, double *z, double *d,
                          const double *dinv, double rel_tol, double abs_tol, int max_iter)
{
    const unsigned g = red_grid(c, c->nl);
    hipLaunchKernelGGL(k_cg_init, dim3(g), dim3(kRedThreads), 0, c->stream, B, x, r, z, d, dinv, c->nl,
                       (int64_t)0, c->d_part);
    hipLaunchKernelGGL(k_cg_init_fin, dim3(1), dim3(1024), 0, c->stream, c->d_part, (int)g, rel_tol,
                       abs_tol, max_iter, c->d_state);
    return hipGetLastError();
}

hipError_t launch_cg_init_nofin(cdfem_ctx *c, const double *B, double *x, double *r, double *z, double *d,
                                const double *dinv)
{
    const unsigned g = red_grid(c, c->nl);
    const int64_t skip = c->skip_lo;
    hipLaunchKernelGGL(k_cg_init, dim3(g), dim3(kRedThreads), 0, c->stream, B, x, r, z, d, dinv, c->nl,
                       skip, c->d_part);
    return launch_fin_sum(c, (int)g, 2);
}

hipError_t launch_fin_sum(cdfem_ctx *c, int nparts, int slot)
{
    hipLaunchKernelGGL(k_fin_sum, dim3(1), dim3(1024), 0, c->stream, c->d_part, nparts, slot, c->d_state);
    return hipGetLastError();
}

hipError_t launch_init_step(cdfem_ctx *c, double rel_tol, double abs_tol, int max_iter)
{
    hipLaunchKernelGGL(k_init_step, dim3(1), dim3(1), 0, c->stream, rel_tol, abs_tol, max_iter, c->d_state);
    return hipGetLastError();
}

hipError_t launch_den_step(cdfem_ctx *c)
{
    hipLaunchKernelGGL(k_den_step, dim3(1), dim3(1), 0, c->stream, c->d_state);
    return hipGetLastError();
}

hipError_t launch_update_step(cdfem_ctx *c)
{
    hipLaunchKernelGGL(k_update_step, dim3(1), dim3(1), 0, c->stream, c->d_state);
    return hipGetLastError();
}

hipError_t launch_cg_update(cdfem_ctx *c, double *x, double *r, double *z, const double *d,
                            const double *dinv)
{
    const unsigned g = red_grid(c, c->nl);
    hipLaunchKernelGGL(k_cg_update<true>, dim3(g), dim3(kRedThreads), 0, c->stream, x, r, z, d, dinv,
                       c->nl, c->skip_lo, c->d_part, c->d_state);
    if (multi_rank(c)) return launch_fin_sum(c, (int)g, 1);  // all-reduced, then the update step
    hipLaunchKernelGGL(k_cg_update_fin, dim3(1), dim3(1024), 0, c->stream, c->d_part, (int)g, c->d_state);
    return hipGetLastError();
}

hipError_t launch_cg_update_noz(cdfem_ctx *c, double *x, double *r, const double *q, const double *d,
                                const double *dinv)
{
    // k_cg_update reads "z" as A d: pass q there; the z output is not written
    const unsigned g = red_grid(c, c->nl);
    hipLaunchKernelGGL(k_cg_update<false>, dim3(g), dim3(kRedThreads), 0, c->stream, x, r,
                       const_cast<double *>(q), d, dinv, c->nl, (int64_t)0, c->d_part, c->d_state);
    hipLaunchKernelGGL(k_cg_update_fin, dim3(1), dim3(1024), 0, c->stream, c->d_part, (int)g, c->d_state);
    return hipGetLastError();
}

__global__ void k_zero(double *__restrict__ y, int64_t n)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = 0.0;
}

hipError_t launch_zero(cdfem_ctx *c, double *y)
{
    hipLaunchKernelGGL(k_zero, dim3(red_grid(c, c->nl)), dim3(kRedThreads), 0, c->stream, y, c->nl);
    return hipGetLastError();
}

hipError_t launch_cg_direction(cdfem_ctx *c, const double *z, double *d)
{
    hipLaunchKernelGGL(k_cg_direction, dim3(red_grid(c, c->nl)), dim3(kRedThreads), 0, c->stream, z,
                       d, c->nl, c->d_state);
    return hipGetLastError();
}

hipError_t launch_dot(cdfem_ctx *c, const double *a, const double *b, double *d_out)
{
    const unsigned g = red_grid(c, c->nl);
    hipLaunchKernelGGL(k_dot, dim3(g), dim3(kRedThreads), 0, c->stream, a, b, c->nl, (int64_t)0, c->d_part);
    hipLaunchKernelGGL(k_dot_fin, dim3(1), dim3(1024), 0, c->stream, c->d_part, (int)g, d_out);
    return hipGetLastError();
}

hipError_t launch_den_local(cdfem_ctx *c, const double *d, const double *q)
{
    const unsigned g = red_grid(c, c->nl);
    const int64_t skip = c->skip_lo;
    hipLaunchKernelGGL(k_dot, dim3(g), dim3(kRedThreads), 0, c->stream, d, q, c->nl, skip, c->d_part);
    return launch_fin_sum(c, (int)g, 0);
}

}  // namespace cdfem
