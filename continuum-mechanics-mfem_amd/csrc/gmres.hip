// gmres.hip — restarted GMRES(m) with left Jacobi preconditioning, device-resident.
//
// Semantics: PETSc KSPGMRES as the reference configures it (Input/petsc.opts:2-6 "-ksp_type gmres
// -pc_type jacobi -ksp_rtol 1e-10 -ksp_atol 1e-12", solver built at
// linear_convection_diffusion_2D.cpp:364-374): restart m (PETSc default 30), LEFT preconditioning,
// classical Gram-Schmidt without refinement, Givens rotations, convergence on the preconditioned
// residual norm  res <= max(rtol * res0, atol)  (KSPConvergedDefault), zero initial guess.
// The CPU restatement is oracle/cdfem_oracle.c:orc_gmres.
//
// MI355X layout: the Krylov basis V is (m + 1) L-vectors contiguous in HBM.  Basis vectors are
// stored UNNORMALISED with a device scalar s_i (v_i = s_i * V_i), which removes the separate
// normalisation pass.  Per inner step j (besides the operator apply):
//   pass 1  w = s_j M^{-1} (A V_j), h_i = s_i (w, V_i) for all i <= j   (reads w once, V_0..j once)
//   fin     h_i summed over blocks in fixed order -> H[:, j]
//   pass 2  V_{j+1} = w - sum_i h_i s_i V_i and the partials of |V_{j+1}|^2
//   fin     h_{j+1,j}, Givens rotation, residual estimate, cycle control flags
// Bytes per step = 8 N (2 j + 7) + apply.  All reductions: fixed grid, fixed order (bitwise
// reproducible).  Every kernel checks the cycle_done flag, so steps the host queued beyond the end
// of a cycle exit at entry.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "brick_core.hpp"
#include "cdfem_internal.hpp"
#include "reduce.hpp"

namespace cdfem {

constexpr int kGmEPT = 4;                         // L-vector entries per thread in the pass kernels
constexpr int kGmBatch = 2;                       // projections per load batch in pass 1
constexpr int kGmBatch2 = 4;                      // basis vectors per load batch in pass 2
constexpr int kGmChunk = kRedThreads * kGmEPT;    // entries per block

int gmres_blocks(int64_t n) { return (int)((n + kGmChunk - 1) / kGmChunk); }

// ---- v0 = M^{-1} (b - A x) and partials of |v0|^2 ------------------------------------------------
__global__ void __launch_bounds__(kRedThreads)
k_gm_residual(const double *__restrict__ b, const double *__restrict__ Ax, const double *__restrict__ dinv,
              double *__restrict__ v0, int64_t n, int64_t skip_lo, double *__restrict__ part,
              const GmresState *__restrict__ st)
{
    __shared__ double sh[kRedThreads / 64];
    if (st->done) return;
    const int64_t base = (int64_t)blockIdx.x * kGmChunk + threadIdx.x;
    double acc = 0.0;
#pragma unroll
    for (int e = 0; e < kGmEPT; ++e) {
        const int64_t k = base + (int64_t)e * kRedThreads;
        if (k < n) {
            double r = Ax ? b[k] - Ax[k] : b[k];
            if (dinv) r *= dinv[k];
            v0[k] = r;
            if (k >= skip_lo) acc += r * r;  // shared plane owned by the rank below
        }
    }
    store_partial(block_sum(acc, sh), part);
}

// host poll without a copy kernel: the last scalar kernel of every polled step writes the head of
// the state (kGmPollBytes: cycle_done, done, converged, its, res, j, kk) straight into the
// pinned host slot the host will wait on (hipHostMalloc memory is device-visible).  A D2H
// hipMemcpyAsync of the same 32 bytes cost a 4 us blit kernel per GMRES step.
__device__ inline void post_poll(const GmresState *st, GmresState *poll)
{
    if (!poll) return;
    poll->cycle_done = st->cycle_done;
    poll->done = st->done;
    poll->converged = st->converged;
    poll->its = st->its;
    poll->res = st->res;
    poll->j = st->j;
    poll->kk = st->kk;
    __threadfence_system();
}

// ---- start of a cycle: beta = |v0|, first-cycle tolerance, convergence / max_it test ------------
__global__ void __launch_bounds__(1024)
k_gm_start(const double *__restrict__ part, int nb, GmresState *__restrict__ st, int first, double rtol,
           double atol, int mode, GmresState *__restrict__ poll)
{
    __shared__ double sh[1024 / 64];
    const double sum = mode == 2 ? st->red[0] : sum_partials(part, nb, sh);
    if (threadIdx.x != 0) return;
    if (mode == 1) {  // multi-rank: local sum, all-reduced before the mode-2 launch
        st->red[0] = sum;
        return;
    }
    if (!st->done) {
        const double beta = sqrt(sum);
        st->res = beta;
        if (first) {
            st->ttol = fmax(rtol * beta, atol);
            st->res0 = beta;
        }
        st->cycle_done = 1;
        if (beta <= st->ttol || beta == 0.0) {
            st->converged = 1;
            st->done = 1;
        } else if (st->its >= st->max_it) {
            st->done = 1;
        } else {
            st->s[0] = 1.0 / beta;
            for (int i = 0; i <= st->m; ++i) st->g[i] = 0.0;
            st->g[0] = beta;
            st->j = 0;
            st->kk = 0;
            st->cycle_done = 0;
        }
    }
    post_poll(st, poll);
}

// ---- pass 1: w = s_j M^{-1} A V_j (in place over the apply output), partial (w, V_i), i <= j ----
// The projections are formed BAT at a time: BAT * kGmEPT loads per lane in flight, all
// unconditional (past V_0 the indices repeat V_0: cache hits whose sums are
// dropped).  Each wave parks its wave sums in LDS, so the whole step needs ONE barrier before the
// block sums.  Measured at C4 (orthogonalisation per step): one barrier per batch of 8, 93.9 us;
// one barrier in all, batches of 8 / 4 / 2 / 1: 85.7 / 83.2 / 82.6 / 82.1 us.
// S > 0 (gm_pb, GmPatchSrc): A_c V_j from the structured Mult's patch buffer (patch_sum8, S = 4p + 1)
// instead of w; w is still written (pass 2 reads it)
template <int BAT, int EPT, int S = 0>
__global__ void __launch_bounds__(kRedThreads)
k_gm_pass1(double *__restrict__ w, const double *__restrict__ dinv, const double *__restrict__ V, int64_t n,
           int64_t ldv, int64_t skip_lo, double *__restrict__ part, int nb, const GmresState *__restrict__ st,
           const GmPatchSrc ps)
{
    __shared__ double sh[kGmMaxRestart + 1][kRedThreads / 64];
    if (st->cycle_done) return;
    const int j = st->j;
    const double sj = st->s[j];
    const int64_t base = (int64_t)blockIdx.x * (kRedThreads * EPT) + threadIdx.x;
    const int lane = threadIdx.x & 63, wv_id = threadIdx.x >> 6;
    double wv[EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        const int64_t k = base + (int64_t)e * kRedThreads;
        double v = 0.0;
        if (k < n) {
            double y;
            if constexpr (S == 0) {
                y = w[k];
            } else {  // (n < 2^28 on the brick path: brick_fits)
                const uint32_t gid = (uint32_t)k, plane = (uint32_t)(ps.g.Lx * ps.g.Ly);
                const uint32_t gz = fdiv(gid, ps.fdxy), rem = gid - gz * plane, gy = fdiv(rem, ps.fdx);
                const uint32_t gx = rem - gy * (uint32_t)ps.g.Lx;
                const auto bp = brsrc(ps.pb, 8u * (uint32_t)ps.g.nbx * ps.g.nby * ps.g.nbz * (S * S * S));
                y = patch_sum8<S>(bp, ps.g, (int)gx, (int)gy, (int)gz);
                if (ps.ess[k]) y = ps.x[k];  // A_c: the identity row
            }
            v = sj * y;
            if (dinv) v *= dinv[k];
            w[k] = v;
        }
        wv[e] = k >= skip_lo ? v : 0.0;  // projections: owned entries only
    }
    // the basis is read from V_j DOWN to V_0 (each projection is its own sum, so the order of the
    // vectors changes nothing): V_0, V_1, ... are then the most recently read lines when pass 2 reads
    // them again in ascending order, so the first ~256 MB of pass 2's basis come from the MALL
    // (Infinity Cache) instead of HBM; with both passes ascending every pass-2 read missed (an LRU
    // scan of more than the cache)
#pragma unroll 1
    for (int r0 = 0; r0 <= j; r0 += BAT) {
        double vv[BAT][EPT];
#pragma unroll
        for (int b = 0; b < BAT; ++b) {
            const double *vi = V + (int64_t)(r0 + b <= j ? j - (r0 + b) : 0) * ldv;
#pragma unroll
            for (int e = 0; e < EPT; ++e) {
                const int64_t k = base + (int64_t)e * kRedThreads;
                vv[b][e] = k < n ? vi[k] : 0.0;
            }
        }
#pragma unroll
        for (int b = 0; b < BAT; ++b) {
            double a = 0.0;
#pragma unroll
            for (int e = 0; e < EPT; ++e) a += wv[e] * vv[b][e];
            const double t = wave_sum(a);
            if (lane == 0 && r0 + b <= j) sh[j - (r0 + b)][wv_id] = t;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i <= j; i += blockDim.x) {
        double t = 0.0;
#pragma unroll
        for (int q = 0; q < kRedThreads / 64; ++q) t += sh[i][q];
        part[(int64_t)i * nb + blockIdx.x] = t;
    }
}

// ---- H[i][j] = s_i * sum_b part[i][b], one wave per i (fixed order) ------------------------------
__global__ void __launch_bounds__(1024)
k_gm_dots_fin(const double *__restrict__ part, int nb, GmresState *__restrict__ st, int mode)
{
    if (st->cycle_done) return;
    const int j = st->j;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (mode == 2) {  // multi-rank: H[i][j] from the all-reduced sums
        if (threadIdx.x <= j) st->H[threadIdx.x * kGmMaxRestart + j] = st->s[threadIdx.x] * st->red[threadIdx.x];
        return;
    }
    for (int i = wv; i <= st->m; i += 16) {
        // 8 independent partial loads per lane in flight, combined in a fixed order
        double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        if (i <= j) {
            const double *pi = part + (int64_t)i * nb;
            int b = lane;
            for (; b + 7 * 64 < nb; b += 8 * 64) {
#pragma unroll
                for (int u = 0; u < 8; ++u) a[u] += pi[b + u * 64];
            }
            for (int u = 0; b < nb; b += 64, ++u) a[u] += pi[b];
        }
        double v = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
        v = wave_sum(v);
        if (lane != 0) continue;
        if (mode == 1) st->red[i] = v;  // multi-rank: local sums (zero past j), all-reduced next
        else if (i <= j) st->H[i * kGmMaxRestart + j] = st->s[i] * v;
    }
}

// ---- H[i][j] = s_i * sum_b part[i][b] (modes 0 / 1 of k_gm_dots_fin), one block per i ------------
// Every projection's partials are summed by a block of its own (fixed order), so the step's
// projections reduce in parallel instead of 16 at a time in one block.
__global__ void __launch_bounds__(kRedThreads)
k_gm_dots_fin_mb(const double *__restrict__ part, int nb, GmresState *__restrict__ st, int mode)
{
    __shared__ double sh[kRedThreads / 64];
    if (st->cycle_done) return;
    const int j = st->j, i = blockIdx.x;  // grid = m + 1
    if (i > j) {
        if (mode == 1 && threadIdx.x == 0) st->red[i] = 0.0;  // multi-rank: zero past j
        return;
    }
    const double *pi = part + (int64_t)i * nb;
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    int b = threadIdx.x;
    for (; b + 3 * kRedThreads < nb; b += 4 * kRedThreads) {
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] += pi[b + u * kRedThreads];
    }
    for (int u = 0; b < nb; b += kRedThreads, ++u) a[u] += pi[b];
    const double v = block_sum((a[0] + a[1]) + (a[2] + a[3]), sh);
    if (threadIdx.x != 0) return;
    if (mode == 1) st->red[i] = v;
    else st->H[i * kGmMaxRestart + j] = st->s[i] * v;
}

// ---- pass 2: V_{j+1} = w - sum_i H[i][j] s_i V_i, partials of |V_{j+1}|^2 ------------------------
// Pass 1's treatment: the coefficients H[i][j] s_i are staged once per block in LDS (one global
// load per i per block instead of one per i per wave), and the basis vectors are read BAT at a time
// with every load unconditional (entry indices clamped to n - 1, basis indices clamped to j with a
// zero coefficient), so BAT * kGmEPT loads per lane are in flight before the first FMA.  The
// subtractions keep the ascending-i order of the one-at-a-time loop (bitwise the same V_{j+1}).
template <int BAT, int EPT>
__global__ void __launch_bounds__(kRedThreads)
k_gm_pass2(const double *__restrict__ w, double *__restrict__ V, int64_t n, int64_t ldv, int64_t skip_lo,
           double *__restrict__ part, const GmresState *__restrict__ st)
{
    __shared__ double sh[kRedThreads / 64];
    __shared__ double coef[kGmMaxRestart + BAT];
    if (st->cycle_done) return;
    const int j = st->j;
    for (int i = threadIdx.x; i < kGmMaxRestart + BAT; i += blockDim.x)
        coef[i] = i <= j ? st->H[i * kGmMaxRestart + j] * st->s[i] : 0.0;
    const int64_t base = (int64_t)blockIdx.x * (kRedThreads * EPT) + threadIdx.x;
    int64_t kc[EPT];
    double acc[EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        const int64_t k = base + (int64_t)e * kRedThreads;
        kc[e] = k < n ? k : n - 1;
        acc[e] = w[kc[e]];
    }
    __syncthreads();
#pragma unroll 1
    for (int i0 = 0; i0 <= j; i0 += BAT) {
        double vv[BAT][EPT];
#pragma unroll
        for (int b = 0; b < BAT; ++b) {
            const double *vi = V + (int64_t)(i0 + b <= j ? i0 + b : j) * ldv;
#pragma unroll
            for (int e = 0; e < EPT; ++e) vv[b][e] = vi[kc[e]];
        }
#pragma unroll
        for (int b = 0; b < BAT; ++b) {
            const double cb = coef[i0 + b];  // 0 past j
#pragma unroll
            for (int e = 0; e < EPT; ++e) acc[e] -= cb * vv[b][e];
        }
    }
    double *vn = V + (int64_t)(j + 1) * ldv;
    double nrm = 0.0;
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
        const int64_t k = base + (int64_t)e * kRedThreads;
        if (k < n) {
            vn[k] = acc[e];
            if (k >= skip_lo) nrm += acc[e] * acc[e];
        }
    }
    store_partial(block_sum(nrm, sh), part);
}

// ---- h_{j+1,j}, Givens rotations, residual estimate, cycle control ------------------------------
__global__ void __launch_bounds__(1024)
k_gm_norm_fin(const double *__restrict__ part, int nb, GmresState *__restrict__ st, int mode,
              GmresState *__restrict__ poll)
{
    constexpr int LD = kGmMaxRestart;
    __shared__ double sh[1024 / 64];
    __shared__ double hc[kGmMaxRestart + 1], cs[kGmMaxRestart], sn[kGmMaxRestart];
    if (st->cycle_done) {  // uniform: every thread reads the same flag before the reduction
        if (threadIdx.x == 0 && mode != 1) post_poll(st, poll);
        return;
    }
    const int j = st->j;
    // the Hessenberg column and the rotations so far, loaded in parallel into LDS: the serial
    // rotation sequence below then runs on LDS instead of dependent global loads
    if ((int)threadIdx.x <= j) hc[threadIdx.x] = st->H[threadIdx.x * LD + j];
    if ((int)threadIdx.x < j) {
        cs[threadIdx.x] = st->cs[threadIdx.x];
        sn[threadIdx.x] = st->sn[threadIdx.x];
    }
    const double sum = mode == 2 ? st->red[0] : sum_partials(part, nb, sh);  // (contains a barrier)
    if (mode == 2) __syncthreads();
    if (threadIdx.x != 0) return;
    if (mode == 1) {  // multi-rank: local sum, all-reduced before the mode-2 launch
        st->red[0] = sum;
        return;
    }
    const double hn = sqrt(sum);
    hc[j + 1] = hn;
    for (int i = 0; i < j; ++i) {
        const double a = hc[i], c2 = hc[i + 1];
        hc[i] = cs[i] * a + sn[i] * c2;
        hc[i + 1] = -sn[i] * a + cs[i] * c2;
    }
    const double a = hc[j], c2 = hc[j + 1];
    const double rr = sqrt(a * a + c2 * c2);
    const double cj = (rr == 0.0) ? 1.0 : a / rr, sj = (rr == 0.0) ? 0.0 : c2 / rr;
    st->cs[j] = cj;
    st->sn[j] = sj;
    hc[j] = rr;
    hc[j + 1] = 0.0;
    for (int i = 0; i <= j + 1; ++i) st->H[i * LD + j] = hc[i];
    const double gj = st->g[j];
    st->g[j + 1] = -sj * gj;
    st->g[j] = cj * gj;
    st->res = fabs(-sj * gj);
    st->kk = j + 1;
    st->its += 1;
    st->s[j + 1] = (hn != 0.0) ? 1.0 / hn : 0.0;
    st->j = j + 1;
    if (hn == 0.0 || st->res <= st->ttol || j + 1 == st->m || st->its >= st->max_it) st->cycle_done = 1;
    post_poll(st, poll);
}

// ---- end of cycle: y = H_k^{-1} g_k (every block, redundantly: k <= 64), x += sum_i y_i s_i V_i --
// cycle end, once: y = H^{-1} g by back substitution (the serial order PETSc's KSPGMRESBuildSoln
// uses), the Hessenberg triangle staged in LDS first, then scaled by the basis scales
__global__ void __launch_bounds__(kRedThreads)
k_gm_solve_y(GmresState *__restrict__ st)
{
    constexpr int LD = kGmMaxRestart;
    __shared__ double h[kGmMaxRestart * kGmMaxRestart];
    __shared__ double g[kGmMaxRestart];
    if (st->done) return;
    const int kk = st->kk;
    for (int t = threadIdx.x; t < kk * kk; t += blockDim.x) {
        const int i = t / kk, l = t - i * kk;
        if (l >= i) h[i * LD + l] = st->H[i * LD + l];
    }
    if ((int)threadIdx.x < kk) g[threadIdx.x] = st->g[threadIdx.x];
    __syncthreads();
    if (threadIdx.x != 0) return;
    // y lives in LDS (a register array with run-time indices would go to scratch); the loads of a
    // row are independent of the chain, so unrolling keeps them in flight ahead of the FMAs
    double *y = g;  // g[i] is read once, before y[i] overwrites it
    for (int i = kk - 1; i >= 0; --i) {
        double acc = g[i];
#pragma unroll 8
        for (int l = i + 1; l < kk; ++l) acc -= h[i * LD + l] * y[l];
        y[i] = acc / h[i * LD + i];
    }
    for (int i = 0; i < kk; ++i) st->y[i] = y[i] * st->s[i];
}

// x += sum_i y_i V_i (y from k_gm_solve_y), 4 basis vectors' loads in flight per batch; each
// entry is summed in ascending i, as before the batching
__global__ void __launch_bounds__(kRedThreads)
k_gm_update(double *__restrict__ x, const double *__restrict__ V, int64_t n, int64_t ldv,
            const GmresState *__restrict__ st)
{
    __shared__ double y[kGmMaxRestart];
    if (st->done) return;
    const int kk = st->kk;
    if ((int)threadIdx.x < kk) y[threadIdx.x] = st->y[threadIdx.x];
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kGmChunk + threadIdx.x;
    double v[kGmEPT];
#pragma unroll
    for (int e = 0; e < kGmEPT; ++e) {
        const int64_t k = base + (int64_t)e * kRedThreads;
        v[e] = k < n ? x[k] : 0.0;
    }
    int i = 0;
    for (; i + 4 <= kk; i += 4) {
        double vv[4][kGmEPT];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int e = 0; e < kGmEPT; ++e) {
                const int64_t k = base + (int64_t)e * kRedThreads;
                vv[u][e] = k < n ? V[(int64_t)(i + u) * ldv + k] : 0.0;
            }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int e = 0; e < kGmEPT; ++e) v[e] += y[i + u] * vv[u][e];
    }
    for (; i < kk; ++i)
#pragma unroll
        for (int e = 0; e < kGmEPT; ++e) {
            const int64_t k = base + (int64_t)e * kRedThreads;
            if (k < n) v[e] += y[i] * V[(int64_t)i * ldv + k];
        }
#pragma unroll
    for (int e = 0; e < kGmEPT; ++e) {
        const int64_t k = base + (int64_t)e * kRedThreads;
        if (k < n) x[k] = v[e];
    }
}

__global__ void k_gm_cycle_end(GmresState *__restrict__ st, GmresState *__restrict__ poll)
{
    if (!st->done) {
        if (st->res <= st->ttol) {
            st->converged = 1;
            st->done = 1;
        } else if (st->its >= st->max_it) {
            st->done = 1;
        }
    }
    post_poll(st, poll);
}

__global__ void k_gm_init(GmresState *__restrict__ st, int m, int max_it)
{
    st->cycle_done = 1;
    st->done = 0;
    st->converged = 0;
    st->its = 0;
    st->j = 0;
    st->kk = 0;
    st->max_it = max_it;
    st->m = m;
    st->res = 0.0;
    st->ttol = 0.0;
    st->res0 = 0.0;
}

// ---- launchers ---------------------------------------------------------------------------------
hipError_t launch_gm_init(cdfem_ctx *c, GmresState *st, int m, int max_it)
{
    hipLaunchKernelGGL(k_gm_init, dim3(1), dim3(1), 0, c->stream, st, m, max_it);
    return hipGetLastError();
}

// multi-rank: partial sums -> local sum (mode 1) -> all-reduce over ranks -> scalar logic (mode 2);
// every rank then runs the same scalar arithmetic on the same sums and takes the same branches
static int64_t owned_from(const cdfem_ctx *c) { return c->skip_lo; }
static double *red_of(GmresState *st) { return st->red; }

hipError_t launch_gm_residual(cdfem_ctx *c, const double *b, const double *Ax, const double *dinv, double *v0,
                              double *part, GmresState *st, bool first, double rtol, double atol, GmresState *poll)
{
    const int nb = gmres_blocks(c->nl);
    const bool mr = multi_rank(c);
    hipLaunchKernelGGL(k_gm_residual, dim3(nb), dim3(kRedThreads), 0, c->stream, b, Ax, dinv, v0,
                       (int64_t)c->nl, owned_from(c), part, st);
    hipLaunchKernelGGL(k_gm_start, dim3(1), dim3(1024), 0, c->stream, part, nb, st, first ? 1 : 0, rtol, atol,
                       mr ? 1 : 0, mr ? nullptr : poll);
    if (mr) {
        comm_allreduce(c, red_of(st), 1);
        hipLaunchKernelGGL(k_gm_start, dim3(1), dim3(1024), 0, c->stream, part, nb, st, first ? 1 : 0, rtol, atol, 2,
                           poll);
    }
    return hipGetLastError();
}

// Entries per thread of the two orthogonalisation passes: the smallest of 4, 5, 6, 8 whose grid is
// resident in one round (blocks <= CUs x resident blocks per CU), so no tail of a few blocks runs
// a second round alone (C2: 2097 blocks of 1024 entries against 2048 resident slots at EPT 4).
static int orth_ept(cdfem_ctx *c)
{
    if (c->gm_ept) return c->gm_ept;                  // set_option("gm_ept")
    if (c->gm_ept_n == c->nl) return c->gm_ept_auto;  // chosen for this size already
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_gm_pass1<kGmBatch, 4, 0>, kRedThreads, 0);
    const int64_t cap = (int64_t)std::max(cus, 1) * std::max(per, 1);
    int ept = 8;
    for (int e : {4, 5, 6, 8})
        if ((c->nl + (int64_t)kRedThreads * e - 1) / ((int64_t)kRedThreads * e) <= cap) {
            ept = e;
            break;
        }
    c->gm_ept_auto = ept;
    c->gm_ept_n = c->nl;
    return ept;
}

template <int EPT>
static void orth_passes(cdfem_ctx *c, double *w, const double *dinv, double *V, int64_t ldv, double *part,
                        GmresState *st, int m, GmresState *poll, const GmPatchSrc *ps)
{
    const int nb = (int)((c->nl + (int64_t)kRedThreads * EPT - 1) / ((int64_t)kRedThreads * EPT));
    const int64_t n = c->nl;
    const bool mr = multi_rank(c);
    const GmPatchSrc src = ps ? *ps : GmPatchSrc{};
#define CDFEM_P1(S_)                                                                                      \
    hipLaunchKernelGGL((k_gm_pass1<kGmBatch, EPT, S_>), dim3(nb), dim3(kRedThreads), 0, c->stream, w, dinv, V, n, \
                       ldv, owned_from(c), part, nb, st, src)
    if (ps && ps->S == 9) CDFEM_P1(9);
    else if (ps && ps->S == 5) CDFEM_P1(5);
    else CDFEM_P1(0);
#undef CDFEM_P1
    hipLaunchKernelGGL(k_gm_dots_fin_mb, dim3(m + 1), dim3(kRedThreads), 0, c->stream, part, nb, st, mr ? 1 : 0);
    if (mr) {
        comm_allreduce(c, red_of(st), m + 1);
        hipLaunchKernelGGL(k_gm_dots_fin, dim3(1), dim3(1024), 0, c->stream, part, nb, st, 2);
    }
    hipLaunchKernelGGL((k_gm_pass2<kGmBatch2, EPT>), dim3(nb), dim3(kRedThreads), 0, c->stream, w, V, n, ldv,
                       owned_from(c), part, st);
    hipLaunchKernelGGL(k_gm_norm_fin, dim3(1), dim3(1024), 0, c->stream, part, nb, st, mr ? 1 : 0,
                       mr ? nullptr : poll);
    if (mr) {
        comm_allreduce(c, red_of(st), 1);
        hipLaunchKernelGGL(k_gm_norm_fin, dim3(1), dim3(1024), 0, c->stream, part, nb, st, 2, poll);
    }
}

hipError_t launch_gm_orth(cdfem_ctx *c, double *w, const double *dinv, double *V, int64_t ldv, double *part,
                          GmresState *st, int m, GmresState *poll, const GmPatchSrc *ps)
{
    if (ps && ps->S != 5 && ps->S != 9) return hipErrorInvalidValue;
    switch (orth_ept(c)) {
    case 5: orth_passes<5>(c, w, dinv, V, ldv, part, st, m, poll, ps); break;
    case 6: orth_passes<6>(c, w, dinv, V, ldv, part, st, m, poll, ps); break;
    case 8: orth_passes<8>(c, w, dinv, V, ldv, part, st, m, poll, ps); break;
    default: orth_passes<4>(c, w, dinv, V, ldv, part, st, m, poll, ps); break;
    }
    return hipGetLastError();
}

hipError_t launch_gm_update(cdfem_ctx *c, double *x, const double *V, int64_t ldv, GmresState *st, GmresState *poll)
{
    const int nb = gmres_blocks(c->nl);
    hipLaunchKernelGGL(k_gm_solve_y, dim3(1), dim3(kRedThreads), 0, c->stream, st);
    hipLaunchKernelGGL(k_gm_update, dim3(nb), dim3(kRedThreads), 0, c->stream, x, V, (int64_t)c->nl, ldv, st);
    hipLaunchKernelGGL(k_gm_cycle_end, dim3(1), dim3(1), 0, c->stream, st, poll);
    return hipGetLastError();
}

}  // namespace cdfem
