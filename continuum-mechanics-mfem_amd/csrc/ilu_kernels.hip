// ilu_kernels.hip — ILU(0) preconditioner for GMRES on the assembled (FA) operator.
//
// Reference: Input/petsc_circle.opts:6-8 ("-pc_type bjacobi -sub_ksp_type preonly -sub_pc_type ilu")
// for linear_convection_diffusion_2D_circle.cpp.  On one rank, block Jacobi has one block, so this is
// PETSc PCILU with zero fill in the natural ordering, no pivoting and no shift, applied on the left
// inside KSPGMRES.  The CPU restatement is oracle/cdfem_oracle.c:orc_ilu0 / orc_ilu_solve.
//
// Factors live in the pattern of the eliminated CSR matrix (unit-lower L and U packed, like the
// oracle).  Both the factorisation and the triangular sweeps are level-scheduled:
//   level_L(i) = 1 + max level_L(k) over k < i in row i      (forward sweep and factorisation)
//   level_U(i) = 1 + max level_U(j) over j > i in row i      (backward sweep)
// One launch per level, one thread per row, each row summed in ascending column order (the
// oracle's order: deterministic, no atomics).  The sweeps of one preconditioner application are a
// fixed sequence of launches on fixed buffers, so they are captured once into a HIP graph and
// replayed (one graph launch per GMRES step instead of 2 x levels kernel launches).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <vector>

#include "cdfem_internal.hpp"

namespace cdfem {

__global__ void __launch_bounds__(256)
k_ilu_factor_level(const int32_t *__restrict__ rp, const int32_t *__restrict__ cols,
                   const int32_t *__restrict__ diag, double *__restrict__ F, const int32_t *__restrict__ rows,
                   int count)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    const int i = rows[t];
    const int e = rp[i + 1];
    for (int pk = rp[i]; pk < e && cols[pk] < i; ++pk) {
        const int k = cols[pk];
        const double lik = F[pk] / F[diag[k]];
        F[pk] = lik;
        int pi = pk + 1, pu = diag[k] + 1;
        const int eu = rp[k + 1];
        while (pi < e && pu < eu) {
            const int ci = cols[pi], cu = cols[pu];
            if (ci < cu) {
                ++pi;
            } else if (ci > cu) {
                ++pu;
            } else {
                F[pi] -= lik * F[pu];
                ++pi;
                ++pu;
            }
        }
    }
}

// forward sweep with the unit lower part: z_i = r_i - sum_{k < i} l_ik z_k
__global__ void __launch_bounds__(256)
k_ilu_lower_level(const int32_t *__restrict__ rp, const int32_t *__restrict__ cols, const double *__restrict__ F,
                  const int32_t *__restrict__ rows, int count, const double *__restrict__ r, double *__restrict__ z)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    const int i = rows[t];
    double v = r[i];
    for (int p = rp[i]; p < rp[i + 1] && cols[p] < i; ++p) v -= F[p] * z[cols[p]];
    z[i] = v;
}

// backward sweep with the upper part: z_i = (z_i - sum_{j > i} u_ij z_j) / u_ii
__global__ void __launch_bounds__(256)
k_ilu_upper_level(const int32_t *__restrict__ rp, const int32_t *__restrict__ cols,
                  const int32_t *__restrict__ diag, const double *__restrict__ F, const int32_t *__restrict__ rows,
                  int count, double *__restrict__ z)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    const int i = rows[t];
    double v = z[i];
    for (int p = rp[i]; p < rp[i + 1]; ++p)
        if (cols[p] > i) v -= F[p] * z[cols[p]];
    z[i] = v / F[diag[i]];
}

// rows grouped by level: ptr[l] .. ptr[l+1] in rows
static void level_sets(const std::vector<int32_t> &rp, const std::vector<int32_t> &cols, int64_t n, bool lower,
                       std::vector<int32_t> &rows, std::vector<int32_t> &ptr)
{
    std::vector<int32_t> lv(n, 0);
    int nlev = 0;
    if (lower) {
        for (int64_t i = 0; i < n; ++i) {
            int l = 0;
            for (int32_t p = rp[i]; p < rp[i + 1] && cols[p] < i; ++p) l = std::max(l, lv[cols[p]] + 1);
            lv[i] = l;
            nlev = std::max(nlev, l + 1);
        }
    } else {
        for (int64_t i = n - 1; i >= 0; --i) {
            int l = 0;
            for (int32_t p = rp[i]; p < rp[i + 1]; ++p)
                if (cols[p] > i) l = std::max(l, lv[cols[p]] + 1);
            lv[i] = l;
            nlev = std::max(nlev, l + 1);
        }
    }
    ptr.assign(nlev + 1, 0);
    for (int64_t i = 0; i < n; ++i) ptr[lv[i] + 1]++;
    for (int l = 0; l < nlev; ++l) ptr[l + 1] += ptr[l];
    rows.resize(n);
    std::vector<int32_t> fill(ptr.begin(), ptr.end() - 1);
    for (int64_t i = 0; i < n; ++i) rows[fill[lv[i]]++] = (int32_t)i;  // ascending rows per level
}

void ilu_free(cdfem_ctx *c)
{
    auto &u = c->ilu;
    if (u.exec) (void)hipGraphExecDestroy(u.exec);
    if (u.graph) (void)hipGraphDestroy(u.graph);
    for (void *p : {(void *)u.F, (void *)u.rows_l, (void *)u.rows_u, (void *)u.z})
        if (p) (void)hipFree(p);
    u = IluState{};
}

// factor the eliminated matrix (values d_vals_c, pattern d_rowptr / d_cols) once per operator and
// capture the sweep graph: in = c->d_w[4] (the GMRES work vector), out = u.z
void ilu_setup(cdfem_ctx *c)
{
    if (c->ilu.ready) return;
    ilu_free(c);
    if (!c->fa_ready) throw std::runtime_error("ILU(0) needs an assembled operator (cdfem_fa_setup)");
    const int64_t n = c->nl;
    std::vector<int32_t> rp(n + 1), cols(c->nnz);
    auto chk = [](hipError_t e) {
        if (e != hipSuccess) throw std::runtime_error(std::string("ILU setup: ") + hipGetErrorString(e));
    };
    chk(hipMemcpyAsync(rp.data(), c->d_rowptr, (n + 1) * 4, hipMemcpyDeviceToHost, c->stream));
    chk(hipMemcpyAsync(cols.data(), c->d_cols, c->nnz * 4, hipMemcpyDeviceToHost, c->stream));
    chk(hipStreamSynchronize(c->stream));
    auto &u = c->ilu;
    std::vector<int32_t> rows_l, rows_u;
    level_sets(rp, cols, n, true, rows_l, u.ptr_l);
    level_sets(rp, cols, n, false, rows_u, u.ptr_u);
    chk(hipMalloc(&u.F, c->nnz * sizeof(double)));
    chk(hipMalloc(&u.rows_l, n * 4));
    chk(hipMalloc(&u.rows_u, n * 4));
    chk(hipMalloc(&u.z, n * sizeof(double)));
    chk(hipMemcpyAsync(u.F, c->d_vals_c, c->nnz * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    chk(hipMemcpyAsync(u.rows_l, rows_l.data(), n * 4, hipMemcpyHostToDevice, c->stream));
    chk(hipMemcpyAsync(u.rows_u, rows_u.data(), n * 4, hipMemcpyHostToDevice, c->stream));
    const int nl_lev = (int)u.ptr_l.size() - 1, nu_lev = (int)u.ptr_u.size() - 1;
    for (int l = 0; l < nl_lev; ++l) {
        const int cnt = u.ptr_l[l + 1] - u.ptr_l[l];
        hipLaunchKernelGGL(k_ilu_factor_level, dim3((cnt + 255) / 256), dim3(256), 0, c->stream, c->d_rowptr,
                           c->d_cols, c->d_diagpos, u.F, u.rows_l + u.ptr_l[l], cnt);
    }
    chk(hipGetLastError());
    // the sweep sequence as a graph on fixed buffers
    const double *in = c->d_w[4];
    chk(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    for (int l = 0; l < nl_lev; ++l) {
        const int cnt = u.ptr_l[l + 1] - u.ptr_l[l];
        hipLaunchKernelGGL(k_ilu_lower_level, dim3((cnt + 255) / 256), dim3(256), 0, c->stream, c->d_rowptr,
                           c->d_cols, u.F, u.rows_l + u.ptr_l[l], cnt, in, u.z);
    }
    for (int l = 0; l < nu_lev; ++l) {
        const int cnt = u.ptr_u[l + 1] - u.ptr_u[l];
        hipLaunchKernelGGL(k_ilu_upper_level, dim3((cnt + 255) / 256), dim3(256), 0, c->stream, c->d_rowptr,
                           c->d_cols, c->d_diagpos, u.F, u.rows_u + u.ptr_u[l], cnt, u.z);
    }
    chk(hipStreamEndCapture(c->stream, &u.graph));
    chk(hipGraphInstantiate(&u.exec, u.graph, nullptr, nullptr, 0));
    chk(hipStreamSynchronize(c->stream));
    u.ready = true;
}

// u.z = (L U)^{-1} c->d_w[4]
hipError_t ilu_apply(cdfem_ctx *c) { return hipGraphLaunch(c->ilu.exec, c->stream); }

}  // namespace cdfem
