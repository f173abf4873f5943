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
// On several ranks (general partition) it is PETSc's bjacobi: one ILU(0) per rank of the owned
// diagonal block of the global matrix (build_owned_block).
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
    if (u.block)
        for (void *p : {(void *)u.rp, (void *)u.cols, (void *)u.diag})
            if (p) (void)hipFree(p);
    u = IluState{};
}

static void chk(hipError_t e)
{
    if (e != hipSuccess) throw std::runtime_error(std::string("ILU setup: ") + hipGetErrorString(e));
}

// PETSc bjacobi on several ranks: rank r's block is the diagonal block of the global eliminated
// matrix on its owned rows and columns, in the local (natural) order of its true dofs.  The global
// matrix is sum_q P_q^T A_q P_q, so an owned row i that other ranks hold also collects their partial
// rows: neighbour q sends every entry (i, j) of its local eliminated matrix with i and j both shared
// with this rank (as positions in the common shared list, the order both sides agree on), and this
// rank keeps those with i and j owned here.  Entries are summed per (i, j) in a fixed order: the own
// partial, then the neighbours in ascending rank.  Essential rows are identity rows, essential
// columns zero (the eliminated matrix of FormLinearSystem, DIAG_ONE).
static void build_owned_block(cdfem_ctx *c, const std::vector<int32_t> &rp, const std::vector<int32_t> &cols,
                              const std::vector<double> &vals, std::vector<int32_t> &brp,
                              std::vector<int32_t> &bcols, std::vector<double> &bvals)
{
    const int64_t n = c->nl, lo = c->skip_lo, no = n - lo;
    const int nn = (int)c->nbr_rank.size();
    const std::vector<int64_t> &off = c->nbr_off;
    const std::vector<int32_t> &idx = c->h_sh_idx;
    // outgoing triples (row position, column position, value) per neighbour
    std::vector<std::vector<double>> out(nn);
    std::vector<int32_t> pos(n, -1);
    for (int k = 0; k < nn; ++k) {
        for (int64_t j = off[k]; j < off[k + 1]; ++j) pos[idx[j]] = (int32_t)(j - off[k]);
        for (int64_t j = off[k]; j < off[k + 1]; ++j) {
            const int32_t i = idx[j];
            for (int32_t p = rp[i]; p < rp[i + 1]; ++p)
                if (pos[cols[p]] >= 0) {
                    out[k].push_back((double)pos[i]);
                    out[k].push_back((double)pos[cols[p]]);
                    out[k].push_back(vals[p]);
                }
        }
        for (int64_t j = off[k]; j < off[k + 1]; ++j) pos[idx[j]] = -1;
    }
    // counts, then the payloads in buffers of the pair's common (larger) size
    std::vector<int64_t> off1(nn + 1);
    for (int k = 0; k <= nn; ++k) off1[k] = k;
    std::vector<double> cnt_send(nn), cnt_recv(nn);
    for (int k = 0; k < nn; ++k) cnt_send[k] = (double)out[k].size();
    double *d_a = nullptr, *d_b = nullptr;
    chk(hipMalloc(&d_a, std::max(nn, 1) * sizeof(double)));
    chk(hipMalloc(&d_b, std::max(nn, 1) * sizeof(double)));
    chk(hipMemcpyAsync(d_a, cnt_send.data(), nn * sizeof(double), hipMemcpyHostToDevice, c->stream));
    comm_exchange_nbr_buf(c, off1, d_a, d_b);
    chk(hipMemcpyAsync(cnt_recv.data(), d_b, nn * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    chk(hipStreamSynchronize(c->stream));
    (void)hipFree(d_a);
    (void)hipFree(d_b);
    std::vector<int64_t> off2(nn + 1, 0);
    for (int k = 0; k < nn; ++k)
        off2[k + 1] = off2[k] + std::max((int64_t)cnt_send[k], (int64_t)cnt_recv[k]);
    const int64_t tot = off2[nn];
    std::vector<double> hs(tot, 0.0), hr(tot, 0.0);
    for (int k = 0; k < nn; ++k) std::copy(out[k].begin(), out[k].end(), hs.begin() + off2[k]);
    chk(hipMalloc(&d_a, std::max<int64_t>(tot, 1) * sizeof(double)));
    chk(hipMalloc(&d_b, std::max<int64_t>(tot, 1) * sizeof(double)));
    chk(hipMemcpyAsync(d_a, hs.data(), tot * sizeof(double), hipMemcpyHostToDevice, c->stream));
    comm_exchange_nbr_buf(c, off2, d_a, d_b);
    chk(hipMemcpyAsync(hr.data(), d_b, tot * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    chk(hipStreamSynchronize(c->stream));
    (void)hipFree(d_a);
    (void)hipFree(d_b);
    // rows of the block: (column, value) in summation order, then merged per column
    std::vector<std::vector<std::pair<int32_t, double>>> row(no);
    for (int64_t i = lo; i < n; ++i)
        for (int32_t p = rp[i]; p < rp[i + 1]; ++p)
            if (cols[p] >= lo) row[i - lo].push_back({cols[p] - (int32_t)lo, vals[p]});
    for (int k = 0; k < nn; ++k) {
        const int64_t m = (int64_t)cnt_recv[k];
        if (m % 3) throw std::runtime_error("ILU setup: malformed block-row exchange");
        for (int64_t t = 0; t < m; t += 3) {
            const int64_t a = (int64_t)hr[off2[k] + t], b = (int64_t)hr[off2[k] + t + 1];
            if (a < 0 || b < 0 || a >= off[k + 1] - off[k] || b >= off[k + 1] - off[k])
                throw std::runtime_error("ILU setup: shared position out of range (neighbour lists disagree)");
            const int32_t i = idx[off[k] + a], j = idx[off[k] + b];
            if (i >= lo && j >= lo) row[i - lo].push_back({j - (int32_t)lo, hr[off2[k] + t + 2]});
        }
    }
    brp.assign(no + 1, 0);
    bcols.clear();
    bvals.clear();
    for (int64_t r = 0; r < no; ++r) {
        auto &e = row[r];
        std::stable_sort(e.begin(), e.end(), [](const auto &x, const auto &y) { return x.first < y.first; });
        const bool ess_row = c->h_ess[lo + r] != 0;
        for (size_t t = 0; t < e.size();) {
            const int32_t col = e[t].first;
            double v = 0.0;
            for (; t < e.size() && e[t].first == col; ++t) v += e[t].second;
            if (ess_row) v = col == r ? 1.0 : 0.0;
            else if (c->h_ess[lo + col]) v = 0.0;
            bcols.push_back(col);
            bvals.push_back(v);
        }
        brp[r + 1] = (int32_t)bcols.size();
    }
}

// factor the eliminated matrix (values d_vals_c, pattern d_rowptr / d_cols; on several ranks the
// owned diagonal block, build_owned_block) once per operator and capture the sweep graph:
// in = c->d_w[4] (the GMRES work vector), out = u.z
void ilu_setup(cdfem_ctx *c)
{
    if (c->ilu.ready) return;
    ilu_free(c);
    if (!c->fa_ready) throw std::runtime_error("ILU(0) needs an assembled operator (cdfem_fa_setup)");
    const int64_t n = c->nl;
    const bool block = c->comm && c->nranks > 1 && c->part_mode == 2;
    const int64_t lo = block ? c->skip_lo : 0, nb = n - lo;
    std::vector<int32_t> rp(n + 1), cols(c->nnz);
    chk(hipMemcpyAsync(rp.data(), c->d_rowptr, (n + 1) * 4, hipMemcpyDeviceToHost, c->stream));
    chk(hipMemcpyAsync(cols.data(), c->d_cols, c->nnz * 4, hipMemcpyDeviceToHost, c->stream));
    chk(hipStreamSynchronize(c->stream));
    auto &u = c->ilu;
    std::vector<int32_t> brp, bcols;
    std::vector<double> bvals;
    if (block) {
        std::vector<double> vals(c->nnz);
        chk(hipMemcpyAsync(vals.data(), c->d_vals_c, c->nnz * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        chk(hipStreamSynchronize(c->stream));
        build_owned_block(c, rp, cols, vals, brp, bcols, bvals);
        std::vector<int32_t> bdiag(nb, -1);
        for (int64_t i = 0; i < nb; ++i)
            for (int32_t p = brp[i]; p < brp[i + 1]; ++p)
                if (bcols[p] == i) bdiag[i] = p;
        for (int64_t i = 0; i < nb; ++i)
            if (bdiag[i] < 0) throw std::runtime_error("ILU setup: owned block row without a diagonal entry");
        u.block = true;
        u.nnz = (int64_t)bcols.size();
        chk(hipMalloc(&u.rp, (nb + 1) * 4));
        chk(hipMalloc(&u.cols, std::max<int64_t>(u.nnz, 1) * 4));
        chk(hipMalloc(&u.diag, std::max<int64_t>(nb, 1) * 4));
        chk(hipMalloc(&u.F, std::max<int64_t>(u.nnz, 1) * sizeof(double)));
        chk(hipMemcpyAsync(u.rp, brp.data(), (nb + 1) * 4, hipMemcpyHostToDevice, c->stream));
        chk(hipMemcpyAsync(u.cols, bcols.data(), u.nnz * 4, hipMemcpyHostToDevice, c->stream));
        chk(hipMemcpyAsync(u.diag, bdiag.data(), nb * 4, hipMemcpyHostToDevice, c->stream));
        chk(hipMemcpyAsync(u.F, bvals.data(), u.nnz * sizeof(double), hipMemcpyHostToDevice, c->stream));
    } else {
        u.rp = c->d_rowptr;
        u.cols = c->d_cols;
        u.diag = c->d_diagpos;
        u.nnz = c->nnz;
        chk(hipMalloc(&u.F, c->nnz * sizeof(double)));
        chk(hipMemcpyAsync(u.F, c->d_vals_c, c->nnz * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    }
    const std::vector<int32_t> &prp = block ? brp : rp;
    const std::vector<int32_t> &pcols = block ? bcols : cols;
    std::vector<int32_t> rows_l, rows_u;
    level_sets(prp, pcols, nb, true, rows_l, u.ptr_l);
    level_sets(prp, pcols, nb, false, rows_u, u.ptr_u);
    chk(hipMalloc(&u.rows_l, std::max<int64_t>(nb, 1) * 4));
    chk(hipMalloc(&u.rows_u, std::max<int64_t>(nb, 1) * 4));
    chk(hipMalloc(&u.z, n * sizeof(double)));
    chk(hipMemsetAsync(u.z, 0, n * sizeof(double), c->stream));
    chk(hipMemcpyAsync(u.rows_l, rows_l.data(), nb * 4, hipMemcpyHostToDevice, c->stream));
    chk(hipMemcpyAsync(u.rows_u, rows_u.data(), nb * 4, hipMemcpyHostToDevice, c->stream));
    const int nl_lev = (int)u.ptr_l.size() - 1, nu_lev = (int)u.ptr_u.size() - 1;
    for (int l = 0; l < nl_lev; ++l) {
        const int cnt = u.ptr_l[l + 1] - u.ptr_l[l];
        hipLaunchKernelGGL(k_ilu_factor_level, dim3((cnt + 255) / 256), dim3(256), 0, c->stream, u.rp, u.cols, u.diag,
                           u.F, u.rows_l + u.ptr_l[l], cnt);
    }
    chk(hipGetLastError());
    // the sweep sequence as a graph on fixed buffers (owned part of the vectors on several ranks)
    const double *in = c->d_w[4] + lo;
    double *z = u.z + lo;
    chk(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    for (int l = 0; l < nl_lev; ++l) {
        const int cnt = u.ptr_l[l + 1] - u.ptr_l[l];
        hipLaunchKernelGGL(k_ilu_lower_level, dim3((cnt + 255) / 256), dim3(256), 0, c->stream, u.rp, u.cols, u.F,
                           u.rows_l + u.ptr_l[l], cnt, in, z);
    }
    for (int l = 0; l < nu_lev; ++l) {
        const int cnt = u.ptr_u[l + 1] - u.ptr_u[l];
        hipLaunchKernelGGL(k_ilu_upper_level, dim3((cnt + 255) / 256), dim3(256), 0, c->stream, u.rp, u.cols, u.diag,
                           u.F, u.rows_u + u.ptr_u[l], cnt, z);
    }
    chk(hipStreamEndCapture(c->stream, &u.graph));
    chk(hipGraphInstantiate(&u.exec, u.graph, nullptr, nullptr, 0));
    chk(hipStreamSynchronize(c->stream));
    u.ready = true;
}

// u.z = (L U)^{-1} c->d_w[4]; on several ranks the owned block's sweeps, then P (the non-owned
// shared entries take their owner's value), so z is a consistent L-vector like a Jacobi product
hipError_t ilu_apply(cdfem_ctx *c)
{
    const hipError_t e = hipGraphLaunch(c->ilu.exec, c->stream);
    if (e != hipSuccess || !c->ilu.block) return e;
    interface_copy_owner(c, c->ilu.z);
    return hipGetLastError();
}

}  // namespace cdfem
