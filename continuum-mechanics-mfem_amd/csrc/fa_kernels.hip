// fa_kernels.hip — full assembly (FA) on simplex meshes: element matrices, deterministic CSR
// assembly and the CSR SpMV that the Krylov solvers run on (BASELINE config C4: unstructured
// tetrahedra, FA CSR SpMV + GMRES(30)/Jacobi — the reference's own solver path,
// linear_convection_diffusion_2D.cpp:339 (Assemble, FA), :349-351 (FormLinearSystem ->
// HypreParMatrix), :364-375 (PETSc MATAIJ + KSPGMRES)).
//
// Pipeline (once per operator, cdfem_fa_setup):
//   host    CSR pattern (sorted columns per row) + for every nonzero the list of element-matrix
//           entries that sum into it, in ascending element order (built once per mesh);
//   k_simplex_elem   one thread per element: affine Jacobian, rule loop, nd x nd element matrix
//                    written element-block-major [blk][i*nd+j][lane] (coalesced stores);
//   k_fa_gather      one thread per nonzero: fixed-order sum of its contributions (bitwise
//                    reproducible, no atomics);
//   k_fa_eliminate   the FormLinearSystem matrix: ess rows/cols zeroed, unit diagonal (DIAG_ONE).
// Hot loop: k_sell_spmv on a SELL-64 copy of the matrix (rows sorted by length, 64-row slices
// stored column-major: one lane per row, each value/column load one coalesced wave access; < 1 %
// padding for Kuhn P2), x gathered (lexicographic numbering keeps it L2-local).
// Algorithmic bytes per SpMV = 12 nnz + 4 (n + 1) + 16 n.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <thread>
#include <vector>

#include "cdfem_internal.hpp"
#include "reduce.hpp"

namespace cdfem {

// ---- host: CSR pattern and contribution lists --------------------------------------------------
template <class F>
static void parallel_rows(int64_t n, F &&f)
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

static inline int64_t ee_index(int e, int i, int j, int nd)
{
    return ((int64_t)(e / kLanes) * nd * nd + (int64_t)i * nd + j) * kLanes + e % kLanes;
}

FaPattern fa_build_pattern(const std::vector<int32_t> &dof, int ne, int nd, int64_t nl, int sell_mode, int dim,
                           const double *dof_xyz, int64_t sell_window, int64_t lds_rows, int lpr)
{
    // dof -> incidences (e * nd + l), ascending
    std::vector<int64_t> cnt(nl + 1, 0);
    for (int64_t k = 0; k < (int64_t)ne * nd; ++k) cnt[dof[k] + 1]++;
    for (int64_t i = 0; i < nl; ++i) cnt[i + 1] += cnt[i];
    std::vector<int64_t> inc((size_t)ne * nd);
    {
        std::vector<int64_t> fill(cnt.begin(), cnt.end() - 1);
        for (int64_t k = 0; k < (int64_t)ne * nd; ++k) inc[fill[dof[k]]++] = k;
    }
    if ((int64_t)ne * nd * nd >= ((int64_t)1 << 31)) throw std::runtime_error("FA contributions exceed int32");
    auto row_cols = [&](int64_t i, std::vector<int32_t> &buf) {
        buf.clear();
        for (int64_t k = cnt[i]; k < cnt[i + 1]; ++k) {
            const int64_t e = inc[k] / nd;
            for (int l = 0; l < nd; ++l) buf.push_back(dof[e * nd + l]);
        }
        std::sort(buf.begin(), buf.end());
        buf.erase(std::unique(buf.begin(), buf.end()), buf.end());
    };
    // pass 1: row lengths
    std::vector<int32_t> rowptr(nl + 1, 0);
    parallel_rows(nl, [&](int64_t lo, int64_t hi) {
        std::vector<int32_t> buf;
        for (int64_t i = lo; i < hi; ++i) {
            row_cols(i, buf);
            rowptr[i + 1] = (int32_t)buf.size();
        }
    });
    int64_t nnz = 0;
    for (int64_t i = 0; i < nl; ++i) {
        nnz += rowptr[i + 1];
        if (nnz >= ((int64_t)1 << 31)) throw std::runtime_error("nnz exceeds int32 indexing");
        rowptr[i + 1] = (int32_t)nnz;
    }
    // pass 2: columns, diagonal positions, contribution lists.  Row i owns the contribution
    // slots [nd * cnt[i], nd * cnt[i+1]) (every incidence of dof i contributes nd entries).
    FaPattern P;
    P.nnz = nnz;
    std::vector<int32_t> &cols = P.cols, &diagpos = P.diagpos, &coff = P.coff, &cpos = P.cpos;
    cols.resize(nnz);
    diagpos.resize(nl);
    coff.resize(nnz + 1);
    cpos.resize((size_t)ne * nd * nd);
    coff[nnz] = (int32_t)((int64_t)ne * nd * nd);
    parallel_rows(nl, [&](int64_t lo, int64_t hi) {
        std::vector<int32_t> buf, hits, slot;
        for (int64_t i = lo; i < hi; ++i) {
            row_cols(i, buf);
            const int32_t base = rowptr[i];
            const int len = (int)buf.size();
            std::copy(buf.begin(), buf.end(), cols.begin() + base);
            diagpos[i] = base + (int32_t)(std::lower_bound(buf.begin(), buf.end(), (int32_t)i) - buf.begin());
            hits.assign(len, 0);
            slot.clear();
            for (int64_t k = cnt[i]; k < cnt[i + 1]; ++k) {  // ascending element
                const int64_t e = inc[k] / nd;
                for (int l = 0; l < nd; ++l) {
                    const int t = (int)(std::lower_bound(buf.begin(), buf.end(), dof[e * nd + l]) - buf.begin());
                    hits[t]++;
                    slot.push_back(t);
                }
            }
            int64_t run = (int64_t)nd * cnt[i];
            for (int t = 0; t < len; ++t) {
                coff[base + t] = (int32_t)run;
                run += hits[t];
            }
            std::fill(hits.begin(), hits.end(), 0);
            size_t s = 0;
            for (int64_t k = cnt[i]; k < cnt[i + 1]; ++k) {
                const int64_t e = inc[k] / nd;
                const int li = (int)(inc[k] % nd);
                for (int l = 0; l < nd; ++l, ++s) {
                    const int t = slot[s];
                    cpos[(size_t)coff[base + t] + hits[t]++] = (int32_t)ee_index((int)e, li, l, nd);
                }
            }
        }
    });
    // SpMV layout: SELL-64 over the rows in the plan's order (sell_plan.cpp)
    P.rowptr = std::move(rowptr);
    SellPlan pl = sell_plan(nl, P.rowptr.data(), P.cols.data(), sell_mode, dim, dof_xyz, sell_window);
    // spmv_lds: > 0 rows per window; -1 (auto): the plan's window when the auto mode chose an
    // unstructured windowed order
    pl.lds_rows = !pl.windowed ? 0 : lds_rows > 0 ? lds_rows : (lds_rows < 0 && pl.auto_lds) ? pl.window : 0;
    // spmv_lpr: 1, 2 or 4 lanes per row; 0 (auto): 4 on the auto mode's unstructured LDS layouts
    // (c4u SpMV 103.3 -> 91.2 us, profiles/r03/ab_c4u_spmv_lanes_per_row.txt), else 1
    if (pl.lds_rows > 0 && lpr <= 0 && pl.auto_lds) {
        // one lane per row pads each 64-row slice to its longest row: where that costs more than 15 %
        // (unstructured meshes' vertex rows) 4 lanes per row, else 2 (measured best on the lattice)
        int64_t st = 0, real = 0;
        for (int64_t k0 = 0; k0 < nl; k0 += kLanes) {
            int32_t mx = 0;
            for (int64_t k = k0; k < std::min<int64_t>(nl, k0 + kLanes); ++k) {
                const int32_t r = pl.perm.empty() ? (int32_t)k : pl.perm[k];
                const int32_t len = P.rowptr[r + 1] - P.rowptr[r];
                mx = std::max(mx, len);
                real += len;
            }
            st += (int64_t)mx * kLanes;
        }
        lpr = st > real + real * 15 / 100 ? 4 : 2;
    }
    pl.lpr = pl.lds_rows <= 0 ? 1 : lpr > 0 ? lpr : 1;
    try {
        sell_build(P, nl, pl);
    } catch (const std::runtime_error &) {
        if (pl.lpr == 1) throw;
        pl.lpr = 1;  // a multi-lane slice's halo exceeds the LDS budget: one lane per row
        P.sptr.clear(); P.srows.clear(); P.scols.clear(); P.smap.clear(); P.sdel.clear(); P.swide.clear();
        P.hptr.clear(); P.hidx.clear(); P.sloc.clear();
        P.nnz_wide = 0; P.lds_rows = 0; P.lds_max = 0;
        sell_build(P, nl, pl);
    }
    return P;
}


// ---- element matrices on affine simplices ----------------------------------------------------------
template <int DIM, int P>
__global__ void __launch_bounds__(64)
k_simplex_elem(const double *__restrict__ verts, int ne, int nqd, int nqc, const double *__restrict__ stab, unsigned kinds,
               double kappa, const double *__restrict__ kq, const double *__restrict__ kmq, double alpha, double c0,
               double c1, double c2,
               const double *__restrict__ cq, double mass, const double *__restrict__ mq, double *__restrict__ Ee)
{
    constexpr int ND = P == 1 ? DIM + 1 : P == 2 ? (DIM + 1) * (DIM + 2) / 2 : 10;
    const int e = blockIdx.x * 64 + threadIdx.x;
    if (e >= ne) return;
    const double *V = verts + (size_t)e * (DIM + 1) * DIM;
    double J[DIM][DIM], A[DIM][DIM];
#pragma unroll
    for (int k = 0; k < DIM; ++k)
#pragma unroll
        for (int m = 0; m < DIM; ++m) J[k][m] = V[(m + 1) * DIM + k] - V[k];
    double det;
    if constexpr (DIM == 3) {
        A[0][0] = J[1][1] * J[2][2] - J[1][2] * J[2][1];
        A[0][1] = J[0][2] * J[2][1] - J[0][1] * J[2][2];
        A[0][2] = J[0][1] * J[1][2] - J[0][2] * J[1][1];
        A[1][0] = J[1][2] * J[2][0] - J[1][0] * J[2][2];
        A[1][1] = J[0][0] * J[2][2] - J[0][2] * J[2][0];
        A[1][2] = J[0][2] * J[1][0] - J[0][0] * J[1][2];
        A[2][0] = J[1][0] * J[2][1] - J[1][1] * J[2][0];
        A[2][1] = J[0][1] * J[2][0] - J[0][0] * J[2][1];
        A[2][2] = J[0][0] * J[1][1] - J[0][1] * J[1][0];
        det = J[0][0] * A[0][0] + J[0][1] * A[1][0] + J[0][2] * A[2][0];
    } else {
        A[0][0] = J[1][1];
        A[0][1] = -J[0][1];
        A[1][0] = -J[1][0];
        A[1][1] = J[0][0];
        det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
    }
    double M[ND][ND];
#pragma unroll
    for (int i = 0; i < ND; ++i)
#pragma unroll
        for (int j = 0; j < ND; ++j) M[i][j] = 0.0;
    const double cc[3] = {c0, c1, c2};
    // two rules (MFEM's GetRule): r = 0 the diffusion rule (order 2p - 2) with the diffusion term,
    // r = 1 the convection + mass rule (order 2p) with those terms; per-point coefficient arrays
    // are indexed in the point order of their own rule
    for (int r = 0; r < 2; ++r) {
        const bool dif = r == 0 && (kinds & CDFEM_DIFFUSION), con = r == 1 && (kinds & CDFEM_CONVECTION),
                   mas = r == 1 && (kinds & CDFEM_MASS);
        if (!dif && !con && !mas) continue;
        const int nq = r == 0 ? nqd : nqc;
        const double *tab = r == 0 ? stab : stab + (size_t)nqd * (ND * (DIM + 1) + 1);
        const double *phi_t = tab, *dphi_t = tab + (size_t)nq * ND, *w_t = tab + (size_t)nq * ND * (DIM + 1);
    for (int q = 0; q < nq; ++q) {
        const double W = w_t[q];
        double D[DIM][DIM] = {}, Cv[DIM] = {}, Ms = 0.0;
        if (dif) {
            const double kap = kq ? kq[(size_t)e * nq + q] : kappa;
            if (kmq) {  // MatrixCoefficient: W adj(J) K adj(J)^T / det J with K = kap I + K_q
                constexpr int NS = DIM * (DIM + 1) / 2;
                const double *km = kmq + ((size_t)e * nq + q) * NS;
                double K[DIM][DIM];
#pragma unroll
                for (int k = 0, m = 0; k < DIM; ++k)
#pragma unroll
                    for (int l = k; l < DIM; ++l, ++m) K[k][l] = K[l][k] = km[m] + (k == l ? kap : 0.0);
#pragma unroll
                for (int a = 0; a < DIM; ++a)
#pragma unroll
                    for (int b = 0; b < DIM; ++b) {
                        double s = 0.0;
#pragma unroll
                        for (int k = 0; k < DIM; ++k) {
                            double t = 0.0;
#pragma unroll
                            for (int l = 0; l < DIM; ++l) t += K[k][l] * A[b][l];
                            s += A[a][k] * t;
                        }
                        D[a][b] = W * s / det;
                    }
            } else {
                const double f = W * kap / det;
#pragma unroll
                for (int a = 0; a < DIM; ++a)
#pragma unroll
                    for (int b = 0; b < DIM; ++b) {
                        double s = 0.0;
#pragma unroll
                        for (int k = 0; k < DIM; ++k) s += A[a][k] * A[b][k];
                        D[a][b] = f * s;
                    }
            }
        }
        if (con) {
#pragma unroll
            for (int a = 0; a < DIM; ++a) {
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < DIM; ++k)
                    s += A[a][k] * (cq ? cq[((size_t)e * nq + q) * DIM + k] : cc[k]);
                Cv[a] = W * alpha * s;
            }
        }
        if (mas) Ms = W * (mq ? mq[(size_t)e * nq + q] : mass) * det;
        double ph[ND], dph[ND][DIM];
#pragma unroll
        for (int i = 0; i < ND; ++i) {
            ph[i] = phi_t[q * ND + i];
#pragma unroll
            for (int k = 0; k < DIM; ++k) dph[i][k] = dphi_t[(q * ND + i) * DIM + k];
        }
#pragma unroll
        for (int j = 0; j < ND; ++j) {
            double Dg[DIM], rest = Ms * ph[j];
#pragma unroll
            for (int a = 0; a < DIM; ++a) {
                Dg[a] = 0.0;
#pragma unroll
                for (int b = 0; b < DIM; ++b) Dg[a] += D[a][b] * dph[j][b];
                rest += Cv[a] * dph[j][a];
            }
#pragma unroll
            for (int i = 0; i < ND; ++i) {
                double v = ph[i] * rest;
#pragma unroll
                for (int a = 0; a < DIM; ++a) v += dph[i][a] * Dg[a];
                M[i][j] += v;
            }
        }
    }
    }
    const int64_t base = (int64_t)(e / kLanes) * ND * ND * kLanes + e % kLanes;
#pragma unroll
    for (int i = 0; i < ND; ++i)
#pragma unroll
        for (int j = 0; j < ND; ++j) Ee[base + (int64_t)(i * ND + j) * kLanes] = M[i][j];
}

// DomainLF on affine simplices: be_l = sum_q w_q det J f_q phi_l(q), element-major E-vector
// (summed by k_e2l).  Tables: phi [nq][ND], w [nq] of the LINEARFORM rule.
template <int DIM, int ND>
__global__ void __launch_bounds__(64)
k_simplex_lf(const double *__restrict__ verts, int ne, int nq, const double *__restrict__ tab,
             const double *__restrict__ fq, double *__restrict__ Ye)
{
    const int e = blockIdx.x * 64 + threadIdx.x;
    if (e >= ne) return;
    const double *V = verts + (size_t)e * (DIM + 1) * DIM;
    double det;
    if constexpr (DIM == 3) {
        double J[3][3];
        for (int k = 0; k < 3; ++k)
            for (int m = 0; m < 3; ++m) J[k][m] = V[(m + 1) * 3 + k] - V[k];
        det = J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) - J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
              J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
    } else {
        det = (V[2] - V[0]) * (V[5] - V[1]) - (V[4] - V[0]) * (V[3] - V[1]);
    }
    double b[ND];
#pragma unroll
    for (int l = 0; l < ND; ++l) b[l] = 0.0;
    for (int q = 0; q < nq; ++q) {
        const double f = tab[(size_t)nq * ND + q] * det * fq[(size_t)e * nq + q];
#pragma unroll
        for (int l = 0; l < ND; ++l) b[l] += f * tab[q * ND + l];
    }
#pragma unroll
    for (int l = 0; l < ND; ++l) Ye[(size_t)e * ND + l] = b[l];
}

__global__ void __launch_bounds__(256)
k_fa_gather(const int32_t *__restrict__ coff, const int32_t *__restrict__ cpos, const double *__restrict__ Ee,
            double *__restrict__ vals, int64_t nnz)
{
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nnz) return;
    double v = 0.0;
    for (int32_t t = coff[k]; t < coff[k + 1]; ++t) v += Ee[cpos[t]];
    vals[k] = v;
}

// FormLinearSystem matrix (MFEM EliminateRowsCols, DIAG_ONE): ess rows and columns zeroed, 1 on
// the diagonal of ess rows
__global__ void __launch_bounds__(256)
k_fa_eliminate(const int32_t *__restrict__ rowptr, const int32_t *__restrict__ cols, const double *__restrict__ vals,
               const uint8_t *__restrict__ ess, double *__restrict__ vals_c, int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const bool ei = ess[i] != 0;
    for (int32_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
        const int32_t j = cols[k];
        vals_c[k] = (ei || ess[j]) ? (j == i ? 1.0 : 0.0) : vals[k];
    }
}

__global__ void __launch_bounds__(256)
k_csr_diag(const double *__restrict__ vals, const int32_t *__restrict__ diagpos, double *__restrict__ d, int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = vals[diagpos[i]];
}

// SELL copies of A and of the eliminated A (after every assembly)
__global__ void __launch_bounds__(256)
k_sell_fill(const int32_t *__restrict__ smap, const double *__restrict__ vals, const double *__restrict__ vals_c,
            double *__restrict__ svals, double *__restrict__ svals_c, int64_t stored)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= stored) return;
    const int32_t k = smap[t];
    svals[t] = k >= 0 ? vals[k] : 0.0;
    svals_c[t] = k >= 0 ? vals_c[k] : 0.0;
}

// y = A x on the SELL-64 layout: one wave per 64-row slice, one lane per row, entries of a row
// summed in CSR order; every value/column load is one coalesced wave access.  CI = int32_t:
// absolute columns; CI = int16_t: column = lane base + delta (10 instead of 12 streamed bytes per
// entry).  PERM: the permuted layout (sell_plan.cpp), lane row = slice * 64 + lane in the SpMV's own
// order (no row index stream, whole-line y stores); otherwise the row comes from srows.  xcd_per > 0:
// workgroup b runs on XCD b mod 8, so logical block (b mod 8) * xcd_per + b / 8 gives every XCD one
// contiguous slice range and its L2 sees each x line once.  CG mode: partials of (x, y) and early
// exit once the Krylov state is done.
template <bool NT, class T>
__device__ __forceinline__ T stream_load(const T *p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// One wave's 64-row slice: returns the row sum of its lane (row index and validity out).
// U entries per lane per step; PIPE: the next step's value/column loads are issued before this
// step's x gathers are consumed (one memory round trip per step instead of two).  NT: values and
// columns are streamed once per SpMV: non-temporal loads, so x stays in L2.
template <typename CI, bool PERM, int U, bool PIPE, bool NT>
__device__ __forceinline__ double sell_slice(const int32_t *__restrict__ sptr, const int32_t *__restrict__ srows,
                                             const CI *__restrict__ scols, const double *__restrict__ svals,
                                             const double *__restrict__ x, int64_t n, int64_t sl, int lane,
                                             int64_t &row, bool &valid)
{
    constexpr bool DELTA = sizeof(CI) == 2;
    const int32_t b = sptr[sl], len = (sptr[sl + 1] - b) >> 6;
    int64_t base;
    if (PERM) {
        row = sl * 64 + lane;
        base = row < n ? row : n - 1;
    } else {
        row = srows[sl * 64 + lane];
        base = row >= 0 ? row : 0;
    }
    valid = PERM ? row < n : row >= 0;
    const double *xr = DELTA ? x + base : x;
    const double *v = svals + b + lane;
    const CI *cidx = scols + b + lane;
    double a0 = 0.0;
    int j = 0;
    if constexpr (PIPE) {
        double vv[U];
        int32_t cc[U];
        if (len >= U) {
#pragma unroll
            for (int k = 0; k < U; ++k) {
                cc[k] = stream_load<NT>(cidx + k * 64);
                vv[k] = stream_load<NT>(v + k * 64);
            }
        }
        for (; j + U <= len; j += U) {
            double xg[U];
#pragma unroll
            for (int k = 0; k < U; ++k) xg[k] = xr[cc[k]];
            const bool more = j + 2 * U <= len;  // wave-uniform
            if (more) {
#pragma unroll
                for (int k = 0; k < U; ++k) cc[k] = stream_load<NT>(cidx + (j + U + k) * 64);
            }
#pragma unroll
            for (int k = 0; k < U; ++k) a0 = fma(vv[k], xg[k], a0);
            if (more) {
#pragma unroll
                for (int k = 0; k < U; ++k) vv[k] = stream_load<NT>(v + (j + U + k) * 64);
            }
        }
    } else {
        for (; j + U <= len; j += U) {  // U independent loads in flight per lane
            double vv[U];
            int32_t cc[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                vv[k] = stream_load<NT>(v + (j + k) * 64);
                cc[k] = stream_load<NT>(cidx + (j + k) * 64);
            }
#pragma unroll
            for (int k = 0; k < U; ++k) a0 = fma(vv[k], xr[cc[k]], a0);
        }
    }
    for (; j < len; ++j) a0 = fma(stream_load<NT>(v + j * 64), xr[(int32_t)stream_load<NT>(cidx + j * 64)], a0);
    return a0;
}

// y = A x on the SELL-64 layout: one wave per 64-row slice, one lane per row, entries of a row
// summed in CSR order; every value/column load is one coalesced wave access.  CI = int32_t:
// absolute columns; CI = int16_t: column = lane base + delta (10 instead of 12 streamed bytes per
// entry).  PERM: the permuted layout (sell_plan.cpp), lane row = slice * 64 + lane in the SpMV's own
// order (no row index stream, whole-line y stores); otherwise the row comes from srows.
// Logical blocks (4 slices each): xcd_per > 0 gives XCD b mod 8 the contiguous range
// [(b mod 8) * xcd_per, + xcd_per), so its L2 sees each x line once (the loop runs once per block
// with the launchers' grids; it keeps any smaller grid correct).
// CG mode: partials of (x, y) and early exit once the Krylov state is done.
// MIX (CI = int16_t): mixed layout, a slice flagged in swide holds a column beyond 16 bits of its
// lane row and streams its 32-bit columns (cols32) instead (the flag is wave-uniform).
template <bool CG, typename CI, bool PERM, int U, bool PIPE, bool NT, bool MIX = false>
__global__ void __launch_bounds__(256)
k_sell_spmv(const int32_t *__restrict__ sptr, const int32_t *__restrict__ srows, const CI *__restrict__ scols,
            const double *__restrict__ svals, const double *__restrict__ x, double *__restrict__ y, int64_t nslices,
            int64_t n, int xcd_per, double *__restrict__ part, const KrylovState *__restrict__ st,
            const int32_t *__restrict__ cols32, const uint8_t *__restrict__ swide)
{
    __shared__ double sh[256 / 64];
    if (CG && st->done) return;
    const int lane = threadIdx.x & 63;
    const int64_t nlb = (nslices + 3) / 4;
    int64_t lb, end, step;
    if (xcd_per > 0) {
        lb = (int64_t)(blockIdx.x & 7) * xcd_per + (blockIdx.x >> 3);
        end = std::min<int64_t>(nlb, (int64_t)((blockIdx.x & 7) + 1) * xcd_per);
        step = gridDim.x >> 3;
    } else {
        lb = blockIdx.x;
        end = nlb;
        step = gridDim.x;
    }
    double dd = 0.0;
    for (; lb < end; lb += step) {
        const int64_t sl = lb * 4 + (threadIdx.x >> 6);
        if (sl >= nslices) continue;
        int64_t row;
        bool valid;
        double acc;
        if (MIX && swide[sl])
            acc = sell_slice<int32_t, PERM, U, PIPE, NT>(sptr, srows, cols32, svals, x, n, sl, lane, row, valid);
        else
            acc = sell_slice<CI, PERM, U, PIPE, NT>(sptr, srows, scols, svals, x, n, sl, lane, row, valid);
        if (valid) {
            y[row] = acc;
            if (CG) dd += acc * x[row];
        }
    }
    if (CG) store_partial(block_sum(dd, sh), part);
}

// LDS-staged windows (windowed layouts, sell_plan.cpp): workgroup = one window of S slices.  The
// window's distinct columns (hidx, ascending) are loaded into LDS once, then every entry reads its x
// value from LDS through its 16-bit window position (sloc): no divergent global gathers, and x leaves
// HBM / L2 once per window.  Each row sums its entries in the stored order (bitwise the windowed
// layout's sums).  Windows run in XCD-contiguous ranges (xcd_per > 0), so neighbouring windows, whose
// halos overlap, share an L2.  CG mode: partials of (x, y) and early exit once the Krylov state is done.
// LPR lanes per row (R = 64 / LPR rows per slice): lane l sums the (l / R)-th contiguous part of row
// l % R's entries, and the parts are combined by a fixed butterfly ((p0 + p1) + (p2 + p3)), so every
// lane of the row holds the same total.
template <bool CG, int LPR>
__global__ void __launch_bounds__(256)
k_sell_spmv_lds(const int32_t *__restrict__ sptr, const uint16_t *__restrict__ sloc, const double *__restrict__ svals,
                const int32_t *__restrict__ hptr, const int32_t *__restrict__ hidx, const double *__restrict__ x,
                double *__restrict__ y, int64_t nslices, int64_t n, int spw, int nwin, int xcd_per,
                double *__restrict__ part, const KrylovState *__restrict__ st)
{
    extern __shared__ double xs[];
    __shared__ double sh[256 / 64];
    if (CG && st->done) return;
    const int w = xcd_per > 0 ? (int)((blockIdx.x & 7) * xcd_per + (blockIdx.x >> 3)) : (int)blockIdx.x;
    double dd = 0.0;
    if (w < nwin) {
        const int h0 = hptr[w], H = hptr[w + 1] - h0;
        for (int i = threadIdx.x; i < H; i += 256) xs[i] = x[hidx[h0 + i]];
        __syncthreads();
        const int lane = threadIdx.x & 63;
        for (int s = threadIdx.x >> 6; s < spw; s += 4) {
            const int64_t sl = (int64_t)w * spw + s;
            if (sl >= nslices) break;
            const int32_t b = sptr[sl], len = (sptr[sl + 1] - b) >> 6;
            const double *v = svals + b + lane;
            const uint16_t *ci = sloc + b + lane;
            double a0 = 0.0;
            int j = 0;
            for (; j + 4 <= len; j += 4) {
                double vv[4];
                uint16_t cc[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    vv[k] = __builtin_nontemporal_load(v + (j + k) * 64);
                    cc[k] = __builtin_nontemporal_load(ci + (j + k) * 64);
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) a0 = fma(vv[k], xs[cc[k]], a0);
            }
            for (; j < len; ++j) a0 = fma(__builtin_nontemporal_load(v + j * 64), xs[__builtin_nontemporal_load(ci + j * 64)], a0);
            constexpr int R = 64 / LPR;
#pragma unroll
            for (int o = R; o < 64; o <<= 1) a0 += __shfl_xor(a0, o, 64);
            const int64_t row = sl * R + (lane % R);
            if (lane < R && row < n) {
                y[row] = a0;
                if (CG) dd += a0 * x[row];
            }
        }
    }
    if (CG) store_partial(block_sum(dd, sh), part);
}

// permuted layout: xp[i] = x[perm[i]] into the SpMV order, y[perm[i]] = yp[i] back to mesh order
__global__ void __launch_bounds__(256)
k_perm_gather(const int32_t *__restrict__ perm, const double *__restrict__ x, double *__restrict__ xp, int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) xp[i] = x[perm[i]];
}

__global__ void __launch_bounds__(256)
k_perm_scatter(const int32_t *__restrict__ perm, const double *__restrict__ yp, double *__restrict__ y, int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[perm[i]] = yp[i];
}

// ---- launchers ---------------------------------------------------------------------------------
hipError_t launch_simplex_elem(cdfem_ctx *c, const double *kq, const double *kmq, double kappa, double alpha,
                               const double *conv, const double *cq, const double *mq, double mass)
{
    const dim3 g((c->ne + 63) / 64), b(64);
    const double c0 = conv ? conv[0] : 0.0, c1 = conv ? conv[1] : 0.0, c2 = (conv && c->dim == 3) ? conv[2] : 0.0;
#define CDFEM_SIMPLEX(D, P)                                                                              \
    hipLaunchKernelGGL((k_simplex_elem<D, P>), g, b, 0, c->stream, c->d_verts, c->ne, c->nq_sd, c->nq_scm, \
                       c->d_stab, c->kinds, kappa, kq, kmq, alpha, c0, c1, c2, cq, mass, mq, c->d_Ee)
    if (c->dim == 3 && c->p == 1) CDFEM_SIMPLEX(3, 1);
    else if (c->dim == 3 && c->p == 2) CDFEM_SIMPLEX(3, 2);
    else if (c->dim == 2 && c->p == 1) CDFEM_SIMPLEX(2, 1);
    else if (c->dim == 2 && c->p == 2) CDFEM_SIMPLEX(2, 2);
    else if (c->dim == 2 && c->p == 3) CDFEM_SIMPLEX(2, 3);
    else return hipErrorInvalidValue;
#undef CDFEM_SIMPLEX
    return hipGetLastError();
}

hipError_t launch_simplex_lf(cdfem_ctx *c, const double *fq, double *Ye)
{
    const dim3 g((c->ne + 63) / 64), b(64);
    if (c->dim == 3 && c->p == 1)
        hipLaunchKernelGGL((k_simplex_lf<3, 4>), g, b, 0, c->stream, c->d_verts, c->ne, c->nq_lf, c->d_stab_lf, fq, Ye);
    else if (c->dim == 3 && c->p == 2)
        hipLaunchKernelGGL((k_simplex_lf<3, 10>), g, b, 0, c->stream, c->d_verts, c->ne, c->nq_lf, c->d_stab_lf, fq, Ye);
    else if (c->dim == 2 && c->p == 1)
        hipLaunchKernelGGL((k_simplex_lf<2, 3>), g, b, 0, c->stream, c->d_verts, c->ne, c->nq_lf, c->d_stab_lf, fq, Ye);
    else if (c->dim == 2 && c->p == 2)
        hipLaunchKernelGGL((k_simplex_lf<2, 6>), g, b, 0, c->stream, c->d_verts, c->ne, c->nq_lf, c->d_stab_lf, fq, Ye);
    else if (c->dim == 2 && c->p == 3)
        hipLaunchKernelGGL((k_simplex_lf<2, 10>), g, b, 0, c->stream, c->d_verts, c->ne, c->nq_lf, c->d_stab_lf, fq, Ye);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_fa_assemble(cdfem_ctx *c)
{
    hipLaunchKernelGGL(k_fa_gather, dim3((unsigned)((c->nnz + 255) / 256)), dim3(256), 0, c->stream, c->d_coff,
                       c->d_cpos, c->d_Ee, c->d_vals, c->nnz);
    hipLaunchKernelGGL(k_fa_eliminate, dim3((unsigned)((c->nl + 255) / 256)), dim3(256), 0, c->stream,
                       c->d_rowptr, c->d_cols, c->d_vals, c->d_ess, c->d_vals_c, (int64_t)c->nl);
    return hipGetLastError();
}

hipError_t launch_csr_diag(cdfem_ctx *c, double *d)
{
    hipLaunchKernelGGL(k_csr_diag, dim3((unsigned)((c->nl + 255) / 256)), dim3(256), 0, c->stream, c->d_vals,
                       c->d_diagpos, d, (int64_t)c->nl);
    return hipGetLastError();
}

hipError_t launch_sell_fill(cdfem_ctx *c)
{
    hipLaunchKernelGGL(k_sell_fill, dim3((unsigned)((c->nstored + 255) / 256)), dim3(256), 0, c->stream, c->d_smap,
                       c->d_vals, c->d_vals_c, c->d_svals, c->d_svals_c, c->nstored);
    return hipGetLastError();
}

// logical SpMV blocks (4 slices each) and the launched grid (a multiple of 8 with the XCD ranges)
static unsigned sell_blocks(const cdfem_ctx *c) { return (unsigned)((c->nslices + 3) / 4); }
static int sell_xcd_per(const cdfem_ctx *c)
{
    // contiguous per-XCD ranges pay on the windowed layout (1.00x traffic); the global length sort
    // puts the longest rows first, and a range split would hand them all to XCD 0
    return c->spmv_xcd && c->sell_windowed ? (int)((sell_blocks(c) + 7) / 8) : 0;
}
unsigned sell_grid(const cdfem_ctx *c)
{
    if (c->lds_rows > 0) {
        const int64_t spw = c->lds_rows / (64 / c->sell_lpr), nwin = (c->nslices + spw - 1) / spw;
        return c->spmv_xcd ? 8u * (unsigned)((nwin + 7) / 8) : (unsigned)nwin;
    }
    return sell_xcd_per(c) ? 8u * (unsigned)sell_xcd_per(c) : sell_blocks(c);
}

bool spmv_delta(const cdfem_ctx *c) { return c->d_sdel && c->spmv_index16; }

static int lds_windows(const cdfem_ctx *c)
{
    const int64_t spw = c->lds_rows / (64 / c->sell_lpr);
    return (int)((c->nslices + spw - 1) / spw);
}

template <bool CG>
static void spmv_launch(cdfem_ctx *c, const double *vals, const double *x, double *y, double *part,
                        const KrylovState *st)
{
    if (c->lds_rows > 0) {
        const int nwin = lds_windows(c), per = c->spmv_xcd ? (nwin + 7) / 8 : 0;
        const dim3 g(per ? 8u * (unsigned)per : (unsigned)nwin), b(256);
        const int spw = (int)(c->lds_rows / (64 / c->sell_lpr));
#define CDFEM_SPMV_LDS(L)                                                                                       \
    CDFEM_LAUNCH(c, (k_sell_spmv_lds<CG, L>), g, b, (size_t)c->lds_max * sizeof(double), c->d_sptr, c->d_sloc, vals, \
                 c->d_hptr, c->d_hidx, x, y, c->nslices, (int64_t)c->nl, spw, nwin, per, part, st)
        if (c->sell_lpr == 4) CDFEM_SPMV_LDS(4);
        else if (c->sell_lpr == 2) CDFEM_SPMV_LDS(2);
        else CDFEM_SPMV_LDS(1);
#undef CDFEM_SPMV_LDS
        return;
    }
    const dim3 g(sell_grid(c)), b(256);
    const int per = sell_xcd_per(c);
    const bool perm = c->sell_windowed;
#define CDFEM_SPMV(CI, PM)                                                                                       \
    CDFEM_LAUNCH(c, (k_sell_spmv<CG, CI, PM, 4, false, true>), g, b, 0, c->d_sptr, c->d_srows,                     \
                 (const CI *)(sizeof(CI) == 2 ? (const void *)c->d_sdel : (const void *)c->d_scols), vals, x, y,  \
                 c->nslices, (int64_t)c->nl, per, part, st, (const int32_t *)nullptr, (const uint8_t *)nullptr)
#define CDFEM_SPMV_MIX(PM)                                                                                       \
    CDFEM_LAUNCH(c, (k_sell_spmv<CG, int16_t, PM, 4, false, true, true>), g, b, 0, c->d_sptr, c->d_srows,          \
                 c->d_sdel, vals, x, y, c->nslices, (int64_t)c->nl, per, part, st, c->d_scols, c->d_swide)
    if (spmv_delta(c) && c->d_swide) {
        if (perm) CDFEM_SPMV_MIX(true);
        else CDFEM_SPMV_MIX(false);
    } else if (spmv_delta(c)) {
        if (perm) CDFEM_SPMV(int16_t, true);
        else CDFEM_SPMV(int16_t, false);
    } else {
        if (perm) CDFEM_SPMV(int32_t, true);
        else CDFEM_SPMV(int32_t, false);
    }
#undef CDFEM_SPMV
#undef CDFEM_SPMV_MIX
}

// y = A x in the mesh's dof order.  Permuted layout: inside a permuted-order solve (perm_space)
// the vectors already are in the SpMV order; otherwise x is gathered and y scattered around it.
hipError_t launch_spmv(cdfem_ctx *c, bool constrained, const double *x, double *y)
{
    const double *vals = constrained ? c->d_svals_c : c->d_svals;
    if (!c->d_rperm || c->perm_space) {
        spmv_launch<false>(c, vals, x, y, nullptr, nullptr);
        return hipGetLastError();
    }
    const dim3 g((unsigned)((c->nl + 255) / 256)), b(256);
    hipLaunchKernelGGL(k_perm_gather, g, b, 0, c->stream, c->d_rperm, x, c->d_pv[0], (int64_t)c->nl);
    spmv_launch<false>(c, vals, c->d_pv[0], c->d_pv[1], nullptr, nullptr);
    hipLaunchKernelGGL(k_perm_scatter, g, b, 0, c->stream, c->d_rperm, c->d_pv[1], y, (int64_t)c->nl);
    return hipGetLastError();
}

hipError_t launch_perm(cdfem_ctx *c, bool to_spmv_order, const double *src, double *dst)
{
    const dim3 g((unsigned)((c->nl + 255) / 256)), b(256);
    if (to_spmv_order)
        hipLaunchKernelGGL(k_perm_gather, g, b, 0, c->stream, c->d_rperm, src, dst, (int64_t)c->nl);
    else
        hipLaunchKernelGGL(k_perm_scatter, g, b, 0, c->stream, c->d_rperm, src, dst, (int64_t)c->nl);
    return hipGetLastError();
}

// q = A_c d and the den partials, then the MFEM CG den step (one-block finalizer).  Vectors in the
// SpMV order (a permuted layout only inside a permuted-order solve).
hipError_t launch_spmv_cg(cdfem_ctx *c, const double *d, double *q)
{
    if (c->d_rperm && !c->perm_space) return hipErrorInvalidValue;
    spmv_launch<true>(c, c->d_svals_c, d, q, c->d_part, (const KrylovState *)c->d_state);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_den_fin(c, (int)sell_grid(c));
}

}  // namespace cdfem
