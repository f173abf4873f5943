// reduce.hpp — deterministic block / grid reductions and the MFEM CG "den" step (device code).
//
// Grid reductions: every block publishes one partial; a one-block finalize kernel sums the
// partials in index order, so the result is bitwise reproducible and independent of dispatch
// order and XCD placement.
#pragma once
#include <hip/hip_runtime.h>

#include "cdfem_internal.hpp"

namespace cdfem {

constexpr int kRedThreads = 256;

__device__ inline double wave_sum(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// block sum, result valid in thread 0
__device__ inline double block_sum(double v, double *sh)
{
    v = wave_sum(v);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) sh[w] = v;
    __syncthreads();
    if (threadIdx.x < 64) {
        v = (threadIdx.x < ((blockDim.x + 63) >> 6)) ? sh[threadIdx.x] : 0.0;
        v = wave_sum(v);
    }
    return v;
}

// Each block stores its partial with a plain store; a separate one-block finalize kernel (the
// kernel boundary is the release/acquire) sums all partials in index order.  No atomics: a
// single-counter "last block" ticket costs ~12 ns per arriving block on MI355X
// (MI355X_MICROARCH.md, fanin row), i.e. ~12 us for a 1024-block grid.
__device__ inline void store_partial(double block_total, double *part)
{
    if (threadIdx.x == 0) part[blockIdx.x] = block_total;
}

// deterministic sum of part[0..n) by one block (fixed order), result valid in thread 0
// The loads of a thread are issued kB at a time before any is added: the partials were just
// written by blocks on all 8 XCDs, so each load is a far round trip, and a load-add loop pays one
// per partial per thread.  The adds keep the loop's order (out-of-range slots add +0.0, which
// leaves every sum unchanged), so the result is bitwise the same.
template <int kB = 8>
__device__ inline double sum_partials(const double *part, int n, double *sh)
{
    const int bd = blockDim.x;
    double v = 0.0;
    for (int i = threadIdx.x; i < n; i += kB * bd) {
        double a[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) a[k] = (i + k * bd < n) ? part[i + k * bd] : 0.0;
#pragma unroll
        for (int k = 0; k < kB; ++k) v += a[k];
    }
    return block_sum(v, sh);
}

// MFEM CGSolver after den = (d, A d): den == 0 stops (not converged); otherwise
// nom = betanom (the previous (r, z)) and alpha = nom / den.
__device__ inline void cg_den_step(KrylovState *st, double den)
{
    st->den = den;
    const int first = (st->first_den != 0);
    st->first_den = 0;
    if (den == 0.0) {
        st->done = 1;
        st->converged = 0;
        st->final_iter = first ? 0 : st->iter;
    } else {
        st->nom = st->betanom;  // (initial den: betanom == nom0)
        st->alpha = st->nom / den;
    }
}

// MFEM CGSolver's decision after betanom = (r, z) at iteration i: 0 go on, 1 breakdown (betanom < 0),
// 2 converged, 3 iteration bound.  The one definition of the stop test: cg_update_logic records it,
// and the betanom-fold apply (k_brick_cg<..., BF>) takes it in every workgroup with i from the host.
enum : int { kCgGoOn = 0, kCgBreakdown = 1, kCgConverged = 2, kCgMaxIter = 3 };
__device__ inline int cg_stop_kind(const KrylovState *st, double betanom, int i)
{
    if (betanom < 0.0) return kCgBreakdown;
    if (betanom <= st->r0) return kCgConverged;
    if (i + 1 > st->max_iter) return kCgMaxIter;
    return kCgGoOn;
}

// MFEM CGSolver after betanom = (r, z): convergence test, iteration bound, beta (at iteration i)
__device__ inline void cg_update_logic_at(KrylovState *st, double betanom, int i)
{
    st->betanom = betanom;
    switch (cg_stop_kind(st, betanom, i)) {
    case kCgBreakdown: st->done = 1; st->converged = 0; st->final_iter = i; st->xflush = 1; break;
    case kCgConverged: st->done = 1; st->converged = 1; st->final_iter = i; st->xflush = 1; break;
    case kCgMaxIter: st->done = 1; st->converged = 0; st->final_iter = st->max_iter; st->xflush = 1; break;
    default:
        st->beta = betanom / st->nom;
        st->iter = i + 1;
    }
}
__device__ inline void cg_update_logic(KrylovState *st, double betanom) { cg_update_logic_at(st, betanom, st->iter); }

// every block's copy of sum(part[0..n)), in one fixed order (so all blocks hold the same bits):
// thread t adds part[t], part[t + bd], ... (loads issued kB at a time), then the block tree;
// the result is returned in every thread (sh: >= blockDim / 64 + 1 doubles)
template <int kB = 8>
__device__ inline double sum_partials_all(const double *part, int n, double *sh)
{
    const double v = sum_partials<kB>(part, n, sh);
    __syncthreads();
    if (threadIdx.x == 0) sh[0] = v;
    __syncthreads();
    const double r = sh[0];
    __syncthreads();
    return r;
}

}  // namespace cdfem
