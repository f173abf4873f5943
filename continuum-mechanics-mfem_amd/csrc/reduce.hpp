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
// kernel boundary is the release/acquire) sums all partials in index order.  On one rank the hot
// CG / GMRES reductions finish in-launch instead (ticket_sum below); no atomics touch data.
__device__ inline void store_partial(double block_total, double *part)
{
    if (threadIdx.x == 0) part[blockIdx.x] = block_total;
}

// deterministic sum of part[0..n) by one block (fixed order), result valid in thread 0
// The loads of a thread are issued kB at a time before any is added: the partials were just
// written by blocks on all 8 XCDs, so each load is a far round trip, and a load-add loop pays one
// per partial per thread.  The adds keep the loop's order (out-of-range slots add +0.0, which
// leaves every sum unchanged), so the result is bitwise the same.
__device__ inline double sum_partials(const double *part, int n, double *sh)
{
    constexpr int kB = 8;
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

// ---- grid sum finished inside the producing launch (no one-block finalize kernel) ---------------
// Blocks are split into 8 groups by blockIdx % 8 (the dispatcher deals blocks round-robin over the
// 8 XCDs, so a group is mostly one XCD's blocks; placement only affects speed).  Each block stores
// its partial write-through (sc1), drains it, and draws a ticket on its group's counter; the block
// drawing the group's last ticket sums the group's partials in index order and draws a ticket on
// the top counter; the block drawing the last top ticket sums the 8 group sums in order.  Every
// sum has a fixed order whichever block arrives last: bitwise reproducible.  The hand-off is the
// write-through form of MI355X_MICROARCH.md's visibility table (sc1 stores, vmcnt(0) before the
// counter add, sc1 loads by the block the returned ticket names): no L2 write-back fence.
// Counters are zero at allocation and reset by the block that drew their last ticket; every block
// of a launch draws exactly one group ticket (kernels that exit early do so in every block).
// (GridTicket: cdfem_internal.hpp.)
__device__ inline void sc1_store(double *p, double v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline double sc1_load(const double *p)
{
    return __hip_atomic_load(const_cast<double *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// block_total valid in thread 0 (block_sum's result).  Returns true in every thread of the one
// block that completes the grid sum; *total is then valid in its thread 0.  flag: an LDS int.
__device__ inline bool ticket_sum(double block_total, double *part, GridTicket *tk, double *sh, int *flag,
                                  double *total)
{
    const unsigned nb = gridDim.x, b = blockIdx.x;
    const unsigned ng = nb < 8 ? nb : 8, g = b & 7u;
    const unsigned n_g = (nb - g + 7u) >> 3;  // blocks g, g + 8, ...
    if (threadIdx.x == 0) {
        sc1_store(part + b, block_total);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev = __hip_atomic_fetch_add(&tk->grp[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = prev == n_g - 1u;
    }
    __syncthreads();
    if (!*flag) return false;
    double v = 0.0;
    for (unsigned i = threadIdx.x; i < n_g; i += blockDim.x) v += sc1_load(part + g + 8u * i);
    v = block_sum(v, sh);
    if (threadIdx.x == 0) {
        __hip_atomic_store(&tk->grp[g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sc1_store(&tk->gsum[g], v);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev = __hip_atomic_fetch_add(&tk->top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = prev == ng - 1u;
    }
    __syncthreads();
    if (!*flag) return false;
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (unsigned k = 0; k < ng; ++k) t += sc1_load(&tk->gsum[k]);
        *total = t;
        __hip_atomic_store(&tk->top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return true;
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

// MFEM CGSolver after betanom = (r, z): convergence test, iteration bound, beta
__device__ inline void cg_update_logic(KrylovState *st, double betanom)
{
    st->betanom = betanom;
    const int i = st->iter;
    if (betanom < 0.0) {
        st->done = 1; st->converged = 0; st->final_iter = i;
    } else if (betanom <= st->r0) {
        st->done = 1; st->converged = 1; st->final_iter = i;
    } else if (i + 1 > st->max_iter) {
        st->done = 1; st->converged = 0; st->final_iter = st->max_iter;
    } else {
        st->beta = betanom / st->nom;
        st->iter = i + 1;
    }
}

}  // namespace cdfem
