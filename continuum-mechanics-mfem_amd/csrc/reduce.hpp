// reduce.hpp — deterministic block / grid reductions and the MFEM CG "den" step (device code).
//
// Grid reductions: every block publishes one partial; the LAST arriving block (agent-scope
// release before the ticket, acquire after it: MI355X_MICROARCH.md "Valid forms") sums the
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
        v = (threadIdx.x < (blockDim.x >> 6)) ? sh[threadIdx.x] : 0.0;
        v = wave_sum(v);
    }
    return v;
}

// Publish this block's partial and find out whether it is the last arriver.  Producer side: plain
// store, every wave drains vmcnt, barrier, lane-0 agent release, asm drain, relaxed agent ticket.
// The last arriver then acquires (agent) before reading other blocks' partials.
__device__ inline bool publish_partial(double v, double *part, unsigned *cnt, int *sh_last)
{
    if (threadIdx.x == 0) part[blockIdx.x] = v;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = (prev == gridDim.x - 1);
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *sh_last = last ? 1 : 0;
    }
    __syncthreads();
    return *sh_last != 0;
}

// deterministic sum of part[0..n) by one block (fixed order), result in thread 0
__device__ inline double sum_partials(const double *part, int n, double *sh)
{
    double v = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) v += part[i];
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

}  // namespace cdfem
