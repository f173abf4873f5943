// brick_kernels.hip — structured-box fast path: fused PA apply + E->L sum through LDS.
//
// On a structured box (BASELINE configs 2, 3, 5) the elements are grouped into 4x4x4 "bricks"
// of 64 elements = one wavefront = one workgroup.  A brick's dofs form an S^3 patch
// (S = 4p + 1: 9^3 = 729 at p = 2).  Per brick:
//   1. the patch of the input vector is gathered into LDS (in CG mode the new search direction
//      d = M^{-1} r + beta d is formed on the fly and written back for the dofs the brick owns);
//   2. each thread applies the fused D + C + M operator to its element (pa_core.hpp, registers);
//   3. the 64 element outputs are summed into a second LDS patch, one local dof at a time for
//      all lanes at once (for a fixed local dof the 64 target positions are distinct), so the
//      order of additions is fixed: deterministic, no atomics;
//   4. patch-interior dofs (owned by exactly this brick: (S-2)^3 = 343 of 729) are complete and
//      written to y directly; patch-face dofs go to a per-brick face buffer.
// k_brick_faces then sums, for every dof on a brick face, the (1, 2, 4 or 8) partials of the
// bricks sharing it, in a fixed order.  This replaces the E-vector round trip of the generic
// path (write + scattered re-read of 27 doubles per element) with 386 face partials per 64
// elements, and removes the element map and E->L index arrays from the stream entirely.
#include <hip/hip_runtime.h>

#include "cdfem_internal.hpp"
#include "pa_core.hpp"
#include "reduce.hpp"

namespace cdfem {

struct BrickGeom {
    int nbx, nby, nbz;  // bricks per axis
    int Lx, Ly, Lz;     // dof lattice per axis
};

// index of boundary position (a, b, c) of an S^3 patch in lexicographic order of the boundary set
template <int S>
__device__ __forceinline__ int face_index(int a, int b, int c)
{
    constexpr int ring = 4 * S - 4;
    if (c == 0) return a + S * b;
    if (c == S - 1) return S * S + (S - 2) * ring + a + S * b;
    const int base = S * S + (c - 1) * ring;
    if (b == 0) return base + a;
    if (b == S - 1) return base + S + 2 * (S - 2) + a;
    return base + S + 2 * (b - 1) + (a == S - 1 ? 1 : 0);
}

template <int S>
constexpr int face_count() { return 2 * S * S + (S - 2) * (4 * S - 4); }

// MODE 0: y = A x;  MODE 1: y = A_c x (ConstrainedOperator);  MODE 2: CG-fused (x := r)
template <int D1, int Q1, unsigned K, int MODE>
__global__ void __launch_bounds__(64)
k_brick3d(const double *__restrict__ x, const double *__restrict__ dinv, double *__restrict__ d,
          double *__restrict__ y, double *__restrict__ face, const double *__restrict__ qd,
          const uint8_t *__restrict__ ess, const Tab<D1, Q1> T, const BrickGeom g,
          double *__restrict__ part, const KrylovState *__restrict__ st)
{
    constexpr int P = D1 - 1;
    constexpr int S = kBrick * P + 1;
    constexpr int S2 = S * S, S3 = S * S * S;
    constexpr int F = face_count<S>();
    constexpr int NC = QLayout<K, 3>::nc;
    constexpr int NQ = Q1 * Q1 * Q1;
    __shared__ double s_in[S3];
    __shared__ double s_out[S3];

    double beta = 0.0;
    if constexpr (MODE == 2) {
        if (st->done) return;
        beta = st->beta;
    }
    const int t = threadIdx.x;
    const int b = blockIdx.x;
    const int bx = b % g.nbx, by = (b / g.nbx) % g.nby, bz = b / (g.nbx * g.nby);
    const int gx0 = (S - 1) * bx, gy0 = (S - 1) * by, gz0 = (S - 1) * bz;

    // 1. gather the input patch (zero outside the lattice and, when constrained, on ess dofs)
    for (int i = t; i < S3; i += 64) {
        const int px = i % S, py = (i / S) % S, pz = i / S2;
        const int gx = gx0 + px, gy = gy0 + py, gz = gz0 + pz;
        double v = 0.0;
        if (gx < g.Lx && gy < g.Ly && gz < g.Lz) {
            const int64_t gid = gx + (int64_t)g.Lx * (gy + (int64_t)g.Ly * gz);
            if constexpr (MODE == 2) {
                const double dn = dinv[gid] * x[gid] + beta * d[gid];
                const bool owned = px > 0 && px < S - 1 && py > 0 && py < S - 1 && pz > 0 && pz < S - 1;
                if (owned) d[gid] = dn;  // no other brick's patch contains this dof
                v = ess[gid] ? 0.0 : dn;
            } else {
                v = x[gid];
                if (MODE == 1 && ess[gid]) v = 0.0;
            }
        }
        s_in[i] = v;
        s_out[i] = 0.0;
    }
    __syncthreads();

    // 2. element apply
    const int ex = t & 3, ey = (t >> 2) & 3, ez = t >> 4;
    const int o0 = P * ez * S2 + P * ey * S + P * ex;
    double X[D1][D1][D1], Y[D1][D1][D1];
#pragma unroll
    for (int dz = 0; dz < D1; ++dz)
#pragma unroll
        for (int dy = 0; dy < D1; ++dy)
#pragma unroll
            for (int dx = 0; dx < D1; ++dx) X[dz][dy][dx] = s_in[o0 + dz * S2 + dy * S + dx];
    elem_apply3d<D1, Q1, K>(X, qd + (size_t)b * NQ * NC * kLanes + t, T, Y);

    // 3. deterministic E->L inside the brick: one local dof per step, all lanes distinct targets
#pragma unroll
    for (int dz = 0; dz < D1; ++dz)
#pragma unroll
        for (int dy = 0; dy < D1; ++dy)
#pragma unroll
            for (int dx = 0; dx < D1; ++dx) {
                const int o = o0 + dz * S2 + dy * S + dx;
                s_out[o] += Y[dz][dy][dx];
                __syncthreads();
            }

    // 4. owned dofs -> y, face dofs -> partial buffer
    double acc = 0.0;
    for (int i = t; i < S3; i += 64) {
        const int px = i % S, py = (i / S) % S, pz = i / S2;
        const double v = s_out[i];
        const bool onface = px == 0 || px == S - 1 || py == 0 || py == S - 1 || pz == 0 || pz == S - 1;
        if (onface) {
            face[(size_t)b * F + face_index<S>(px, py, pz)] = v;
            continue;
        }
        const int gx = gx0 + px, gy = gy0 + py, gz = gz0 + pz;
        if (gx >= g.Lx || gy >= g.Ly || gz >= g.Lz) continue;
        const int64_t gid = gx + (int64_t)g.Lx * (gy + (int64_t)g.Ly * gz);
        if constexpr (MODE == 0) {
            y[gid] = v;
        } else if constexpr (MODE == 1) {
            y[gid] = ess[gid] ? x[gid] : v;
        } else {
            const bool e = ess[gid] != 0;
            const double dn = e ? d[gid] : s_in[i];  // this thread wrote d[gid] in step 1
            const double q = e ? dn : v;
            y[gid] = q;
            acc += dn * q;
        }
    }
    if constexpr (MODE == 2) {
        acc = wave_sum(acc);
        if (t == 0) part[b] = acc;
    }
}

// sum the brick-face partials of every dof lying on a brick face
template <int S, int MODE>
__global__ void __launch_bounds__(kRedThreads)
k_brick_faces(const double *__restrict__ x, const double *__restrict__ dinv, double *__restrict__ d,
              double *__restrict__ y, const double *__restrict__ face, const uint8_t *__restrict__ ess,
              const BrickGeom g, double *__restrict__ part, int n_apply_parts,
              KrylovState *__restrict__ st)
{
    constexpr int F = face_count<S>();
    constexpr int s1 = S - 1;
    __shared__ double sh[kRedThreads / 64];
    __shared__ int sh_last;
    double beta = 0.0;
    if constexpr (MODE == 2) {
        if (st->done) return;
        beta = st->beta;
    }
    const int64_t n = (int64_t)g.Lx * g.Ly * g.Lz;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    double acc = 0.0;
    for (int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; gid < n; gid += stride) {
        const int gx = (int)(gid % g.Lx), gy = (int)((gid / g.Lx) % g.Ly), gz = (int)(gid / ((int64_t)g.Lx * g.Ly));
        const bool fx = gx % s1 == 0, fy = gy % s1 == 0, fz = gz % s1 == 0;
        if (!(fx || fy || fz)) continue;
        int bxs[2], pxs[2], nxc = 0, bys[2], pys[2], nyc = 0, bzs[2], pzs[2], nzc = 0;
        auto cand = [](int gc, bool f, int nb, int *bs, int *ps, int &nc) {
            const int q = gc / s1;
            if (f) {
                if (q - 1 >= 0 && q - 1 < nb) { bs[nc] = q - 1; ps[nc] = s1; ++nc; }
                if (q < nb) { bs[nc] = q; ps[nc] = 0; ++nc; }
            } else {
                bs[0] = q; ps[0] = gc - q * s1; nc = 1;
            }
        };
        cand(gx, fx, g.nbx, bxs, pxs, nxc);
        cand(gy, fy, g.nby, bys, pys, nyc);
        cand(gz, fz, g.nbz, bzs, pzs, nzc);
        double sum = 0.0;
        for (int kz = 0; kz < nzc; ++kz)
            for (int ky = 0; ky < nyc; ++ky)
                for (int kx = 0; kx < nxc; ++kx) {
                    const int bb = bxs[kx] + g.nbx * (bys[ky] + g.nby * bzs[kz]);
                    sum += face[(size_t)bb * F + face_index<S>(pxs[kx], pys[ky], pzs[kz])];
                }
        if constexpr (MODE == 0) {
            y[gid] = sum;
        } else if constexpr (MODE == 1) {
            y[gid] = ess[gid] ? x[gid] : sum;
        } else {
            const double dn = dinv[gid] * x[gid] + beta * d[gid];
            d[gid] = dn;
            const double q = ess[gid] ? dn : sum;
            y[gid] = q;
            acc += dn * q;
        }
    }
    if constexpr (MODE == 2) {
        const double bs = block_sum(acc, sh);
        if (!publish_partial(bs, part + n_apply_parts, &st->cnt[0], &sh_last)) return;
        // den = sum over the apply kernel's per-brick partials, then this kernel's, fixed order
        double v = 0.0;
        for (int i = threadIdx.x; i < n_apply_parts + (int)gridDim.x; i += blockDim.x) v += part[i];
        const double den = block_sum(v, sh);
        if (threadIdx.x == 0) {
            st->cnt[0] = 0;
            cg_den_step(st, den);
        }
    }
}

// ------------------------------------------------------------------------------------------------
bool brick_supported(int dim, int p) { return dim == 3 && (p == 1 || p == 2); }

static BrickGeom geom_of(const cdfem_ctx *c)
{
    return BrickGeom{c->nbx, c->nby, c->nbz, (int)c->Lx, (int)c->Ly, (int)c->Lz};
}

static unsigned faces_grid(const cdfem_ctx *c)
{
    const int64_t need = (c->nl + kRedThreads - 1) / kRedThreads;
    return (unsigned)(need < c->red_blocks ? (need < 1 ? 1 : need) : c->red_blocks);
}

template <int D1, int Q1, unsigned K, int MODE>
static hipError_t brick_launch(cdfem_ctx *c, const double *x, const double *dinv, double *d, double *y,
                               int which)
{
    constexpr int S = kBrick * (D1 - 1) + 1;
    const BrickGeom g = geom_of(c);
    if (which & 1) {
        const Tab<D1, Q1> T = make_tab<D1, Q1>(c->rule_op);
        hipLaunchKernelGGL((k_brick3d<D1, Q1, K, MODE>), dim3(c->nblk), dim3(64), 0, c->stream, x, dinv,
                           d, y, c->d_face, c->d_qd, c->d_ess, T, g, c->d_part, c->d_state);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (which & 2)
        hipLaunchKernelGGL((k_brick_faces<S, MODE>), dim3(faces_grid(c)), dim3(kRedThreads), 0,
                           c->stream, x, dinv, d, y, c->d_face, c->d_ess, g, c->d_part, c->nblk,
                           c->d_state);
    return hipGetLastError();
}

template <int D1, int Q1, int MODE>
static hipError_t brick_kinds(cdfem_ctx *c, const double *x, const double *dinv, double *d, double *y,
                              int which)
{
    switch (c->kinds) {
    case 1: return brick_launch<D1, Q1, 1, MODE>(c, x, dinv, d, y, which);
    case 2: return brick_launch<D1, Q1, 2, MODE>(c, x, dinv, d, y, which);
    case 3: return brick_launch<D1, Q1, 3, MODE>(c, x, dinv, d, y, which);
    case 4: return brick_launch<D1, Q1, 4, MODE>(c, x, dinv, d, y, which);
    case 5: return brick_launch<D1, Q1, 5, MODE>(c, x, dinv, d, y, which);
    case 6: return brick_launch<D1, Q1, 6, MODE>(c, x, dinv, d, y, which);
    case 7: return brick_launch<D1, Q1, 7, MODE>(c, x, dinv, d, y, which);
    default: return hipErrorInvalidValue;
    }
}

template <int MODE>
static hipError_t brick_dispatch(cdfem_ctx *c, const double *x, const double *dinv, double *d, double *y,
                                 int which)
{
    const int q1 = c->rule_op.q1;
    if (c->p == 1 && q1 == 3) return brick_kinds<2, 3, MODE>(c, x, dinv, d, y, which);
    if (c->p == 2 && q1 == 4) return brick_kinds<3, 4, MODE>(c, x, dinv, d, y, which);
    return hipErrorInvalidValue;
}

hipError_t launch_brick_mult(cdfem_ctx *c, const double *x, double *y, bool constrained, int which)
{
    return constrained ? brick_dispatch<1>(c, x, nullptr, nullptr, y, which)
                       : brick_dispatch<0>(c, x, nullptr, nullptr, y, which);
}

hipError_t launch_brick_cg(cdfem_ctx *c, const double *r, const double *dinv, double *d, double *q,
                           int which)
{
    return brick_dispatch<2>(c, r, dinv, d, q, which);
}

}  // namespace cdfem
