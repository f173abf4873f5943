// brick_geom.hpp — structured-box brick geometry shared by the brick kernels (brick_kernels.hip)
// and the kernels that consume brick-face partial sums (the CG update, the GMRES pass 1).
//
// A brick is kBrick^3 elements; its dofs form an S^3 patch (S = kBrick p + 1).  Patch-interior dofs
// belong to one brick; a dof on a brick face (lattice coordinate a multiple of s1 = S - 1 along some
// axis) is shared by the 2, 4 or 8 bricks around it, each of which stores its partial sum in its
// face buffer (F = face_count<S>() values per brick, boundary-lexicographic order, face_index).
#pragma once
#include <hip/hip_runtime.h>

#include "cdfem_internal.hpp"
#include "pa_core.hpp"

namespace cdfem {

struct BrickGeom {
    int nbx, nby, nbz;  // bricks per axis
    int Lx, Ly, Lz;     // dof lattice per axis
    int xcd;            // 1: XCD-contiguous brick order (default; set_option "brick_xcd")
    int bz0, bzs;       // k_brick_cg: the launch covers brick layers bz0, bz0 + bzs, ... (all: 0, 1)
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

template <int S>
__device__ __forceinline__ bool on_brick_face(int gx, int gy, int gz)
{
    constexpr int s1 = S - 1;
    return gx % s1 == 0 || gy % s1 == 0 || gz % s1 == 0;
}

// the bricks holding lattice coordinate q along one axis and the patch coordinate in each
// (1 brick inside a brick, 2 on a brick boundary, 1 at the lattice ends)
template <int S>
__device__ __forceinline__ int brick_axis(int gq, int nb, int *bq, int *pq)
{
    constexpr int s1 = S - 1;
    const int qq = gq / s1;
    int n = 0;
    if (gq - qq * s1 == 0) {
        if (qq - 1 >= 0) { bq[n] = qq - 1; pq[n] = s1; ++n; }
        if (qq < nb) { bq[n] = qq; pq[n] = 0; ++n; }
    } else {
        bq[0] = qq; pq[0] = gq - qq * s1; n = 1;
    }
    return n;
}

// sum of the face partials of a brick-face dof, bricks in a fixed (z, y, x) order
template <int S>
__device__ __forceinline__ double brick_face_sum(int gx, int gy, int gz, const BrickGeom &g,
                                                 const double *__restrict__ face)
{
    constexpr int F = face_count<S>();
    int bxs[2], pxs[2], bys[2], pys[2], bzs[2], pzs[2];
    const int nxc = brick_axis<S>(gx, g.nbx, bxs, pxs);
    const int nyc = brick_axis<S>(gy, g.nby, bys, pys);
    const int nzc = brick_axis<S>(gz, g.nbz, bzs, pzs);
    double sum = 0.0;
    for (int kz = 0; kz < nzc; ++kz)
        for (int ky = 0; ky < nyc; ++ky)
            for (int kx = 0; kx < nxc; ++kx) {
                const int bb = bxs[kx] + g.nbx * (bys[ky] + g.nby * bzs[kz]);
                sum += face[(size_t)bb * F + face_index<S>(pxs[kx], pys[ky], pzs[kz])];
            }
    return sum;
}

// GMRES pass 1 on a brick apply whose face dofs are still partials (k_brick3d<MODE 1> without
// k_brick_faces): the constrained operator's value of dof k is x_k on essential dofs, the face sum
// on brick-face dofs, and the brick's own store otherwise
struct GmFaces {
    const double *face;
    const uint8_t *ess;
    const double *x;  // the operator's input (V_j)
    BrickGeom g;
    FastDiv fdx, fdxy;
    int s;            // S (dispatch)
};

}  // namespace cdfem
