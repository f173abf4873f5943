// brick_common.hpp — the brick decomposition of a structured box (brick_kernels.hip) as seen by
// kernels outside it: the face-partial layout of a brick's S^3 patch and the fixed-order sum of the
// partials of a dof on a brick face.
#pragma once
#include <hip/hip_runtime.h>

namespace cdfem {

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

// (A x)_i of a dof on a brick face: the partials of the (1, 2, 4 or 8) bricks sharing it, summed
// z-outer / x-inner over the bricks (the order k_brick_faces and k_cg_update_faces use)
template <int S>
__device__ __forceinline__ double brick_face_sum(const double *__restrict__ face, int gx, int gy, int gz, int nbx,
                                                 int nby, int nbz)
{
    constexpr int F = face_count<S>();
    constexpr int s1 = S - 1;
    int bxs[2], pxs[2], nxc = 0, bys[2], pys[2], nyc = 0, bzs[2], pzs[2], nzc = 0;
    const int qx = gx / s1, qy = gy / s1, qz = gz / s1;
    if (gx - qx * s1 == 0) {
        if (qx - 1 >= 0) { bxs[nxc] = qx - 1; pxs[nxc] = s1; ++nxc; }
        if (qx < nbx) { bxs[nxc] = qx; pxs[nxc] = 0; ++nxc; }
    } else { bxs[0] = qx; pxs[0] = gx - qx * s1; nxc = 1; }
    if (gy - qy * s1 == 0) {
        if (qy - 1 >= 0) { bys[nyc] = qy - 1; pys[nyc] = s1; ++nyc; }
        if (qy < nby) { bys[nyc] = qy; pys[nyc] = 0; ++nyc; }
    } else { bys[0] = qy; pys[0] = gy - qy * s1; nyc = 1; }
    if (gz - qz * s1 == 0) {
        if (qz - 1 >= 0) { bzs[nzc] = qz - 1; pzs[nzc] = s1; ++nzc; }
        if (qz < nbz) { bzs[nzc] = qz; pzs[nzc] = 0; ++nzc; }
    } else { bzs[0] = qz; pzs[0] = gz - qz * s1; nzc = 1; }
    double v = 0.0;
    for (int kz = 0; kz < nzc; ++kz)
        for (int ky = 0; ky < nyc; ++ky)
            for (int kx = 0; kx < nxc; ++kx) {
                const int bb = bxs[kx] + nbx * (bys[ky] + nby * bzs[kz]);
                v += face[(size_t)bb * F + face_index<S>(pxs[kx], pys[ky], pzs[kz])];
            }
    return v;
}

}  // namespace cdfem
