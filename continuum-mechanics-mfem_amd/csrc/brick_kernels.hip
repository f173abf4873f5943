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

#include <type_traits>
#include <vector>
#include <algorithm>
#include <cmath>

#include "cdfem_internal.hpp"
#include "brick_core.hpp"
#include "pa_core.hpp"
#include "reduce.hpp"

// LDS of the brick CG apply (k_brick_cg): 0 = three linear S^3 patches (in, out, essential d), 1 = the
// essential d in registers, 2 = that plus the padded patch pitch
#ifndef CDFEM_BRICK_LDS
#define CDFEM_BRICK_LDS 1
#endif

namespace cdfem {

// workgroup b runs on XCD b % 8; with xcd = 1 each XCD takes a contiguous range of bricks, so a
// brick's neighbours (which re-read its patch faces) are mostly on the same L2.  Measured in
// process (tools/ab.py, 64^3 p=2, two boxes): 242.8 vs 258.6 us per k_brick_cg launch; at 256^3
// no difference (14444 vs 14470 us).
__device__ __forceinline__ int brick_id(const BrickGeom &g)
{
    if (!g.xcd) return blockIdx.x;
    const unsigned G = gridDim.x, b = blockIdx.x, x = b % 8, k = b / 8, q = G / 8, r = G % 8;
    return (int)(x * q + (x < r ? x : r) + k);
}

// Patch positions i = t, t + STEP, t + 2 STEP, ... of an S^3 patch (x fastest), advanced incrementally:
// STEP = dz S^2 + dy S + dx, so each step adds (dx, dy, dz) with carries (a few adds and selects
// instead of two constant divisions per position; STEP < S^3)
template <int S, int STEP = 64>
struct PatchWalk {
    int x, y, z;
    __device__ __forceinline__ explicit PatchWalk(unsigned t) : x((int)(t % S)), y((int)((t / S) % S)), z((int)(t / (S * S))) {}
    __device__ __forceinline__ void next()
    {
        constexpr int dx = STEP % S, dy = (STEP / S) % S, dz = STEP / (S * S);
        x += dx;
        const int cx = x >= S ? 1 : 0;
        x -= S & -cx;
        y += dy + cx;
        const int cy = y >= S ? 1 : 0;
        y -= S & -cy;
        z += dz + cy;
    }
};

// PatchWalk plus the lattice index gid = gx + Lx gy + Lxy gz of the position, advanced with the walk's
// carries (no per-position 32-bit multiplies: v_mul_lo_u32 issues at a quarter of the VALU rate)
template <int S, int STEP = 64>
struct LatWalk {
    int x, y, z;
    uint32_t gid;
    __device__ __forceinline__ LatWalk(unsigned t, uint32_t g0, uint32_t Lx, uint32_t Lxy)
        : x((int)(t % S)), y((int)((t / S) % S)), z((int)(t / (S * S)))
    {
        gid = g0 + (uint32_t)x + Lx * (uint32_t)y + Lxy * (uint32_t)z;
    }
    __device__ __forceinline__ void next(uint32_t dgid, uint32_t cxd, uint32_t cyd)
    {
        constexpr int dx = STEP % S, dy = (STEP / S) % S, dz = STEP / (S * S);
        x += dx;
        const int cx = x >= S ? 1 : 0;
        x -= S & -cx;
        y += dy + cx;
        const int cy = y >= S ? 1 : 0;
        y -= S & -cy;
        z += dz + cy;
        // dgid = dx + dy Lx + dz Lxy; a carry out of x adds Lx - S, out of y Lxy - S Lx
        gid += dgid + (cxd & (uint32_t)-cx) + (cyd & (uint32_t)-cy);
    }
};

// index of boundary position (a, b, c) of an S^3 patch in lexicographic order of the boundary set.
// Bit-mask selects, no ?: on expressions: the callers run it in every lane, and the compiler turns
// conditional expressions into divergent branches.
__device__ __forceinline__ int bsel(bool c, int a, int b)
{
    const int m = -(int)c;
    return (a & m) | (b & ~m);
}
template <int S>
__device__ __forceinline__ int face_index(int a, int b, int c)
{
    constexpr int ring = 4 * S - 4;
    const int cap = a + S * b;                                   // planes c == 0 and c == S - 1
    const int mid = bsel(b == 0, a, bsel(b == S - 1, S + 2 * (S - 2) + a, S + 2 * (b - 1) + (int)(a == S - 1)));
    return bsel(c == 0, cap, bsel(c == S - 1, S * S + (S - 2) * ring + cap, S * S + (c - 1) * ring + mid));
}

template <int S>
constexpr int face_count() { return 2 * S * S + (S - 2) * (4 * S - 4); }

// The CG apply's patch-output buffer, x rows of the brick lattice contiguous ([bz][pz][by][py][bx][px]):
// a brick writes 81 runs of S, and the update kernel's wave over a lattice x row reads one contiguous
// run (each dof's 1-8 entries: its own brick's, plus the neighbours' on brick faces)
template <int S, int SZ = S>
__device__ __forceinline__ size_t patch_idx(const BrickGeom &g, int bx, int by, int bz, int px, int py, int pz)
{
    return ((((size_t)bz * SZ + pz) * g.nby + by) * S + py) * ((size_t)g.nbx * S) + (size_t)bx * S + px;
}

// f(std::integral_constant<int, k>) for k = B .. E - 1, unrolled at compile time (array indices
// stay compile-time, so the arrays stay in registers)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F &&f)
{
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// v unchanged, but opaque to the optimiser: index arithmetic that depends on it cannot be hoisted
// above this point (LLVM otherwise computes a later phase's per-position indices at kernel entry
// and spills them across the element apply)
__device__ __forceinline__ int opaque(int v)
{
    asm volatile("" : "+v"(v));
    return v;
}

// In-LDS E->L schedule.  At P = 2 an element's local dof d lands on patch position 2e + d per axis,
// so two (element, local dof) pairs meet on one position only if their local dofs agree mod 2: the
// 27 local dofs split into 8 parity classes (dx & 1, dy & 1, dz & 1) of 8, 4, 4, 2, 4, 2, 2, 1 dofs
// that never collide with each other, and round r adds member r of every class (8 rounds instead of
// one dof per step, 27).  Member r of class cls (members in lexicographic order), -1 past the end.
__host__ __device__ constexpr int e2l_member(int cls, int r)
{
    const int a = cls & 1, b = (cls >> 1) & 1, c = (cls >> 2) & 1;
    const int nx = a ? 1 : 2, ny = b ? 1 : 2, nz = c ? 1 : 2;
    if (r >= nx * ny * nz) return -1;
    const int ix = r % nx, iy = (r / nx) % ny, iz = r / (nx * ny);
    const int dx = a ? 1 : 2 * ix, dy = b ? 1 : 2 * iy, dz = c ? 1 : 2 * iz;
    return dx + 3 * (dy + 3 * dz);
}

// s_out[o0 + patch offset of local dof] += Y for the 64 elements of a brick, deterministic order
// (patch strides SY per row, S2 per plane in LDS: S, S^2 unpadded)
template <int D1, int S, int SY = S, int S2 = S * S>
__device__ __forceinline__ void brick_e2l(double *s_out, int o0, const double (&Y)[D1][D1][D1])
{
    if constexpr (D1 == 3) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
#pragma unroll
            for (int cls = 0; cls < 8; ++cls) {
                const int l = e2l_member(cls, r);
                if (l < 0) continue;
                const int dz = l / 9, dy = (l / 3) % 3, dx = l % 3;
                s_out[o0 + dz * S2 + dy * SY + dx] += Y[dz][dy][dx];
            }
            __syncthreads();
        }
    } else {
        // P = 1: every pair of local dofs can meet (positions e + d), one dof per step
#pragma unroll
        for (int dz = 0; dz < D1; ++dz)
#pragma unroll
            for (int dy = 0; dy < D1; ++dy)
#pragma unroll
                for (int dx = 0; dx < D1; ++dx) {
                    s_out[o0 + dz * S2 + dy * SY + dx] += Y[dz][dy][dx];
                    __syncthreads();
                }
    }
}

// MODE 0: y = A x;  MODE 1: y = A_c x (ConstrainedOperator).  (The CG loop runs k_brick_cg.)
// PBO (set_option "brick_mult_pb"): the whole patch sum goes to the patch buffer (patch_idx, as the CG
// kernel writes it) and k_brick_patch_sum forms y; otherwise owned dofs go to y, face dofs to the
// brick's face partials (k_brick_faces).
// One wave per SIMD with the per-point stream, unconstrained registers: 241.5 vs 272.2 us per C2
// apply in the GMRES leg against a two-waves-per-SIMD build (<= 256 registers, 124 B/lane of
// spills; tools/ab_gmres.py, profiles/r02_ab_c2_gmres_brick_waves.txt); two with the Kronecker form.
template <int D1, int Q1, unsigned K, int MODE, int AF, bool PBO = false>
__global__ void __launch_bounds__(64, AF == 2 ? 2 : 1)
k_brick3d(const double *__restrict__ x, double *__restrict__ y, double *__restrict__ face,
          const double *__restrict__ qd, const uint8_t *__restrict__ ess, const Tab<D1, Q1> T, const BrickGeom g)
{
    constexpr int P = D1 - 1;
    constexpr int S = kBrick * P + 1;
    constexpr int S2 = S * S, S3 = S * S * S;
    constexpr int F = face_count<S>();
    constexpr int NC = QLayout<K, 3>::nc;
    constexpr int NQ = Q1 * Q1 * Q1;
    constexpr int NI = (S3 + 63) / 64;
    __shared__ double s_in[S3];
    __shared__ double s_out[S3];

    const int t = threadIdx.x;
    const int b = blockIdx.x;
    const int bx = b % g.nbx, by = (b / g.nbx) % g.nby, bz = b / (g.nbx * g.nby);
    const int gx0 = (S - 1) * bx, gy0 = (S - 1) * by, gz0 = (S - 1) * bz;
    const int Lx = g.Lx, Lxy = g.Lx * g.Ly;

    // 1. gather the input patch (zero outside the lattice and, when constrained, on ess dofs);
    //    every load issued before any is consumed
    double xv[NI];
    uint8_t ev[NI];
    bool inv[NI];
    PatchWalk<S> pw0(t);
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const unsigned i = t + 64 * k;
        const int px = pw0.x, py = pw0.y, pz = pw0.z;
        pw0.next();
        const int gx = gx0 + px, gy = gy0 + py, gz = gz0 + pz;
        inv[k] = i < S3 && gx < g.Lx && gy < g.Ly && gz < g.Lz;
        const int gid = inv[k] ? gx + Lx * gy + Lxy * gz : 0;
        xv[k] = x[gid];
        ev[k] = MODE == 1 ? ess[gid] : 0;
    }
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const unsigned i = t + 64 * k;
        if (k == NI - 1 && i >= S3) break;
        s_in[i] = (inv[k] && !ev[k]) ? xv[k] : 0.0;
        s_out[i] = 0.0;
    }
    __syncthreads();

    // 2. element apply
    const int ex = t & 3, ey = (t >> 2) & 3, ez = t >> 4;
    const int o0 = P * ez * S2 + P * ey * S + P * ex;
    double Y[D1][D1][D1];
    auto xl = [&](int dz, int dy, int dx) { return s_in[o0 + dz * S2 + dy * S + dx]; };
    elem_apply3d_af<D1, Q1, K, AF>(xl, qd + (size_t)b * (AF ? 1 : NQ) * NC * kLanes, t, T, Y);

    // 3. deterministic E->L inside the brick (brick_e2l: all lanes of a step write distinct targets)
    brick_e2l<D1, S>(s_out, o0, Y);

    if constexpr (PBO) {
        // 4'. the whole patch -> the patch buffer (32-bit index: base + pz A + py R + px)
        const uint32_t R = (uint32_t)g.nbx * S, A = (uint32_t)g.nby * S * R;
        const int bxp = b % g.nbx, byp = (b / g.nbx) % g.nby, bzp = b / (g.nbx * g.nby);
        const uint32_t base = (uint32_t)bzp * S * A + (uint32_t)byp * S * R + (uint32_t)bxp * S;
        const auto bp = brsrc(face, 8u * (uint32_t)g.nbx * g.nby * g.nbz * S3);
        const unsigned tp = (unsigned)opaque(t);
        PatchWalk<S> pw(tp);
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const unsigned i = tp + 64 * k;
            if (k == NI - 1 && i >= S3) break;
            bstore(bp, 8u * (base + (uint32_t)pw.z * A + (uint32_t)pw.y * R + (uint32_t)pw.x), s_out[i]);
            pw.next();
        }
        return;
    }
    // 4. owned dofs -> y (constrained: y = x on ess rows), face dofs -> this brick's partials
    double *const fb = face + (size_t)b * F;
    const unsigned to = (unsigned)opaque(t);
    PatchWalk<S> pw1(to);
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const unsigned i = to + 64 * k;
        const int px = pw1.x, py = pw1.y, pz = pw1.z;
        pw1.next();
        const bool onface = px == 0 || px == S - 1 || py == 0 || py == S - 1 || pz == 0 || pz == S - 1;
        const int gx = gx0 + px, gy = gy0 + py, gz = gz0 + pz;
        const bool in = i < S3 && gx < g.Lx && gy < g.Ly && gz < g.Lz;
        if (in && !onface) {
            const int gid = gx + Lx * gy + Lxy * gz;
            const double v = s_out[i];
            if constexpr (MODE == 0) y[gid] = v;
            else y[gid] = ess[gid] ? x[gid] : v;
        }
    }
    PatchWalk<S> pw2(to);
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const unsigned i = to + 64 * k;
        const int px = pw2.x, py = pw2.y, pz = pw2.z;
        pw2.next();
        const bool onface = px == 0 || px == S - 1 || py == 0 || py == S - 1 || pz == 0 || pz == S - 1;
        if (i < S3 && onface) fb[face_index<S>(px, py, pz)] = s_out[i];
    }
}

// Sum the brick-face partials of every dof lying on a brick face: one thread per face dof.
// Grid (x, z-plane): a plane gz = multiple of 4p is all face dofs; any other plane holds full
// lines (gy = multiple of 4p) and, on the remaining lines, the dofs gx = 0, 4p, 8p, ...
// CG mode also forms d = M^{-1} r + beta d for these dofs and the partial (d, A d).
template <int S, int MODE>
__global__ void __launch_bounds__(kRedThreads)
k_brick_faces(const double *__restrict__ x, const double *__restrict__ dinv, double *__restrict__ d,
              double *__restrict__ y, const double *__restrict__ face, const uint8_t *__restrict__ ess,
              const BrickGeom g, double *__restrict__ part, const KrylovState *__restrict__ st)
{
    constexpr int F = face_count<S>();
    constexpr int s1 = S - 1;
    __shared__ double sh[kRedThreads / 64];
    double beta = 0.0;
    if constexpr (MODE == 2) {
        if (st->done) return;
        beta = st->beta;
    }
    const int gz = blockIdx.y;
    const bool fz = gz % s1 == 0;
    const int Lx = g.Lx, Ly = g.Ly;
    const int nfx = (Lx - 1) / s1 + 1, nfy = (Ly - 1) / s1 + 1;
    const int per = Lx + (s1 - 1) * nfx;                     // dofs per s1-line period (sparse plane)
    const int count = fz ? Lx * Ly : nfy * Lx + (Ly - nfy) * nfx;
    int bzs[2], pzs[2], nzc = 0;
    {
        const int qz = gz / s1;
        if (fz) {
            if (qz - 1 >= 0) { bzs[nzc] = qz - 1; pzs[nzc] = s1; ++nzc; }
            if (qz < g.nbz) { bzs[nzc] = qz; pzs[nzc] = 0; ++nzc; }
        } else { bzs[0] = qz; pzs[0] = gz - qz * s1; nzc = 1; }
    }
    double acc = 0.0;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < count; k += gridDim.x * blockDim.x) {
        int gx, gy;
        if (fz) {
            gy = k / Lx; gx = k - gy * Lx;
        } else {
            const int pi = k / per, rem = k - pi * per;
            if (rem < Lx) { gy = s1 * pi; gx = rem; }
            else { const int j = rem - Lx, jl = j / nfx; gy = s1 * pi + 1 + jl; gx = (j - jl * nfx) * s1; }
        }
        int bxs[2], pxs[2], nxc = 0, bys[2], pys[2], nyc = 0;
        {
            const int qx = gx / s1, qy = gy / s1;
            if (gx - qx * s1 == 0) {
                if (qx - 1 >= 0) { bxs[nxc] = qx - 1; pxs[nxc] = s1; ++nxc; }
                if (qx < g.nbx) { bxs[nxc] = qx; pxs[nxc] = 0; ++nxc; }
            } else { bxs[0] = qx; pxs[0] = gx - qx * s1; nxc = 1; }
            if (gy - qy * s1 == 0) {
                if (qy - 1 >= 0) { bys[nyc] = qy - 1; pys[nyc] = s1; ++nyc; }
                if (qy < g.nby) { bys[nyc] = qy; pys[nyc] = 0; ++nyc; }
            } else { bys[0] = qy; pys[0] = gy - qy * s1; nyc = 1; }
        }
        double sum = 0.0;
        for (int kz = 0; kz < nzc; ++kz)
            for (int ky = 0; ky < nyc; ++ky)
                for (int kx = 0; kx < nxc; ++kx) {
                    const int bb = bxs[kx] + g.nbx * (bys[ky] + g.nby * bzs[kz]);
                    sum += face[(size_t)bb * F + face_index<S>(pxs[kx], pys[ky], pzs[kz])];
                }
        const int64_t gid = gx + (int64_t)Lx * (gy + (int64_t)Ly * gz);
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
        if (threadIdx.x == 0) part[blockIdx.x + gridDim.x * blockIdx.y] = bs;
    }
}

// The structured Mult's row sums from k_brick3d<..., PBO>'s patch buffer: y = the dof's 1-8 patch
// entries (patch_sum8), constrained (MODE 1): y = x on essential rows.  Rank-local: the interface
// planes of a slab get this rank's partial sums, as from k_brick_faces.
template <int S, int MODE>
__global__ void __launch_bounds__(kRedThreads)
k_brick_patch_sum(const double *__restrict__ x, double *__restrict__ y, const double *__restrict__ pb,
                  const uint8_t *__restrict__ ess, const BrickGeom g, const FastDiv fdx, const FastDiv fdxy)
{
    const int n = g.Lx * g.Ly * g.Lz, plane = g.Lx * g.Ly;
    const auto bp = brsrc(pb, 8u * (uint32_t)g.nbx * g.nby * g.nbz * (S * S * S));
    for (int gid = blockIdx.x * blockDim.x + threadIdx.x; gid < n; gid += gridDim.x * blockDim.x) {
        const int gz = (int)fdiv((uint32_t)gid, fdxy);
        const int rem = gid - gz * plane;
        const int gy = (int)fdiv((uint32_t)rem, fdx);
        const int gx = rem - gy * g.Lx;
        double v = patch_sum8<S>(bp, g, gx, gy, gz);
        if constexpr (MODE == 1) {
            if (ess[gid]) v = x[gid];
        }
        __builtin_nontemporal_store(v, &y[gid]);
    }
}

// ------------------------------------------------------------------------------------------------
bool brick_supported(int dim, int p) { return dim == 3 && (p == 1 || p == 2); }
int brick_count(const cdfem_ctx *c);
int brick_patch_side(const cdfem_ctx *c);

// kOOB = 2^31 is out of range only for buffers below 2^31 bytes: the lattice vectors (8 N_L) and the
// patch buffer (8 S^3 per brick) must both fit, else an out-of-lattice load would read real data and a
// dropped store would land inside the buffer
bool brick_fits(const cdfem_ctx *c)
{
    const double S = brick_patch_side(c), SZ = brick_patch_side_z(c), lim = (double)c->brick_limit;
    // a slab partition decides on the largest rank's sizes (cdfem_set_slab), the same on every rank
    const double nl = (double)std::max<int64_t>(c->nl, c->part_mode == 1 ? c->slab_nl_max : 0);
    const double nb = (double)std::max<int64_t>(brick_count(c), c->part_mode == 1 ? c->slab_nb_max : 0);
    return 8.0 * nl < lim && 8.0 * nb * S * S * SZ < lim;
}

// the brick lattice of the context: 4^3-element bricks at p <= 2, 2^3-element blocks at p = 3, 4 (ho_brick)
static BrickGeom geom_of(const cdfem_ctx *c)
{
    if (c->p >= 3) return BrickGeom{c->hb_nbx, c->hb_nby, c->hb_nbz, (int)c->Lx, (int)c->Ly, (int)c->Lz, c->brick_xcd, 0, 1, c->d_bess};
    // brick_stagger: -1 automatic (shift log2 CUs when the CU count is a power of two; n = 4 sleeps, 2 for
    // the matrix-core apply of a uniform box, whose compute phase is shorter: profiles/r06/ab_c2_stagger_um/),
    // 0 off
    int stag = c->brick_stagger;
    if (stag < 0) {
        int sh = 0;
        while ((1 << sh) < c->ncu) ++sh;
        const int n = (uniform_elem(c) && c->p == 2) ? 2 : 4;
        stag = (c->ncu > 0 && (1 << sh) == c->ncu) ? (sh | (n << 4)) : 0;
    }
    return BrickGeom{c->nbx, c->nby, c->nbz, (int)c->Lx, (int)c->Ly, (int)c->Lz, c->brick_xcd, 0, 1, c->d_bess,
                     stag, 8 * c->ncu};
}

int brick_count(const cdfem_ctx *c) { return c->p >= 3 ? c->hb_nblk : c->nblk; }
int brick_patch_side(const cdfem_ctx *c) { return c->p >= 3 ? kHoBrickEdge * c->p + 1 : kBrick * c->p + 1; }
int brick_patch_side_z(const cdfem_ctx *c) { return c->p >= 3 ? c->hb_ez * c->p + 1 : kBrick * c->p + 1; }

// patch-buffer Mult (Kronecker form, byte offsets within 32 bits)
bool brick_mult_pb_on(const cdfem_ctx *c) { return c->brick_mult_pb != 0 && pa_af(c) == 2 && brick_fits(c); }

GmPatchSrc gm_patch_src(const cdfem_ctx *c, const double *x)
{
    return GmPatchSrc{c->d_face, c->d_ess, x, geom_of(c), make_fastdiv((uint32_t)c->Lx),
                      make_fastdiv((uint32_t)(c->Lx * c->Ly)), kBrick * c->p + 1};
}

static dim3 faces_grid(const cdfem_ctx *c)
{
    const int64_t plane = c->Lx * c->Ly;
    int64_t bx = (plane + kRedThreads - 1) / kRedThreads;
    if (bx > 64) bx = 64;  // grid-stride beyond 64 blocks per plane (keeps the partial count small)
    return dim3((unsigned)bx, (unsigned)c->Lz);
}

template <int D1, int Q1, unsigned K, int MODE>
static hipError_t brick_launch(cdfem_ctx *c, const double *x, const double *dinv, double *d, double *y,
                               int which)
{
    constexpr int S = kBrick * (D1 - 1) + 1;
    const BrickGeom g = geom_of(c);
    const bool mpb = brick_mult_pb_on(c);
    if (which & 1) {
        const Tab<D1, Q1> T = make_tab<D1, Q1>(c->rule_op);
#define CDFEM_B3(AF_, QD_)                                                                                    \
    hipLaunchKernelGGL((k_brick3d<D1, Q1, K, MODE, AF_>), dim3(c->nblk), dim3(64), 0, c->stream, x, y, c->d_face, \
                       QD_, c->d_ess, T, g)
        if (pa_af(c) == 2 && mpb)
            hipLaunchKernelGGL((k_brick3d<D1, Q1, K, MODE, 2, true>), dim3(c->nblk), dim3(64), 0, c->stream, x, y,
                               c->d_face, c->d_qaff, c->d_ess, T, g);
        else if (pa_af(c) == 2) CDFEM_B3(2, c->d_qaff);
        else if (pa_af(c) == 1) CDFEM_B3(1, c->d_qaff);
        else CDFEM_B3(0, c->d_qd);
#undef CDFEM_B3
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if ((which & 2) && mpb) {
        const FastDiv fdx = make_fastdiv((uint32_t)c->Lx), fdxy = make_fastdiv((uint32_t)(c->Lx * c->Ly));
        const int64_t need = (c->nl + kRedThreads - 1) / kRedThreads;
        hipLaunchKernelGGL((k_brick_patch_sum<S, MODE>), dim3((unsigned)std::min<int64_t>(need, 16384)),
                           dim3(kRedThreads), 0, c->stream, x, y, c->d_face, c->d_ess, g, fdx, fdxy);
        return hipGetLastError();
    }
    if (which & 2) {
        const dim3 fg = faces_grid(c);
        hipLaunchKernelGGL((k_brick_faces<S, MODE>), fg, dim3(kRedThreads), 0, c->stream, x, dinv, d, y,
                           c->d_face, c->d_ess, g, c->d_part + c->nblk, c->d_state);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;

    }
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





// ================================================================================================
// Brick CG, version 2 (the Krylov hot loop on structured boxes): 2 streaming kernels + 2 one-block
// finalizers per iteration.
//   k_brick_cg:         d_new = M^{-1} r + beta d_old for the whole patch (recomputed by every brick
//                       containing a dof: same inputs, bitwise-identical values), written once by its
//                       writer brick into the OTHER d buffer (double-buffered: no brick ever reads a
//                       d entry another brick writes in the same launch); element apply; den
//                       contribution computed ELEMENT-WISE, den = sum_e d0_e . A_e d0_e + sum_ess d^2
//                       (= (d, A_c d) exactly in exact arithmetic); in-LDS E->L; interior q and face
//                       partials out.
//   k_cg_update_faces:  q = interior q | sum of face partials | d (ess), then the CG update
//                       x += alpha d, r -= alpha q, betanom = (r, M^{-1} r).  Face dofs are never
//                       touched by a strided pass of their own.
// Multi-rank slabs: zlo_shared = 1 when the local gz = 0 plane is the interface with the rank
// below, which owns it for the dot products (remote_lo / remote_hi carry the neighbours' partial
// sums of the interface planes; nullptr on a single GPU).
// ================================================================================================
// W: waves per SIMD the register allocation targets (the Kronecker form fits 2 without spills; three
// waves, 168 registers with a few spilled values, measured slower twice: profiles/r04/ab_c2_xfold_waves.json,
// ab_c2_xfold_pb.json; the point-data forms take 1)
// BF (set_option "cg_beta_fold", one rank, with the den fold): the betanom step of the previous
// update runs here: every workgroup (one wave) loads the update's nupart <= 1024 partials together
// with its patch gather, sums them in one fixed order, takes MFEM's decision (workgroup 0 records it,
// cg_update_logic; kk = updates so far, from the host) and forms beta itself, so the one-block update
// finalizer is not launched.
// MX (set_option "brick_mfma", kinds 7, the Kronecker form): the x stage of the brick's
// 64 elements on the matrix cores.  Per input plane jz and row jy, four v_mfma_f64_16x16x4_f64 (16 elements
// each): A = the 1D matrices stacked as rows (q, ix) = 4 q + ix (M, K, C, C^T; 12 of 16 rows), k = jx (3 of
// 4), B = the 16 elements' input rows from the LDS patch (column = element).  Lane (ix, element) then holds
// that element's four x-applied values for column ix and stores them to LDS, where each element's thread
// reads them back for the combinations and the y / z stages (kron_core otherwise).  A/B in DESIGN.md 4.1.
// MX 2 (pa_uniform, a uniformly refined box: every element has the same factors, so the same 27 x 27
// matrix A_e, formed once by setup_uniform_elem): the brick's 64 element applies as one GEMM on the
// matrix cores, Y (27 x 64) = A_e (27 x 27) X (27 x 64), 2 x 4 tiles of 16 x 16 over 7 k-steps of 4 = 56
// v_mfma_f64_16x16x4_f64 per brick (729 useful MACs per element against ~1,560 f64 FMAs of the Kronecker
// form on the VALU).  qd is then A_e in operand order: [mt][ks][lane] = A_e[16 mt + (lane & 15)][4 ks +
// (lane >> 4)] (0 past 27), 14 doubles per lane held for the whole kernel.  B (lane: input node 4 ks +
// (lane >> 4) of element 16 nt + (lane & 15)) comes straight from the LDS patch; accumulator i of a lane is
// row 16 mt + 4 i + (lane >> 4) of element 16 nt + (lane & 15).  The den terms are taken in
// the accumulator layout, then the accumulators go through LDS (over the two patches) to the
// thread-per-element layout of brick_e2l.
template <int D1, int Q1, unsigned K, int AF, int W = 1, bool XF = false, bool BF = false, bool FULL = false,
          int MX = 0>
__global__ void __launch_bounds__(64, W)
k_brick_cg(const double *__restrict__ r, const double *__restrict__ dinv,
           const double *__restrict__ d_old, double *__restrict__ d_new, double *__restrict__ q,
           double *__restrict__ face, const double *__restrict__ qd, const uint8_t *__restrict__ ess,
           const Tab<D1, Q1> T, const BrickGeom g, int zlo_shared, double *__restrict__ part,
           KrylovState *__restrict__ st, double *__restrict__ x, const double *__restrict__ upart, int nupart,
           int kk, double *__restrict__ gsum, uint32_t *__restrict__ gcnt, int grp, int nbrick)
{
    constexpr int P = D1 - 1;
    constexpr int S = kBrick * P + 1;
    constexpr int S2 = S * S, S3 = S * S * S;
    constexpr int NC = QLayout<K, 3>::nc;
    constexpr int NQ = Q1 * Q1 * Q1;
    // LDS patch layout (CDFEM_BRICK_LDS 2, p = 2): rows padded to SY = 12 and planes to SZ = 112 doubles,
    // so the 32 element origins of a ds_read_b64 half-wave (2 ex + 2 SY ey + 2 SZ ez) fall on 16
    // distinct bank pairs (2-way, the floor for even origins) instead of up to 4-way at SY = 9, SZ = 81
    constexpr bool PAD = CDFEM_BRICK_LDS == 2 && P == 2;
    constexpr int SY = PAD ? 12 : S, SZ = PAD ? 112 : S2, PS = (S - 1) * SZ + (S - 1) * SY + S;
    constexpr bool UM = MX == 2;
    constexpr int NDE = D1 * D1 * D1;
    // UM: the accumulators' trip to the thread-per-element layout reuses both patches ([node][element],
    // 13.8 KB against the patches' 11.7).  Measured (profiles/r06/ab_c2_uniform_mfma/): two trips of half
    // the brick each (11.7 KB) at 2 waves per SIMD 1.5 % slower per CG iteration; at 3 waves (168
    // registers, 31 spilled) 20 % slower
    constexpr int UMB = UM ? (2 * PS > NDE * 64 ? 2 * PS : NDE * 64) : PS;
    __shared__ double s_in[UMB];
    __shared__ double s_out_own[UM ? 1 : PS];
    double *const s_out = UM ? s_in + PS : s_out_own;
    // EP (the Kronecker form, AF 2): the essential rows' patch entries carry (A_c d)_i = d_i, the
    // writer brick's d (0 where the den ownership bit is off: non-writers, and the slab plane the rank
    // below owns), so the update's sum of a row's entries is its q with no essential flag or d read.
    // CDFEM_BRICK_LDS 0 keeps those d in a third LDS patch; >= 1 in registers (each position is formed
    // and stored by the same thread: 12 doubles live through the core, the LDS round trip gone)
    constexpr bool EP = AF == 2;
    constexpr bool EPL = EP && CDFEM_BRICK_LDS == 0;
    __shared__ double s_d[EPL ? S3 : 1];
    static_assert(!MX || (AF == 2 && D1 == 3), "the MFMA stages are built for the p = 2 Kronecker form");
    __shared__ double s_x[MX == 1 ? 3 * 3 * 4 * 64 : 1];  // MX 1: [jy][ix][q][element] of one input plane
    if (st->done) return;
    brick_stagger(g);
    double beta = st->beta;
    constexpr int NPL = 16;  // BF: partials per lane (nupart <= 64 NPL)
    double pv[NPL];
    if constexpr (BF) {
        if (kk > 0) {  // (buffer loads: past nupart they read 0, no branch per load)
            const auto bu = brsrc(upart, 8u * (uint32_t)nupart);
#pragma unroll
            for (int i = 0; i < NPL; ++i) pv[i] = bload(bu, 8u * ((uint32_t)threadIdx.x + 64u * i));
        }
    }
    // x-fold (XF, set_option "cg_xfold"): the previous iteration's x += alpha d_old, for the dofs
    // this brick writes d_new for (each dof has exactly one writer brick); the update kernel then
    // leaves x alone.  Bitwise the unfolded update (same fma on the same values).  A template flag:
    // a run-time one costs every position's writer mask a scalar register pair.
    const double alpha_prev = XF ? st->alpha : 0.0;
    const int t = threadIdx.x;
    // launch-local brick -> global brick (a launch covers every g.bzs-th layer from g.bz0)
    const int bl = brick_id(g), nxy = g.nbx * g.nby;
    const int bz = g.bz0 + (bl / nxy) * g.bzs;
    const int b = bl % nxy + nxy * bz;
    const int bx = b % g.nbx, by = (b / g.nbx) % g.nby;
    const int gx0 = (S - 1) * bx, gy0 = (S - 1) * by, gz0 = (S - 1) * bz;
    const bool lastx = bx == g.nbx - 1, lasty = by == g.nby - 1, lastz = bz == g.nbz - 1;
    const double *q0 = qd + (size_t)b * (AF ? 1 : NQ) * NC * kLanes;  // AF: per-element factors
    double den = 0.0;
    // patch gather: every load of the patch is issued before any is consumed (clamped indices,
    // no branches between them): one memory latency per brick instead of one per patch row.
    // Measured (tools/ab.py, in process): 241.1 vs 242.4 us per launch for the per-row form; the
    // other waves of the CU hide most of that latency.
    // Buffer access (brsrc): byte offsets fit 32 bits (8 N_L < 2^32 on one context: N_L <= 1.35e8,
    // SURVEY 8a); out-of-lattice positions of partial bricks use kOOB (loads 0, stores dropped).
    constexpr int NI = (S3 + 63) / 64;
    const int Lx = g.Lx, Lxy = g.Lx * g.Ly;
    const uint32_t nl = (uint32_t)Lxy * (uint32_t)g.Lz;
    const auto br = brsrc(r, 8u * nl), bm = brsrc(dinv, 8u * nl), bo = brsrc(d_old, 8u * nl);
    const auto be = brsrc(ess, nl), bd = brsrc(d_new, 8u * nl), bxf = brsrc(x, XF ? 8u * nl : 0u);
    // (the essential flags are loaded in every brick: skipping them where g.bess says the patch has
    // none, as k_hobrick_cg does, splits the gather's back-to-back loads and cost 2 us per launch,
    // profiles/r05/ab_bess/)
    // per position: the writer's byte offset (kOOB where this brick does not write the dof) and one
    // bit of dbits for "writer, and its d^2 counts in den" (not on a slab plane the rank below owns),
    // formed once here: the second pass then needs neither the patch walk nor the lane masks (which
    // the compiler kept in scalar registers and spilled to VGPR lanes across the loads)
    double rv[NI], mv[NI], ov[NI], xv[NI];
    uint32_t woffv[NI];
    uint32_t dbits = 0, ebits = 0;
    uint8_t ev[NI];
    uint32_t liv[PAD ? NI : 1];     // PAD: the position's LDS index
    double dev[EP && !EPL ? NI : 1];  // EP in registers: the essential entries' d
    // FULL (every brick of the box has its whole patch inside the lattice: the element counts are
    // multiples of 4): no lattice bound per position
    const uint32_t uLx = (uint32_t)Lx, uLxy = (uint32_t)Lxy;
    constexpr uint32_t wdx = 64 % S, wdy = (64 / S) % S, wdz = 64 / (S * S);
    const uint32_t dgid = wdx + wdy * uLx + wdz * uLxy, cxd = uLx - S, cyd = uLxy - S * uLx;
    LatWalk<S> pw0(t, (uint32_t)gx0 + uLx * (uint32_t)gy0 + uLxy * (uint32_t)gz0, uLx, uLxy);
    // W >= 3 waves per SIMD: the patch is gathered and formed in two halves, so only half of its
    // loads are in registers at once (round 5: the gather is not the register peak, the Kronecker
    // core is; at 168 registers the kernel still spills 22, so the default stays at 2 waves)
    constexpr int NG = W >= 3 ? 2 : 1, GK = (NI + NG - 1) / NG;
    auto gather = [&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const unsigned i = t + 64 * k;
        const int px = pw0.x, py = pw0.y, pz = pw0.z;
        const uint32_t gid = pw0.gid;
        if constexpr (PAD) liv[k] = (uint32_t)px + SY * (uint32_t)py + SZ * (uint32_t)pz;
        pw0.next(dgid, cxd, cyd);
        const int gz = gz0 + pz;
        const bool in = i < S3 && (FULL || (gx0 + px < g.Lx && gy0 + py < g.Ly && gz < g.Lz));
        const uint32_t off = in ? 8u * gid : kOOB;
        rv[k] = bload(br, off);
        mv[k] = bload(bm, off);
        ov[k] = bload(bo, off);
        ev[k] = __builtin_amdgcn_raw_buffer_load_b8(be, in ? gid : kOOB, 0, 0);
        const bool writer = in && (px < S - 1 || lastx) && (py < S - 1 || lasty) && (pz < S - 1 || lastz);
        woffv[k] = writer ? off : kOOB;
        dbits |= (uint32_t)(writer && !(zlo_shared && gz == 0)) << k;
        if constexpr (XF) xv[k] = bload(bxf, woffv[k]);
    };
    auto form = [&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const unsigned i = t + 64 * k;
        if (k == NI - 1 && i >= S3) return;
        const double dn = mv[k] * rv[k] + beta * ov[k];  // 0 outside the lattice
        const bool e = ev[k] != 0;
        bstore(bd, woffv[k], dn);
        if constexpr (XF) bstore(bxf, woffv[k], xv[k] + alpha_prev * ov[k]);
        // (A_c d)_i = d_i on ess dofs
        den += (e && ((dbits >> k) & 1u)) ? dn * dn : 0.0;
        const unsigned li = PAD ? liv[PAD ? k : 0] : i;
        s_in[li] = e ? 0.0 : dn;
        if constexpr (!UM) s_out[li] = 0.0;  // (UM: after the accumulators' trip through LDS)
        if constexpr (EP) {  // (unconditional: a predicated LDS store compiles to a branch per position)
            ebits |= (uint32_t)e << k;
            if constexpr (EPL) s_d[i] = ((dbits >> k) & 1u) ? dn : 0.0;
            else dev[EPL ? 0 : k] = ((dbits >> k) & 1u) ? dn : 0.0;
        }
    };
    static_for<0, GK>(gather);
    if constexpr (BF) {
        if (kk > 0) {
            double v = 0.0;
#pragma unroll
            for (int q = 0; q < NPL; ++q) v += pv[q];
            const double B = wave_sum(v);
            // cg_update_logic's decision (cg_stop_kind), taken identically by every workgroup at the
            // host's update count kk; workgroup 0 records it at the same kk
            const bool stop = cg_stop_kind(st, B, kk) != kCgGoOn;
            if (b == 0 && t == 0) {  // (global brick 0: one launch records, also when a slab is split in two)
#ifdef CDFEM_DEBUG
                assert(st->iter == kk);
#endif
                cg_update_logic_at(st, B, kk);
            }
            if (stop) return;
            beta = B / st->nom;
        }
    }
    static_for<0, GK>(form);
    if constexpr (NG == 2) {
        static_for<GK, NI>(gather);
        static_for<GK, NI>(form);
    }
    __syncthreads();

    const int ex = t & 3, ey = (t >> 2) & 3, ez = t >> 4;
    const int o0 = P * ez * SZ + P * ey * SY + P * ex;
    auto xl = [&](int dz, int dy, int dx) { return s_in[o0 + dz * SZ + dy * SY + dx]; };
    double Y[D1][D1][D1];
    if constexpr (UM) {
        const int n16 = t & 15, kg = t >> 4;
        double av[2][7];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int ks = 0; ks < 7; ++ks) av[mt][ks] = qd[(mt * 7 + ks) * 64 + t];
        // element 16 nt + n16 of the brick: (ex, ey, ez) = (n16 & 3, n16 >> 2, nt)
        const int ob0 = P * (n16 >> 2) * SY + P * (n16 & 3);
        auto node_off = [&](int j) { return (j / 9) * SZ + ((j / 3) % 3) * SY + j % 3; };
        v4d_t acc[2][4];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = v4d_t{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int ks = 0; ks < 7; ++ks) {
            const int j = 4 * ks + kg;  // this lane's input node (27 = the k padding: B = 0)
            const int jo = node_off(j < NDE ? j : 0);
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const double bv = j < NDE ? s_in[P * nt * SZ + ob0 + jo] : 0.0;
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
                    acc[mt][nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[mt][ks], bv, acc[mt][nt], 0, 0, 0);
            }
        }
        // den: sum over (node m, element n) of X[m][n] Y[m][n], in the accumulator layout (lane: acc[i]
        // = row 16 mt + 4 i + kg of element 16 nt + n16; the layout the MX 1 stage relies on too)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int m = 16 * mt + 4 * i + kg;
                const int mo = node_off(m < NDE ? m : 0);
#pragma unroll
                for (int nt = 0; nt < 4; ++nt)
                    den += m < NDE ? s_in[P * nt * SZ + ob0 + mo] * acc[mt][nt][i] : 0.0;
            }
        __syncthreads();
        double *const yb = s_in;  // [node][element] over both patches
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int m = 16 * mt + 4 * i + kg;
                if (mt == 0 || m < NDE) {
#pragma unroll
                    for (int nt = 0; nt < 4; ++nt) yb[m * 64 + 16 * nt + n16] = acc[mt][nt][i];
                }
            }
        __syncthreads();
#pragma unroll
        for (int dz = 0; dz < D1; ++dz)
#pragma unroll
            for (int dy = 0; dy < D1; ++dy)
#pragma unroll
                for (int dx = 0; dx < D1; ++dx) Y[dz][dy][dx] = yb[((dz * D1 + dy) * D1 + dx) * 64 + t];
        __syncthreads();
        // the output patch, zeroed now that the accumulators have left it
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const unsigned i = t + 64 * k;
            if (k == NI - 1 && i >= S3) break;
            s_out[PAD ? liv[PAD ? k : 0] : i] = 0.0;
        }
        __syncthreads();
    } else if constexpr (MX == 1) {
        double gk[NC];
        kron_load_g<K>(q0, t, gk);
        // A operand: lane (row = l & 15 = 4 q + ix, k = l >> 4 = jx) -> F_q[ix][jx] (0 in the padding)
        const int row = t & 15, kq = t >> 4, qa = row >> 2, ia = row & 3;
        double av = 0.0;
        static_for<0, D1>([&](auto ic) {
            static_for<0, D1>([&](auto jc) {
                constexpr int i = decltype(ic)::value, j = decltype(jc)::value;
                const double fm = tM(T, i, j), fk = tK(T, i, j), fc = tCacc(T, i, j, 1.0, 0.0),
                             fct = tCacc(T, j, i, 1.0, 0.0);
                if (ia == i && kq == j) av = qa == 0 ? fm : qa == 1 ? fk : qa == 2 ? fc : fct;
            });
        });
#pragma unroll
        for (int dz = 0; dz < D1; ++dz)
#pragma unroll
            for (int dy = 0; dy < D1; ++dy)
#pragma unroll
                for (int dx = 0; dx < D1; ++dx) Y[dz][dy][dx] = 0.0;
#pragma unroll
        for (int jz = 0; jz < D1; ++jz) {
#pragma unroll
            for (int jy = 0; jy < D1; ++jy)
#pragma unroll
                for (int tl = 0; tl < 4; ++tl) {
                    const int eb = 16 * tl + row;  // B column = element of tile tl
                    const int ob = P * (eb >> 4) * SZ + P * ((eb >> 2) & 3) * SY + P * (eb & 3);
                    const double bv = kq < D1 ? s_in[ob + jz * SZ + jy * SY + kq] : 0.0;
                    const v4d_t acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, v4d_t{0.0, 0.0, 0.0, 0.0}, 0, 0, 0);
                    if (kq < D1) {  // lane (ix = kq, element eb): its (M, K, C, C^T) X row values
#pragma unroll
                        for (int q = 0; q < 4; ++q) s_x[((jy * 3 + kq) * 4 + q) * 64 + eb] = acc[q];
                    }
                }
            __syncthreads();
#pragma unroll
            for (int ix = 0; ix < D1; ++ix) {
                double v[D1][5];
#pragma unroll
                for (int jy = 0; jy < D1; ++jy) {
                    const double *xr = &s_x[((jy * 3 + ix) * 4) * 64 + t];
                    kron_xcombine<K>(gk, xr[0], xr[64], xr[128], xr[192], v[jy]);
                }
                auto col = [&](int q, int jy) { return v[jy][q]; };
#pragma unroll
                for (int iy = 0; iy < D1; ++iy) {
                    double Yz[D1];
#pragma unroll
                    for (int iz = 0; iz < D1; ++iz) Yz[iz] = Y[iz][iy][ix];
                    kron_yz<D1, Q1, K>(T, gk, col, iy, jz, Yz);
#pragma unroll
                    for (int iz = 0; iz < D1; ++iz) Y[iz][iy][ix] = Yz[iz];
                }
            }
            __syncthreads();
        }
    } else {
        elem_apply3d_af<D1, Q1, K, AF>(xl, q0, t, T, Y);
    }

    // element-wise den contribution d0_e . (A_e d0_e) (UM: taken above) and deterministic in-LDS E->L
    if constexpr (!UM) {
#pragma unroll
        for (int dz = 0; dz < D1; ++dz)
#pragma unroll
            for (int dy = 0; dy < D1; ++dy)
#pragma unroll
                for (int dx = 0; dx < D1; ++dx) den += s_in[o0 + dz * SZ + dy * SY + dx] * Y[dz][dy][dx];
    }
    brick_e2l<D1, S, SY, SZ>(s_out, o0, Y);

    // the brick's whole patch output (interior rows complete, face rows partial) -> the patch buffer
    // (patch_idx, here in 32-bit arithmetic with the brick's part uniform: index = base + pz A + py R
    // + px); k_cg_update_faces sums each dof's 1-8 patch entries
    {
        const uint32_t R = (uint32_t)g.nbx * S, A = (uint32_t)g.nby * S * R;
        const uint32_t base = (uint32_t)bz * S * A + (uint32_t)by * S * R + (uint32_t)bx * S;
        const auto bp = brsrc(face, 8u * (uint32_t)g.nbx * g.nby * g.nbz * S3);
        const unsigned to = (unsigned)opaque(t);
        PatchWalk<S> pw(to);
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const unsigned i = to + 64 * k;
            if (k == NI - 1 && i >= S3) break;
            double v = s_out[PAD ? (uint32_t)pw.x + SY * (uint32_t)pw.y + SZ * (uint32_t)pw.z : i];
            if constexpr (EPL) v = ((ebits >> k) & 1u) ? s_d[i] : v;
            else if constexpr (EP) v = ((ebits >> k) & 1u) ? dev[EPL ? 0 : k] : v;
            bstore(bp, 8u * (base + (uint32_t)pw.z * A + (uint32_t)pw.y * R + (uint32_t)pw.x), v);
            pw.next();
        }
    }
    den = wave_sum(den);
    if (grp <= 1) {
        if (t == 0) part[b] = den;
        return;
    }
    // grouped partials (den_grp > 1): the partial goes out write-through (sc1: an agent-scope relaxed
    // store), the wave waits for it, then counts its arrival on the group's agent-scope counter; the
    // brick whose add returns the group's last count reads the group's partials with sc1 loads (L2 and
    // L1 bypassed: correct wherever the group's bricks ran, MI355X_MICROARCH.md inter-workgroup
    // visibility) and sums them by the fixed wave tree, so the group sum does not depend on the order
    // of arrival.  The counter is reset for the next launch by the same brick.
    const int gi = b / grp, g0 = gi * grp, gn = min(grp, nbrick - g0);
    uint32_t prev = 0;
    if (t == 0) {
        __hip_atomic_store(&part[b], den, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        prev = __hip_atomic_fetch_add(&gcnt[gi], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    prev = (uint32_t)__shfl((int)prev, 0, 64);
    if (prev != (uint32_t)(gn - 1)) return;
    double v = t < gn ? __hip_atomic_load(&part[g0 + t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
    v = wave_sum(v);
    if (t == 0) {
        gsum[gi] = v;
        __hip_atomic_store(&gcnt[gi], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// PB (set_option "brick_upd_pb"): the 1-8 patch entries of every dof as eight unconditional buffer
// loads at fixed offsets from its own brick's entry P (the lower brick's face entry along x / y / z
// sits at P - 1 / P - R / P - A in the pencil layout), the missing ones at kOOB (read as 0), summed
// in the branchy form's order (lower brick first per face axis, z outermost): bitwise the same q.
// DS (set_option "cg_den_fold", one rank): every workgroup sums the apply's den partials (apart,
// napart) in one fixed order and takes MFEM's den step itself (workgroup 0 records it), so the
// one-block den finalizer and its launch go away; the grid is a few hundred to a few thousand
// workgroups (grid-stride loop) to keep the redundant sums small, and its partials go to part.
template <int S, bool XF, bool PB = false, bool DS = false, bool EP = false, int SZ = S>
__global__ void __launch_bounds__(kRedThreads)
k_cg_update_faces(double *__restrict__ x, double *__restrict__ r, const double *__restrict__ d,
                  const double *__restrict__ dinv, const double *__restrict__ pb,
                  const uint8_t *__restrict__ ess, const BrickGeom g,
                  const FastDiv fdx, const FastDiv fdxy, int zlo_shared,
                  const double *__restrict__ remote_lo, const double *__restrict__ remote_hi,
                  double *__restrict__ part, KrylovState *__restrict__ st, int den_step,
                  const double *__restrict__ apart, int napart)
{
    constexpr int s1 = S - 1, sz1 = SZ - 1;
    constexpr uint32_t PV = (uint32_t)S * S * SZ;  // patch entries per brick / block
    __shared__ double sh[kRedThreads / 64 + 1];
    if (st->done) return;
    double alpha = 0.0;
    if constexpr (DS) {
        // (16 loads per thread in flight at once: the apply's 4096 partials in one round trip)
        const double den = sum_partials_all<16>(apart, napart, sh);
        if (blockIdx.x == 0 && threadIdx.x == 0) cg_den_step(st, den);
        if (den == 0.0) return;
        alpha = st->betanom / den;  // = cg_den_step's nom / den (block 0 may not have stored it yet)
    } else if (den_step) {
        // multi-rank: the MFEM den step on the all-reduced den, folded in (no one-thread kernel
        // between the all-reduce and the update).  Every block forms alpha = betanom / den as
        // cg_den_step does; block 0 alone writes the state (den, nom, alpha; done if den == 0).
        // No block reads a field block 0 writes, except done at entry, which only turns on
        // when every block returns here anyway.
        const double den = st->red[0];
        if (blockIdx.x == 0 && threadIdx.x == 0) cg_den_step(st, den);
        if (den == 0.0) return;
        alpha = st->betanom / den;
    } else {
        alpha = st->alpha;
    }
    const int n = g.Lx * g.Ly * g.Lz;
    const int plane = g.Lx * g.Ly;
    double acc = 0.0;
    if constexpr (EP) {
        // the apply's essential-row patch entries (EP in k_brick_cg): q is the sum of the row's 1-8
        // entries everywhere (with the neighbour's plane sums on a slab), so the loop reads r, M^-1 and
        // the patch only, every load independent of the others (no essential flag, no d).  Measured and
        // not kept (profiles/r05/ab_c2_update_pipe.json): the loop software-pipelined with the den sum
        // under the first loads (59.2-59.4 against 59.05 us per iteration) and two dofs per pass (62.5
        // against 59.8)
        static_assert(PB, "EP reads the patch buffer with the predicated loads");
        const auto bp = brsrc(pb, 8u * (uint32_t)g.nbx * g.nby * g.nbz * PV);
        for (int gid = blockIdx.x * blockDim.x + threadIdx.x; gid < n; gid += gridDim.x * blockDim.x) {
            const int gz = (int)fdiv((uint32_t)gid, fdxy);
            const int rem = gid - gz * plane;
            const int gy = (int)fdiv((uint32_t)rem, fdx);
            const int gx = rem - gy * g.Lx;
            const double rold = r[gid], mi = dinv[gid];
            const double xi = XF ? 0.0 : x[gid], di = XF ? 0.0 : d[gid];
            double qi = patch_sum8<S, SZ>(bp, g, gx, gy, gz);
            if (remote_lo && gz == 0) qi += remote_lo[rem];
            if (remote_hi && gz == g.Lz - 1) qi += remote_hi[rem];
            if constexpr (!XF) __builtin_nontemporal_store(xi + alpha * di, &x[gid]);
            const double ri = rold - alpha * qi;
            __builtin_nontemporal_store(ri, &r[gid]);
            if (!(zlo_shared && gz == 0)) acc += ri * (mi * ri);
        }
    } else {
        for (int gid = blockIdx.x * blockDim.x + threadIdx.x; gid < n; gid += gridDim.x * blockDim.x) {
            const int gz = (int)fdiv((uint32_t)gid, fdxy);
            const int rem = gid - gz * plane;
            const int gy = (int)fdiv((uint32_t)rem, fdx);
            const int gx = rem - gy * g.Lx;
            // every load is issued before any is consumed: which bricks' patch outputs hold this dof's
            // row sum depends on its lattice position only, and the essential flag selects last
            const bool is_ess = ess[gid] != 0;
            // XF: x was advanced by the apply (x-fold); d is then needed on essential rows only
            const double di = (!XF || is_ess) ? d[gid] : 0.0, xi = XF ? 0.0 : x[gid];
            const double rold = r[gid], mi = dinv[gid];
            double qi;
            if constexpr (PB) {
                qi = patch_sum8<S, SZ>(brsrc(pb, 8u * (uint32_t)g.nbx * g.nby * g.nbz * PV), g, gx, gy, gz);
            } else if (gx % s1 == 0 || gy % s1 == 0 || gz % sz1 == 0) {
                int bxs[2], pxs[2], nxc = 0, bys[2], pys[2], nyc = 0, bzs[2], pzs[2], nzc = 0;
                const int qx = gx / s1, qy = gy / s1, qz = gz / sz1;
                if (gx - qx * s1 == 0) {
                    if (qx - 1 >= 0) { bxs[nxc] = qx - 1; pxs[nxc] = s1; ++nxc; }
                    if (qx < g.nbx) { bxs[nxc] = qx; pxs[nxc] = 0; ++nxc; }
                } else { bxs[0] = qx; pxs[0] = gx - qx * s1; nxc = 1; }
                if (gy - qy * s1 == 0) {
                    if (qy - 1 >= 0) { bys[nyc] = qy - 1; pys[nyc] = s1; ++nyc; }
                    if (qy < g.nby) { bys[nyc] = qy; pys[nyc] = 0; ++nyc; }
                } else { bys[0] = qy; pys[0] = gy - qy * s1; nyc = 1; }
                if (gz - qz * sz1 == 0) {
                    if (qz - 1 >= 0) { bzs[nzc] = qz - 1; pzs[nzc] = sz1; ++nzc; }
                    if (qz < g.nbz) { bzs[nzc] = qz; pzs[nzc] = 0; ++nzc; }
                } else { bzs[0] = qz; pzs[0] = gz - qz * sz1; nzc = 1; }
                qi = 0.0;
                for (int kz = 0; kz < nzc; ++kz)
                    for (int ky = 0; ky < nyc; ++ky)
                        for (int kx = 0; kx < nxc; ++kx) {
                            qi += pb[patch_idx<S, SZ>(g, bxs[kx], bys[ky], bzs[kz], pxs[kx], pys[ky], pzs[kz])];
                        }
            } else {  // inside one brick's patch
                const int qx = gx / s1, qy = gy / s1, qz = gz / sz1;
                qi = pb[patch_idx<S, SZ>(g, qx, qy, qz, gx - qx * s1, gy - qy * s1, gz - qz * sz1)];
            }
            // interface planes: add the neighbour rank's partial sums
            if (remote_lo && gz == 0) qi += remote_lo[rem];
            if (remote_hi && gz == g.Lz - 1) qi += remote_hi[rem];
            if (is_ess) qi = di;
            if constexpr (!XF) __builtin_nontemporal_store(xi + alpha * di, &x[gid]);
            const double ri = rold - alpha * qi;
            __builtin_nontemporal_store(ri, &r[gid]);
            if (!(zlo_shared && gz == 0)) acc += ri * (mi * ri);
        }
    }
    const double bs = block_sum(acc, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = bs;
}


// ================================================================================================
// High-order brick CG apply (3D p = 3, 4 on a structured affine box; set_option "ho_brick"): the brick
// CG protocol of k_brick_cg on blocks of 2 x 2 x 2 elements (an S^3 patch, S = 2p + 1: 9^3 at p = 4),
// with the Kronecker-form element core of k_apply3d_ktile (ho_kernels.hip) spread over one D1 x D1
// thread tile per element.  Per block (8 D1^2 threads, 256 at p = 4):
//   1. patch: d_new = M^-1 r + beta d_old on every position (the writer block stores it, and x +=
//      alpha d_old under the x-fold), the essential entries zeroed in LDS, their d^2 into den;
//   2. the eight elements' tiles: x + y stages (thread (ix, jz)) -> LDS groups, z stage (thread
//      (ix, iy)) -> the element output Y in LDS, d~_e . Y_e into den;
//   3. E->L inside the block: every patch position sums its 1-8 element entries in a fixed order
//      and the whole patch goes to the patch buffer (patch_idx, the p = 2 brick's layout), so
//      k_cg_update_faces (S = 2p + 1) forms q and updates r exactly as on the p = 2 brick.
// This replaces the tile path's E-vector round trip (125 entries per element written, then read by
// the flat E->L update) with 729 patch entries per 8 elements, and the update's x, d and z streams
// with the brick CG's r, M^-1.
// ================================================================================================
constexpr int kHoBrick = kHoBrickEdge;  // elements per block edge (high order)

// MF (set_option "ho_brick_mfma", kinds 7): the x stage of the eight elements as block GEMMs on
// v_mfma_f64_16x16x4_f64 (block_mfma, pa_core.hpp): rows = the block's 8 x 25 element rows
// (element, jz, jy), k = jx (5, padded to 8), columns = (matrix, ix) for M, K, C, C^T (20, as a
// 16-column and a 4-column GEMM), staged through LDS (aliased on the y-stage groups) to the tile
// threads, which form the element combinations and the y / z stages on the VALU as before.  The
// north star's "MFMA for the per-element B^T D B contraction at high order", A/B'd against the VALU
// x stage.
// EZ (set_option "ho_block_z"): elements per block along z, 2 (2^3 blocks: 8 tiles = 200 of 256 threads busy
// at p = 4, 1.42 patch entries per dof) or 4 (2 x 2 x 4 blocks: 16 tiles = 400 of 448, 1.34 entries per dof;
// an S x S x SZ patch, SZ = 4p + 1)
template <int D1, int Q1, unsigned K, bool XF, bool MF = false, int EZ = kHoBrick>
__global__ void __launch_bounds__(((kHoBrick * kHoBrick * EZ * D1 * D1 + 63) / 64) * 64, 4)
k_hobrick_cg(const double *__restrict__ r, const double *__restrict__ dinv, const double *__restrict__ d_old,
             double *__restrict__ d_new, double *__restrict__ face, const double *__restrict__ qaff,
             const uint8_t *__restrict__ ess, const Tab<D1, Q1> T, const BrickGeom g, int nex, int ney, int nez,
             double *__restrict__ part, const KrylovState *__restrict__ st, double *__restrict__ x,
             const double *__restrict__ ktab, int zlo_shared)
{
    using L = QLayout<K, 3>;
    constexpr int P = D1 - 1, EB = kHoBrick, S = EB * P + 1, SZ = EZ * P + 1, S2 = S * S, S3 = S * S * SZ;
    constexpr int DD = D1 * D1, ND = DD * D1, NEB = EB * EB * EZ, NC = L::nc;
    constexpr int NT = ((NEB * DD + 63) / 64) * 64, NI = (S3 + NT - 1) / NT;
    __shared__ double s_in[S3];
    __shared__ double sP[NEB][4][ND];  // [element][grp][jz][iy][ix]
    // element outputs Y [dz][dy][dx], in place of group 0 of the element's y-stage output: thread (a, bb)
    // reads all its groups' (jz, bb, a) entries before it writes its Y at (dz, bb, a), and no other
    // thread reads or writes those (8 KB less LDS: four blocks per CU)
    auto sE = [&](int e8, int idx) -> double & { return sP[e8][0][idx]; };
    __shared__ double shd[NT / 64];
    if (st->done) return;
    const double beta = st->beta;
    const double alpha_prev = XF ? st->alpha : 0.0;
    const int tid = threadIdx.x;
    const int b = brick_id(g);
    const int nxy = g.nbx * g.nby;
    const int bz = b / nxy, by = (b - bz * nxy) / g.nbx, bx = b - bz * nxy - by * g.nbx;
    const int gx0 = (S - 1) * bx, gy0 = (S - 1) * by, gz0 = (SZ - 1) * bz;
    const bool lastx = bx == g.nbx - 1, lasty = by == g.nby - 1, lastz = bz == g.nbz - 1;
    const int Lx = g.Lx, Lxy = g.Lx * g.Ly;
    const uint32_t nl = (uint32_t)Lxy * (uint32_t)g.Lz;
    const auto br = brsrc(r, 8u * nl), bm = brsrc(dinv, 8u * nl), bo = brsrc(d_old, 8u * nl);
    const auto be = brsrc(ess, nl), bd = brsrc(d_new, 8u * nl), bxf = brsrc(x, XF ? 8u * nl : 0u);
    // blocks with no essential dof in their patch (g.bess, formed at cdfem_mesh_set_structured: all but
    // the boundary layer) load no essential flags (a wave-uniform branch; C3 apply 2,948 -> 2,786 us,
    // profiles/r05/ab_bess/)
    const bool bhas = g.bess == nullptr || g.bess[b] != 0;
    // this thread's element tile and x-stage rows (ix = a), loaded with the patch
    const int le = tid / DD, tt = tid - le * DD, a = tt % D1, bb = tt / D1;
    const int lex = le & 1, ley = (le >> 1) & 1, lez = le >> 2;
    const int ex = EB * bx + lex, ey = EB * by + ley, ez = EZ * bz + lez;
    const bool tile = le < NEB, valid = tile && ex < nex && ey < ney && ez < nez;
    const int64_t ec = valid ? (int64_t)ex + (int64_t)nex * (ey + (int64_t)ney * ez) : 0;
    double Mr[D1], Kr[D1], Cr[D1], Ctr[D1], gf[NC];
#pragma unroll
    for (int j = 0; j < D1; ++j) {
        Mr[j] = ktab[(0 * D1 + a) * D1 + j];
        Kr[j] = ktab[(1 * D1 + a) * D1 + j];
        Cr[j] = ktab[(2 * D1 + a) * D1 + j];
        Ctr[j] = ktab[(3 * D1 + a) * D1 + j];
    }
#pragma unroll
    for (int k = 0; k < NC; ++k) gf[k] = qaff[ec * NC + k];
    // 1. the patch: all loads issued before any is consumed (kOOB outside the lattice: 0)
    double den = 0.0;
    {
        double rv[NI], mv[NI], ov[NI], xv[NI];
        uint32_t offv[NI];
        uint8_t ev[NI];
        PatchWalk<S, NT> pw0(tid);
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const unsigned i = tid + NT * k;
            const int px = pw0.x, py = pw0.y, pz = pw0.z;
            pw0.next();
            const int gx = gx0 + px, gy = gy0 + py, gz = gz0 + pz;
            const bool in = i < S3 && gx < g.Lx && gy < g.Ly && gz < g.Lz;
            const uint32_t gid = (uint32_t)opaque(gx + Lx * gy + Lxy * gz);
            offv[k] = in ? 8u * gid : kOOB;
            rv[k] = bload(br, offv[k]);
            mv[k] = bload(bm, offv[k]);
            ov[k] = bload(bo, offv[k]);
            ev[k] = 0;
            if (bhas) ev[k] = __builtin_amdgcn_raw_buffer_load_b8(be, in ? gid : kOOB, 0, 0);
            const bool writer = in && (px < S - 1 || lastx) && (py < S - 1 || lasty) && (pz < SZ - 1 || lastz);
            if constexpr (XF) xv[k] = bload(bxf, writer ? offv[k] : kOOB);
        }
        PatchWalk<S, NT> pw1(tid);
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const unsigned i = tid + NT * k;
            const int px = pw1.x, py = pw1.y, pz = pw1.z;
            pw1.next();
            if (i >= S3) break;
            const bool in = offv[k] != kOOB;
            const double dn = mv[k] * rv[k] + beta * ov[k];  // 0 outside the lattice
            const bool e = ev[k] != 0;
            const bool writer = in && (px < S - 1 || lastx) && (py < S - 1 || lasty) && (pz < SZ - 1 || lastz);
            const uint32_t woff = writer ? offv[k] : kOOB;
            bstore(bd, woff, dn);
            if constexpr (XF) bstore(bxf, woff, xv[k] + alpha_prev * ov[k]);
            // (A_c d)_i = d_i on ess dofs; on a slab the lower plane's are the rank below's
            den += (writer && e && !(zlo_shared && gz0 + pz == 0)) ? dn * dn : 0.0;
            s_in[i] = e ? 0.0 : dn;
        }
    }
    __syncthreads();
    // 2. element tiles: x + y stages, thread (ix = a, jz = bb)
    const int o0 = P * lez * S2 + P * ley * S + P * lex;
    double xq[MF ? 4 : 1][MF ? D1 : 1];  // MF: this thread's (M, K, C, C^T) X rows, from the GEMM
    if constexpr (MF) {
        static_assert(EZ == kHoBrick, "the MFMA x stage is built for 2^3 blocks");
        constexpr int NR = NEB * DD, NCOL = 4 * D1;
        static_assert(NR * NCOL <= NEB * 4 * ND, "the x-stage output aliases the y-stage groups");
        double *xs = &sP[0][0][0];
        auto arow = [&](int row, int k) {
            const int e8 = row / DD, rr = row - e8 * DD, jz = rr / D1, jy = rr - jz * D1;
            const int ob = P * (e8 >> 2) * S2 + P * ((e8 >> 1) & 1) * S + P * (e8 & 1);
            return k < D1 ? s_in[ob + jz * S2 + jy * S + k] : 0.0;
        };
        auto bcol = [&](int k, int col) { return (k < D1 && col < NCOL) ? ktab[col * D1 + k] : 0.0; };
        auto o16 = [&](int row, int col, double v) { xs[row * NCOL + col] = v; };
        auto b16 = [&](int k, int col) { return bcol(k, 16 + col); };
        auto o4 = [&](int row, int col, double v) {
            if (16 + col < NCOL) xs[row * NCOL + 16 + col] = v;
        };
        block_mfma<NR, (D1 + 3) / 4, decltype(arow), decltype(bcol), decltype(o16), NT / 64>(arow, bcol, o16);
        if constexpr (NCOL > 16)  // (p = 4: C^T's last 4 columns; p = 3 fits one 16-column GEMM)
            block_mfma<NR, (D1 + 3) / 4, decltype(arow), decltype(b16), decltype(o4), NT / 64>(arow, b16, o4);
        __syncthreads();
        if (tile) {
#pragma unroll
            for (int jy = 0; jy < D1; ++jy) {
                const int row = le * DD + bb * D1 + jy;
#pragma unroll
                for (int q = 0; q < 4; ++q) xq[q][jy] = xs[row * NCOL + q * D1 + a];
            }
        }
        __syncthreads();  // (the y stage's groups overwrite xs)
    }
    if (tile) {
        double v[D1][5];
#pragma unroll
        for (int jy = 0; jy < D1; ++jy) {
            double mm = 0.0, kk = 0.0, cc = 0.0, ct = 0.0;
            if constexpr (MF) {
                mm = xq[0][jy];
                kk = xq[1][jy];
                cc = xq[2][jy];
                ct = xq[3][jy];
            } else {
                const double *xrow = &s_in[o0 + bb * S2 + jy * S];
#pragma unroll
                for (int jx = 0; jx < D1; ++jx) {
                    const double xv = xrow[jx];
                    mm += Mr[jx] * xv;
                    if constexpr (L::kD) {
                        kk += Kr[jx] * xv;
                        ct += Ctr[jx] * xv;
                    }
                    if constexpr (L::kD || L::kC) cc += Cr[jx] * xv;
                }
            }
            kron_xcombine<K>(gf, mm, kk, cc, ct, v[jy]);
        }
        auto col = [&](int q, int jy) { return v[jy][q]; };
#pragma unroll
        for (int iy = 0; iy < D1; ++iy) {
            double Pg[4];
            kron_y<D1, Q1, K>(T, gf, col, iy, Pg);
#pragma unroll
            for (int k = 0; k < 4; ++k) sP[le][k][(bb * D1 + iy) * D1 + a] = Pg[k];
        }
    }
    __syncthreads();
    // z stage, thread (ix = a, iy = bb): Y -> LDS and the element's d~ . A_e d~
    if (tile) {
        double Yz[D1];
#pragma unroll
        for (int iz = 0; iz < D1; ++iz) Yz[iz] = 0.0;
#pragma unroll
        for (int jz = 0; jz < D1; ++jz) {
            double Pg[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) Pg[k] = sP[le][k][(jz * D1 + bb) * D1 + a];
            kron_z<D1, Q1, K>(T, Pg, jz, Yz);
        }
#pragma unroll
        for (int dz = 0; dz < D1; ++dz) {
            const double y = valid ? Yz[dz] : 0.0;
            den += s_in[o0 + dz * S2 + bb * S + a] * y;
            sE(le, (dz * D1 + bb) * D1 + a) = y;
        }
    }
    __syncthreads();
    // 3. E->L in the block: position (px, py, pz) takes the entries of the 1-8 elements holding it
    //    (lower element first per axis, z outermost) -> the patch buffer
    {
        const uint32_t R = (uint32_t)g.nbx * S, A = (uint32_t)g.nby * S * R;
        const uint32_t base = (uint32_t)bz * SZ * A + (uint32_t)by * S * R + (uint32_t)bx * S;
        const auto bp = brsrc(face, 8u * (uint32_t)g.nbx * g.nby * g.nbz * S3);
        const unsigned to = (unsigned)opaque(tid);
        PatchWalk<S, NT> pw(to);
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const unsigned i = to + NT * k;
            if (i >= S3) break;
            const int px = pw.x, py = pw.y, pz = pw.z;
            // per axis: element 0 holds positions 0..P, element 1 positions P..2P (local P + 0..P); along z
            // the pair of candidate elements is (kz - 1, kz) around position pz = kz P + lz (lower first)
            const int x0 = px < P ? px : P, y0 = py < P ? py : P;
            const bool hx1 = px >= P, hy1 = py >= P;
            const bool hx0 = px <= P, hy0 = py <= P;
            const int x1 = px - P, y1 = py - P;
            int kz = pz / P;
            kz = kz < EZ ? kz : EZ - 1;
            const int zl = pz - kz * P;  // 0..P: local z in element kz
            const bool zlow = zl == 0 && kz > 0;  // also the top face of element kz - 1
            double sum = 0.0;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const int cx = c & 1, cy = (c >> 1) & 1, cz = c >> 2;
                // cz = 0: the lower z element (kz - 1 at local P when zlow, else kz), cz = 1: element kz
                // when zlow (at local 0); the same order as the 2^3 form's (lower element first)
                const bool okz = cz ? zlow : true;
                const int ez8 = cz ? kz : (zlow ? kz - 1 : kz), lz = cz ? 0 : (zlow ? P : zl);
                const bool ok = (cx ? hx1 : hx0) && (cy ? hy1 : hy0) && okz;
                const int lx = cx ? x1 : x0, ly = cy ? y1 : y0;
                const double t = sE(cx + 2 * cy + 4 * ez8, ok ? (lz * D1 + ly) * D1 + lx : 0);
                sum += ok ? t : 0.0;
            }
            bstore(bp, 8u * (base + (uint32_t)pw.z * A + (uint32_t)pw.y * R + (uint32_t)pw.x), sum);
            pw.next();
        }
    }
    const double bs = block_sum(den, shd);
    if (tid == 0) part[b] = bs;
}

// one launch of k_brick_cg over brick layers bz0, bz0 + bzs, ... (nlay of them) on stream s;
// the whole slab (0, 1, nbz) on the context stream goes through CDFEM_LAUNCH (profiling events)
struct BrickRun {
    int bz0, bzs, nlay;
    hipStream_t s;
    int kk = -1;      // >= 0: the betanom-fold apply (k_brick_cg<..., BF>) after kk updates
    int nupart = 0;   //   with the update's partial count
};

template <int D1, int Q1, unsigned K>
static hipError_t brick_cg2_launch(cdfem_ctx *c, const double *r, const double *dinv,
                                   const double *d_old, double *d_new, double *q, const BrickRun &run, double *x)
{
    const Tab<D1, Q1> T = make_tab<D1, Q1>(c->rule_op);
    BrickGeom g = geom_of(c);
    g.bz0 = run.bz0;
    g.bzs = run.bzs;
    const dim3 grid((unsigned)(c->nbx * c->nby * run.nlay)), block(64);
    const bool whole = run.nlay == c->nbz && run.s == c->stream;
    const double *qd = c->d_qaff ? c->d_qaff : c->d_qd;  // (pa_uniform: the element matrix, below)
    const double *upart = c->d_part + c->nblk;  // the den-fold update's partials
    double *const dpart = c->den_out ? c->den_out : c->d_part;  // the apply's den partials
    const int grp = c->den_grp, nbrick = c->nblk;               // (grouped: sums into d_gsum)
#define CDFEM_BCG6(AFF_, W_, XF_, BF_, FU_, MX_)                                                            \
    if (whole)                                                                                               \
        CDFEM_LAUNCH(c, (k_brick_cg<D1, Q1, K, AFF_, W_, XF_, BF_, FU_, MX_>), grid, block, 0, r, dinv, d_old, d_new, q, \
                     c->d_face, qd, c->d_ess, T, g, c->zlo_shared, dpart, c->d_state, x, upart, run.nupart,     \
                     run.kk, c->d_gsum, c->d_gcnt, grp, nbrick);                                             \
    else                                                                                                     \
        hipLaunchKernelGGL((k_brick_cg<D1, Q1, K, AFF_, W_, XF_, BF_, FU_, MX_>), grid, block, 0, run.s, r, dinv, \
                           d_old, d_new, q, c->d_face, qd, c->d_ess, T, g, c->zlo_shared, dpart, c->d_state, x, \
                           upart, run.nupart, run.kk, c->d_gsum, c->d_gcnt, grp, nbrick)
    // (brick_mfma: the MFMA x stage, built for the Kronecker form of the full operator at p = 2;
    // pa_uniform: the common element matrix on the matrix cores, p = 2, instantiated for the full
    // operator and the symmetric kK + sM of the bench (kinds 7, 5); other kinds keep the Kronecker form)
    constexpr bool kMX = K == 7 && D1 == 3;
    constexpr bool kUM = (K == 7 || K == 5) && D1 == 3;
    const bool mx = kMX && c->brick_mfma != 0;
    const bool um = kUM && uniform_elem(c);
    if (um) qd = c->d_uelem;
#define CDFEM_BCG5(AFF_, W_, XF_, BF_, FU_)                                                                 \
    if constexpr (kUM && AFF_ == 2) {                                                                        \
        if (um) { CDFEM_BCG6(AFF_, W_, XF_, BF_, FU_, 2); }                                                  \
        else if (mx) { CDFEM_BCG6(AFF_, W_, XF_, BF_, FU_, (kMX ? 1 : 0)); }                                 \
        else { CDFEM_BCG6(AFF_, W_, XF_, BF_, FU_, 0); }                                                     \
    } else {                                                                                                 \
        CDFEM_BCG6(AFF_, W_, XF_, BF_, FU_, 0);                                                              \
    }
#define CDFEM_BCG4(AFF_, W_, XF_, BF_)                                                                      \
    if (full) { CDFEM_BCG5(AFF_, W_, XF_, BF_, true); } else { CDFEM_BCG5(AFF_, W_, XF_, BF_, false); }
#define CDFEM_BCG3(AFF_, W_, XF_) CDFEM_BCG5(AFF_, W_, XF_, false, false)
#define CDFEM_BCG(AFF_, W_) CDFEM_BCG3(AFF_, W_, false)
    // every brick's patch inside the lattice (element counts multiples of 4): no per-position bounds
    const bool full = c->sx % kBrick == 0 && c->sy % kBrick == 0 && c->sz % kBrick == 0;
    if (pa_af(c) == 2 && run.kk >= 0) {
        if (x) { CDFEM_BCG4(2, 2, true, true); }
        else { CDFEM_BCG4(2, 2, false, true); }
    } else if (pa_af(c) == 2) {
        if (x) { CDFEM_BCG4(2, 2, true, false); }
        else { CDFEM_BCG4(2, 2, false, false); }
    } else if (pa_af(c) == 1) {
        CDFEM_BCG(1, 1);
    } else {
        CDFEM_BCG(0, 1);
    }
#undef CDFEM_BCG
#undef CDFEM_BCG3
#undef CDFEM_BCG4
#undef CDFEM_BCG5
#undef CDFEM_BCG6
    return hipGetLastError();
}

template <int D1, int Q1, unsigned K, int EZ = kHoBrick>
static hipError_t hobrick_launch(cdfem_ctx *c, const double *r, const double *dinv, const double *d_old, double *d_new,
                                 double *x)
{
    if constexpr (EZ == kHoBrick) {
        if (c->hb_ez == 4) return hobrick_launch<D1, Q1, K, 4>(c, r, dinv, d_old, d_new, x);
    }
    if (c->hb_ez != EZ) return hipErrorInvalidValue;
    constexpr int NT = ((kHoBrick * kHoBrick * EZ * D1 * D1 + 63) / 64) * 64;
    const Tab<D1, Q1> T = make_tab<D1, Q1>(c->rule_op);
    const double *kt = nullptr;
    if (c->d_hbpart == nullptr) return hipErrorInvalidValue;
    const hipError_t e = ho_ktab(c, &kt);
    if (e != hipSuccess || kt == nullptr) return e != hipSuccess ? e : hipErrorInvalidValue;
    const BrickGeom g = geom_of(c);
    const dim3 grid((unsigned)c->hb_nblk), block(NT);
#define CDFEM_HB(XF_, MF_)                                                                                     \
    CDFEM_LAUNCH(c, (k_hobrick_cg<D1, Q1, K, XF_, MF_, EZ>), grid, block, 0, r, dinv, d_old, d_new, c->d_face, c->d_qaff, \
                 c->d_ess, T, g, c->sx, c->sy, c->sz, c->d_hbpart, c->d_state, x, kt, c->zlo_shared)
    if constexpr (K == 7 && EZ == kHoBrick) {  // the MFMA x stage: the full operator on 2^3 blocks (ho_brick_mfma)
        if (c->ho_brick_mfma) {
            if (x) { CDFEM_HB(true, true); } else { CDFEM_HB(false, true); }
            return hipGetLastError();
        }
    }
    if (x) { CDFEM_HB(true, false); } else { CDFEM_HB(false, false); }
#undef CDFEM_HB
    return hipGetLastError();
}

static hipError_t brick_cg2_run(cdfem_ctx *c, const double *r, const double *dinv, const double *d_old,
                                double *d_new, double *q, const BrickRun &run, double *x)
{
    const int q1 = c->rule_op.q1;
    if (c->p >= 3) {  // 2^3-element blocks, one launch (one rank)
        if (run.nlay != c->hb_nbz || run.kk >= 0) return hipErrorInvalidValue;
#define CDFEM_HK(D1_, Q1_)                                                                          \
    switch (c->kinds) {                                                                             \
    case 1: return hobrick_launch<D1_, Q1_, 1>(c, r, dinv, d_old, d_new, x);                        \
    case 2: return hobrick_launch<D1_, Q1_, 2>(c, r, dinv, d_old, d_new, x);                        \
    case 3: return hobrick_launch<D1_, Q1_, 3>(c, r, dinv, d_old, d_new, x);                        \
    case 4: return hobrick_launch<D1_, Q1_, 4>(c, r, dinv, d_old, d_new, x);                        \
    case 5: return hobrick_launch<D1_, Q1_, 5>(c, r, dinv, d_old, d_new, x);                        \
    case 6: return hobrick_launch<D1_, Q1_, 6>(c, r, dinv, d_old, d_new, x);                        \
    case 7: return hobrick_launch<D1_, Q1_, 7>(c, r, dinv, d_old, d_new, x);                        \
    default: return hipErrorInvalidValue;                                                           \
    }
        if (c->p == 3 && q1 == 5) { CDFEM_HK(4, 5) }
        if (c->p == 4 && q1 == 6) { CDFEM_HK(5, 6) }
#undef CDFEM_HK
        return hipErrorInvalidValue;
    }
#define CDFEM_K(D1_, Q1_)                                                                           \
    switch (c->kinds) {                                                                             \
    case 1: return brick_cg2_launch<D1_, Q1_, 1>(c, r, dinv, d_old, d_new, q, run, x);                 \
    case 2: return brick_cg2_launch<D1_, Q1_, 2>(c, r, dinv, d_old, d_new, q, run, x);                 \
    case 3: return brick_cg2_launch<D1_, Q1_, 3>(c, r, dinv, d_old, d_new, q, run, x);                 \
    case 4: return brick_cg2_launch<D1_, Q1_, 4>(c, r, dinv, d_old, d_new, q, run, x);                 \
    case 5: return brick_cg2_launch<D1_, Q1_, 5>(c, r, dinv, d_old, d_new, q, run, x);                 \
    case 6: return brick_cg2_launch<D1_, Q1_, 6>(c, r, dinv, d_old, d_new, q, run, x);                 \
    case 7: return brick_cg2_launch<D1_, Q1_, 7>(c, r, dinv, d_old, d_new, q, run, x);                 \
    default: return hipErrorInvalidValue;                                                           \
    }
    if (c->p == 1 && q1 == 3) { CDFEM_K(2, 3) }
    if (c->p == 2 && q1 == 4) { CDFEM_K(3, 4) }
#undef CDFEM_K
    return hipErrorInvalidValue;
}

hipError_t launch_brick_cg2(cdfem_ctx *c, const double *r, const double *dinv, const double *d_old,
                            double *d_new, double *q, double *x, int bfkk)
{
    BrickRun run{0, 1, c->p >= 3 ? c->hb_nbz : c->nbz, c->stream};
    if (bfkk >= 0) {
        run.kk = bfkk;
        run.nupart = cg_den_fold_grid(c);
    }
    return brick_cg2_run(c, r, dinv, d_old, d_new, q, run, x);
}

// the den-fold update's workgroups (k_cg_update_faces<..., DS>), one per partial
int cg_den_fold_grid(const cdfem_ctx *c)
{
    const int64_t need = (c->nl + kRedThreads - 1) / kRedThreads;
    return (int)std::min<int64_t>(c->cg_den_fold, need);
}

// the betanom step folded into the next apply (one rank, Kronecker form, den fold on, <= 1024 partials)
// both scalar steps folded (den in the update, betanom in the next apply): p <= 2, Kronecker form, and
// partial counts the kernels' fixed-order sums are sized for (the apply's 4,096 per 64^3 slab, the
// update's <= 1024)
static bool cg_folds_fit(const cdfem_ctx *c)
{
    return c->cg_den_fold != 0 && c->cg_beta_fold != 0 && c->p <= 2 && pa_af(c) == 2 && cg_den_fold_grid(c) <= 1024 &&
           den_parts(c) <= kDenFoldMaxParts;
}

// den partial groups (p <= 2, several ranks): none while the bricks fit the fold bound (kMrFoldMaxParts; C2's
// 4,096 bricks per rank), else the smallest power of two <= 64 leaving <= kDenGroupParts group sums (C5's
// per-rank slab of 32,768 bricks: 8 -> 4,096), so the multi-rank fold stays on; 1 when even 64 leaves too many.
// One rank keeps per-brick partials (its 256^3 p = 2 box: the two-stage den sum, 3,491 us of kernels per
// iteration against 3,503 with groups of 64, profiles/r06/r06c_c5_1gpu*.json); set_option "den_group"
// forces a size on any box (tests)
int den_group(const cdfem_ctx *c)
{
    const int nb = brick_count(c);
    if (c->p > 2) return 1;
    if (c->den_group_opt > 0) return c->den_group_opt;
    if (!multi_rank(c) || nb <= kMrFoldMaxParts) return 1;
    for (int g = 2; g <= 64; g *= 2)
        if ((nb + g - 1) / g <= kDenGroupParts) return g;
    return 1;
}
int den_parts(const cdfem_ctx *c)
{
    const int g = den_group(c);
    return (brick_count(c) + g - 1) / g;
}

// several ranks (set_option "cg_mr_fold"): the ranks all-reduce the apply's den partials and the
// update's betanom partials as vectors (element-wise sum over ranks: every rank then holds the same
// partials and forms the same scalars in the same order), so the update and the next apply take the
// den and betanom steps as on one rank; no sum / step kernels between them
bool cg_mr_fold(const cdfem_ctx *c)
{
    return multi_rank(c) && c->cg_mr_fold != 0 && cg_folds_fit(c) && den_parts(c) <= kMrFoldMaxParts;
}

bool cg_beta_fold_ok(const cdfem_ctx *c)
{
    return cg_folds_fit(c) && (!multi_rank(c) || cg_mr_fold(c));
}

// den step inside the update (p <= 2: every update workgroup sums the apply's partials, one per
// 64-element brick; the high-order blocks leave too many partials and keep the finalizer)
bool cg_den_fold_on(const cdfem_ctx *c)
{
    return c->cg_den_fold != 0 && c->p <= 2 && den_parts(c) <= kDenFoldMaxParts && (!multi_rank(c) || cg_mr_fold(c));
}

// the first and last brick layers (the shared planes' partial sums) on stream s, the interior
// layers on the context stream; nbz >= 3
hipError_t launch_brick_cg2_split(cdfem_ctx *c, const double *r, const double *dinv, const double *d_old,
                                  double *d_new, double *q, hipStream_t s, double *x, int bfkk)
{
    if (c->nbz < 3) return hipErrorInvalidValue;
    BrickRun edge{0, c->nbz - 1, 2, s}, inner{1, 1, c->nbz - 2, c->stream};
    if (bfkk >= 0) {
        edge.kk = inner.kk = bfkk;
        edge.nupart = inner.nupart = cg_den_fold_grid(c);
    }
    const hipError_t e = brick_cg2_run(c, r, dinv, d_old, d_new, q, edge, x);
    if (e != hipSuccess) return e;
    return brick_cg2_run(c, r, dinv, d_old, d_new, q, inner, x);
}

hipError_t launch_cg_update_faces(cdfem_ctx *c, double *x, double *r, const double *q, const double *d,
                                  const double *dinv, const double *remote_lo, const double *remote_hi,
                                  bool den_step, bool xfold)
{
    const BrickGeom g = geom_of(c);
    const FastDiv fdx = make_fastdiv((uint32_t)c->Lx), fdxy = make_fastdiv((uint32_t)(c->Lx * c->Ly));
    // one dof per thread (no grid-stride up to 16384 blocks): the face gathers are dependent
    // loads, so every dof's chain must be in flight at once
    const int64_t need = (c->nl + kRedThreads - 1) / kRedThreads;
    const unsigned grid = (unsigned)(need < 16384 ? need : 16384);
    // den fold (one rank): a grid of cg_den_fold workgroups, partials after the apply's
    const bool ds = !den_step && cg_den_fold_on(c);
    const unsigned ugrid = ds ? (unsigned)cg_den_fold_grid(c) : grid;
    double *const upart = ds ? c->d_part + c->nblk : c->d_part;
    // the apply's den partials the den fold sums: one per brick, or the group sums (den_grp > 1)
    const double *const apart = c->den_grp > 1 ? c->d_gsum : c->d_part;
    const int napart = c->den_grp > 1 ? den_parts(c) : c->nblk;
#define CDFEM_UPD4(S_, XF_, PB_, DS_, EP_)                                                                 \
    hipLaunchKernelGGL((k_cg_update_faces<S_, XF_, PB_, DS_, EP_, SZ_>), dim3(ugrid), dim3(kRedThreads), 0, c->stream, x, \
                       r, d, dinv, c->d_face, c->d_ess, g, fdx, fdxy, c->zlo_shared, remote_lo, remote_hi, upart, \
                       c->d_state, (int)den_step, apart, napart)
    // the apply's essential-row patch entries (k_brick_cg EP: the Kronecker form at p <= 2)
    const bool ep = pa_af(c) == 2 && c->p <= 2;
#define CDFEM_UPD3(S_, XF_, PB_, DS_)                                                                      \
    if (ep && PB_) { CDFEM_UPD4(S_, XF_, PB_, DS_, PB_); } else { CDFEM_UPD4(S_, XF_, PB_, DS_, false); }
#define CDFEM_UPD2(S_, XF_, PB_)                                                                           \
    if (ds) { CDFEM_UPD3(S_, XF_, PB_, true); } else { CDFEM_UPD3(S_, XF_, PB_, false); }
    // predicated-load face sums: the patch buffer's byte offsets must fit 32 bits
    const bool pb = c->brick_upd_pb != 0 && brick_fits(c);
#define CDFEM_UPD(S_)                                                                                       \
    if (xfold) {                                                                                            \
        if (pb) { CDFEM_UPD2(S_, true, true); } else { CDFEM_UPD2(S_, true, false); }                       \
    } else {                                                                                                \
        if (pb) { CDFEM_UPD2(S_, false, true); } else { CDFEM_UPD2(S_, false, false); }                     \
    }
    // (SZ_: the patch's z side, in scope of CDFEM_UPD4; p = 3, 4 with ho_block_z 4: 2 x 2 x 4 blocks)
    if (c->p == 1) {
        constexpr int SZ_ = kBrick * 1 + 1;
        CDFEM_UPD(kBrick * 1 + 1);
    } else if (c->p == 2 || (c->p == 4 && c->hb_ez == 2)) {  // (p = 4: 2^3-element blocks, the same 9^3 patch)
        constexpr int SZ_ = kBrick * 2 + 1;
        CDFEM_UPD(kBrick * 2 + 1);
    } else if (c->p == 4 && c->hb_ez == 4) {
        constexpr int SZ_ = 4 * 4 + 1;
        CDFEM_UPD(kHoBrickEdge * 4 + 1);
    } else if (c->p == 3 && c->hb_ez == 2) {
        constexpr int SZ_ = kHoBrickEdge * 3 + 1;
        CDFEM_UPD(kHoBrickEdge * 3 + 1);
    } else if (c->p == 3 && c->hb_ez == 4) {
        constexpr int SZ_ = 4 * 3 + 1;
        CDFEM_UPD(kHoBrickEdge * 3 + 1);
    } else {
        return hipErrorInvalidValue;
    }
#undef CDFEM_UPD
#undef CDFEM_UPD2
#undef CDFEM_UPD3
#undef CDFEM_UPD4
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (ds && cg_beta_fold_ok(c)) return hipSuccess;  // the next apply takes the betanom step
    if (multi_rank(c)) return launch_fin_sum(c, (int)grid, 1);
    return launch_update_fin(c, (int)ugrid, ds ? c->nblk : 0);
}


// local partial sums of q = A d on the shared interface planes (what the neighbour must add)
template <int S>
__global__ void __launch_bounds__(256)
k_pack_qplanes(const double *__restrict__ q, const double *__restrict__ face, const BrickGeom g,
               int lo, int hi, double *__restrict__ out_lo, double *__restrict__ out_hi,
               const KrylovState *__restrict__ st)
{
    constexpr int s1 = S - 1;
    if (st->done) return;
    const int n = g.Lx * g.Ly;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const int gy = k / g.Lx, gx = k - gy * g.Lx;
    for (int side = 0; side < 2; ++side) {
        if (side == 0 ? !lo : !hi) continue;
        const int gz = side == 0 ? 0 : g.Lz - 1;
        double v;
        if (gx % s1 == 0 || gy % s1 == 0 || gz % s1 == 0) {
            int bxs[2], pxs[2], nxc = 0, bys[2], pys[2], nyc = 0, bzs[2], pzs[2], nzc = 0;
            const int qx = gx / s1, qy = gy / s1, qz = gz / s1;
            if (gx - qx * s1 == 0) {
                if (qx - 1 >= 0) { bxs[nxc] = qx - 1; pxs[nxc] = s1; ++nxc; }
                if (qx < g.nbx) { bxs[nxc] = qx; pxs[nxc] = 0; ++nxc; }
            } else { bxs[0] = qx; pxs[0] = gx - qx * s1; nxc = 1; }
            if (gy - qy * s1 == 0) {
                if (qy - 1 >= 0) { bys[nyc] = qy - 1; pys[nyc] = s1; ++nyc; }
                if (qy < g.nby) { bys[nyc] = qy; pys[nyc] = 0; ++nyc; }
            } else { bys[0] = qy; pys[0] = gy - qy * s1; nyc = 1; }
            if (gz - qz * s1 == 0) {
                if (qz - 1 >= 0) { bzs[nzc] = qz - 1; pzs[nzc] = s1; ++nzc; }
                if (qz < g.nbz) { bzs[nzc] = qz; pzs[nzc] = 0; ++nzc; }
            } else { bzs[0] = qz; pzs[0] = gz - qz * s1; nzc = 1; }
            v = 0.0;
            for (int kz = 0; kz < nzc; ++kz)
                for (int ky = 0; ky < nyc; ++ky)
                    for (int kx = 0; kx < nxc; ++kx) {
                        v += face[patch_idx<S>(g, bxs[kx], bys[ky], bzs[kz], pxs[kx], pys[ky], pzs[kz])];
                    }
        } else {  // inside one brick's patch
            const int qx = gx / s1, qy = gy / s1, qz = gz / s1;
            v = face[patch_idx<S>(g, qx, qy, qz, gx - qx * s1, gy - qy * s1, gz - qz * s1)];
        }
        (side == 0 ? out_lo : out_hi)[k] = v;
    }
}

hipError_t launch_pack_qplanes(cdfem_ctx *c, const double *q, hipStream_t s)
{
    const BrickGeom g = geom_of(c);
    const int n = (int)(c->Lx * c->Ly);
    const dim3 grid((n + 255) / 256), block(256);
    if (!s) s = c->stream;
    // (p = 3, 4: the 2^3-element blocks' cubic patches, S = 2p + 1; p = 4 shares S = 9 with p = 2)
    if (c->p >= 3 && c->hb_ez != kHoBrickEdge) return hipErrorInvalidValue;
    if (c->p == 1)
        hipLaunchKernelGGL(k_pack_qplanes<kBrick * 1 + 1>, grid, block, 0, s, q, c->d_face, g,
                           c->zlo_shared, c->zhi_shared, c->d_if[0], c->d_if[2], c->d_state);
    else if (c->p == 2 || c->p == 4)
        hipLaunchKernelGGL(k_pack_qplanes<kBrick * 2 + 1>, grid, block, 0, s, q, c->d_face, g,
                           c->zlo_shared, c->zhi_shared, c->d_if[0], c->d_if[2], c->d_state);
    else if (c->p == 3)
        hipLaunchKernelGGL(k_pack_qplanes<kHoBrickEdge * 3 + 1>, grid, block, 0, s, q, c->d_face, g,
                           c->zlo_shared, c->zhi_shared, c->d_if[0], c->d_if[2], c->d_state);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// ---- pa_uniform: the common element matrix of a uniformly refined box (k_brick_cg<..., MX 2>) ------
// Every element slot's factors against slot 0's (brick 0, lane 0: element (0, 0, 0)); any component
// further than tol flags the box as not uniform (plain vector stores of the same value).
__global__ void __launch_bounds__(256)
k_uniform_check(const double *__restrict__ gaff, const int32_t *__restrict__ perm, int nslots, int nc, int ne,
                double tol, int *__restrict__ bad)
{
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nslots) return;
    const int e = perm[s];
    if (e < 0 || e >= ne) return;
    const size_t b = (size_t)(s / kLanes), lane = (size_t)(s % kLanes);
    bool diff = false;
    for (int k = 0; k < nc; ++k) diff |= fabs(gaff[(b * nc + k) * kLanes + lane] - gaff[(size_t)k * kLanes]) > tol;
    if (diff) *bad = 1;
}

// column j of the element matrix = the Kronecker core (what k_brick_cg<..., AF 2> applies) on the unit
// vector e_j with element 0's factors: thread j writes A[i][j], row-major N x N
template <int D1, int Q1, unsigned K>
__global__ void __launch_bounds__(64)
k_uniform_elem(const double *__restrict__ gaff, const Tab<D1, Q1> T, double *__restrict__ A)
{
    constexpr int N = D1 * D1 * D1;
    const int j = threadIdx.x;
    if (j >= N) return;
    double g[QLayout<K, 3>::nc];
    kron_load_g<K>(gaff, 0, g);
    auto xl = [&](int z, int y, int x) { return (z * D1 + y) * D1 + x == j ? 1.0 : 0.0; };
    double Y[D1][D1][D1];
    kron_core<D1, Q1, K>(xl, g, T, Y);
    for (int i = 0; i < N; ++i) A[i * N + j] = Y[i / (D1 * D1)][(i / D1) % D1][i % D1];
}

hipError_t setup_uniform_elem(cdfem_ctx *c)
{
    if (c->d_uelem) {
        const hipError_t e = hipFree(c->d_uelem);
        c->d_uelem = nullptr;
        if (e != hipSuccess) return e;
    }
    if (!c->pa_uniform || !c->structured || c->qlay != 0 || c->dim != 3 || pa_af(c) != 2 || c->p != 2 ||
        c->rule_op.q1 != 4 || c->ncomp < 1 || (c->kinds != 7 && c->kinds != 5))
        return hipSuccess;
    const int nc = c->ncomp;
    std::vector<double> g0(nc);
    hipError_t e = hipMemcpy2D(g0.data(), sizeof(double), c->d_qaff, kLanes * sizeof(double), sizeof(double), nc,
                               hipMemcpyDeviceToHost);
    if (e != hipSuccess) return e;
    double gmax = 0.0;
    for (double v : g0) gmax = std::max(gmax, std::fabs(v));
    // one scratch allocation: the flag, then the N x N matrix
    constexpr int N = 27;
    void *scratch = nullptr;
    if ((e = hipMalloc(&scratch, sizeof(double) * (N * N + 1))) != hipSuccess) return e;
    int *bad = static_cast<int *>(scratch);
    double *A = static_cast<double *>(scratch) + 1;
    int hbad = 0;
    const int nslots = c->nblk * kLanes;
    e = hipMemsetAsync(bad, 0, sizeof(int), c->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_uniform_check, dim3((nslots + 255) / 256), dim3(256), 0, c->stream, c->d_qaff, c->d_perm,
                           nslots, nc, (int)c->ne, 1e-14 * gmax, bad);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    std::vector<double> h(N * N), op(2 * 7 * 64, 0.0);
    if (e == hipSuccess && !hbad) {
        const Tab<3, 4> T = make_tab<3, 4>(c->rule_op);
        if (c->kinds == 7) hipLaunchKernelGGL((k_uniform_elem<3, 4, 7>), dim3(1), dim3(64), 0, c->stream, c->d_qaff, T, A);
        else hipLaunchKernelGGL((k_uniform_elem<3, 4, 5>), dim3(1), dim3(64), 0, c->stream, c->d_qaff, T, A);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipMemcpyAsync(h.data(), A, sizeof(double) * N * N, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    }
    const hipError_t ef = hipFree(scratch);
    if (e != hipSuccess) return e;
    if (ef != hipSuccess) return ef;
    if (hbad) return hipSuccess;  // not uniform: the Kronecker form
    // the A operands of v_mfma_f64_16x16x4_f64 in lane order: [mt][ks][lane] = A[16 mt + (lane & 15)][4 ks + (lane >> 4)]
    for (int mt = 0; mt < 2; ++mt)
        for (int ks = 0; ks < 7; ++ks)
            for (int l = 0; l < 64; ++l) {
                const int i = 16 * mt + (l & 15), j = 4 * ks + (l >> 4);
                op[(mt * 7 + ks) * 64 + l] = (i < N && j < N) ? h[i * N + j] : 0.0;
            }
    void *d = nullptr;
    if ((e = hipMalloc(&d, sizeof(double) * op.size())) != hipSuccess) return e;
    e = hipMemcpy(d, op.data(), sizeof(double) * op.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(d);
        return e;
    }
    c->d_uelem = static_cast<double *>(d);
    return hipSuccess;
}

}  // namespace cdfem
