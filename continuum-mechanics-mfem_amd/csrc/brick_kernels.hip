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

#include "cdfem_internal.hpp"
#include "pa_core.hpp"
#include "reduce.hpp"

namespace cdfem {

struct BrickGeom {
    int nbx, nby, nbz;  // bricks per axis
    int Lx, Ly, Lz;     // dof lattice per axis
    int xcd;            // 1: XCD-contiguous brick order (default; set_option "brick_xcd")
    int bz0, bzs;       // k_brick_cg: the launch covers brick layers bz0, bz0 + bzs, ... (all: 0, 1)
};

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

// Patch positions i = t, t + 64, t + 128, ... of an S^3 patch (x fastest), advanced incrementally:
// 64 = dz S^2 + dy S + dx, so each step adds (dx, dy, dz) with carries (a few adds and selects
// instead of two constant divisions per position)
template <int S>
struct PatchWalk {
    int x, y, z;
    __device__ __forceinline__ explicit PatchWalk(unsigned t) : x((int)(t % S)), y((int)((t / S) % S)), z((int)(t / (S * S))) {}
    __device__ __forceinline__ void next()
    {
        constexpr int dx = 64 % S, dy = (64 / S) % S, dz = 64 / (S * S);
        x += dx;
        const int cx = x >= S ? 1 : 0;
        x -= S & -cx;
        y += dy + cx;
        const int cy = y >= S ? 1 : 0;
        y -= S & -cy;
        z += dz + cy;
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
template <int S>
__device__ __forceinline__ size_t patch_idx(const BrickGeom &g, int bx, int by, int bz, int px, int py, int pz)
{
    return ((((size_t)bz * S + pz) * g.nby + by) * S + py) * ((size_t)g.nbx * S) + (size_t)bx * S + px;
}

// v unchanged, but opaque to the optimiser: index arithmetic that depends on it cannot be hoisted
// above this point (LLVM otherwise computes a later phase's per-position indices at kernel entry
// and spills them across the element apply)
__device__ __forceinline__ int opaque(int v)
{
    asm volatile("" : "+v"(v));
    return v;
}

// Raw buffer access (MI355X buffer resources): a 32-bit byte offset from a scalar base instead of a
// 64-bit address per lane, and an offset past num_records (kOOB) reads 0 and drops a store, so the
// brick kernels' out-of-lattice positions and predicated stores need neither branches nor clamps.
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
constexpr uint32_t kOOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void *p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ double bload(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, uint32_t off, double v)
{
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, off, 0, 0);
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
template <int D1, int S>
__device__ __forceinline__ void brick_e2l(double *s_out, int o0, const double (&Y)[D1][D1][D1])
{
    constexpr int S2 = S * S;
    if constexpr (D1 == 3) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
#pragma unroll
            for (int cls = 0; cls < 8; ++cls) {
                const int l = e2l_member(cls, r);
                if (l < 0) continue;
                const int dz = l / 9, dy = (l / 3) % 3, dx = l % 3;
                s_out[o0 + dz * S2 + dy * S + dx] += Y[dz][dy][dx];
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
                    s_out[o0 + dz * S2 + dy * S + dx] += Y[dz][dy][dx];
                    __syncthreads();
                }
    }
}

// The 1-8 patch-buffer entries of lattice dof (gx, gy, gz) summed in a fixed order (lower brick first
// per face axis, z outermost): eight buffer loads at fixed offsets from its own brick's entry P (the
// lower brick's face entry along x / y / z sits at P - 1 / P - R / P - A in the pencil layout of
// patch_idx), the absent ones at kOOB (read as 0).
template <int S>
__device__ __forceinline__ double patch_sum8(__amdgpu_buffer_rsrc_t bp, const BrickGeom &g, int gx, int gy, int gz)
{
    constexpr int s1 = S - 1;
    const int qx = min(gx / s1, g.nbx - 1), qy = min(gy / s1, g.nby - 1), qz = min(gz / s1, g.nbz - 1);
    const int px = gx - qx * s1, py = gy - qy * s1, pz = gz - qz * s1;
    const bool fx = px == 0 && qx > 0, fy = py == 0 && qy > 0, fz = pz == 0 && qz > 0;
    const uint32_t R = (uint32_t)g.nbx * S, A = (uint32_t)g.nby * S * R;
    const uint32_t P = (((uint32_t)qz * S + pz) * g.nby + qy) * S * R + (uint32_t)py * R + (uint32_t)qx * S + px;
    double t[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int sz = (k >> 2) & 1 ? 0 : 1, sy = (k >> 1) & 1 ? 0 : 1, sx = k & 1 ? 0 : 1;
        const bool ok = (!sx || fx) && (!sy || fy) && (!sz || fz);
        const uint32_t o = P - (uint32_t)sx - (uint32_t)sy * R - (uint32_t)sz * A;
        t[k] = bload(bp, ok ? 8u * o : kOOB);
    }
    double q = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) q += t[k];
    return q;
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

// kOOB = 2^31 is out of range only for buffers below 2^31 bytes: the lattice vectors (8 N_L) and the
// patch buffer (8 S^3 per brick) must both fit, else an out-of-lattice load would read real data and a
// dropped store would land inside the buffer
bool brick_fits(const cdfem_ctx *c)
{
    const double S = kBrick * c->p + 1.0, lim = (double)c->brick_limit;
    return 8.0 * (double)c->nl < lim && 8.0 * (double)c->nblk * S * S * S < lim;
}

static BrickGeom geom_of(const cdfem_ctx *c)
{
    return BrickGeom{c->nbx, c->nby, c->nbz, (int)c->Lx, (int)c->Ly, (int)c->Lz, c->brick_xcd, 0, 1};
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
    // patch-buffer Mult (Kronecker form, byte offsets within 32 bits)
    const bool mpb = c->brick_mult_pb != 0 && pa_af(c) == 2 && brick_fits(c);
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
template <int D1, int Q1, unsigned K, int AF, int W = 1, bool XF = false, bool BF = false>
__global__ void __launch_bounds__(64, W)
k_brick_cg(const double *__restrict__ r, const double *__restrict__ dinv,
           const double *__restrict__ d_old, double *__restrict__ d_new, double *__restrict__ q,
           double *__restrict__ face, const double *__restrict__ qd, const uint8_t *__restrict__ ess,
           const Tab<D1, Q1> T, const BrickGeom g, int zlo_shared, double *__restrict__ part,
           KrylovState *__restrict__ st, double *__restrict__ x, const double *__restrict__ upart, int nupart,
           int kk)
{
    constexpr int P = D1 - 1;
    constexpr int S = kBrick * P + 1;
    constexpr int S2 = S * S, S3 = S * S * S;
    constexpr int NC = QLayout<K, 3>::nc;
    constexpr int NQ = Q1 * Q1 * Q1;
    __shared__ double s_in[S3];
    __shared__ double s_out[S3];
    if (st->done) return;
    double beta = st->beta;
    constexpr int NPL = 16;  // BF: partials per lane (nupart <= 64 NPL)
    double pv[NPL];
    if constexpr (BF) {
        if (kk > 0) {
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                const int j = (int)threadIdx.x + 64 * i;
                pv[i] = j < nupart ? upart[j] : 0.0;
            }
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
    double rv[NI], mv[NI], ov[NI], xv[NI];
    uint32_t offv[NI];
    uint8_t ev[NI];
    PatchWalk<S> pw0(t);
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const unsigned i = t + 64 * k;
        const int px = pw0.x, py = pw0.y, pz = pw0.z;
        pw0.next();
        const int gx = gx0 + px, gy = gy0 + py, gz = gz0 + pz;
        const bool in = i < S3 && gx < g.Lx && gy < g.Ly && gz < g.Lz;
        const uint32_t gid = (uint32_t)opaque(gx + Lx * gy + Lxy * gz);  // computed in every lane, selected
        offv[k] = in ? 8u * gid : kOOB;
        rv[k] = bload(br, offv[k]);
        mv[k] = bload(bm, offv[k]);
        ov[k] = bload(bo, offv[k]);
        ev[k] = __builtin_amdgcn_raw_buffer_load_b8(be, in ? gid : kOOB, 0, 0);
        const bool writer = in && (px < S - 1 || lastx) && (py < S - 1 || lasty) && (pz < S - 1 || lastz);
        if constexpr (XF) xv[k] = bload(bxf, writer ? offv[k] : kOOB);
    }
    if constexpr (BF) {
        if (kk > 0) {
            double v = 0.0;
#pragma unroll
            for (int i = 0; i < NPL; ++i) v += pv[i];
            const double B = wave_sum(v);
            // cg_update_logic's decision (cg_stop_kind), taken identically by every workgroup at the
            // host's update count kk; workgroup 0 records it at the same kk
            const bool stop = cg_stop_kind(st, B, kk) != kCgGoOn;
            if (blockIdx.x == 0 && t == 0) {
#ifdef CDFEM_DEBUG
                assert(st->iter == kk);
#endif
                cg_update_logic_at(st, B, kk);
            }
            if (stop) return;
            beta = B / st->nom;
        }
    }
    PatchWalk<S> pw1(t);
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        const unsigned i = t + 64 * k;
        if (k == NI - 1 && i >= S3) break;
        const int px = pw1.x, py = pw1.y, pz = pw1.z;
        pw1.next();
        const int gz = gz0 + pz;
        const bool in = offv[k] != kOOB;
        const double dn = mv[k] * rv[k] + beta * ov[k];  // 0 outside the lattice
        const bool e = ev[k] != 0;
        const bool writer = in && (px < S - 1 || lastx) && (py < S - 1 || lasty) && (pz < S - 1 || lastz);
        const uint32_t woff = writer ? offv[k] : kOOB;
        bstore(bd, woff, dn);
        if constexpr (XF) bstore(bxf, woff, xv[k] + alpha_prev * ov[k]);
        // (A_c d)_i = d_i on ess dofs
        den += (writer && e && !(zlo_shared && gz == 0)) ? dn * dn : 0.0;
        s_in[i] = e ? 0.0 : dn;
        s_out[i] = 0.0;
    }
    __syncthreads();

    const int ex = t & 3, ey = (t >> 2) & 3, ez = t >> 4;
    const int o0 = P * ez * S2 + P * ey * S + P * ex;
    auto xl = [&](int dz, int dy, int dx) { return s_in[o0 + dz * S2 + dy * S + dx]; };
    double Y[D1][D1][D1];
    elem_apply3d_af<D1, Q1, K, AF>(xl, q0, t, T, Y);

    // element-wise den contribution d0_e . (A_e d0_e) and deterministic in-LDS E->L
#pragma unroll
    for (int dz = 0; dz < D1; ++dz)
#pragma unroll
        for (int dy = 0; dy < D1; ++dy)
#pragma unroll
            for (int dx = 0; dx < D1; ++dx) den += s_in[o0 + dz * S2 + dy * S + dx] * Y[dz][dy][dx];
    brick_e2l<D1, S>(s_out, o0, Y);

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
            bstore(bp, 8u * (base + (uint32_t)pw.z * A + (uint32_t)pw.y * R + (uint32_t)pw.x), s_out[i]);
            pw.next();
        }
    }
    den = wave_sum(den);
    if (t == 0) part[b] = den;
}

// PB (set_option "brick_upd_pb"): the 1-8 patch entries of every dof as eight unconditional buffer
// loads at fixed offsets from its own brick's entry P (the lower brick's face entry along x / y / z
// sits at P - 1 / P - R / P - A in the pencil layout), the missing ones at kOOB (read as 0), summed
// in the branchy form's order (lower brick first per face axis, z outermost): bitwise the same q.
// DS (set_option "cg_den_fold", one rank): every workgroup sums the apply's den partials (apart,
// napart) in one fixed order and takes MFEM's den step itself (workgroup 0 records it), so the
// one-block den finalizer and its launch go away; the grid is a few hundred to a few thousand
// workgroups (grid-stride loop) to keep the redundant sums small, and its partials go to part.
template <int S, bool XF, bool PB = false, bool DS = false>
__global__ void __launch_bounds__(kRedThreads)
k_cg_update_faces(double *__restrict__ x, double *__restrict__ r, const double *__restrict__ d,
                  const double *__restrict__ dinv, const double *__restrict__ pb,
                  const uint8_t *__restrict__ ess, const BrickGeom g,
                  const FastDiv fdx, const FastDiv fdxy, int zlo_shared,
                  const double *__restrict__ remote_lo, const double *__restrict__ remote_hi,
                  double *__restrict__ part, KrylovState *__restrict__ st, int den_step,
                  const double *__restrict__ apart, int napart)
{
    constexpr int s1 = S - 1;
    __shared__ double sh[kRedThreads / 64 + 1];
    if (st->done) return;
    double alpha;
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
            qi = patch_sum8<S>(brsrc(pb, 8u * (uint32_t)g.nbx * g.nby * g.nbz * (S * S * S)), g, gx, gy, gz);
        } else if (gx % s1 == 0 || gy % s1 == 0 || gz % s1 == 0) {
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
            qi = 0.0;
            for (int kz = 0; kz < nzc; ++kz)
                for (int ky = 0; ky < nyc; ++ky)
                    for (int kx = 0; kx < nxc; ++kx) {
                        qi += pb[patch_idx<S>(g, bxs[kx], bys[ky], bzs[kz], pxs[kx], pys[ky], pzs[kz])];
                    }
        } else {  // inside one brick's patch
            const int qx = gx / s1, qy = gy / s1, qz = gz / s1;
            qi = pb[patch_idx<S>(g, qx, qy, qz, gx - qx * s1, gy - qy * s1, gz - qz * s1)];
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
    const double bs = block_sum(acc, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = bs;
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
    const double *qd = c->d_qaff ? c->d_qaff : c->d_qd;
    const double *upart = c->d_part + c->nblk;  // the den-fold update's partials
#define CDFEM_BCG4(AFF_, W_, XF_, BF_)                                                                      \
    if (whole)                                                                                               \
        CDFEM_LAUNCH(c, (k_brick_cg<D1, Q1, K, AFF_, W_, XF_, BF_>), grid, block, 0, r, dinv, d_old, d_new, q,  \
                     c->d_face, qd, c->d_ess, T, g, c->zlo_shared, c->d_part, c->d_state, x, upart, run.nupart, \
                     run.kk);                                                                                \
    else                                                                                                     \
        hipLaunchKernelGGL((k_brick_cg<D1, Q1, K, AFF_, W_, XF_, BF_>), grid, block, 0, run.s, r, dinv, d_old,   \
                           d_new, q, c->d_face, qd, c->d_ess, T, g, c->zlo_shared, c->d_part, c->d_state, x, upart, \
                           run.nupart, run.kk)
#define CDFEM_BCG3(AFF_, W_, XF_) CDFEM_BCG4(AFF_, W_, XF_, false)
#define CDFEM_BCG(AFF_, W_) CDFEM_BCG3(AFF_, W_, false)
    if (pa_af(c) == 2 && run.kk >= 0) {
        if (x) { CDFEM_BCG4(2, 2, true, true); }
        else { CDFEM_BCG4(2, 2, false, true); }
    } else if (pa_af(c) == 2) {
        if (x) { CDFEM_BCG3(2, 2, true); }
        else { CDFEM_BCG(2, 2); }
    } else if (pa_af(c) == 1) {
        CDFEM_BCG(1, 1);
    } else {
        CDFEM_BCG(0, 1);
    }
#undef CDFEM_BCG
#undef CDFEM_BCG3
#undef CDFEM_BCG4
    return hipGetLastError();
}

static hipError_t brick_cg2_run(cdfem_ctx *c, const double *r, const double *dinv, const double *d_old,
                                double *d_new, double *q, const BrickRun &run, double *x)
{
    const int q1 = c->rule_op.q1;
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
    BrickRun run{0, 1, c->nbz, c->stream};
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
bool cg_beta_fold_ok(const cdfem_ctx *c)
{
    return c->cg_beta_fold != 0 && c->cg_den_fold != 0 && !multi_rank(c) && pa_af(c) == 2 &&
           cg_den_fold_grid(c) <= 1024;
}

// the first and last brick layers (the shared planes' partial sums) on stream s, the interior
// layers on the context stream; nbz >= 3
hipError_t launch_brick_cg2_split(cdfem_ctx *c, const double *r, const double *dinv, const double *d_old,
                                  double *d_new, double *q, hipStream_t s, double *x)
{
    if (c->nbz < 3) return hipErrorInvalidValue;
    const hipError_t e = brick_cg2_run(c, r, dinv, d_old, d_new, q, BrickRun{0, c->nbz - 1, 2, s}, x);
    if (e != hipSuccess) return e;
    return brick_cg2_run(c, r, dinv, d_old, d_new, q, BrickRun{1, 1, c->nbz - 2, c->stream}, x);
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
    const bool ds = !den_step && !multi_rank(c) && c->cg_den_fold != 0;
    const unsigned ugrid = ds ? (unsigned)cg_den_fold_grid(c) : grid;
    double *const upart = ds ? c->d_part + c->nblk : c->d_part;
#define CDFEM_UPD3(S_, XF_, PB_, DS_)                                                                      \
    hipLaunchKernelGGL((k_cg_update_faces<S_, XF_, PB_, DS_>), dim3(ugrid), dim3(kRedThreads), 0, c->stream, x, r, \
                       d, dinv, c->d_face, c->d_ess, g, fdx, fdxy, c->zlo_shared, remote_lo, remote_hi, upart,  \
                       c->d_state, (int)den_step, c->d_part, c->nblk)
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
    if (c->p == 1) {
        CDFEM_UPD(kBrick * 1 + 1);
    } else if (c->p == 2) {
        CDFEM_UPD(kBrick * 2 + 1);
    } else {
        return hipErrorInvalidValue;
    }
#undef CDFEM_UPD
#undef CDFEM_UPD2
#undef CDFEM_UPD3
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (multi_rank(c)) return launch_fin_sum(c, (int)grid, 1);
    if (ds && cg_beta_fold_ok(c)) return hipSuccess;  // the next apply takes the betanom step
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
    if (c->p == 1)
        hipLaunchKernelGGL(k_pack_qplanes<kBrick * 1 + 1>, grid, block, 0, s, q, c->d_face, g,
                           c->zlo_shared, c->zhi_shared, c->d_if[0], c->d_if[2], c->d_state);
    else if (c->p == 2)
        hipLaunchKernelGGL(k_pack_qplanes<kBrick * 2 + 1>, grid, block, 0, s, q, c->d_face, g,
                           c->zlo_shared, c->zhi_shared, c->d_if[0], c->d_if[2], c->d_state);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace cdfem
