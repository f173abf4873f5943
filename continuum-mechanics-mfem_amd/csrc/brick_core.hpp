// brick_core.hpp — the structured-box lattice geometry, raw buffer access and the patch-buffer row
// sum, shared by the brick kernels (brick_kernels.hip) and the GMRES passes that read the structured
// Mult's patch buffer directly (gmres.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pa_core.hpp"

#ifndef CDFEM_PS8_SKIP
#define CDFEM_PS8_SKIP 1
#endif

namespace cdfem {

struct BrickGeom {
    int nbx, nby, nbz;  // bricks per axis
    int Lx, Ly, Lz;     // dof lattice per axis
    int xcd;            // 1: XCD-contiguous brick order (default; set_option "brick_xcd")
    int bz0, bzs;       // k_brick_cg: the launch covers brick layers bz0, bz0 + bzs, ... (all: 0, 1)
    const uint8_t *bess;  // per brick: 1 if a dof of its patch is essential (nullptr: assume so)
    // first-round stagger of the brick CG apply (k_brick_cg; set_option "brick_stagger"):
    // stag bits 0-3 a shift s, bits 4-8 a count n; stag_round = the workgroups resident at once (2 per SIMD)
    int stag = 0, stag_round = 0;
};

// The first round of a brick kernel's workgroups starts together, so every wave gathers its patch at
// once (one HBM burst) and then every wave computes (one VALU crush).  Workgroups b < stag_round with bit
// s of b set (s = log2 CUs: half of every CU's waves) sleep n x 2,048 cycles first, so half the first
// round gathers while the other half computes.  Launches of at least two rounds only.  C2 (4,096 bricks
// on 256 CUs, n = 4): k_brick_cg 39.0 -> 37.4 us (profiles/r06/ab_c2_stagger/); the GMRES leg's Mult
// (k_brick3d, whose gather is one vector) ran 35.0 -> 35.8 us with it and is left alone.
__device__ __forceinline__ void brick_stagger(const BrickGeom &g)
{
    if (g.stag == 0 || gridDim.x < 2u * (unsigned)g.stag_round) return;
    const unsigned wb = blockIdx.x;
    if (wb < (unsigned)g.stag_round && ((wb >> (g.stag & 15)) & 1u))
        for (int i = 0; i < ((g.stag >> 4) & 31); ++i) __builtin_amdgcn_s_sleep(32);
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

// The 1-8 patch-buffer entries of lattice dof (gx, gy, gz) summed in a fixed order (lower brick first
// per face axis, z outermost): eight buffer loads at fixed offsets from its own brick's entry P (the
// lower brick's face entry along x / y / z sits at P - 1 / P - R / P - A in the pencil layout of
// patch_idx), the absent ones at kOOB (read as 0).  Patches are S x S x SZ (SZ > S: the z-elongated
// high-order blocks, set_option "ho_block_z").
template <int S, int SZ = S>
__device__ __forceinline__ double patch_sum8(__amdgpu_buffer_rsrc_t bp, const BrickGeom &g, int gx, int gy, int gz)
{
    constexpr int s1 = S - 1, sz1 = SZ - 1;
    const int qx = min(gx / s1, g.nbx - 1), qy = min(gy / s1, g.nby - 1), qz = min(gz / sz1, g.nbz - 1);
    const int px = gx - qx * s1, py = gy - qy * s1, pz = gz - qz * sz1;
    const bool fx = px == 0 && qx > 0, fy = py == 0 && qy > 0, fz = pz == 0 && qz > 0;
    const uint32_t R = (uint32_t)g.nbx * S, A = (uint32_t)g.nby * S * R;
    const uint32_t P = (((uint32_t)qz * SZ + pz) * g.nby + qy) * S * R + (uint32_t)py * R + (uint32_t)qx * S + px;
    // (CDFEM_PS8_SKIP: a wave none of whose dofs sits on a y or z brick face issues no load for those
    // neighbours: the 64 consecutive dofs of a wave share one or two lattice rows, so most waves load
    // 2 entries, not 8.  An out-of-range buffer load moves no memory but still returns 64 lanes of
    // data; the skipped terms are the zeros they would have read, so the sum is unchanged)
    bool ax = true, ay = true, az = true;
    if constexpr (CDFEM_PS8_SKIP) {
        ax = __builtin_amdgcn_ballot_w64(fx) != 0;
        ay = __builtin_amdgcn_ballot_w64(fy) != 0;
        az = __builtin_amdgcn_ballot_w64(fz) != 0;
    }
    double t[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int sz = (k >> 2) & 1 ? 0 : 1, sy = (k >> 1) & 1 ? 0 : 1, sx = k & 1 ? 0 : 1;
        const bool ok = (!sx || fx) && (!sy || fy) && (!sz || fz);
        const uint32_t o = P - (uint32_t)sx - (uint32_t)sy * R - (uint32_t)sz * A;
        t[k] = 0.0;
        if ((!sx || ax) && (!sy || ay) && (!sz || az)) t[k] = bload(bp, ok ? 8u * o : kOOB);
    }
    double q = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) q += t[k];
    return q;
}

// GMRES on the structured Mult (set_option "gm_pb"): A_c V_j is each row's 1-8 patch entries of the
// patch-buffer Mult (k_brick3d<..., PBO>), V_j itself on the essential rows; pass 1 forms it there
// (k_gm_pass1<..., S>), so the E->L kernel's y write and pass 1's re-read of it go away
struct GmPatchSrc {
    const double *pb;    // the patch buffer
    const uint8_t *ess;  // essential flags
    const double *x;     // the Mult's input V_j
    BrickGeom g;
    FastDiv fdx, fdxy;   // lattice row / plane
    int S;               // patch side (4p + 1)
};
// the patch-buffer Mult is in use (brick_mult_pb, Kronecker form, offsets within 32 bits)
bool brick_mult_pb_on(const cdfem_ctx *c);
GmPatchSrc gm_patch_src(const cdfem_ctx *c, const double *x);

}  // namespace cdfem
