// cdfem_internal.hpp — context layout and kernel-launch declarations shared by the HIP sources.
//
// Device data layout (HBM), chosen for the thread-per-element PA kernels:
//   elements are grouped in blocks of 64 (one wavefront, lane = element within the block);
//   elem map   : int32 [nblk][nd][64]      L-dof of local dof l of element 64*b+lane; essential
//                                           dofs stored as -(gid+1) so the constrained gather
//                                           reads 0 without a second array
//   qdata      : f64   [nblk][nq][nc][64]  per quadrature point: D (sym, dim(dim+1)/2), C (dim),
//                                           M (1), only the kinds present (nc = 7 for K+M, 10 all)
//   E-vector Y : f64   [nblk][nd][64]      element outputs before the E->L sum
//   E->L map   : CSR over L-dofs, entries = positions in Y, element order ascending (deterministic)
// Every wave reads 512 contiguous bytes per qdata component, so the dominant stream is fully
// coalesced; the x gather is served by L2/MALL (x is 17 MB at 64^3 p=2).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/cdfem.h"

namespace cdfem {

constexpr int kLanes = 64;        // elements per element-block (= wavefront width)
constexpr int kMaxD1 = 6;
constexpr int kMaxQ1 = 8;

// 1D tables for one quadrature rule: B[q][d] = phi_d(xi_q), G[q][d] = phi_d'(xi_q), points, weights
struct Rule1D {
    int d1 = 0, q1 = 0;
    double B[kMaxQ1][kMaxD1] = {};
    double G[kMaxQ1][kMaxD1] = {};
    double pts[kMaxQ1] = {};
    double wts[kMaxQ1] = {};
};

// Product implementation of the 1D rules (independent of the oracle): basis.cpp
void gll_nodes(int p, double *x);
void gauss_legendre(int n, double *x, double *w);
// simplices (basis.cpp)
int simplex_rule(int dim, int n, std::vector<double> &xi, std::vector<double> &w);
// MFEM's tabulated triangle (order <= 9) / tetrahedron (order <= 6) rules; 0 when not tabulated
int mfem_simplex_rule(int dim, int order, std::vector<double> &xi, std::vector<double> &w);
// the rule IntRules.Get(simplex, order) returns: MFEM's table, else collapsed Gauss of that order
int simplex_rule_for_order(int dim, int order, std::vector<double> &xi, std::vector<double> &w);
int simplex_ndofs(int dim, int p);
void simplex_basis(int dim, int p, const double *xi, double *phi, double *dphi);
extern const int kSimplexEdge[6][2];
double p3_edge_t(int k);
// element partition helpers (partition.cpp, host only)
void partition_rcb(int dim, int ne, int nv, const double *elem_verts, int nranks, int32_t *part);
void p3_tri_nodes(double (*X)[2]);
extern const int kTriEdge[3][2];
Rule1D make_rule(int p, int q1);
// MFEM default rule sizes on multilinear tensor elements (which: 0 operator, 1 LF, 2 L2 error)
int rule_points_1d(int which, int dim, int p);

// High-order qdata layout (cdfem_ctx::qlay = 1, 3D p >= 3, ho_kernels.hip): per element and
// quadrature plane qz one block of nc * Q1^2 doubles (padded to an even count so every block is
// 16-byte aligned), components paired as [pair][qxy][2] with an odd last component as [qxy].
__host__ __device__ constexpr int qd_ho_plane(int nc, int q1) { return (nc * q1 * q1 + 1) & ~1; }
__host__ __device__ inline size_t qd_ho_index(int64_t e, int c, int q, int nc, int q1)
{
    const int qq = q1 * q1, qz = q / qq, qxy = q - qz * qq;
    const size_t base = ((size_t)e * q1 + qz) * qd_ho_plane(nc, q1);
    return base + ((c < (nc & ~1)) ? ((size_t)(c >> 1) * qq + qxy) * 2 + (c & 1) : (size_t)(nc & ~1) * qq + qxy);
}

// Device-side Krylov state (one per context), updated only by kernels.
struct KrylovState {
    double nom, nom0, den, alpha, beta, betanom, r0;
    double red[4];  // rank-local reductions awaiting the all-reduce (0 den, 1 betanom, 2 nom)
    int iter, done, converged, final_iter, max_iter, first_den;
    int xflush;     // x-fold CG (cg_xfold): the last update's x += alpha d is still pending (stopped by
                    // the update logic, so no further apply folded it): k_cg_xflush applies it
};

// Device-side GMRES(m) state (gmres.hip).  The first 32 bytes are what the host polls.
constexpr int kGmMaxRestart = 64;
struct GmresState {
    int cycle_done, done, converged, its;
    double res;
    int j, kk;
    // ----
    int max_it, m;
    double ttol, res0;
    double s[kGmMaxRestart + 1];   // basis scales: v_i = s_i * V_i
    double g[kGmMaxRestart + 1], cs[kGmMaxRestart], sn[kGmMaxRestart];
    double H[(kGmMaxRestart + 1) * kGmMaxRestart];  // row-major, leading dimension kGmMaxRestart
    double red[kGmMaxRestart + 1];  // multi-rank: rank-local sums awaiting the all-reduce
    double y[kGmMaxRestart];        // cycle end: the least-squares solution, scaled by s
};
constexpr size_t kGmPollBytes = 32;

// ILU(0) preconditioner state (ilu_kernels.hip)
struct IluState {
    bool ready = false;
    double *F = nullptr;                 // factors in the CSR pattern (unit-lower L, U packed)
    int32_t *rows_l = nullptr, *rows_u = nullptr;  // rows grouped by level
    std::vector<int32_t> ptr_l, ptr_u;   // level pointers (host)
    double *z = nullptr;                 // output of one application
    // multi-rank (PETSc bjacobi, one ILU(0) block per rank): the factored matrix is the owned
    // diagonal block of the global eliminated matrix, on rows/columns [skip_lo, nl), in its own
    // pattern; the sweeps write the owned part of z and the owners' values are then copied to the
    // non-owned shared entries
    bool block = false;
    int32_t *rp = nullptr, *cols = nullptr, *diag = nullptr;  // block pattern (owned; else the CSR's)
    int64_t nnz = 0;
    hipGraph_t graph = nullptr;          // the captured forward + backward sweeps
    hipGraphExec_t exec = nullptr;
};

struct Comm;  // comm.hip

struct ProfileSlot {
    std::vector<hipEvent_t> ev;  // pairs
    int used = 0;
    double total_ms = 0.0;
    int64_t count = 0;
    std::vector<float> each;  // per-launch ms since the last reset (cdfem_profile_launches)
};

}  // namespace cdfem

struct cdfem_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;

    // mesh / space
    int dim = 0, p = 0, d1 = 0, nd = 0, ne = 0, nblk = 0, nv = 0;
    int qlay = 0;                       // 0: element blocks of 64 (thread per element), 1: element-major
                                        //    map / E-vector / qdata (wave per element, 3D p >= 3)
    int64_t nl = 0;
    int n_ess = 0;
    bool mesh_ready = false;
    double *d_verts = nullptr;          // [ne][nv][dim]
    int32_t *d_map = nullptr;           // [nblk][nd][64], ess negative
    int32_t *d_e2l_off = nullptr;       // [nl+1]
    int32_t *d_e2l_pos = nullptr;       // [ne*nd]
    uint8_t *d_ess = nullptr;           // [nl]
    int32_t *d_ess_list = nullptr;      // [n_ess]
    int32_t *d_perm = nullptr;          // [nblk*64] element at (block, lane), -1 = padding
    std::vector<int32_t> h_dofs;        // host copy of the element dof map (ne*nd)
    std::vector<uint8_t> h_ess;         // host essential marker (nl)

    // structured-box fast path (cdfem_mesh_set_structured): 4x4x4-element bricks
    bool structured = false;
    bool epencil = false;               // qlay 1 on a structured box: pencil E-vector layout (ho_eidx)
    int sx = 0, sy = 0, sz = 0;         // elements per axis of the local box
    int nbx = 0, nby = 0, nbz = 0;      // bricks per axis
    // 3D p = 3, 4 on a structured box: blocks of kHoBrickEdge^3 elements for the high-order brick CG
    // (brick_kernels.hip k_hobrick_cg; set_option "ho_brick")
    int hb_nbx = 0, hb_nby = 0, hb_nbz = 0, hb_nblk = 0;
    int ho_block_z = 2;                 // set_option "ho_block_z": elements per block along z (2 or 4), read by
                                        // cdfem_mesh_set_structured; 4 = 2 x 2 x 4 blocks
    int hb_ez = 2;                      //   the block depth of the current structured box
    uint8_t *d_bess = nullptr;          // per brick (block): 1 if a dof of its patch is essential
    int ho_brick = 1;                   // set_option "ho_brick": high-order CG through k_hobrick_cg + the brick update
    double *d_hbpart = nullptr;         // den partials summed in two stages: k_hobrick_cg's, and k_brick_cg's past
                                        // kDenFoldMaxParts bricks on one rank (one per brick)
    double *den_out = nullptr;          // k_brick_cg writes its den partials here instead of d_part (set by the solve)
    // grouped den partials (p <= 2 past the fold bounds: C5's per-rank slab of 32,768 bricks, its 262,144 on one
    // GPU): the last-arriving brick of each group of den_grp sums the group's partials in a fixed order
    // (k_brick_cg tail: write-through partial, agent-scope arrival count), so the folds sum <= 4,096 values
    int den_grp = 1;                    // group size of the running solve (1: one partial per brick)
    int den_group_opt = 0;              // set_option "den_group": 0 automatic, else this group size (tests)
    double *d_gsum = nullptr;           // [ceil(nblk / den_grp)] group sums
    uint32_t *d_gcnt = nullptr;         // [same] arrival counters (0 between launches)
    int64_t gsum_cap = 0;
    int ho_brick_mfma = 0;              // set_option "ho_brick_mfma": its x stage on v_mfma_f64_16x16x4_f64 (kinds 7)
    int brick_stagger = -1;             // set_option "brick_stagger": BrickGeom::stag (-1 automatic, 0 off)
    int brick_mfma = 0;                 // set_option "brick_mfma": k_brick_cg's x stage on the matrix cores (p = 2, kinds 7)
    int pa_uniform = 1;                 // set_option "pa_uniform": when every element's factors equal the first
                                        // element's (a uniformly refined box, what MFEM's MakeCartesian3D
                                        // gives), the p = 2 brick CG applies that element's 27 x 27 matrix on
                                        // the matrix cores (k_brick_cg<..., MX 2>); 0 keeps the Kronecker form
    double *d_uelem = nullptr;          // pa_uniform: the common element matrix in MFMA A-operand order
    int64_t Lx = 0, Ly = 0, Lz = 0;     // dof lattice per axis
    double *d_face = nullptr;           // [nblk][F] brick-face partial sums
    double *d_ones = nullptr;           // all-ones vector (unpreconditioned brick CG)
    double *d_dalt = nullptr;           // second search-direction buffer (brick CG)
    int nface = 0;                      // F
    int gm_ept = 0;                     // set_option "gm_ept": GMRES orthogonalisation entries per thread (0: auto, orth_ept)
    int gm_ept_auto = 4;                // the automatic choice for vectors of gm_ept_n entries
    int gm_pb = 1;                      // set_option "gm_pb": GMRES pass 1 reads the structured Mult's patch buffer
    int gm_poll = 4;                    // set_option "gm_poll": the host polls the GMRES state every k inner steps
    int64_t gm_ept_n = -1;
    int brick_xcd = 1;                  // k_brick_cg brick order: 0 dispatch, 1 XCD-contiguous (default)
    // the brick kernels address r, M^-1, d, x, ess and the patch buffer through buffer resources with
    // 32-bit byte offsets and the out-of-range marker kOOB = 2^31, so every such buffer must stay below
    // 2^31 bytes (8 N_L and 8 S^3 nblk); larger boxes take the generic 64-bit-indexed element kernels.
    // set_option "brick_byte_limit" lowers the bound (tests force the fallback on small boxes).
    int64_t brick_limit = (int64_t)1 << 31;
    // slab partition: the largest L-vector and brick count over all ranks (all-reduced by cdfem_set_slab),
    // so brick_fits takes the same decision on every rank (slabs of different sizes near the
    // bound would otherwise send ranks down CG paths with different collective sequences)
    int64_t slab_nl_max = 0, slab_nb_max = 0;
    int ncu = 0;                        // compute units of the device
    int zlo_shared = 0;                 // local gz=0 plane owned by the rank below (slabs)
    int zhi_shared = 0;                 // local gz=Lz-1 plane shared with the rank above
    cdfem::Comm *comm = nullptr;        // rank communicator (comm.hip), nullptr on one GPU
    int rank = 0, nranks = 1;
    double *d_if[4] = {};               // interface planes: send_lo, recv_lo, send_hi, recv_hi
    // rank partition of the L-vector: 0 none, 1 z-slab (cdfem_set_slab), 2 general element
    // partition (cdfem_set_shared).  Both number the dofs owned by a lower rank first, so the
    // owned (true) dofs are the suffix [skip_lo, nl) and every dot product skips the prefix.
    int part_mode = 0;
    int64_t skip_lo = 0;
    // general partition: per neighbour rank (ascending) the shared local dofs, same order on both
    // sides; send/recv buffers concatenated in neighbour order
    std::vector<int32_t> nbr_rank;
    std::vector<int64_t> nbr_off;       // [n_nbr + 1]
    std::vector<int32_t> h_sh_idx;      // [n_sh] local dof of send/recv slot (host copy)
    int32_t *d_sh_idx = nullptr;        // [n_sh] local dof of send/recv slot
    double *d_sh_send = nullptr, *d_sh_recv = nullptr;
    int32_t n_shd = 0;                  // distinct shared dofs
    int32_t *d_shd = nullptr;           // [n_shd] their local index
    int32_t *d_shd_off = nullptr;       // [n_shd + 1] contributions, ascending rank (own = -1)
    int32_t *d_shd_src = nullptr;       //   source: -1 own partial, else recv slot
    int32_t *d_shd_owner = nullptr;     // [n_shd] recv slot of the owner's copy, -1 if owned here

    // rules
    cdfem::Rule1D rule_op, rule_lf, rule_err;

    // geometry family: 0 tensor (quad/hex: PA), 1 simplex (tri/tet: FA, cdfem_mesh_upload_simplex)
    int geom = 0;
    // simplex integrator rules (MFEM's GetRule on affine simplices): diffusion order 2p - 2,
    // convection and mass order 2p, each on MFEM's tabulated rule (simplex_rule_for_order)
    int nq_sd = 0, nq_scm = 0;          // points of the diffusion / convection + mass rules
    double *d_stab = nullptr;           // rule tables, diffusion rule first then the convection + mass
                                        // rule, each phi [nq][nd], dphi [nq][nd][dim], w [nq]
    std::vector<double> h_verts;        // simplex host geometry (quadrature points for coefficients)
    std::vector<double> h_sxi_d, h_sxi_cm;  // the two rules' points (reference coordinates)
    int nq_lf = 0;                      // simplex LINEARFORM rule (collapsed Gauss, n = p + 3)
    std::vector<double> h_sxi_lf;
    double *d_stab_lf = nullptr;        // phi [nq_lf][nd], w [nq_lf]
    // full assembly (cdfem_fa_setup): CSR with sorted columns + deterministic contribution lists
    bool fa_ready = false;
    int64_t nnz = 0;
    int32_t *d_rowptr = nullptr, *d_cols = nullptr, *d_diagpos = nullptr;
    int32_t *d_coff = nullptr, *d_cpos = nullptr;  // per-nonzero contribution lists into d_Ee
    double *d_vals = nullptr;           // A
    double *d_vals_c = nullptr;         // eliminated A (FormLinearSystem, DIAG_ONE)
    double *d_Ee = nullptr;             // element matrices [blk][nd*nd][64]
    int64_t nslices = 0, nstored = 0;   // SELL-64 copy (the SpMV layout)
    int32_t *d_sptr = nullptr, *d_srows = nullptr, *d_scols = nullptr, *d_smap = nullptr;
    double *d_tpart = nullptr;          // den partials of the fused high-order CG apply (one per tile block)
    double *d_ktab = nullptr;           // k_apply3d_ktile's rows of M, K, C, C^T (canonical entries, [4][D1][D1])
    double h_ktab[4 * 5 * 5] = {};      //   host copy (source of the async upload)
    int ktab_key = -1;                  //   (p, rule) the table was built for
    int16_t *d_sdel = nullptr;          // 16-bit column deltas (null when the bandwidth does not fit)
    uint8_t *d_swide = nullptr;         // per slice: 1 = streams 32-bit columns (mixed layout; null: none)
    int64_t sell_nnz_wide = 0;          // real entries in the 32-bit slices of a mixed layout
    int mr_overlap = 1;                 // set_option "mr_overlap": slab CG exchange overlapped with interior bricks
    hipStream_t stream2 = nullptr;      // side stream of the overlapped exchange (created on first use)
    hipEvent_t ov_ev[2] = {};           // fork / join of the side stream
    int brick_mult_pb = 1;              // set_option "brick_mult_pb": structured Mult through the patch buffer
    int cg_beta_fold = 1;               // set_option "cg_beta_fold": brick CG betanom step in the next apply
    int cg_mr_fold = 1;                 // set_option "cg_mr_fold": both folds on several ranks (partials all-reduced)
    double *d_small = nullptr;          // a few doubles of device scratch (mr_fold_agreed's all-reduce)
    int cg_den_fold = 1024;             // set_option "cg_den_fold": brick CG den step in the update (N workgroups; 0 off)
    int brick_upd_pb = 1;               // set_option "brick_upd_pb": predicated-load face sums in the brick CG update
    int ho_dfold = 1;                   // set_option "ho_dfold": CG direction folded into the Kronecker tile apply
    int ho_mfma = 0;                    // set_option "ho_mfma": bit 0 = stage x of the p >= 3 tile apply on MFMA
    int cg_fused = 1;                   // set_option "cg_fused": fused high-order CG iteration (p >= 3 boxes)
    int cg_xfold = 1;                   // set_option "cg_xfold": brick CG folds x += alpha d into the next apply
    int spmv_index16 = 1;               // set_option "spmv_index16": SpMV streams d_sdel when present
    int sell_mode = 8;                  // set_option "sell_order" (read when the FA pattern is built)
    int sell_window = 0;                // set_option "sell_window": rows per window of a windowed order (0 auto)
    int spmv_lds = -1;                  // set_option "spmv_lds": rows per LDS-staged SpMV window (0 off, -1 auto)
    int32_t *d_hptr = nullptr, *d_hidx = nullptr;  // LDS-staged windows (FaPattern::hptr / hidx / sloc)
    uint16_t *d_sloc = nullptr;
    int64_t lds_rows = 0;               // rows per window of the current LDS layout (0: none)
    int32_t lds_max = 0;                // largest window halo (doubles)
    int64_t lds_halo = 0;               // staged columns over all windows
    int spmv_lpr = 0;                   // set_option "spmv_lpr": lanes per row of the LDS layouts (0 auto, 1, 2, 4)
    int sell_lpr = 1;                   // lanes per row of the current SELL copy
    int spmv_xcd = 1;                   // set_option "spmv_xcd": contiguous slice range per XCD (windowed layout)
    int32_t *d_rperm = nullptr;         // SpMV space order: space row -> mesh row (null: mesh order)
    bool sell_windowed = false;         // slices cut from the space order (kernel row = slice * 64 + lane)
    double *d_pv[2] = {};               // permuted-space scratch (apply in mesh order; solve B / X)
    bool perm_space = false;            // inside a solve that runs in the permuted order
    double *d_dinv_p = nullptr;         // the Jacobi scale in permuted order (during such a solve)
    double *d_svals = nullptr, *d_svals_c = nullptr;
    cdfem::IluState ilu;                // ILU(0) of the eliminated matrix (GMRES pc = ILU)

    // partial assembly
    unsigned kinds = 0;
    int ncomp = 0;
    bool pa_ready = false;
    double *d_qd = nullptr;             // [nblk][nq][nc][64]
    double *d_qaff = nullptr;           // [nblk][nc][64] per-element factors of an affine mesh (qd = W_q * g)
    bool mesh_affine = false;           // every element a parallelepiped (checked at upload)
    int pa_affine = 2;                  // set_option "pa_affine": when the mesh allows, 1 form the point data
                                        // from the affine factors, 2 the Kronecker form of the same factors
                                        // (3D p <= 2 applies; the p >= 3 tile apply takes 2 as 1); 0 stream
    double *d_Ye = nullptr;             // [nblk][nd][64]
    double *d_dinv = nullptr;           // Jacobi (constrained: ess -> 1)
    bool dinv_ready = false;

    // work vectors (L-size)
    double *d_w[8] = {};                // staging + Krylov vectors
    double *d_part = nullptr;           // reduction partials [red_blocks + nblk]
    int red_blocks = 1024;
    cdfem::KrylovState *d_state = nullptr;
    cdfem::KrylovState *h_state = nullptr;  // pinned
    double *d_gm = nullptr;             // GMRES basis (restart+1) * nl
    int gm_cap = 0;
    double *d_gm_part = nullptr;        // GMRES partials [(restart+1) * blocks]
    double *d_lfq = nullptr;            // cdfem_lf_assemble: the point values (kept across calls)
    size_t lfq_cap = 0;
    cdfem::GmresState *d_gmst = nullptr;   // device GMRES state
    cdfem::GmresState *h_gmpoll = nullptr; // pinned, 2 poll slots of kGmPollBytes
    hipEvent_t gm_ev[2] = {};

    // profiling
    bool profile = false;
    cdfem::ProfileSlot prof[CDFEM_K_COUNT];
    unsigned prof_mask = ~0u;  // kernels that get HIP events while profiling (set_option profile_mask)
    hipEvent_t ext_ev[2] = {};  // armed by prof_mark(begin): the next CDFEM_LAUNCH records these
                                // events at its own dispatch start / end (hipExtLaunchKernelGGL)
};

// Launch on the context stream; when a profiling mark is armed (prof_mark), the kernel records the
// mark's event pair itself at dispatch start and completion (hipExtLaunchKernelGGL), so the timed
// interval is the kernel alone, without the ~5-10 us an event record adds ahead of a ~100 us
// kernel.  Used for the dominant (roofline) kernels.
#define CDFEM_LAUNCH(c, kernel, grid, block, shm, ...)                                                       \
    do {                                                                                                     \
        if ((c)->ext_ev[0]) {                                                                                \
            hipExtLaunchKernelGGL(kernel, grid, block, shm, (c)->stream, (c)->ext_ev[0], (c)->ext_ev[1], 0,   \
                                  __VA_ARGS__);                                                              \
            (c)->ext_ev[0] = (c)->ext_ev[1] = nullptr;                                                       \
        } else {                                                                                             \
            hipLaunchKernelGGL(kernel, grid, block, shm, (c)->stream, __VA_ARGS__);                          \
        }                                                                                                    \
    } while (0)

namespace cdfem {

// the high-order tile apply forms the point data from the affine factors; with MFMA stages
// (ho_mfma) only on the full operator (kinds 7) and the masks 1, 8, 9, else ho_mfma keeps the stream
inline bool tile_affine(const cdfem_ctx *c)
{
    if (c->d_qaff == nullptr) return false;
    if (c->ho_mfma == 0) return true;
    return c->kinds == 7 && (c->ho_mfma == 1 || c->ho_mfma == 8 || c->ho_mfma == 9);
}
// the high-order tile apply in the Kronecker form of the affine factors (k_apply3d_ktile)
inline bool tile_kron(const cdfem_ctx *c) { return c->d_qaff != nullptr && c->ho_mfma == 0 && c->pa_affine == 2; }
// the element core of the 3D p <= 2 applies (pa_core.hpp elem_apply3d_af): 0 per-point stream,
// 1 point data from the affine factors, 2 Kronecker form of the factors
inline int pa_af(const cdfem_ctx *c) { return c->d_qaff == nullptr ? 0 : (c->pa_affine == 2 ? 2 : 1); }
// the brick CG applies the common element matrix of a uniform box (pa_uniform: formed at the PA setup;
// set_option "pa_uniform" 0 switches back to the Kronecker form without a new setup)
inline bool uniform_elem(const cdfem_ctx *c) { return c->d_uelem != nullptr && c->pa_uniform != 0 && pa_af(c) == 2; }

// ---- kernel launchers (pa_kernels.hip) -------------------------------------------------------
hipError_t launch_setup_qdata(cdfem_ctx *c, const double *d_kappa_q, const double *d_kmat_q, double kappa, double alpha,
                              const double *conv, const double *d_conv_q, const double *d_mass_q,
                              double mass);
hipError_t launch_apply(cdfem_ctx *c, const double *x, double *Ye, bool constrained);
hipError_t launch_apply_wpe(cdfem_ctx *c, const double *x, double *Ye, bool con, const KrylovState *st);
hipError_t launch_apply_st(cdfem_ctx *c, const double *x, double *Ye, bool constrained,
                           const KrylovState *st);
hipError_t launch_diag_elem(cdfem_ctx *c, double *Ye);
hipError_t launch_lf_elem(cdfem_ctx *c, const double *d_fq, double *Ye);
hipError_t launch_quad_points(cdfem_ctx *c, const Rule1D &r, double *xyz);
bool apply_supported(int dim, int p);

// ---- structured brick kernels (brick_kernels.hip) --------------------------------------------
constexpr int kBrick = 4;               // elements per brick edge (4^3 = 64 = one wavefront)
constexpr int kHoBrickEdge = 2;         // p = 3, 4: elements per block edge of the high-order brick CG
bool brick_supported(int dim, int p);
int brick_count(const cdfem_ctx *c);        // bricks (p <= 2) or high-order blocks (p = 3, 4)
int brick_patch_side(const cdfem_ctx *c);   // S: 4p + 1 (p <= 2), 2p + 1 (p = 3, 4)
int brick_patch_side_z(const cdfem_ctx *c); // the patch's z side: S, or hb_ez p + 1 (p = 3, 4)
bool cg_den_fold_on(const cdfem_ctx *c);
bool cg_mr_fold(const cdfem_ctx *c);
// den partial groups of the brick CG apply at p <= 2: 1 when the bricks fit the fold bounds, else the
// power of two (<= 64) that brings them to <= kDenGroupParts sums; den_parts = the folds' partial count
constexpr int kDenGroupParts = 4096;
int den_group(const cdfem_ctx *c);
int den_parts(const cdfem_ctx *c);
constexpr int kMrFoldMaxParts = 8192;   // cg_mr_fold: apply partials every update workgroup re-sums
constexpr int kDenFoldMaxParts = 16384; // cg_den_fold: beyond (C5's 256^3 on one GPU: 262,144 bricks) the
                                        // den finalizer (the update workgroups' redundant sums grow with it)
// the Kronecker tile's x-stage table (ho_kernels.hip), built for the context's p and rule
hipError_t ho_ktab(cdfem_ctx *c, const double **out);
// every buffer the brick kernels reach through a 32-bit buffer resource is below c->brick_limit bytes
bool brick_fits(const cdfem_ctx *c);
// y = A x (constrained: ess in -> 0, y[ess] = x[ess]); fused E->L through LDS + face partials
hipError_t launch_brick_mult(cdfem_ctx *c, const double *x, double *y, bool constrained, int which);


// ---- vector kernels (vec_kernels.hip) --------------------------------------------------------
// y = E->L sum of Ye; constrained: y[ess] = x[ess]; if dot_part != nullptr also reduces
// partial sums of y.x into dot_part[blockIdx] and the last block writes state->den and alpha.
hipError_t launch_e2l(cdfem_ctx *c, const double *Ye, const double *x, double *y, bool constrained,
                      int cg_mode);
hipError_t launch_set_ess(cdfem_ctx *c, double *y, const double *x);          // y[ess] = x[ess]
hipError_t launch_mask_ess(cdfem_ctx *c, const double *x, double *y);        // y = x, y[ess] = 0
hipError_t launch_axpby(cdfem_ctx *c, double a, const double *x, double b, double *y);  // y = a x + b y
hipError_t launch_axpby_n(cdfem_ctx *c, int64_t n, double a, const double *x, double b, double *y);  // n entries
hipError_t launch_dinv(cdfem_ctx *c, const double *diag, double *dinv);      // 1/diag, ess -> 1
// CG pieces (MFEM CGSolver semantics)
hipError_t launch_cg_init(cdfem_ctx *c, const double *B, double *x, double *r, double *z, double *d,
                          const double *dinv, double rel_tol, double abs_tol, int max_iter);
hipError_t launch_cg_update(cdfem_ctx *c, double *x, double *r, double *z, const double *d,
                            const double *dinv);
hipError_t launch_cg_direction(cdfem_ctx *c, const double *z, double *d);
// x += alpha d, r -= alpha q, betanom = (r, M^{-1} r); z is not stored (brick path recomputes it)
hipError_t launch_cg_update_noz(cdfem_ctx *c, double *x, double *r, const double *q, const double *d,
                                const double *dinv);
hipError_t launch_zero(cdfem_ctx *c, double *y);
// one-block finalizers: den = sum(d_part[0..nparts)) (MFEM CG den step); betanom (update step)
hipError_t launch_den_fin(cdfem_ctx *c, int nparts);
hipError_t launch_update_fin(cdfem_ctx *c, int nparts, int64_t off = 0);
// brick CG v2 (brick_kernels.hip): d_new = M^{-1} r + beta d_old, q/face partials, den partials
// pa_uniform: after the PA setup of a structured p = 2 box in the Kronecker form (kinds 7 or 5), checks
// that every element's factors equal the first element's (within 1e-14 of the largest) and, if so, forms
// that element's 27 x 27 matrix (column j = the Kronecker core on e_j) in d_uelem (freed otherwise)
hipError_t setup_uniform_elem(cdfem_ctx *c);
hipError_t launch_brick_cg2(cdfem_ctx *c, const double *r, const double *dinv, const double *d_old,
                            double *d_new, double *q, double *x = nullptr, int bfkk = -1);
int cg_den_fold_grid(const cdfem_ctx *c);
bool cg_beta_fold_ok(const cdfem_ctx *c);
// x-fold CG after the loop: x += alpha d_m when the last update's x term is still pending
// (d_m in dbuf[(m - 1) & 1], m = the final iteration)
hipError_t launch_cg_xflush(cdfem_ctx *c, double *x, const double *d0, const double *d1);
// q from interior/face partials (+ remote interface sums), x += alpha d, r -= alpha q, betanom
hipError_t launch_cg_update_faces(cdfem_ctx *c, double *x, double *r, const double *q, const double *d,
                                  const double *dinv, const double *remote_lo, const double *remote_hi,
                                  bool den_step = false, bool xfold = false);
// generic deterministic dot into host-visible scalar via state (used by GMRES / tests)
hipError_t launch_dot(cdfem_ctx *c, const double *a, const double *b, double *d_out);
// multi-rank CG: rank-local (d, q) over owned entries into the state's den slot (all-reduce next)
hipError_t launch_den_local(cdfem_ctx *c, const double *d, const double *q);

// ---- communication (comm.hip) -----------------------------------------------------------------
void comm_destroy(cdfem_ctx *c);
void comm_allreduce(cdfem_ctx *c, double *dbuf, int n);
void comm_exchange(cdfem_ctx *c, const double *send_lo, double *recv_lo, const double *send_hi,
                   double *recv_hi, int64_t n, hipStream_t s = nullptr);
void interface_sum(cdfem_ctx *c, double *v);  // L-vector interface planes summed over ranks
// non-owned shared entries of an L-vector <- the owner's value (MFEM P applied to R v)
void interface_copy_owner(cdfem_ctx *c, double *v);
// general partition: send[off[k]..off[k+1]) -> nbr_rank[k], recv[same range] <- it (device buffers)
void comm_exchange_nbr_buf(cdfem_ctx *c, const std::vector<int64_t> &off, const double *dsend, double *drecv,
                           hipStream_t s = nullptr);
void partition_free(cdfem_ctx *c);
inline bool multi_rank(const cdfem_ctx *c) { return c->nranks > 1; }
// split CG finalizers for the multi-rank path: local sum -> all-reduce -> step
hipError_t launch_fin_sum(cdfem_ctx *c, int nparts, int slot);
hipError_t launch_den_step(cdfem_ctx *c);
hipError_t launch_update_step(cdfem_ctx *c);
hipError_t launch_init_step(cdfem_ctx *c, double rel_tol, double abs_tol, int max_iter);
hipError_t launch_cg_init_nofin(cdfem_ctx *c, const double *B, double *x, double *r, double *z, double *d,
                                const double *dinv);
// pack the local partial sums of q on the shared interface planes into d_if[0] / d_if[2]
hipError_t launch_pack_qplanes(cdfem_ctx *c, const double *q, hipStream_t s = nullptr);
hipError_t launch_brick_cg2_split(cdfem_ctx *c, const double *r, const double *dinv, const double *d_old,
                                  double *d_new, double *q, hipStream_t s, double *x = nullptr, int bfkk = -1);

// ---- bandwidth probes (stream_kernels.hip): mode 0 read 16 B/lane, 1 read 8 B/lane, 2 copy 16 B
// full assembly on simplices (fa_kernels.hip)
constexpr int kSpmvMaxBlocks = 65536;  // partial slots reserved for the SpMV-CG den
constexpr int kLdsHaloMax = 7936;      // doubles of x one LDS-staged SpMV window may stage (62 KiB)
struct FaPattern {
    int64_t nnz = 0;
    std::vector<int32_t> rowptr, cols, diagpos, coff, cpos;
    // SELL-64 (sigma = global sort by row length) copy of the pattern for the SpMV
    std::vector<int32_t> sptr;   // [nslices + 1] first stored entry of each 64-row slice
    std::vector<int32_t> srows;  // [nslices * 64] original row of (slice, lane), -1 = padding
    std::vector<int32_t> scols;  // [stored] column, slice-major then entry-major then lane
    std::vector<int32_t> smap;   // [stored] CSR index of the stored entry, -1 = padding
    std::vector<int16_t> sdel;   // [stored] column - lane row where it fits 16 bits (see swide), else empty
    std::vector<uint8_t> swide;  // [nslices] 1: this slice has a delta beyond 16 bits and streams scols
                                 // (empty: every slice fits); nnz_wide = real entries in such slices
    int64_t nnz_wide = 0;
    // LDS-staged windows (windowed layouts, sell_build with lds_rows > 0): window w = slices
    // [w S, (w + 1) S), S = lds_rows / 64; its distinct columns hidx[hptr[w] .. hptr[w + 1]) (ascending)
    // are staged in LDS and every stored entry addresses them by sloc (16-bit position in the window)
    int64_t lds_rows = 0;
    int lpr = 1;                  // lanes per row (R = 64 / lpr rows per slice; LDS layouts only)
    int32_t lds_max = 0;          // largest window halo (doubles of LDS)
    std::vector<int32_t> hptr, hidx;
    std::vector<uint16_t> sloc;
    std::vector<int32_t> perm;   // SpMV space order (sell_plan.cpp): space row -> mesh row; empty = mesh order
    bool windowed = false;       // slices cut from the space order directly (no srows)
};
// SpMV order (sell_plan.cpp): 0 natural + global sort, 1 natural + windows, 2 RCM + windows,
// 3 auto (mode 0, geometric or RCM + global), 4 RCM + global, 5 geometric + global
struct SellPlan {
    int mode = 0, base = 1;  // base: 1 natural, 2 RCM, 3 geometric, 4 Morton
    bool windowed = false;
    int64_t window = 0, max_delta = 0, bw_natural = 0, bw_rcm = 0, bw_geometric = 0;
    std::vector<int32_t> perm;   // space row -> mesh row (empty: mesh order)
    int64_t lds_rows = 0;        // windowed: rows per LDS-staged window (set_option "spmv_lds"; 0 off)
    bool auto_lds = false;       // the auto mode chose a windowed unstructured order: LDS windows
    int lpr = 1;                 // LDS layouts: lanes per row (set_option "spmv_lpr")
};
constexpr int64_t kAutoLdsRows = 768;  // rows per window of the auto LDS orders (profiles/r03/ab_c4_lds_windows.txt)
std::vector<int32_t> rcm_order(int64_t nl, const int32_t *rowptr, const int32_t *cols);
SellPlan sell_plan(int64_t nl, const int32_t *rowptr, const int32_t *cols, int mode, int dim = 0,
                   const double *xyz = nullptr, int64_t window = 0);
// dof coordinates of a simplex space (P1, P2, triangle P3 nodes; element-affine map), nl * dim
std::vector<double> simplex_dof_coords(int dim, int p, int ne, int nd, int64_t nl, const std::vector<double> &verts,
                                       const std::vector<int32_t> &dofs);
void sell_build(FaPattern &P, int64_t nl, const SellPlan &pl);
FaPattern fa_build_pattern(const std::vector<int32_t> &elem_dofs, int ne, int nd, int64_t nl, int sell_mode,
                           int dim = 0, const double *dof_xyz = nullptr, int64_t sell_window = 0,
                           int64_t lds_rows = 0, int lpr = 1);
hipError_t launch_simplex_elem(cdfem_ctx *c, const double *kq, const double *kmq, double kappa, double alpha,
                               const double *conv, const double *cq, const double *mq, double mass);
hipError_t launch_fa_assemble(cdfem_ctx *c);
hipError_t launch_simplex_lf(cdfem_ctx *c, const double *fq, double *Ye);
hipError_t launch_sell_fill(cdfem_ctx *c);
hipError_t launch_csr_diag(cdfem_ctx *c, double *d);
hipError_t launch_spmv(cdfem_ctx *c, bool constrained, const double *x, double *y);
hipError_t launch_spmv_cg(cdfem_ctx *c, const double *d, double *q);
// permuted SpMV layout: dst = src gathered into the SpMV order (to_spmv_order) or scattered back
hipError_t launch_perm(cdfem_ctx *c, bool to_spmv_order, const double *src, double *dst);
bool spmv_delta(const cdfem_ctx *c);
// fused high-order CG iteration (ho_kernels.hip / vec_kernels.hip)
bool tile_den_ok(const cdfem_ctx *c);
int tile_den_blocks(const cdfem_ctx *c, bool most = false);
hipError_t launch_apply_den(cdfem_ctx *c, const double *d, double *Ye, const KrylovState *st, double *part);
// the same with the CG direction folded in (ho_dfold, Kronecker tile): d_new = z + beta d_old
bool tile_dfold_ok(const cdfem_ctx *c);
hipError_t launch_apply_den_dfold(cdfem_ctx *c, const double *z, const double *dold, double *dnew, double *Ye,
                                  const KrylovState *st, double *part);
bool e2l_box_ok(const cdfem_ctx *c);
hipError_t launch_den_from_partials(cdfem_ctx *c, const double *in, int64_t n);
hipError_t launch_den_local_from_partials(cdfem_ctx *c, const double *in, int64_t n);
hipError_t launch_e2l_cg_update(cdfem_ctx *c, const double *Ye, const double *d, double *x, double *r, double *z,
                                const double *dinv);

// GMRES(m) (gmres.hip)
int gmres_blocks(int64_t n);
hipError_t launch_gm_init(cdfem_ctx *c, GmresState *st, int m, int max_it);
// poll: pinned host slot the step's last scalar kernel writes the state head into (solve_gmres)
hipError_t launch_gm_residual(cdfem_ctx *c, const double *b, const double *Ax, const double *dinv, double *v0,
                              double *part, GmresState *st, bool first, double rtol, double atol, GmresState *poll);
// ps (gm_pb): pass 1 reads the structured Mult's patch buffer for A_c V_j instead of w (brick_core.hpp)
struct GmPatchSrc;
hipError_t launch_gm_orth(cdfem_ctx *c, double *w, const double *dinv, double *V, int64_t ldv, double *part,
                          GmresState *st, int m, GmresState *poll, const GmPatchSrc *ps = nullptr);
hipError_t launch_gm_update(cdfem_ctx *c, double *x, const double *V, int64_t ldv, GmresState *st, GmresState *poll);
hipError_t launch_stream(cdfem_ctx *c, int mode, const double *a, double *b, int64_t n);
// ILU(0) (ilu_kernels.hip): factor + capture once per operator; apply: ilu.z = (LU)^{-1} d_w[4]
void ilu_setup(cdfem_ctx *c);
void ilu_free(cdfem_ctx *c);
hipError_t ilu_apply(cdfem_ctx *c);
// f64 compute-rate probes: mode 0 VALU v_fma_f64, 1 v_mfma_f64_16x16x4_f64; *flops per launch
hipError_t launch_fp64_probe(cdfem_ctx *c, int mode, double *out, double *flops);

}  // namespace cdfem
