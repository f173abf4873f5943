/*
 * cdfem.h — C-ABI of the MI355X-native convection-diffusion FE hot path (libcdfem.so).
 *
 * One opaque context per GPU (per process / rank).  All entry points return CDFEM_OK (0) or an
 * error code; the message is in cdfem_last_error(ctx).  No C++ exception crosses this boundary;
 * the C++ MFEM-shaped layer (continuum-mechanics-mfem_amd/cpp/cdfem_mfem.hpp) turns a status into
 * std::runtime_error, which the reference drivers already map to exit code 3
 * (linear_convection_diffusion_2D.cpp:435-442).
 *
 * Each entry point names the reference interface it replaces.  The reference calls MFEM, hypre
 * and PETSc (not vendored: SURVEY.md §8b/c), so the "replaces" lines cite the reference CALL SITE.
 *
 * Ownership: the caller owns every host array; the context owns every device buffer it allocates;
 * no caller pointer is retained after a call returns.  Pointers tagged `where` are host memory
 * when where == CDFEM_HOST and device memory (hipMalloc / cdfem_alloc) when where == CDFEM_DEVICE.
 * A context is not thread-safe.  Calls with where == CDFEM_HOST are synchronous on return.
 *
 * Vector spaces.  L-vector = all dofs of the rank's elements (for one rank this is also MFEM's
 * T-vector: P = I on a conforming mesh).  DoF numbering and element-dof maps are supplied by the
 * caller; element dofs are LEXICOGRAPHIC on the tensor element (l = dx + (p+1)(dy + (p+1)dz)),
 * element vertices lexicographic (v = a + 2b + 4c), reference element [0,1]^dim.
 */
#ifndef CDFEM_H
#define CDFEM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CDFEM_ABI_VERSION 1

typedef struct cdfem_ctx cdfem_ctx;

enum cdfem_status {
    CDFEM_OK = 0,
    CDFEM_ERR_ARG = 1,          /* bad argument / shape mismatch                          */
    CDFEM_ERR_HIP = 2,          /* HIP runtime error (no device, OOM, launch failure)     */
    CDFEM_ERR_STATE = 3,        /* call order violated (e.g. mult before setup)          */
    CDFEM_ERR_UNSUPPORTED = 4,  /* dim/order/kernel combination not built                 */
    CDFEM_ERR_NOT_CONVERGED = 5,/* Krylov solve hit max_iter (result still returned)      */
    CDFEM_ERR_COMM = 6          /* RCCL error                                             */
};

/* integrator kinds (bit mask) */
enum { CDFEM_DIFFUSION = 1, CDFEM_CONVECTION = 2, CDFEM_MASS = 4 };
/* pointer locations */
enum { CDFEM_HOST = 0, CDFEM_DEVICE = 1 };
/* Krylov methods and preconditioners */
enum { CDFEM_CG = 0, CDFEM_GMRES = 1 };
enum { CDFEM_PC_NONE = 0, CDFEM_PC_JACOBI = 1, CDFEM_PC_ILU = 2 };
/* quadrature rules whose points the host may need for coefficient evaluation.  Quads / hexes: one
 * operator rule (Gauss n = p + 2, shared by the three integrators; DIFFUSION / CONVECTION / MASS
 * name it too).  Simplices: each integrator its own rule, MFEM's GetRule on affine simplices on
 * MFEM's tabulated rules: DIFFUSION order 2p - 2, CONVECTION and MASS order 2p (OPERATOR refused). */
enum { CDFEM_RULE_OPERATOR = 0, CDFEM_RULE_LINEARFORM = 1, CDFEM_RULE_ERROR = 2, CDFEM_RULE_DIFFUSION = 3,
       CDFEM_RULE_CONVECTION = 4, CDFEM_RULE_MASS = 5 };
/* kernel ids for cdfem_profile_read */
enum { CDFEM_K_APPLY = 0, CDFEM_K_E2L = 1, CDFEM_K_UPDATE = 2, CDFEM_K_DIRECTION = 3, CDFEM_K_ORTH = 4,
       CDFEM_K_COUNT = 8 };

int cdfem_abi_version(void);

/* ---- context ------------------------------------------------------------------------------- */
/* replaces: Device device("cpu") (linear_convection_diffusion_2D.cpp:287) — here: one MI355X.  */
int cdfem_create(int device, cdfem_ctx **out);
void cdfem_destroy(cdfem_ctx *ctx);
const char *cdfem_last_error(const cdfem_ctx *ctx);
int cdfem_synchronize(cdfem_ctx *ctx);
/* number of visible HIP devices (0 on a CPU-only host; never fails) */
int cdfem_device_count(void);

/* ---- device memory helpers (for where == CDFEM_DEVICE callers and benchmarks) ---------------- */
int cdfem_alloc(cdfem_ctx *ctx, size_t bytes, void **dptr);
int cdfem_free(cdfem_ctx *ctx, void *dptr);
int cdfem_memcpy(cdfem_ctx *ctx, void *dst, int dst_where, const void *src, int src_where, size_t bytes);
/* y = a x + b y on n doubles of device memory, synchronous.  replaces: Vector::Add(a, x) on device
 * vectors (MFEM's forall kernel; diffusion_mms.cpp:433 rhs.Add(dt, f), linear_convection_diffusion_1D.cpp
 * the same rhs update), so the shim's time loop keeps rhs in HBM.                                  */
int cdfem_vec_axpby(cdfem_ctx *ctx, int64_t n, double a, const double *x, double b, double *y);

/* ---- mesh + H1 space -------------------------------------------------------------------------
 * replaces: ParMesh + H1_FECollection(order, dim) + ParFiniteElementSpace + GetEssentialTrueDofs
 *           (linear_convection_diffusion_2D.cpp:300-322; diffusion_mms.cpp:275-285).
 * elem_verts: ne * 2^dim * dim doubles (multilinear geometry), elem_dofs: ne * (order+1)^dim
 * L-dof indices in [0, nldofs), ess_dofs: essential L-dofs (Dirichlet on the marked boundary).  */
int cdfem_mesh_upload(cdfem_ctx *ctx, int dim, int order, int ne, const double *elem_verts,
                      int64_t nldofs, const int32_t *elem_dofs, int n_ess, const int32_t *ess_dofs);

/* Declare the uploaded mesh a structured nx*ny*nz box with the lexicographic numbering of
 * cdfem_box_mesh (validated; element vertices may be perturbed).  Enables the brick fast path:
 * 4x4x4-element bricks per wavefront, E->L sum fused into the apply through LDS, CG direction
 * update fused into the operator gather.  Same results as the generic path to rounding.
 * Call before cdfem_pa_setup.  (Specialisation of ParFiniteElementSpace for Cartesian meshes.)  */
int cdfem_mesh_set_structured(cdfem_ctx *ctx, int nx, int ny, int nz);

/* Physical coordinates of the quadrature points of a rule (CDFEM_RULE_*), ne * nq * dim doubles,
 * element-major, q lexicographic (qx fastest): where a host Coefficient::Eval is sampled
 * (linear_convection_diffusion_2D.cpp:165-215).  cdfem_rule_size returns nq per element.       */
int cdfem_rule_size(cdfem_ctx *ctx, int rule, int *nq_per_elem);
int cdfem_quadrature_points(cdfem_ctx *ctx, int rule, double *xyz, int where);

/* ---- partial assembly (the hot operator) -----------------------------------------------------
 * replaces: a.AddDomainIntegrator(new DiffusionIntegrator(kappa))          :336
 *           a.AddDomainIntegrator(new ConvectionIntegrator(c, alpha))      :337
 *           a.AddDomainIntegrator(new MassIntegrator(s))                   :338
 *           a.Assemble()                                                   :339
 * with MFEM partial-assembly semantics: per-quadrature-point data
 *   D = W kappa adj(J) adj(J)^T / det J,  C = W alpha adj(J) c,  M = W s det J.
 * *_q arrays (ne*nq of the OPERATOR rule = the DIFFUSION / CONVECTION / MASS rules on quads and hexes;
 * conv_q ne*nq*dim) override the constants when
 * non-NULL (host pointers): a variable Coefficient / VectorCoefficient sampled on the host.     */
int cdfem_pa_setup(cdfem_ctx *ctx, unsigned kinds, double kappa, const double *kappa_q,
                   double alpha, const double *conv, const double *conv_q, double mass,
                   const double *mass_q);

/* The same setup with every coefficient form in one struct, including a MatrixCoefficient for the
 * diffusion: DiffusionIntegrator(MatrixCoefficient&) (diffusion_mms_ale.cpp:474-496,1019), the ALE
 * metric alpha dt / J cof(A) cof(A)^T.  The diffusion tensor at a point is K = k I + K_q with k =
 * kappa_q[i] (or kappa) and K_q the symmetric tensor kappa_mat_q[i] (NULL: 0), stored as
 * xx, xy, yy (2D) / xx, xy, xz, yy, yz, zz (3D); qdata D = W adj(J) K adj(J)^T / det J keeps its
 * dim(dim+1)/2 components.  Non-symmetric matrix coefficients are not accepted (the shim checks).  */
typedef struct {
    unsigned kinds;
    double kappa;
    const double *kappa_q;      /* ne*nq, or NULL */
    const double *kappa_mat_q;  /* ne*nq*dim(dim+1)/2, or NULL */
    double alpha;
    const double *conv;         /* 3 doubles (unused components 0) */
    const double *conv_q;       /* ne*nq*dim, or NULL */
    double mass;
    const double *mass_q;       /* ne*nq, or NULL */
} cdfem_form_coeffs;
int cdfem_pa_setup_form(cdfem_ctx *ctx, const cdfem_form_coeffs *form);

/* ---- full assembly on simplex meshes (BASELINE config C4: unstructured tetrahedra) -------------
 * replaces: the same ParMesh / H1_FECollection(p, dim) / ParFiniteElementSpace calls on a triangle
 * or tetrahedral mesh (gmsh input, Input/input_2d.yaml:1), and ParBilinearForm::Assemble +
 * FormLinearSystem -> HypreParMatrix (linear_convection_diffusion_2D.cpp:339,349-351) whose CSR
 * PETSc's KSPGMRES then multiplies (MATAIJ, :364-375).
 * cdfem_mesh_upload_simplex: Lagrange P1/P2 (triangles also P3) on affine simplices; elem_verts
 * ne*(dim+1)*dim, elem_dofs ne*nd with nd = dim+1 (P1) / (dim+1)(dim+2)/2 (P2) / 10 (P3 triangle),
 * local order: vertices, then edge nodes along a->b for edges (0,1),(0,2),(0,3),(1,2),(1,3),(2,3)
 * [2D: (0,1),(0,2),(1,2)], then the P3 centroid; det J > 0 required.  cdfem_lf_assemble works on
 * simplex meshes with f sampled at the CDFEM_RULE_LINEARFORM points (MFEM's tabulated rule of order
 * 2p, cdfem_simplex_rule_order).  Each integrator has MFEM's rule (GetRule on affine simplices):
 * diffusion order 2p - 2, convection and mass order 2p, on MFEM's tabulated rules.
 * cdfem_fa_setup: same coefficients as cdfem_pa_setup, per-point arrays on the rule of their
 * integrator: kappa_q / kappa_mat_q on CDFEM_RULE_DIFFUSION, conv_q on CDFEM_RULE_CONVECTION,
 * mass_q on CDFEM_RULE_MASS (cdfem_rule_size / cdfem_quadrature_points);
 * assembles A (CSR, columns sorted) and the eliminated matrix of FormLinearSystem on the GPU.
 * Afterwards cdfem_pa_mult / cdfem_pa_diagonal / cdfem_form_linear_system / cdfem_solve run on the
 * CSR operator.  cdfem_fa_csr exports it (rowptr n+1, cols/vals nnz; pass NULLs to query nnz).   */
int cdfem_mesh_upload_simplex(cdfem_ctx *ctx, int dim, int order, int ne, const double *elem_verts,
                              int64_t nldofs, const int32_t *elem_dofs, int n_ess, const int32_t *ess_dofs);
int cdfem_fa_setup(cdfem_ctx *ctx, unsigned kinds, double kappa, const double *kappa_q, double alpha,
                   const double *conv, const double *conv_q, double mass, const double *mass_q);
int cdfem_fa_setup_form(cdfem_ctx *ctx, const cdfem_form_coeffs *form);
int cdfem_fa_csr(cdfem_ctx *ctx, int constrained, int64_t *nnz, int32_t *rowptr, int32_t *cols, double *vals);

/* replaces: Operator::Mult on the assembled operator when constrained == 0 (shared dofs summed over
 * the ranks: P^T A P on a consistent L-vector), the ConstrainedOperator built by FormLinearSystem
 * (:349-351) when constrained == 1 (input essential entries treated as 0, output y[ess] = x[ess]),
 * and BilinearForm::Mult on a ParBilinearForm (diffusion_mms.cpp:430) when constrained == 2: the
 * rank-local product, a partial L-vector (no exchange; the same as 0 on one rank).             */
int cdfem_pa_mult(cdfem_ctx *ctx, const double *x, double *y, int constrained, int where);

/* replaces: BilinearForm::AssembleDiagonal (PA) — unconstrained operator diagonal.             */
int cdfem_pa_diagonal(cdfem_ctx *ctx, double *diag, int where);

/* ---- linear form -----------------------------------------------------------------------------
 * replaces: b.AddDomainIntegrator(new DomainLFIntegrator(f)); b.Assemble()  (:341-343).
 * f_q: values of f at the CDFEM_RULE_LINEARFORM points (ne * nq, host), output b is an L-vector. */
int cdfem_lf_assemble(cdfem_ctx *ctx, const double *f_q, double *b, int where);

/* ---- constrained linear system -----------------------------------------------------------------
 * replaces: a.FormLinearSystem(ess_tdof_list, x, b, A, X, B)  (:349-351), PA/ConstrainedOperator
 * semantics: X = x,  B = b - A x_e (x_e = x on ess dofs, 0 elsewhere),  B[ess] = x[ess].        */
int cdfem_form_linear_system(cdfem_ctx *ctx, const double *x, const double *b, double *X,
                             double *B, int where);

/* ---- Krylov solve ------------------------------------------------------------------------------
 * replaces: PetscLinearSolver(A).Mult(B, X) (:364-375; Input/petsc.opts: gmres, rtol 1e-10,
 * atol 1e-12, max_it 500, pc jacobi) and CGSolver (mesh_recession_handler.cpp:270-276).
 * CG follows MFEM CGSolver (convergence (r,z) <= max(nom0 rel^2, abs^2)); GMRES follows PETSc
 * KSPGMRES (left PC, classical Gram-Schmidt, restart, ||M^{-1} r|| <= max(rtol ||M^{-1}b||, atol)).
 * X on input is ignored (zero initial guess, iterative_mode = false), on output the solution.
 * GMRES: restart 1..64; iterations = inner steps; final_norm = last preconditioned residual
 * estimate (PETSc rnorm).  CDFEM_PC_ILU = ILU(0), natural ordering, no shift: PETSc
 * "-pc_type bjacobi -sub_pc_type ilu" on one rank (Input/petsc_circle.opts:6-8); GMRES on assembled
 * (cdfem_fa_setup) operators, single rank.  Multi-rank slabs: CG and GMRES with none / Jacobi.
 * Returns CDFEM_ERR_NOT_CONVERGED (result filled) when max_iter is reached.                     */
typedef struct {
    int method;        /* CDFEM_CG / CDFEM_GMRES */
    int pc;            /* CDFEM_PC_NONE / CDFEM_PC_JACOBI / CDFEM_PC_ILU (GMRES on FA operators) */
    int max_iter;
    int restart;       /* GMRES restart (PETSc default 30) */
    double rel_tol;
    double abs_tol;
    int check_every;   /* host convergence poll interval in iterations (0: default 16) */
    int print_level;
} cdfem_solver_params;

typedef struct {
    int converged;
    int iterations;
    double final_norm;
    double initial_norm;
    double seconds;    /* wall time of the Krylov loop (device-synchronised) */
} cdfem_solver_result;

int cdfem_solve(cdfem_ctx *ctx, const cdfem_solver_params *prm, const double *B, double *X,
                int where, cdfem_solver_result *res);

/* ---- HBM bandwidth probe: mode 0 read (16 B/lane), 1 read (8 B/lane), 2 copy (16 B/lane) of a
 * `bytes`-sized buffer, `reps` launches; returns achieved GB/s (bytes moved / time).
 * Modes 3-7: per-wave private 320 KiB chunks (16 B/lane), 8/16/8/4/32 loads in flight; 3, 4, 6, 7
 * limited to one wave per SIMD by an LDS reservation, 5 unrestricted.  Modes 8, 9: the same
 * per-wave work (8 / 4 loads in flight, one wave per SIMD) on an interleaved layout.  Modes 10-13:
 * mode 3 with chunks skewed by 256 B / 512 B / 1 KiB / 4 KiB.  Modes 14, 15: 4 (one workgroup per
 * CU) / 2 waves of a workgroup streaming one shared chunk, 4 / 2 KiB per step.  Modes 16, 17: the
 * 16-byte grid-stride read with 64-thread blocks at one wave per SIMD, 1024 / 4096 blocks.       */
int cdfem_stream_bench(cdfem_ctx *ctx, int mode, size_t bytes, int reps, double *gbps);

/* f64 compute-rate probe (diagnostic; backs DESIGN.md's VALU-vs-MFMA choice for the high-order
 * contractions): mode 0 = v_fma_f64 (8 independent chains per lane), 1 = v_mfma_f64_16x16x4_f64
 * (4 independent accumulators per wave), 2 / 3 / 4 = both in one loop (4 MFMA chains interleaved
 * with 16 / 32 / 64 v_fma_f64 per lane: does the matrix core run beside the VALU?);
 * *tflops = achieved f64 TFLOP/s over `reps` launches. */
int cdfem_fp64_bench(cdfem_ctx *ctx, int mode, int reps, double *tflops);

/* ---- tuning knobs (performance only; results identical to rounding) --------------------------
 * "profile_mask": bit k set = kernel slot k (CDFEM_K_*) gets HIP events while profiling is on
 *                 (default all; events around every kernel cost ~1 us each on the stream).
 * "brick_xcd": 1 (default) — XCD-contiguous brick order of the structured CG kernel; 0 = the
 *              dispatcher's round-robin order.
 * "mr_overlap": 1 (default) — slab (multi-rank) structured CG: the first/last brick layers, the
 *               interface pack and the exchange run on a side stream under the interior layers;
 *               0 = one launch, then the exchange (bitwise the same results).
 * "brick_mult_pb": 1 (default) — the structured Mult (GMRES, cdfem_pa_mult; Kronecker form) writes
 *              each brick's whole patch sum to the patch buffer and a second pass forms every row from
 *              its 1-8 entries (predicated loads); 0 = owned rows + face partials + face sums
 *              (k_brick_faces).  Same sums in the same order (bitwise); C2 GMRES step 195.0 -> 189.4 us,
 *              profiles/r04/ab_c2_gmres_dpp_multpb.json.
 * "cg_beta_fold": 1 (default) — with cg_den_fold (one rank, Kronecker form, <= 1024 update
 *              workgroups) the brick CG apply also takes MFEM's betanom step of the previous update:
 *              every workgroup sums the update's partials with its patch gather in flight, and the
 *              one-block update finalizer is not launched (iterates agree with 0 to rounding; C2:
 *              60.8 against 62.6 us per iteration, profiles/r04/ab_c2_beta_fold.json).
 * "cg_den_fold": 1024 (default) — N (64..16384): the one-rank brick CG takes MFEM's den step inside
 *              the update kernel, run as N workgroups that each sum the apply's den partials in one
 *              fixed order; the one-block den finalizer is not launched (iterates agree with the
 *              finalizer path, 0, to rounding; C2: 62.4 against 64.6 us per iteration,
 *              profiles/r04/ab_c2_den_fold.json).
 * "cg_mr_fold": 1 (default) — several ranks (slab partition, p <= 2, both folds on): the ranks
 *              all-reduce the apply's den partials and the update's betanom partials as vectors, so the
 *              update and the next apply take MFEM's den and betanom steps as on one rank (no sum or
 *              step kernels between them); taken only when every rank holds as many partials (checked
 *              once, collectively); 0 = per-rank sums, 8-byte all-reduces and step kernels.
 * "gm_poll": 4 (default) — the GMRES host loop records an event and checks the device state every k
 *              inner steps (and at every cycle's last step) instead of after every step (1: every step).
 *              Steps queued past a converged step exit at entry; their Mult runs (at most k - 1 per solve).
 * "brick_stagger": -1 (default, automatic: s = log2 CUs, n = 4), 0 off, or bits 0-3 a shift s and bits
 *              4-8 a count n: the first round of the brick CG apply (k_brick_cg workgroups b < 8 x CUs,
 *              launches of >= 2 rounds) with bit s of b set sleeps n x 2,048 cycles at entry, so half the
 *              round gathers its patches while the other half computes (C2: 39.0 -> 37.4 us per apply,
 *              DESIGN.md 4.1).
 * "pa_uniform": 1 (default) — under pa_affine 2 on a structured p = 2 box (kinds 7 or 5), cdfem_pa_setup
 *              checks whether every element's factors equal the first element's (each within 1e-14 of the
 *              largest factor: a uniformly refined box, what MFEM's MakeCartesian3D gives) and, if so,
 *              forms that element's 27 x 27 matrix once (column j = the Kronecker apply of e_j); the brick
 *              CG apply then runs it as a GEMM on the matrix cores (56 v_mfma_f64_16x16x4_f64 per 64
 *              elements; the same operator to rounding).  0 = the Kronecker form (takes effect without a
 *              new setup; 1 needs one).  The GMRES Mult and the other applies keep the Kronecker form.
 * "brick_mfma": 0 (default) or 1 — the p = 2 brick CG apply's x stage (kinds 7, Kronecker form) on
 *              v_mfma_f64_16x16x4_f64: 16 elements per GEMM, outputs staged through LDS to the element
 *              threads.  Parity-green, measured slower.
 * "ho_block_z": 2 (default) or 4 — elements per block along z of the high-order brick CG (read by
 *              cdfem_mesh_set_structured): 2 x 2 x 2 blocks (8 element tiles, 200 of 256 threads busy at
 *              p = 4) or 2 x 2 x 4 (16 tiles, 400 of 448; 1.34 patch entries per dof against 1.42).
 * "ho_brick": 1 (default) — the CG solve on a structured affine box at 3D p = 3, 4 (one rank,
 *              Kronecker form) runs on blocks of 2^3 elements (k_hobrick_cg: the tile core, the block's
 *              E->L in LDS, the 9^3 patch buffer of the p = 2 brick) and the brick update, instead of the
 *              tile apply's E-vector and the flat E->L update (0).  Iterates agree to rounding; C3:
 *              4114 against 4287 us per iteration (profiles/r05/ab_c3_ho_brick_occ4.json).
 * "ho_brick_mfma": 0 (default) — with ho_brick on the full operator (kinds 7): the x stage of the
 *              block's eight elements as GEMMs on v_mfma_f64_16x16x4_f64 (rows = element rows, k = the
 *              five input points padded to eight, columns = M, K, C, C^T per output point), staged to
 *              the tile threads through LDS; the y and z stages stay on the VALU.  Same operator to
 *              rounding; the north star's MFMA contraction, A/B'd in DESIGN.md 4.2.
 * "den_group": 0 (default) — on several ranks the brick CG apply's den partials (one per 64-element brick)
 *              are summed in groups by the group's last-arriving brick once there are more than the
 *              multi-rank fold sums (8,192: C5's per-rank slab of 32,768 bricks -> groups of 8), so the
 *              fold stays on; one rank keeps per-brick partials (measured: its 256^3 box runs the
 *              two-stage den sum 0.3 % faster); a power of two up to 64 forces that size (tests).
 * "brick_byte_limit": 2^31 (default) — the structured brick kernels address their vectors and patch
 *              buffer with 32-bit buffer offsets (out-of-range marker 2^31), so a box whose 8 N_L or
 *              8 S^3 bricks reach the limit runs the generic element kernels instead; lower values
 *              force that fallback (tests); 0 restores the default.  On a slab partition the
 *              decision is taken on the largest rank's sizes (all-reduced by cdfem_set_slab), so
 *              every rank runs the same CG path.
 * "brick_upd_pb": 1 (default) — the brick CG update (k_cg_update_faces) reads each dof's 1-8 patch
 *              entries as eight predicated buffer loads (absent ones out of range) instead of
 *              branching on the face planes (0); bitwise the same sums.
 * "ho_dfold": 1 (default) — read by the CG solve on structured boxes (one rank, fused high-order CG,
 *              Kronecker tile: pa_affine 2, ho_mfma 0): the apply gathers z and the previous
 *              direction, forms d = z + beta d_old itself (each dof's owner element stores it to a
 *              second direction buffer), and the direction pass is skipped (same formula); 0 = the
 *              direction pass.
 * "ho_mfma": 0 (default) — the LDS stages of the high-order (3D p = 3, 4) tile apply as block GEMMs on
 *            v_mfma_f64_16x16x4_f64, bit 0 = stage x, 1 = y, 2 = y^T, 3 = x^T; the masks 1, 3, 8, 9
 *            and 15 are built (results agree to rounding; the north star's MFMA alternative,
 *            measured even to slower).
 * "pa_affine": 2 (default) — read by cdfem_pa_setup: on a mesh whose elements are all
 *              parallelepipeds (checked at upload: every vertex within 32 ulp of the coordinates plus
 *              1e-12 of the element's longest edge of v0 + sum of the edge vectors) with constant
 *              coefficients, the Jacobian is the element's edge matrix, the per-point data are stored
 *              as W_q * g_e (so the diagonal and the 2D / FA paths see the same operator), and the
 *              3D applies read the 10 per-element factors g_e instead of the per-point stream:
 *                2 — the structured brick kernels (p <= 2, CG and Mult) and the generic 3D
 *                    element-block apply (p <= 2) apply the factors in their Kronecker form
 *                    (1D rule matrices M, K, C per axis, pa_core.hpp elem_apply3d_kron);
 *                1 — the same applies form each point's data W_q * g_e from the factors;
 *                the p >= 3 tile apply forms the point data from the factors under 1 and 2 (and
 *                streams them when "ho_mfma" is non-zero).  The 2D applies always stream the per-point
 *                data.  All forms apply the operator of the per-point multilinear-map setup to rounding
 *                (the Kronecker form is an algebraic identity of the tensor rule, not an exactness
 *                argument); 0 = the per-point map and stream everywhere.
 * "cg_xfold": 1 (default) — structured brick CG (p <= 2, Kronecker form): each apply after the first
 *             advances x by the previous iteration's alpha d on the dofs it writes the new direction
 *             for, so the update kernel streams neither x nor d (bitwise the same iterates; 1 % faster
 *             at C2 in two A/B runs, profiles/r04/ab_c2_patchbuf_xfold.json, ab_c2_xfold_pb.json);
 *             0 = x += alpha d in the update.
 * "cg_fused": 1 (default) — high-order (p = 3, 4) CG on a structured box, one rank: (d, A d) from the
 *             apply's element outputs and the E->L sum fused into the CG update; 0 = separate
 *             E->L kernel (results agree to rounding).
 * "spmv_index16": 1 (default) — the assembled-operator SpMV streams 16-bit column deltas
 *                 (column - lane row); a 64-row slice with a delta beyond 2^15 streams its 32-bit
 *                 columns instead (mixed layout, when at least half the entries fit); 0 = 32-bit
 *                 columns everywhere.
 * "sell_order": 0..8, default 8 — the FA SpMV's order, read when the pattern is built
 *               (cdfem_fa_setup on a new mesh; see cdfem_sell_plan): 0 natural, 1 natural +
 *               windows, 2 RCM + windows, 3 auto (banded mesh order, geometric, RCM), 4 RCM, 5
 *               geometric, 6 Morton + windows, 7 Morton, 8 Morton windows of 768 rows staged in LDS
 *               (2 or 4 lanes per row by the padding) when the dof coordinates are known, else 3.
 *               A permuted order runs the Krylov solve in that order (Mult to rounding, iterates to
 *               1e-12).
 * "sell_window": 0 (default, auto) or a multiple of 64 — rows per window of the windowed orders.
 * "spmv_lpr": 0 (default, auto), 1, 2 or 4 — lanes per row of the LDS-staged layouts (read when
 *             the pattern is built): each lane sums a contiguous part of its row and the parts are
 *             combined in a fixed order (less padding where row lengths vary; results to rounding);
 *             auto = 4 where one lane per row would pad slices by more than 15 %, else 2, on the
 *             auto modes' LDS layouts; 1 elsewhere.
 * "spmv_lds": -1 (default, auto), 0 or rows per window — LDS-staged SpMV windows for the windowed
 *             orders: each workgroup stages its window's distinct columns in LDS and the entries
 *             address them by 16-bit window positions (bitwise the windowed sums); auto = on for the
 *             auto orders (sell_order 8, and the RCM windows sell_order 3 picks on unstructured meshes
 *             without coordinates: 768 rows).
 * "spmv_xcd": 1 (default) — contiguous slice range per XCD for the windowed SpMV layout.
 * "gm_ept": 0 (default, auto) — entries per thread of the GMRES orthogonalisation passes (4, 5, 6
 *           or 8); auto takes the smallest whose grid is resident in one round (same results).
 * "gm_pb": 1 (default) — GMRES on the structured patch-buffer Mult (one rank, Jacobi or no
 *          preconditioner): the first orthogonalisation pass sums each row's patch entries itself, so
 *          the Mult's row-sum kernel and its output vector's write and re-read go away (same sums in
 *          the same order: bitwise the same iterates); 0 = the Mult's own row sums.
 * Variants measured slower and removed in round 3 (their records stay under profiles/r02_ab_*):
 * brick element cores 1-10 and the four-waves-per-brick kernel, x-fold / paired x updates, the
 * folded high-order direction, the derived mass weight, per-XCD SpMV sort, SpMV stream offsets and
 * the software-pipelined SpMV loop, the two-waves-per-SIMD structured Mult, 2 / 4 lanes per SpMV row
 * (profiles/r03/ab_c4_spmv_lanes_per_row.txt), a spinning / less frequent GMRES host poll
 * (profiles/r03/ab_c2_gmres_poll.txt), in-launch grid sums for the CG / GMRES scalars
 * (profiles/r03/ab_c2_grid_fin.txt), brick-face sums in GMRES pass 1
 * (profiles/r03/ab_c2_gmres_faces_pass1.txt), chunked SELL storage with wide loads
 * (profiles/r03/ab_c4_spmv_chunk.txt), XCD-ordered blocks of the p >= 3 tile apply
 * (profiles/r03/ab_c3_tile_xcd_order.txt).                                                         */
int cdfem_set_option(cdfem_ctx *ctx, const char *key, int value);

/* ---- profiling (live HIP-event timing of the hot kernels, on the context's stream) ------------ */
int cdfem_profile_enable(cdfem_ctx *ctx, int on);
int cdfem_profile_reset(cdfem_ctx *ctx);
/* total milliseconds and launch count of kernel id (CDFEM_K_*) since the last reset */
int cdfem_profile_read(cdfem_ctx *ctx, int kernel, double *total_ms, int64_t *count);
/* per-launch milliseconds of kernel id since the last reset, in launch order: the first min(cap, count)
 * into ms, the count into *count (bench.py separates the full launches from the early-return ones) */
int cdfem_profile_launches(cdfem_ctx *ctx, int kernel, double *ms, int64_t cap, int64_t *count);
/* algorithmic bytes moved by one launch of kernel id (see DESIGN.md for the per-unit figures); on
 * structured boxes the figure is that of the kernel the CG solve launches (the brick CG kernels, the
 * fused high-order apply with its direction fold)                                                 */
int cdfem_kernel_bytes(cdfem_ctx *ctx, int kernel, double *bytes);
/* algorithmic f64 flops of one launch of the 3D partial-assembly apply (CDFEM_K_APPLY; FMA = 2):
 * the sum-factorized element apply (plus the point data W_q * g_e under pa_affine 1), or the
 * Kronecker-form element apply under pa_affine 2                                 */
int cdfem_kernel_flops(cdfem_ctx *ctx, int kernel, double *flops);
/* the HIP kernel name (without template arguments) kernel id runs as in the current configuration,
 * as rocprof reports it: the operator apply of a CG solve (CDFEM_K_APPLY) only — the SpMV after
 * cdfem_fa_setup, else the partial-assembly apply of the path the context takes (brick CG, the
 * high-order block CG, the tile applies, the element-block apply)                                  */
int cdfem_kernel_name(cdfem_ctx *ctx, int kernel, char *buf, size_t n);

/* ---- multi-GPU (element-partitioned z-slabs, one context per GPU / rank) ----------------------
 * replaces: MPI_COMM_WORLD + ParMesh partition (linear_convection_diffusion_2D.cpp:300) and the MPI
 * traffic inside hypre/PETSc (halo sums, Krylov all-reduces).  Each rank uploads its slab
 * (cdfem_box_mesh with [z0,z1)), declares it structured, then attaches a communicator and marks
 * which of its z-end planes are shared with a neighbour (the lower rank owns a shared plane).
 * Backends: RCCL (stream-ordered, over xGMI) or host callbacks (any transport: gloo, MPI).      */
typedef int (*cdfem_allreduce_fn)(double *buf, int n, void *user);  /* in-place sum over ranks */
/* send_lo -> rank-1, recv_lo <- rank-1, send_hi -> rank+1, recv_hi <- rank+1 (NULL if absent) */
typedef int (*cdfem_exchange_fn)(const double *send_lo, double *recv_lo, const double *send_hi,
                                 double *recv_hi, int64_t n, void *user);
int cdfem_comm_unique_id(unsigned char *id /* 128 bytes */);
int cdfem_comm_init_rccl(cdfem_ctx *ctx, int rank, int nranks, const unsigned char *id);
int cdfem_comm_init_host(cdfem_ctx *ctx, int rank, int nranks, cdfem_allreduce_fn allreduce,
                         cdfem_exchange_fn exchange, void *user);
int cdfem_set_slab(cdfem_ctx *ctx, int zlo_shared, int zhi_shared);

/* General element partition of any conforming mesh (ParMesh(MPI_COMM_WORLD, *mesh) and the
 * ParFiniteElementSpace shared-dof groups, linear_convection_diffusion_2D.cpp:300,312; used where the
 * mesh is not a structured box, e.g. the reference's gmsh triangles).  After uploading its local mesh
 * and attaching a communicator, each rank lists per neighbour rank (strictly ascending) the local dofs
 * it shares with that rank, in the same order on both sides (ascending global id).  A shared dof is
 * OWNED by the lowest rank holding it, and the local numbering must list the dofs owned by lower ranks
 * first: the true dofs are the suffix of the L-vector (cdfem_local_space produces this numbering).
 * Shared sums add every holder's partial in ascending rank order, so all copies are bitwise equal.
 * nbr_off: n_nbr + 1 offsets into nbr_idx (n_nbr = 0: a rank that shares nothing).                 */
int cdfem_set_shared(cdfem_ctx *ctx, int n_nbr, const int32_t *nbr_ranks, const int64_t *nbr_off,
                     const int32_t *nbr_idx);
/* Collective between neighbours, after cdfem_set_shared: sends the global id (l2g, nl entries) of
 * every shared entry and checks that each neighbour's list holds the same id at the same position
 * (the shared sums pair entries by position).  CDFEM_ERR_ARG on a mismatch, on both ranks of the
 * pair, naming the neighbour and the first differing entry.                                     */
int cdfem_check_shared(cdfem_ctx *ctx, const int64_t *l2g);
/* Host backend of the general partition: send[nbr_off[k] .. nbr_off[k+1]) goes to nbr_ranks[k] and
 * recv[same range] receives from it (MPI_Isend/Irecv, gloo, ...).  RCCL contexts need none.      */
typedef int (*cdfem_nbr_exchange_fn)(int n_nbr, const int32_t *nbr_ranks, const int64_t *nbr_off,
                                     const double *send, double *recv, void *user);
int cdfem_comm_set_host_nbr_exchange(cdfem_ctx *ctx, cdfem_nbr_exchange_fn fn, void *user);
/* dst uses src's communicator (reference counted): every form of one ParFiniteElementSpace is its
 * own context, and they share one RCCL communicator instead of bootstrapping one each.          */
int cdfem_comm_share(cdfem_ctx *dst, const cdfem_ctx *src);

/* True dofs (MFEM T-vector) = the owned L-dofs, the suffix [first_owned, nl) of the L-vector
 * (slab: the lower interface plane belongs to the rank below; one rank: everything).
 * replaces: ParFiniteElementSpace::TrueVSize / GetTrueDofs (:313,353).                          */
int cdfem_true_size(cdfem_ctx *ctx, int64_t *ntrue, int64_t *first_owned);
/* x = P X: the L-vector (nl) of the true-dof vector X (ntrue): owned entries from X, the other
 * shared entries received from their owner.  replaces: RecoverFEMSolution's P (:377).           */
int cdfem_prolongate(cdfem_ctx *ctx, const double *X, double *x, int where);

/* Communicator report: "backend=<none|rccl|host> rccl_version=<ncclGetVersion> rccl_path=<file>",
 * the RCCL build libcdfem.so is bound to in this process (ctx may be NULL).                      */
int cdfem_comm_info(const cdfem_ctx *ctx, char *buf, size_t n);

/* ---- structured mesh helper (host only, no device needed) ---------------------------------------
 * Box [0,1]^dim into nx*ny(*nz) quads/hexes with the conventions above; rank-slab variant for
 * the element-partitioned multi-GPU path: elements with iz in [z0, z1) only, dofs renumbered
 * locally (L-vector of the slab).  Sizes: see cdfem_box_sizes.                                 */
int cdfem_box_sizes(int dim, int nx, int ny, int nz, int order, int z0, int z1, int *ne,
                    int64_t *nldofs, int *n_ess);
int cdfem_box_mesh(int dim, int nx, int ny, int nz, int order, int z0, int z1, double perturb,
                   double *elem_verts, int32_t *elem_dofs, int32_t *ess_dofs, double *dof_xyz);

/* Kuhn simplex mesh of [0,1]^dim (config C4): n^dim cubes, dim! simplices each, P1/P2 dofs on the
 * (order n + 1)^dim lattice; perturb moves interior vertices (returns CDFEM_ERR_ARG if that inverts
 * an element).  Host only.                                                                      */
/* Element partition for the general path (host only): recursive coordinate bisection of the element
 * centroids into nranks parts, part[e] = rank (MFEM's ParMesh calls METIS, which is absent here; any
 * partition defines the same global operator).  Deterministic: every rank computes the same one.  */
int cdfem_partition_rcb(int dim, int ne, int nv, const double *elem_verts, int nranks, int32_t *part);
/* Order of the assembled operator's SpMV (host only; what cdfem_fa_setup builds with set_option
 * "sell_order" = mode: 0 mesh order + global length sort, 1 natural + windows, 2 reverse
 * Cuthill-McKee + windows, 3 auto (the mesh order when banded, else the geometric order when xyz is
 * given and banded, else RCM + global when it halves the bandwidth), 4 RCM + global, 5 geometric +
 * global).  xyz: nl * dim dof coordinates or NULL (cdfem_fa_setup passes the simplex space's nodes).
 * perm[space row] = mesh row; info[0..6] = base order (1 natural, 2 RCM, 3 geometric), window rows
 * (0: global length sort), max |column - row| in the space order, natural bandwidth, RCM bandwidth
 * (0 if not computed), stored SELL entries / nnz * 1e6, geometric bandwidth (0 if not computed).
 * Internal layout choice with no reference counterpart (the reference multiplies in mesh order,
 * PETSc MatMult on MATAIJ); exported for tests and tools.  */
int cdfem_sell_plan(int64_t nl, const int32_t *rowptr, const int32_t *cols, int mode, int dim, const double *xyz,
                    int32_t *perm, int64_t *info);
/* The rank-local H1 space of a partition (host only): elems = the rank's elements (ascending global
 * index), loc_dofs = their dofs in local numbering (dofs owned by lower ranks first, then the owned
 * ones, each by ascending global id), l2g = global id of each local dof, and the neighbour lists that
 * cdfem_set_shared takes.                                                                        */
int cdfem_local_space_sizes(int ne, int nd, int64_t nldofs, const int32_t *elem_dofs, const int32_t *part,
                            int rank, int *ne_loc, int64_t *nl_loc, int *n_nbr, int64_t *n_shared,
                            int64_t *n_not_owned);
int cdfem_local_space(int ne, int nd, int64_t nldofs, const int32_t *elem_dofs, const int32_t *part, int rank,
                      int32_t *elems, int32_t *loc_dofs, int64_t *l2g, int32_t *nbr_ranks, int64_t *nbr_off,
                      int32_t *nbr_idx);

int cdfem_kuhn_sizes(int dim, int n, int order, int *ne, int64_t *nldofs, int *n_ess);
int cdfem_kuhn_mesh(int dim, int n, int order, double perturb, double *elem_verts, int32_t *elem_dofs,
                    int32_t *ess_dofs, double *dof_xyz);

/* gmsh v2.2 ASCII simplex meshes (the reference's inputs, e.g. Mesh/unit_square.msh); replaces
 * Mesh(mesh_file, 1, 1) + H1_FECollection(order, dim) + ParFiniteElementSpace
 * (linear_convection_diffusion_2D.cpp:290,311-313).  Triangles (order 1-3) in MFEM's vertex order
 * (Finalize: orientation fix, then the longest edge first, Triangle::MarkEdge) or tetrahedra (1-2,
 * re-oriented to det J > 0); dofs: vertices (increasing gmsh node id), then (order-1) per edge (edges
 * numbered as MFEM first meets them) along increasing vertex dof, then P3 triangle centroids.
 * Boundary physical tags must be 1..31 (a larger tag is an error).  dof_bdr_mask[i] has bit (a-1) set when dof i
 * lies on a boundary element of physical attribute a (GetEssentialTrueDofs with an ess_bdr marker).
 * Host only; the element arrays feed cdfem_mesh_upload_simplex.                               */
int cdfem_gmsh_sizes(const char *path, int order, int *dim, int *ne, int64_t *nldofs);
int cdfem_gmsh_mesh(const char *path, int order, double *elem_verts, int32_t *elem_dofs, int32_t *dof_bdr_mask,
                    double *dof_xyz);
/* The same in two steps, for callers that refine or partition the mesh first (Mesh /
 * UniformRefinement / ParMesh, linear_convection_diffusion_2D.cpp:290-305): the gmsh file's simplex
 * topology (vertices in increasing node id, xyz nvert*dim; domain elements ne*(dim+1) vertex indices;
 * boundary elements nbe*dim vertex indices with their physical tags), and the H1 space of order p on
 * any such topology (the arrays of cdfem_gmsh_mesh; boundary masks from the tagged boundary
 * elements).  Host only.                                                                        */
int cdfem_gmsh_topology_sizes(const char *path, int *dim, int64_t *nvert, int *ne, int *nbe);
int cdfem_gmsh_topology(const char *path, double *vxyz, int32_t *elem_v, int32_t *bdr_v, int32_t *bdr_attr);
int cdfem_simplex_space_sizes(int dim, int64_t nvert, const double *vxyz, int ne, const int32_t *elem_v, int order,
                              int64_t *nldofs);
int cdfem_simplex_space(int dim, int64_t nvert, const double *vxyz, int ne, const int32_t *elem_v, int nbe,
                        const int32_t *bdr_v, const int32_t *bdr_attr, int order, double *elem_verts,
                        int32_t *elem_dofs, int32_t *dof_bdr_mask, double *dof_xyz);

/* Host helpers: the collapsed-Gauss simplex rule (returns the point count; xi/w may be NULL to
 * query it) and the nodal simplex basis phi [npts][nd], dphi [npts][nd][dim] in the local dof
 * order above — for host-side functionals (ComputeL2Error, :383-392).                         */
int cdfem_simplex_rule(int dim, int n, double *xi, double *w);
/* The rule IntRules.Get(TRIANGLE / TETRAHEDRON, order) returns in MFEM: its tabulated symmetric rules
 * (triangles order <= 9, tetrahedra order <= 6; tools/simplex_rules.py), else a collapsed-Gauss rule
 * exact to that order.  Returns the point count (xi / w may be NULL to query it).  The linear-form
 * rule of cdfem_mesh_upload_simplex is this rule at order 2p (DomainLFIntegrator's default).     */
int cdfem_simplex_rule_order(int dim, int order, double *xi, double *w);
int cdfem_simplex_basis(int dim, int order, int npts, const double *xi, double *phi, double *dphi);

#ifdef __cplusplus
}
#endif
#endif /* CDFEM_H */
