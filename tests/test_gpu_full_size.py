"""The BASELINE headline configurations at full size against the oracle, on the bench's exact paths.

C2 (BASELINE configs[1], the metric's workload, bench.py main): 64^3 hex, p = 2, 2,146,689 DoFs, the
convection-diffusion-reaction operator kinds 7 (kappa 0.1, c (1, -2, 0.5), s 1), structured brick
path with every default on: the Kronecker form of the affine factors (pa_affine 2), the x-fold
(cg_xfold), the den step in the update (cg_den_fold: 1,024 update workgroups, each summing the
apply's 4,096 partials) and the betanom step in the apply (cg_beta_fold: each of the 4,096 apply
workgroups summing the update's 1,024 partials, its limit of 64 lanes x 16).  Those folds reach the
sizes they are written for only here.  Checks (SURVEY.md 8d ladder):
  * Mult, constrained Mult, diagonal, FormLinearSystem: <= 1e-13 of max |y| against the oracle's
    assembled CSR of the same mesh;
  * 100 fixed Jacobi-CG iterates from x0 = 0 (tolerances 0, check_every 100, the bench's RHS seed
    20261015): relative L2 <= 1e-11 against the oracle's MFEM CGSolver restatement;
  * the symmetric kK + sM operator (kinds 5) solved to rel_tol 1e-13 on both sides: relative L2
    <= 1e-10, iteration counts within 2.
C4 (configs[3]): Kuhn 55^3 x 6 tets, P2, 1,367,631 DoFs, GPU-assembled FA CSR (pattern exact, values
1e-13), Mult / diagonal / FormLinearSystem 1e-13, and 60 GMRES(30) + Jacobi inner steps (two restart
cycles, the bench's step) with tolerances 0: relative L2 <= 1e-11 against the oracle's PETSc KSPGMRES
restatement.
C3 (configs[2]): 128^3 hex, p = 4, 135,005,697 DoFs, kinds 7, through the block CG (k_hobrick_cg: 2^3-element
blocks, the den partials summed in two stages, 262,144 blocks and a 1.53 GB patch buffer) and C5's mesh
(configs[4]): 256^3 hex, p = 2, 135,005,697 DoFs on ONE GPU (262,144 bricks: past kDenFoldMaxParts, so the
den step goes through the two-stage finalizer).  Both against the oracle's host partial assembly (O.PA:
MFEM's per-integrator point data and sum-factorised element loops, pinned to the FA CSR by
tests/test_oracle.py): Mult, constrained Mult, diagonal (orc_pa_diag) and FormLinearSystem <= 1e-13, and
20 fixed Jacobi-CG iterates on the bench's RHS seed <= 1e-11.  The size-dependent code of both paths runs
only at these sizes.  Host memory of the oracle: ~36 GB of point data at C3, ~86 GB at C5.

The oracle runs on the box's CPU share (OpenMP): assembling either matrix takes seconds
(bench.py's cpu_baseline assembles both), the CG and GMRES legs a few seconds more.
Reference call sites: linear_convection_diffusion_2D.cpp:335-374, Input/petsc.opts:2-6,
mesh_recession_handler.cpp:270-276 (CGSolver semantics).
"""
import numpy as np
import pytest

import cdfem
from oracle import oracle as O

pytestmark = pytest.mark.gpu
C3 = (1.0, -2.0, 0.5)
TOL_MULT = 1e-13


def _relmax(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


@pytest.fixture(scope="module")
def c2(gpu_ctx):
    n, p = 64, 2
    om = O.BoxMesh(3, n, p)
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)).set_structured(n, n, n)
    return om


def test_c2_headline_full_size_parity(gpu_ctx, c2):
    om = c2
    assert om.nl == 129 ** 3
    gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    # the affine (Kronecker) form is in use: the apply reads factors, not the 64-point stream
    assert gpu_ctx.kernel_bytes(cdfem.K_APPLY) < 8.0 * 10 * 64 * om.ne
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3)
    x = np.random.default_rng(20261016).uniform(-1, 1, om.nl)
    yo = A.mult(x)
    assert _relmax(gpu_ctx.mult(x), yo) <= TOL_MULT
    xz = x.copy()
    xz[om.ess] = 0.0
    yco = A.mult(xz)
    yco[om.ess] = x[om.ess]
    assert _relmax(gpu_ctx.mult(x, constrained=True), yco) <= TOL_MULT
    assert _relmax(gpu_ctx.diagonal(), A.diag()) <= TOL_MULT
    # bench.py: B = FormLinearSystem(u_bc = 0, b ~ U[-1, 1) seed 20261015), 100 iterations per solve
    b = np.random.default_rng(20261015).uniform(-1, 1, om.nl)
    u = np.zeros(om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    del A
    _, B = gpu_ctx.form_linear_system(u, b)
    assert _relmax(B, Bo) <= TOL_MULT
    xo, io = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=100)
    xg, ig = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=100, check_every=100)
    assert io["iterations"] == ig["iterations"] == 100 and not ig["converged"]
    assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)
    assert abs(ig["final_norm"] - io["final_norm"]) <= 1e-9 * io["final_norm"]
    # and with the host polling every 16 iterations (the default), bitwise the same
    xg2, ig2 = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=100)
    np.testing.assert_array_equal(xg2, xg)


def test_c2_full_size_converged_spd(gpu_ctx, c2):
    om = c2
    gpu_ctx.pa_setup(kinds=5, kappa=0.1, mass=1.0)
    A = O.fa_assemble(om, kappa=0.1, s=1.0, kinds=O.DIFFUSION | O.MASS)
    rng = np.random.default_rng(4)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    del A
    _, B = gpu_ctx.form_linear_system(u, b)
    xo, io = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=1e-13, max_iter=4000)
    xg, ig = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=1e-13, max_iter=4000)
    assert io["converged"] and ig["converged"]
    assert abs(ig["iterations"] - io["iterations"]) <= 2
    assert np.linalg.norm(xg - xo) <= 1e-10 * np.linalg.norm(xo)


def test_c4_full_size_parity(gpu_ctx):
    n, p = 55, 2
    gm = cdfem.kuhn_mesh(3, n, p, with_coords=False)      # bench.py main_c4's mesh
    om = O.KuhnMesh(3, n, p)
    np.testing.assert_array_equal(om.dofmap, gm.dofmap)
    np.testing.assert_array_equal(om.verts, gm.verts)
    assert gm.nl == 1367631
    gpu_ctx.upload_mesh(gm)
    gpu_ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    assert gpu_ctx.kernel_name(cdfem.K_APPLY) == "k_sell_spmv_lds"
    A = O.fa_assemble_simplex(om, kappa=0.1, alpha=1.0, s=1.0, c=C3)
    rp, cols, vals = gpu_ctx.fa_csr()
    orp, ocol, oval = A.export()
    np.testing.assert_array_equal(rp, orp)
    np.testing.assert_array_equal(cols, ocol)
    assert np.abs(vals - oval).max() <= TOL_MULT * np.abs(oval).max()
    del rp, cols, vals, orp, ocol, oval
    x = np.random.default_rng(20261016).uniform(-1, 1, gm.nl)
    assert _relmax(gpu_ctx.mult(x), A.mult(x)) <= TOL_MULT
    assert _relmax(gpu_ctx.diagonal(), A.diag()) <= TOL_MULT
    b = np.random.default_rng(20261015).uniform(-1, 1, gm.nl)
    u = np.zeros(gm.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    del A
    _, B = gpu_ctx.form_linear_system(u, b)
    assert _relmax(B, Bo) <= TOL_MULT
    xo, io = O.gmres(Ac, Bo, dinv=1.0 / Ac.diag(), restart=30, rtol=0.0, atol=0.0, max_it=60)
    xg, ig = gpu_ctx.solve(B, method="gmres", pc="jacobi", restart=30, rel_tol=0.0, abs_tol=0.0, max_iter=60)
    assert io["iterations"] == ig["iterations"] == 60
    assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)


def test_c5_one_gpu_folds_bounded(gpu_ctx):
    """BASELINE configs[4]'s 256^3 p = 2 mesh on one GPU (262,144 bricks): past kDenFoldMaxParts
    apply partials the den step goes back to the one-block finalizer, and with it the betanom step (the
    two folds are taken together).  20 fixed Jacobi-CG iterates on the full operator equal the
    finalizer path's (cg_den_fold 0) to rounding and give the same residual norm."""
    n, p = 256, 2
    gm = cdfem.box_mesh(3, n, p, with_coords=False)
    b = np.random.default_rng(20261015).uniform(-1, 1, gm.nl)
    out = {}
    try:
        for fold in (1024, 0):
            gpu_ctx.set_option("cg_den_fold", fold)
            gpu_ctx.upload_mesh(gm).set_structured(n, n, n)
            gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            _, B = gpu_ctx.form_linear_system(np.zeros(gm.nl), b)
            out[fold] = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=20)
    finally:
        gpu_ctx.set_option("cg_den_fold", 1024)
    (x1, i1), (x0, i0) = out[1024], out[0]
    assert i1["iterations"] == i0["iterations"] == 20
    assert np.linalg.norm(x1 - x0) <= 1e-12 * np.linalg.norm(x0)
    assert abs(i1["final_norm"] - i0["final_norm"]) <= 1e-10 * i0["initial_norm"]


def _pa_full_size(gpu_ctx, n, p, kernel):
    """Full-size parity of the default CG path on an n^3 box of order p against the host PA."""
    om = O.BoxMesh(3, n, p)
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)).set_structured(n, n, n)
    gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    assert gpu_ctx.kernel_name(cdfem.K_APPLY) == kernel
    pa = O.PA(om, kappa=0.1, alpha=1.0, s=1.0, c=C3, kinds=7)
    om.verts = None  # (the point data is formed; the host copy of the geometry is not needed again)
    x = np.random.default_rng(20261016).uniform(-1, 1, om.nl)
    assert _relmax(gpu_ctx.mult(x), pa.mult(x)) <= TOL_MULT
    assert _relmax(gpu_ctx.mult(x, constrained=True), pa.mult(x, constrained=True)) <= TOL_MULT
    del x
    diag = pa.diag()
    assert _relmax(gpu_ctx.diagonal(), diag) <= TOL_MULT
    ess = om.bdr != 0
    dinv = np.where(ess, 1.0, 1.0 / np.where(ess, 1.0, diag))
    del diag
    b = np.random.default_rng(20261015).uniform(-1, 1, om.nl)   # bench.py's RHS
    u = np.zeros(om.nl)
    Bo = pa.form_linear_system(u, b)
    _, B = gpu_ctx.form_linear_system(u, b)
    assert _relmax(B, Bo) <= TOL_MULT
    del b, B
    xo, io = pa.cg(Bo, dinv=dinv, rel_tol=0.0, abs_tol=0.0, max_iter=20)
    xg, ig = gpu_ctx.solve(Bo, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=20)
    assert io["iterations"] == ig["iterations"] == 20 and not ig["converged"]
    assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)
    assert abs(ig["final_norm"] - io["final_norm"]) <= 1e-9 * io["final_norm"]


def test_c3_full_size_oracle_parity(gpu_ctx):
    """BASELINE configs[2] (128^3, p = 4) on the bench's block CG against the host PA oracle."""
    _pa_full_size(gpu_ctx, 128, 4, "k_hobrick_cg")


def test_c5_one_gpu_full_size_oracle_parity(gpu_ctx):
    """BASELINE configs[4]'s 256^3 p = 2 mesh on one GPU (262,144 bricks, the two-stage den sum)
    against the host PA oracle."""
    _pa_full_size(gpu_ctx, 256, 2, "k_brick_cg")
