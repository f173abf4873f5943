"""Brick CG (the BASELINE metric's loop) options that must not change the iterates.

cg_xfold (option, default 1) moves x += alpha d of iteration k into the apply of iteration k + 1 (the dofs a
brick writes the new direction for), with k_cg_xflush adding the last update's term after the loop
when the update logic stopped the solve.  Against cg_xfold 0 the solution must be bitwise equal for
every way a solve ends: fixed iteration counts (max_iter, including 0, 1 and 2), convergence inside a
host-poll batch (check_every), and on partial bricks with essential values.  MFEM CGSolver semantics
(mesh_recession_handler.cpp:270-276) are pinned against the oracle elsewhere (test_gpu_parity.py)."""
import numpy as np
import pytest

import cdfem
from oracle import oracle as O

pytestmark = pytest.mark.gpu
C3 = (1.0, -2.0, 0.5)


def _solve(gpu_ctx, om, shape, kinds, xfold, B, **kw):
    gpu_ctx.set_option("cg_xfold", xfold)
    try:
        return gpu_ctx.solve(B, method="cg", pc="jacobi", **kw)
    finally:
        gpu_ctx.set_option("cg_xfold", 1)


@pytest.mark.parametrize("shape,p,kinds,pert", [((8, 8, 8), 2, 7, 0.0), ((9, 6, 7), 2, 5, 0.1), ((6, 5, 7), 1, 7, 0.0)])
def test_xfold_bitwise(gpu_ctx, shape, p, kinds, pert):
    om = O.BoxMesh(3, shape, p, perturb=pert)
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)).set_structured(*shape)
    gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    rng = np.random.default_rng(5)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    _, B = gpu_ctx.form_linear_system(u, rng.uniform(-1, 1, om.nl))
    cases = [dict(rel_tol=0.0, abs_tol=0.0, max_iter=m, check_every=ce) for m, ce in ((0, 16), (1, 16), (2, 1), (30, 7))]
    if kinds == 5:  # SPD: a converged stop inside a poll batch
        cases.append(dict(rel_tol=1e-8, max_iter=2000, check_every=7))
    for kw in cases:
        x0, i0 = _solve(gpu_ctx, om, shape, kinds, 0, B, **kw)
        x1, i1 = _solve(gpu_ctx, om, shape, kinds, 1, B, **kw)
        assert i0["iterations"] == i1["iterations"] and i0["converged"] == i1["converged"], kw
        np.testing.assert_array_equal(x1, x0)



@pytest.mark.parametrize("shape,p,kinds,xfold", [((8, 8, 8), 2, 7, 0), ((9, 6, 7), 2, 5, 1), ((6, 5, 7), 1, 7, 0),
                                                 ((5, 9, 10), 2, 3, 0)])
def test_brick_update_predicated_faces_bitwise(gpu_ctx, shape, p, kinds, xfold):
    """brick_upd_pb: the update's face sums as eight predicated patch-buffer loads summed in the
    branchy form's order: bitwise the same iterates (partial bricks in every direction, essential
    values, with and without the x-fold)."""
    om = O.BoxMesh(3, shape, p)
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)).set_structured(*shape)
    gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    rng = np.random.default_rng(11)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    _, B = gpu_ctx.form_linear_system(u, rng.uniform(-1, 1, om.nl))
    out = {}
    try:
        gpu_ctx.set_option("cg_xfold", xfold)
        for pb in (1, 0):
            gpu_ctx.set_option("brick_upd_pb", pb)
            out[pb] = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=25, check_every=7)
    finally:
        gpu_ctx.set_option("brick_upd_pb", 1)
        gpu_ctx.set_option("cg_xfold", 1)
    assert out[1][1]["iterations"] == out[0][1]["iterations"] == 25
    np.testing.assert_array_equal(out[1][0], out[0][0])


@pytest.mark.parametrize("shape,p,kinds,fold", [((8, 8, 8), 2, 7, 256), ((9, 6, 7), 2, 5, 1024), ((6, 5, 7), 1, 7, 64)])
def test_den_fold_matches_den_finalizer(gpu_ctx, shape, p, kinds, fold):
    """cg_den_fold N: the update kernel (N workgroups) sums the apply's den partials itself and takes
    MFEM's den step, instead of the one-block finalizer (which sums them with 1024 threads, so den
    differs by rounding): 30 fixed iterates within 1e-12 of the finalizer path and 1e-11 of the
    oracle; on the SPD operator a converging solve stops on the same iteration."""
    om = O.BoxMesh(3, shape, p)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3,
                      kinds=(O.DIFFUSION if kinds & 1 else 0) | (O.CONVECTION if kinds & 2 else 0) |
                      (O.MASS if kinds & 4 else 0))
    rng = np.random.default_rng(31)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    xo, _ = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=30)
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)).set_structured(*shape)
    gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    _, B = gpu_ctx.form_linear_system(u, b)
    out, conv = {}, {}
    try:
        for f in (fold, 0):
            gpu_ctx.set_option("cg_den_fold", f)
            out[f] = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=30, check_every=7)
            if kinds == 5:
                conv[f] = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=1e-8, max_iter=2000, check_every=7)
    finally:
        gpu_ctx.set_option("cg_den_fold", 1024)
    for f, (xg, ig) in out.items():
        assert ig["iterations"] == 30
        assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo), f
    assert np.linalg.norm(out[fold][0] - out[0][0]) <= 1e-12 * np.linalg.norm(out[0][0])
    if conv:
        assert conv[fold][1]["converged"] and conv[fold][1]["iterations"] == conv[0][1]["iterations"]
        assert np.linalg.norm(conv[fold][0] - conv[0][0]) <= 1e-10 * np.linalg.norm(conv[0][0])


@pytest.mark.parametrize("shape,pert", [((8, 8, 8), 0.0), ((9, 6, 7), 0.0), ((5, 9, 10), 0.0)])
def test_brick_mfma_x_stage_parity(gpu_ctx, shape, pert):
    """brick_mfma: k_brick_cg's x stage (p = 2, kinds 7, Kronecker form) on v_mfma_f64_16x16x4_f64, 16
    elements per GEMM, the outputs staged through LDS to the element threads.  Partial bricks, non-zero
    essential values: 40 fixed Jacobi-CG iterates against the oracle (1e-11) and against the VALU x stage
    (1e-12; the matrix core sums each length-3 row in its own order), bitwise repeatable."""
    p = 2
    om = O.BoxMesh(3, shape, p, perturb=pert)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3)
    rng = np.random.default_rng(43)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    xo, _ = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=40)
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)).set_structured(*shape)
    gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    _, B = gpu_ctx.form_linear_system(u, b)
    out = {}
    try:
        gpu_ctx.set_option("pa_uniform", 0)  # (a uniform box: the x stage belongs to the Kronecker form)
        for mx in (1, 0):
            gpu_ctx.set_option("brick_mfma", mx)
            out[mx] = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=40, check_every=7)
        gpu_ctx.set_option("brick_mfma", 1)
        again = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=40)
    finally:
        gpu_ctx.set_option("brick_mfma", 0)
        gpu_ctx.set_option("pa_uniform", 1)
    np.testing.assert_array_equal(again[0], out[1][0])
    for mx, (xg, ig) in out.items():
        assert ig["iterations"] == 40
        assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo), mx
    assert np.linalg.norm(out[1][0] - out[0][0]) <= 1e-12 * np.linalg.norm(out[0][0])


@pytest.mark.parametrize("shape,p,kinds,grp", [((12, 16, 8), 2, 7, 8), ((12, 16, 8), 2, 5, 16), ((9, 6, 7), 2, 7, 4),
                                                ((10, 8, 13), 1, 7, 64)])
def test_den_group_matches_ungrouped(gpu_ctx, shape, p, kinds, grp):
    """den_group G (automatic past the fold bounds: C5's per-rank slab, its 256^3 on one GPU; forced here on
    small boxes): each group of G bricks' den partials is summed by the group's last-arriving brick (a
    write-through partial, an agent-scope arrival count, sc1 loads of the group) and the folds sum the
    group sums.  Groups of 8 / 16 / 4 / 64 over 24 / 24 / 24 / 48 bricks (a partial last group in three
    of them): 30 fixed iterates within 1e-12 of the ungrouped fold and 1e-11 of the oracle, bitwise
    repeatable (the group sum does not depend on the order the bricks arrive in)."""
    om = O.BoxMesh(3, shape, p)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3,
                      kinds=(O.DIFFUSION if kinds & 1 else 0) | (O.CONVECTION if kinds & 2 else 0) |
                      (O.MASS if kinds & 4 else 0))
    rng = np.random.default_rng(37)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    xo, _ = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=30)
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)).set_structured(*shape)
    gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    _, B = gpu_ctx.form_linear_system(u, b)
    out = {}
    try:
        for g in (grp, 0):
            gpu_ctx.set_option("den_group", g)
            out[g] = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=30, check_every=7)
        gpu_ctx.set_option("den_group", grp)
        again = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=30)
    finally:
        gpu_ctx.set_option("den_group", 0)
    np.testing.assert_array_equal(again[0], out[grp][0])
    for g, (xg, ig) in out.items():
        assert ig["iterations"] == 30
        assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo), g
    assert np.linalg.norm(out[grp][0] - out[0][0]) <= 1e-12 * np.linalg.norm(out[0][0])
    with pytest.raises(cdfem.CdfemError):
        gpu_ctx.set_option("den_group", 3)


@pytest.mark.parametrize("shape,p,kinds", [((8, 8, 8), 2, 7), ((9, 6, 7), 2, 5), ((6, 5, 7), 1, 7), ((5, 9, 10), 2, 3)])
def test_brick_mult_patch_buffer_bitwise(gpu_ctx, shape, p, kinds):
    """brick_mult_pb: the structured Mult through the patch buffer (k_brick3d<..., PBO> +
    k_brick_patch_sum) sums each row's 1-8 brick entries in k_brick_faces' order, so Mult,
    constrained Mult and 40 GMRES(30) iterates are bitwise those of the owned-row / face-partial form,
    and the Mult matches the oracle to 1e-13 (partial bricks in every direction)."""
    om = O.BoxMesh(3, shape, p)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3,
                      kinds=(O.DIFFUSION if kinds & 1 else 0) | (O.CONVECTION if kinds & 2 else 0) |
                      (O.MASS if kinds & 4 else 0))
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)).set_structured(*shape)
    gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    rng = np.random.default_rng(41)
    x = rng.uniform(-1, 1, om.nl)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    _, B = gpu_ctx.form_linear_system(u, rng.uniform(-1, 1, om.nl))
    out = {}
    try:
        for pb in (1, 0):
            gpu_ctx.set_option("brick_mult_pb", pb)
            xg, ig = gpu_ctx.solve(B, method="gmres", pc="jacobi", restart=30, rel_tol=0.0, abs_tol=0.0, max_iter=40)
            out[pb] = (gpu_ctx.mult(x), gpu_ctx.mult(x, constrained=True), xg, ig["iterations"])
    finally:
        gpu_ctx.set_option("brick_mult_pb", 1)
    for k in range(3):
        np.testing.assert_array_equal(out[1][k], out[0][k])
    assert out[1][3] == out[0][3] == 40
    yo = A.mult(x)
    assert np.abs(out[1][0] - yo).max() <= 1e-13 * np.abs(yo).max()


@pytest.mark.parametrize("shape,p,kinds", [((8, 8, 8), 2, 7), ((9, 6, 7), 2, 5), ((6, 5, 7), 1, 7)])
def test_beta_fold_matches_update_finalizer(gpu_ctx, shape, p, kinds):
    """cg_beta_fold: the apply takes the betanom step of the previous update (every workgroup sums the
    update's partials, workgroup 0 records MFEM's decision) instead of the one-block finalizer: fixed
    iterate counts 0 / 1 / 2 / 30 within 1e-12 of the finalizer path and 1e-11 of the oracle, and on
    the SPD operator a converging solve stops on the same iteration with the same flags."""
    om = O.BoxMesh(3, shape, p)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3,
                      kinds=(O.DIFFUSION if kinds & 1 else 0) | (O.CONVECTION if kinds & 2 else 0) |
                      (O.MASS if kinds & 4 else 0))
    rng = np.random.default_rng(37)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    xo, _ = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=30)
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)).set_structured(*shape)
    gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    _, B = gpu_ctx.form_linear_system(u, b)
    cases = [dict(rel_tol=0.0, abs_tol=0.0, max_iter=m, check_every=ce) for m, ce in ((0, 16), (1, 16), (2, 1), (30, 7))]
    if kinds == 5:
        cases.append(dict(rel_tol=1e-8, max_iter=2000, check_every=7))
    try:
        for kw in cases:
            res = {}
            for bf in (1, 0):
                gpu_ctx.set_option("cg_beta_fold", bf)
                res[bf] = gpu_ctx.solve(B, method="cg", pc="jacobi", **kw)
            (x1, i1), (x0, i0) = res[1], res[0]
            assert i1["iterations"] == i0["iterations"] and i1["converged"] == i0["converged"], kw
            assert np.linalg.norm(x1 - x0) <= 1e-12 * max(np.linalg.norm(x0), 1e-300), kw
            if kw["max_iter"] == 30:
                assert np.linalg.norm(x1 - xo) <= 1e-11 * np.linalg.norm(xo)
    finally:
        gpu_ctx.set_option("cg_beta_fold", 1)


def test_beta_fold_breakdown_paths(gpu_ctx):
    """The two early exits the betanom fold must take exactly as the finalizer path does:
    (a) an indefinite Jacobi preconditioner (kappa K + s M with s = -124 on a 6 x 5 x 7 p = 2 box: 210
    negative diagonal entries), where MFEM's CGSolver stops on betanom < 0 at iteration 4 — the fold's
    workgroups take that decision from the shared cg_stop_kind at the host's update count; (b) den == 0
    at the first den step (a zero operator away from the boundary, zero boundary values, pc none), where
    the den-fold update returns before any update.  Both: same iteration count and flags with
    cg_beta_fold 0 and 1 and the oracle, x within 1e-12 of each other and 1e-11 of the oracle."""
    shape, p = (6, 5, 7), 2
    om = O.BoxMesh(3, shape, p)
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)).set_structured(*shape)
    rng = np.random.default_rng(3)
    u, b = np.zeros(om.nl), rng.uniform(-1, 1, om.nl)
    cases = []
    # (a) betanom < 0 after four updates
    A = O.fa_assemble(om, kappa=0.1, s=-124.0, kinds=O.DIFFUSION | O.MASS)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    xo, io = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=1e-12, max_iter=200)
    assert not io["converged"] and io["iterations"] == 4
    cases.append((dict(kinds=5, kappa=0.1, mass=-124.0), "jacobi", xo, io))
    # (b) den == 0 at the first den step: convection with c = 0 is the zero operator, the constrained
    # operator is the identity on the (zero) boundary values only
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, c=(0.0, 0.0, 0.0), kinds=O.CONVECTION)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    xo, io = O.cg(Ac, Bo, dinv=None, rel_tol=1e-12, max_iter=200)
    assert not io["converged"] and io["iterations"] == 0
    cases.append((dict(kinds=2, alpha=1.0, conv=(0.0, 0.0, 0.0)), "none", xo, io))
    try:
        for setup, pc, xo, io in cases:
            gpu_ctx.pa_setup(**setup)
            _, B = gpu_ctx.form_linear_system(u, b)
            res = {}
            for bf in (1, 0):
                gpu_ctx.set_option("cg_beta_fold", bf)
                res[bf] = gpu_ctx.solve(B, method="cg", pc=pc, rel_tol=1e-12, max_iter=200, check_every=3)
            (x1, i1), (x0, i0) = res[1], res[0]
            assert i1["iterations"] == i0["iterations"] == io["iterations"], setup
            assert not i1["converged"] and not i0["converged"], setup
            scale = max(np.linalg.norm(xo), 1e-300)
            assert np.linalg.norm(x1 - x0) <= 1e-12 * scale, setup
            assert np.linalg.norm(x1 - xo) <= 1e-11 * scale, setup
    finally:
        gpu_ctx.set_option("cg_beta_fold", 1)


def test_brick_byte_limit_falls_back_to_generic(gpu_ctx):
    """The brick kernels reach their vectors and patch buffer through buffer resources whose 32-bit
    offsets use kOOB = 2^31 as the out-of-range marker, so the brick path is taken only when every such
    buffer is below 2^31 bytes; a larger box runs the generic element kernels.  Forced
    here on a small box with brick_byte_limit: the generic path takes over (its CG launches the
    direction kernel, which the brick CG does not have) and gives the brick path's Mult (1e-13),
    diagonal and CG iterates (1e-11 of the oracle)."""
    shape, p = (8, 8, 8), 2
    om = O.BoxMesh(3, shape, p)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3)
    rng = np.random.default_rng(71)
    x, b = rng.uniform(-1, 1, om.nl), rng.uniform(-1, 1, om.nl)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    xo, _ = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=30)
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)).set_structured(*shape)
    gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    _, B = gpu_ctx.form_linear_system(u, b)
    out = {}
    try:
        for lim in (None, 4096):
            if lim:
                gpu_ctx.set_option("brick_byte_limit", lim)
            gpu_ctx.set_option("profile_mask", -1)
            gpu_ctx.profile(True)
            xg, ig = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=30)
            _, ndir = gpu_ctx.profile_read(cdfem.K_DIRECTION)
            gpu_ctx.profile(False)
            out[lim] = dict(y=gpu_ctx.mult(x), yc=gpu_ctx.mult(x, constrained=True), x=xg, it=ig["iterations"],
                            ndir=ndir)
    finally:
        gpu_ctx.set_option("brick_byte_limit", 0)  # 0: back to the default bound, 2^31 bytes
        gpu_ctx.profile(False)
    assert out[None]["ndir"] == 0 and out[4096]["ndir"] > 0
    yo = A.mult(x)
    for lim in (None, 4096):
        assert np.abs(out[lim]["y"] - yo).max() <= 1e-13 * np.abs(yo).max()
        assert out[lim]["it"] == 30
        assert np.linalg.norm(out[lim]["x"] - xo) <= 1e-11 * np.linalg.norm(xo)
    assert np.abs(out[4096]["yc"] - out[None]["yc"]).max() <= 1e-13 * np.abs(out[None]["yc"]).max()
    with pytest.raises(cdfem.CdfemError):
        gpu_ctx.set_option("brick_byte_limit", -1)
