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
