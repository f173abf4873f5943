"""pa_uniform: the brick CG apply on a uniformly refined box as one GEMM on the matrix cores.

Every element of a uniform box (MFEM's MakeCartesian3D meshes, the BASELINE configurations) has the
same factors and so the same 27 x 27 element matrix; cdfem_pa_setup detects that (every element's factors
within 1e-14 of element 0's) and forms the matrix once from the Kronecker core (column j = the core on
e_j), and k_brick_cg<..., MX 2> applies it to the brick's 64 elements with 56 v_mfma_f64_16x16x4_f64.
The operator is the Kronecker form's to rounding, so the iterates are checked against the oracle (CG
on the assembled constrained matrix, mesh_recession_handler.cpp:270-276 semantics, 1e-11), against
the Kronecker form (pa_uniform 0, 1e-12) and for bitwise repeatability; a graded box (affine, not
uniform) must keep the Kronecker form."""
import numpy as np
import pytest

import cdfem
from oracle import oracle as O

pytestmark = pytest.mark.gpu
C3 = (1.0, -2.0, 0.5)


def _problem(om, kinds, seed):
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3,
                      kinds=(O.DIFFUSION if kinds & 1 else 0) | (O.CONVECTION if kinds & 2 else 0) |
                      (O.MASS if kinds & 4 else 0))
    rng = np.random.default_rng(seed)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    return Ac, Bo, u, b


@pytest.mark.parametrize("shape,kinds", [((8, 8, 8), 7), ((9, 6, 7), 7), ((5, 9, 10), 5), ((4, 4, 12), 5)])
def test_uniform_matrix_parity(gpu_ctx, shape, kinds):
    """Full and partial bricks, non-zero essential values, kinds 7 (D + C + M) and 5 (kK + sM): 40
    fixed Jacobi-CG iterates of the matrix-core apply against the oracle (1e-11) and the Kronecker form
    (1e-12), bitwise repeatable; the apply's algorithmic bytes drop by the factor stream."""
    p = 2
    om = O.BoxMesh(3, shape, p)
    Ac, Bo, u, b = _problem(om, kinds, 17)
    xo, _ = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=40)
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)).set_structured(*shape)
    gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    _, B = gpu_ctx.form_linear_system(u, b)
    out, nbytes = {}, {}
    try:
        for uni in (1, 0):
            gpu_ctx.set_option("pa_uniform", uni)
            nbytes[uni] = gpu_ctx.kernel_bytes(cdfem.K_APPLY)
            out[uni] = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=40, check_every=7)
        gpu_ctx.set_option("pa_uniform", 1)
        again = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=40)
    finally:
        gpu_ctx.set_option("pa_uniform", 1)
    assert nbytes[1] < nbytes[0]
    np.testing.assert_array_equal(again[0], out[1][0])
    for uni, (xg, ig) in out.items():
        assert ig["iterations"] == 40
        assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo), uni
    assert np.linalg.norm(out[1][0] - out[0][0]) <= 1e-12 * np.linalg.norm(out[0][0])


def test_uniform_matrix_converging_spd(gpu_ctx):
    """kK + sM (kinds 5, SPD): a converging Jacobi-CG solve (rel_tol 1e-10) stops on the same iteration
    with the matrix-core apply and with the Kronecker form, and matches the oracle's solve (1e-9)."""
    shape, p = (8, 8, 8), 2
    om = O.BoxMesh(3, shape, p)
    Ac, Bo, u, b = _problem(om, 5, 5)
    xo, io = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=1e-10, max_iter=2000)
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)).set_structured(*shape)
    gpu_ctx.pa_setup(kinds=5, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    _, B = gpu_ctx.form_linear_system(u, b)
    out = {}
    try:
        for uni in (1, 0):
            gpu_ctx.set_option("pa_uniform", uni)
            out[uni] = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=1e-10, max_iter=2000, check_every=7)
    finally:
        gpu_ctx.set_option("pa_uniform", 1)
    assert out[1][1]["converged"] and out[1][1]["iterations"] == out[0][1]["iterations"]
    assert abs(out[1][1]["iterations"] - io["iterations"]) <= 1
    assert np.linalg.norm(out[1][0] - xo) <= 1e-9 * np.linalg.norm(xo)


@pytest.mark.parametrize("perturb", ["graded", "perturbed"])
def test_nonuniform_box_keeps_kronecker_form(gpu_ctx, perturb):
    """A box graded along x and y (affine, element sizes differ) or with perturbed vertices (not even
    affine) is not taken for uniform: the apply's bytes equal pa_uniform 0's, and 30 CG iterates match
    the oracle (1e-11)."""
    shape, p = (8, 6, 5), 2
    om = O.BoxMesh(3, shape, p, perturb=0.1 if perturb == "perturbed" else 0.0)
    if perturb == "graded":
        v = om.verts.copy()
        v[..., 0] = v[..., 0] ** 1.5
        v[..., 1] = 0.5 * (v[..., 1] + v[..., 1] ** 2)
        om.verts = np.ascontiguousarray(v)
    Ac, Bo, u, b = _problem(om, 7, 11)
    xo, _ = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=30)
    nbytes = {}
    try:
        for uni in (1, 0):
            gpu_ctx.set_option("pa_uniform", uni)
            gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)).set_structured(*shape)
            gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            nbytes[uni] = gpu_ctx.kernel_bytes(cdfem.K_APPLY)
            _, B = gpu_ctx.form_linear_system(u, b)
            xg, ig = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=30)
            assert ig["iterations"] == 30
            assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo), uni
    finally:
        gpu_ctx.set_option("pa_uniform", 1)
    assert nbytes[1] == nbytes[0]
