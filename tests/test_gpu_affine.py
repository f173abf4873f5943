"""The affine-factor PA forms on genuine parallelepipeds.

`pa_affine` 1 forms every point's data as W_q g_e from ten factors per element; `pa_affine` 2 (the
default) applies the same factors in their Kronecker form (pa_core.hpp elem_apply3d_kron).  Both
are exact only where the element map is affine, and every earlier test ran them on the axis-aligned
unit cube, where J = hI: the three off-diagonal diffusion factors vanish and the diagonal ones are
equal, so a swapped factor would pass.  Here the box is mapped through a fixed rotation x shear x
anisotropic scale (plus a translation), on a non-cubic shape, so every factor is distinct and
non-zero.  Checked on every apply that takes the factors: the structured brick kernels (p = 1, 2,
CG and the GMRES Mult), the generic element-block apply (p = 1, 2) and the high-order tile apply
(p = 3, 4, structured and generic), for kinds 7 / 5 / 3, against the oracle (Mult, constrained
Mult, diagonal 1e-13; 30 CG and 40 GMRES iterates 1e-11) and against the per-point stream
(pa_affine 0, 1e-13).  Reference semantics: PA qdata W kappa adj(J) adj(J)^T / det J,
alpha W adj(J) c, W s det J (linear_convection_diffusion_2D.cpp:336-338).
"""
import numpy as np
import pytest

import cdfem
from oracle import oracle as O

pytestmark = pytest.mark.gpu
C3 = (1.0, -2.0, 0.5)
TOL = 1e-13


def _kinds_o(k):
    return (O.DIFFUSION if k & 1 else 0) | (O.CONVECTION if k & 2 else 0) | (O.MASS if k & 4 else 0)


def _relmax(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def _affine_map():
    """A fixed non-diagonal affine map: [0,1]x[0,2]x[0,0.5] (anisotropic scale), sheared, rotated
    about (1, 2, 3) by 0.7 rad, translated."""
    D = np.diag([1.0, 2.0, 0.5])
    S = np.array([[1.0, 0.3, 0.1], [0.0, 1.0, 0.2], [0.0, 0.0, 1.0]])
    a = np.array([1.0, 2.0, 3.0]) / np.sqrt(14.0)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    t = 0.7
    R = np.eye(3) + np.sin(t) * K + (1 - np.cos(t)) * K @ K
    return R @ S @ D, np.array([0.3, -1.2, 2.5])


def _mapped_box(shape, p):
    om = O.BoxMesh(3, shape, p)
    A, t = _affine_map()
    om.verts = np.ascontiguousarray(om.verts @ A.T + t)
    return om


def _run(gpu_ctx, om, shape, p, kinds, structured, aff, u, b, x):
    gpu_ctx.set_option("pa_affine", aff)
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess))
    if structured:
        gpu_ctx.set_structured(*shape)
    gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    out = dict(y=gpu_ctx.mult(x), yc=gpu_ctx.mult(x, constrained=True), dg=gpu_ctx.diagonal(),
               bytes=gpu_ctx.kernel_bytes(cdfem.K_APPLY))
    _, B = gpu_ctx.form_linear_system(u, b)
    out["B"] = B
    out["cg"], icg = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=30,
                                   check_every=7)
    out["gm"], igm = gpu_ctx.solve(B, method="gmres", pc="jacobi", restart=30, rel_tol=0.0, abs_tol=0.0,
                                   max_iter=40)
    assert icg["iterations"] == 30 and igm["iterations"] == 40
    return out


def _check(gpu_ctx, shape, p, kinds, structured):
    om = _mapped_box(shape, p)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3, kinds=_kinds_o(kinds))
    rng = np.random.default_rng(7 + p + kinds)
    x = rng.uniform(-1, 1, om.nl)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    dinv = 1.0 / Ac.diag()
    xcg, _ = O.cg(Ac, Bo, dinv=dinv, rel_tol=0.0, abs_tol=0.0, max_iter=30)
    xgm, _ = O.gmres(Ac, Bo, dinv=dinv, restart=30, rtol=0.0, atol=0.0, max_it=40)
    yo = A.mult(x)
    xz = x.copy()
    xz[om.ess] = 0.0
    yco = A.mult(xz)
    yco[om.ess] = x[om.ess]
    out = {}
    try:
        for aff in (2, 1, 0):
            out[aff] = _run(gpu_ctx, om, shape, p, kinds, structured, aff, u, b, x)
    finally:
        gpu_ctx.set_option("pa_affine", 2)
    # the mapped box is recognised as affine: both factor forms read the factors, not the stream
    assert out[2]["bytes"] < out[0]["bytes"] and out[1]["bytes"] < out[0]["bytes"]
    for aff in (2, 1, 0):
        o = out[aff]
        assert _relmax(o["y"], yo) <= TOL, aff
        assert _relmax(o["yc"], yco) <= TOL, aff
        assert _relmax(o["dg"], A.diag()) <= TOL, aff
        assert _relmax(o["B"], Bo) <= TOL, aff
        assert np.linalg.norm(o["cg"] - xcg) <= 1e-11 * np.linalg.norm(xcg), aff
        assert np.linalg.norm(o["gm"] - xgm) <= 1e-11 * np.linalg.norm(xgm), aff
    for aff in (2, 1):
        for k in ("y", "yc", "dg"):
            assert _relmax(out[aff][k], out[0][k]) <= TOL, (aff, k)


@pytest.mark.parametrize("p", [1, 2])
@pytest.mark.parametrize("kinds", [7, 5, 3])
def test_affine_map_brick(gpu_ctx, p, kinds):
    """Structured brick kernels (k_brick_cg for CG, k_brick3d for the GMRES Mult), partial bricks."""
    _check(gpu_ctx, (6, 5, 7), p, kinds, structured=True)


@pytest.mark.parametrize("p", [1, 2])
@pytest.mark.parametrize("kinds", [7, 5, 3])
def test_affine_map_generic(gpu_ctx, p, kinds):
    """Generic element-block apply (k_apply3d) + CSR E->L."""
    _check(gpu_ctx, (6, 5, 7), p, kinds, structured=False)


@pytest.mark.parametrize("p,structured", [(3, True), (4, True), (3, False), (4, False)])
@pytest.mark.parametrize("kinds", [7, 5, 3])
def test_affine_map_tile(gpu_ctx, p, structured, kinds):
    """High-order tile apply (k_apply3d_tile, p = 3, 4), fused CG on structured boxes."""
    shape = (3, 4, 2) if p == 4 else (4, 3, 5)
    _check(gpu_ctx, shape, p, kinds, structured=structured)


@pytest.mark.parametrize("p,structured", [(4, True), (3, False)])
@pytest.mark.parametrize("mf", [1, 9])
def test_affine_map_tile_mfma(gpu_ctx, p, structured, mf):
    """The affine-factor tile apply with its x / x^T stages on v_mfma_f64_16x16x4_f64 (ho_mfma 1, 9;
    kinds 7, the BASELINE operator)."""
    shape = (3, 4, 2) if p == 4 else (4, 3, 5)
    gpu_ctx.set_option("ho_mfma", mf)
    try:
        _check(gpu_ctx, shape, p, 7, structured=structured)
    finally:
        gpu_ctx.set_option("ho_mfma", 0)


def test_affine_tolerance_is_element_relative(gpu_ctx):
    """mesh_is_affine compares each vertex's parallelepiped defect with 32 ulp of the coordinates
    plus 1e-12 of the element's edge: small elements far from the origin (|x| ~ 100, edges 0.01) are
    accepted unperturbed, and a defect of 1e-9 of one element's edge keeps the per-point stream
    (the round-3 tolerance, 1e-13 of max(|x|, edge) = 1e-11 here, admitted it)."""
    n, p = 4, 2
    om = O.BoxMesh(3, n, p)
    om.verts = np.ascontiguousarray(om.verts * 0.04 + 100.0)
    stream = 8.0 * 10 * (p + 2) ** 3 * om.ne

    def apply_bytes(verts):
        gpu_ctx.upload_mesh(cdfem.Mesh(3, p, verts, om.dofmap, om.nl, om.ess)).set_structured(n, n, n)
        gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
        return gpu_ctx.kernel_bytes(cdfem.K_APPLY)

    assert apply_bytes(om.verts) < stream
    v2 = om.verts.copy()
    v2[13, 7, :] += 1e-9 * 0.01  # vertex (1,1,1) of one element, 1e-9 of its edge
    assert apply_bytes(v2) >= stream


@pytest.mark.parametrize("p", [1, 2])
def test_graded_box_brick_cg(gpu_ctx, p):
    """A box graded along x and y (every element a box, the sizes differ: affine, each element its own
    factors) through the brick CG in the Kronecker form: the apply reads the factors, not the stream,
    and 30 Jacobi-CG iterates match the oracle to 1e-11."""
    shape = (8, 6, 5)
    om = O.BoxMesh(3, shape, p)
    v = om.verts.copy()
    v[..., 0] = v[..., 0] ** 1.5
    v[..., 1] = 0.5 * (v[..., 1] + v[..., 1] ** 2)
    om.verts = np.ascontiguousarray(v)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3)
    rng = np.random.default_rng(11)
    b = rng.uniform(-1, 1, om.nl)
    u = np.zeros(om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    xo, _ = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=30)
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)).set_structured(*shape)
    gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    assert gpu_ctx.kernel_bytes(cdfem.K_APPLY) < 8.0 * 10 * (p + 2) ** 3 * om.ne
    _, B = gpu_ctx.form_linear_system(u, b)
    assert _relmax(B, Bo) <= TOL
    xg, ig = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=30)
    assert ig["iterations"] == 30
    assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)
