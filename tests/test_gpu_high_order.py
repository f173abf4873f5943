"""GPU high-order hex path (3D p = 3, 4: wave-per-element kernel, element-major layout; BASELINE
config C3 is 128^3 at p = 4) against the oracle, same parity ladder as tests/test_gpu_parity.py:
Mult / diagonal / linear form to 1e-13, fixed CG iterates to 1e-11, MMS error to 1e-6 relative.
At a full-size-class mesh (32^3, p = 4: 2.1 M DoFs) size-independent properties are checked.
"""
import numpy as np
import pytest

import cdfem
from oracle import oracle as O

pytestmark = pytest.mark.gpu
C3 = (1.0, -2.0, 0.5)


def _kinds_o(k):
    return (O.DIFFUSION if k & 1 else 0) | (O.CONVECTION if k & 2 else 0) | (O.MASS if k & 4 else 0)


def _pair(gpu_ctx, n, p, pert, kinds):
    om = O.BoxMesh(3, n, p, perturb=pert)
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    gpu_ctx.upload_mesh(gm)
    gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3, kinds=_kinds_o(kinds))
    return om, A


@pytest.mark.parametrize("n,p,pert", [(2, 3, 0.1), (3, 3, 0.0), (2, 4, 0.15), (3, 4, 0.1), (5, 4, 0.0)])
@pytest.mark.parametrize("kinds", [7, 5, 1, 2, 4])
def test_ho_mult_parity(gpu_ctx, n, p, pert, kinds):
    om, A = _pair(gpu_ctx, n, p, pert, kinds)
    x = np.random.default_rng(13).uniform(-1, 1, om.nl)
    yo = A.mult(x)
    assert np.abs(gpu_ctx.mult(x) - yo).max() <= 1e-13 * np.abs(yo).max()
    xz = x.copy()
    xz[om.ess] = 0.0
    yc = A.mult(xz)
    yc[om.ess] = x[om.ess]
    assert np.abs(gpu_ctx.mult(x, constrained=True) - yc).max() <= 1e-13 * np.abs(yc).max()


@pytest.mark.parametrize("n,p", [(2, 3), (3, 4)])
def test_ho_diagonal_and_lf(gpu_ctx, n, p):
    om, A = _pair(gpu_ctx, n, p, 0.1, 7)
    d = gpu_ctx.diagonal()
    assert np.abs(d - A.diag()).max() <= 1e-13 * np.abs(A.diag()).max()
    prm = O.mms_params(O.MMS_SIN, 3, kappa=0.1, s=1.0, c=C3, p=p)
    xyz = gpu_ctx.quadrature_points(cdfem.RULE_LINEARFORM)
    b = gpu_ctx.lf_assemble(O.mms_f(prm, xyz).reshape(-1))
    bo = O.lf_assemble(om, prm)
    assert np.abs(b - bo).max() <= 1e-12 * np.abs(bo).max()


@pytest.mark.parametrize("n,p,pert,structured", [(2, 3, 0.1, False), (3, 4, 0.1, False), (3, 3, 0.0, True),
                                                 (4, 4, 0.0, True)])
@pytest.mark.parametrize("kinds", [1, 2, 3, 4, 5, 6, 7])
def test_ho_diagonal_every_kinds(gpu_ctx, n, p, pert, structured, kinds):
    """The staged sum-factorised diagonal (k_diag_ho: z contraction per point column, y and x through
    LDS; compile-time term groups per kinds mask) against the oracle's assembled diagonal, 1e-13,
    for every integrator combination, generic and structured (pencil E-vector) layouts."""
    om, A = _pair(gpu_ctx, n, p, pert, kinds)
    if structured:
        gpu_ctx.set_structured(n, n, n)
        gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    d, do = gpu_ctx.diagonal(), A.diag()
    assert np.abs(d - do).max() <= 1e-13 * np.abs(do).max()


@pytest.mark.parametrize("n,p", [(3, 3), (4, 4)])
def test_ho_structured_e2l_bitwise(gpu_ctx, n, p):
    """cdfem_mesh_set_structured at p >= 3 switches to the lattice E->L (k_e2l_box): same sums,
    same order as the generic position-array E->L -> bitwise-identical results."""
    m = cdfem.box_mesh(3, n, p, perturb=0.1)
    x = np.random.default_rng(21).uniform(-1, 1, m.nl)
    gpu_ctx.upload_mesh(m)
    gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    y0, yc0, d0 = gpu_ctx.mult(x), gpu_ctx.mult(x, constrained=True), gpu_ctx.diagonal()
    gpu_ctx.upload_mesh(m).set_structured(n, n, n)
    gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    np.testing.assert_array_equal(gpu_ctx.mult(x), y0)
    np.testing.assert_array_equal(gpu_ctx.mult(x, constrained=True), yc0)
    np.testing.assert_array_equal(gpu_ctx.diagonal(), d0)
    om = O.BoxMesh(3, n, p, perturb=0.0)
    assert np.array_equal(om.dofmap, m.dofmap)


def test_ho_cg_parity(gpu_ctx):
    om, A = _pair(gpu_ctx, 3, 4, 0.1, 5)
    rng = np.random.default_rng(2)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    _, B = gpu_ctx.form_linear_system(u, b)
    assert np.abs(B - Bo).max() <= 1e-13 * np.abs(Bo).max()
    xo, io = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=50)
    xg, ig = gpu_ctx.solve(B, method="cg", rel_tol=0.0, abs_tol=0.0, max_iter=50, check_every=11)
    assert io["iterations"] == ig["iterations"] == 50
    assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)
    xo, io = O.gmres(Ac, Bo, dinv=1.0 / Ac.diag(), restart=30, rtol=1e-10, atol=1e-12, max_it=500)
    om2, A2 = _pair(gpu_ctx, 3, 4, 0.1, 5)
    _, B2 = gpu_ctx.form_linear_system(u, b)
    xg, ig = gpu_ctx.solve(B2, method="gmres", restart=30, rel_tol=1e-10, abs_tol=1e-12, max_iter=500)
    assert io["converged"] and ig["converged"] and abs(io["iterations"] - ig["iterations"]) <= 1
    assert np.linalg.norm(xg - xo) <= 1e-8 * np.linalg.norm(xo)


@pytest.mark.parametrize("n,p,pert", [(3, 4, 0.1), (3, 3, 0.15)])
def test_ho_fused_cg_parity(gpu_ctx, n, p, pert):
    """Structured boxes run the fused high-order CG iteration (den from the apply's E-vector, E->L
    inside the update): fixed iterates against the oracle with non-zero essential values (so the
    essential DoFs' d_i^2 term of den is exercised), and against the unfused path."""
    om = O.BoxMesh(3, n, p, perturb=pert)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3, kinds=_kinds_o(5))
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    rng = np.random.default_rng(12)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    xo, io = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=50)
    out = {}
    try:
        for fused in (1, 0):
            gpu_ctx.set_option("cg_fused", fused)
            gpu_ctx.upload_mesh(gm).set_structured(n, n, n)
            gpu_ctx.pa_setup(kinds=5, kappa=0.1, mass=1.0)
            _, B = gpu_ctx.form_linear_system(u, b)
            out[fused] = gpu_ctx.solve(B, method="cg", rel_tol=0.0, abs_tol=0.0, max_iter=50, check_every=7)
    finally:
        gpu_ctx.set_option("cg_fused", 1)
    for fused, (xg, ig) in out.items():
        assert io["iterations"] == ig["iterations"] == 50
        assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo), fused
    # the residual norms agree to rounding relative to the initial norm (after 50 iterations the
    # small p = 3 case has converged to ~1e-12, where only rounding is left)
    assert abs(out[1][1]["final_norm"] - out[0][1]["final_norm"]) <= 1e-12 * out[0][1]["initial_norm"]


@pytest.mark.parametrize("shape,p", [((4, 3, 5), 4), ((5, 4, 3), 3)])
def test_ho_fused_cg_box_shapes(gpu_ctx, shape, p):
    """Fused vs unfused high-order CG on non-cubic boxes (the essential-DoF ownership rule on each
    axis), converging to tolerance with the same iteration count and solution."""
    m = cdfem.box_mesh(3, shape, p, perturb=0.1, with_coords=False)
    rng = np.random.default_rng(13)
    u = np.zeros(m.nl)
    u[m.ess] = rng.uniform(-1, 1, len(m.ess))
    b = rng.uniform(-1, 1, m.nl)
    out = {}
    try:
        for fused in (1, 0):
            gpu_ctx.set_option("cg_fused", fused)
            gpu_ctx.upload_mesh(m).set_structured(*shape)
            gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=(0.0, 0.0, 0.0), mass=1.0)
            _, B = gpu_ctx.form_linear_system(u, b)
            out[fused] = gpu_ctx.solve(B, method="cg", rel_tol=1e-12, abs_tol=0.0, max_iter=2000)
    finally:
        gpu_ctx.set_option("cg_fused", 1)
    (x1, i1), (x0, i0) = out[1], out[0]
    assert i1["converged"] and i0["converged"] and abs(i1["iterations"] - i0["iterations"]) <= 1
    assert np.linalg.norm(x1 - x0) <= 1e-10 * np.linalg.norm(x0)


@pytest.mark.parametrize("shape,p,kinds", [((3, 3, 3), 4, 7), ((4, 3, 5), 3, 5), ((3, 4, 2), 4, 3)])
def test_ho_dfold_matches_direction_pass(gpu_ctx, shape, p, kinds):
    """ho_dfold: the Kronecker tile's fused CG apply forms d = z + beta d_old itself (its owner element
    writes it to the other direction buffer) and the direction pass is skipped (default).  Affine
    boxes with non-zero essential values: 40 fixed iterates against the oracle (1e-11) and against
    the direction pass (same formula: 1e-13), same residual norms to rounding; a converging solve
    (stopped by the tolerance inside a check interval) gives the same iteration count and solution."""
    om = O.BoxMesh(3, shape, p)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3, kinds=_kinds_o(kinds))
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    rng = np.random.default_rng(17)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    xo, _ = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=40)
    out, conv = {}, {}
    try:
        gpu_ctx.set_option("ho_brick", 0)  # the tile path's fused CG (the block CG has its own tests)
        for df in (1, 0):
            gpu_ctx.set_option("ho_dfold", df)
            gpu_ctx.upload_mesh(gm).set_structured(*shape)
            gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            _, B = gpu_ctx.form_linear_system(u, b)
            out[df] = gpu_ctx.solve(B, method="cg", rel_tol=0.0, abs_tol=0.0, max_iter=40, check_every=7)
            conv[df] = gpu_ctx.solve(B, method="cg", rel_tol=1e-6, abs_tol=0.0, max_iter=400, check_every=16)
    finally:
        gpu_ctx.set_option("ho_dfold", 1)
        gpu_ctx.set_option("ho_brick", 1)
    for df, (xg, ig) in out.items():
        assert ig["iterations"] == 40
        assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo), df
    for df in (1,):
        assert np.linalg.norm(out[df][0] - out[0][0]) <= 1e-13 * np.linalg.norm(out[0][0]), df
        assert abs(out[df][1]["final_norm"] - out[0][1]["final_norm"]) <= 1e-12 * out[0][1]["initial_norm"]
        assert conv[df][1]["iterations"] == conv[0][1]["iterations"], df
        assert np.linalg.norm(conv[df][0] - conv[0][0]) <= 1e-12 * np.linalg.norm(conv[0][0]), df


def test_ho_mms_error_matches_oracle(gpu_ctx):
    n, p = 3, 4
    om = O.BoxMesh(3, n, p)
    prm = O.mms_params(O.MMS_SIN, 3, kappa=0.1, s=1.0, c=C3, modes=(1, 1, 1), p=p)
    Xo, io, eo = O.solve_mms(om, prm, kappa=0.1, s=1.0, c=C3, solver="gmres", tol=1e-12, atol=1e-14)
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    gpu_ctx.upload_mesh(gm)
    gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    xyz = gpu_ctx.quadrature_points(cdfem.RULE_LINEARFORM)
    b = gpu_ctx.lf_assemble(O.mms_f(prm, xyz).reshape(-1))
    u = np.zeros(om.nl)
    u[om.ess] = O.mms_u(prm, om.dof_coords()[om.ess])
    _, B = gpu_ctx.form_linear_system(u, b)
    X, ig = gpu_ctx.solve(B, method="gmres", restart=30, rel_tol=1e-12, abs_tol=1e-14, max_iter=2000)
    assert ig["converged"]
    eg = O.l2_error(om, X, prm)
    assert abs(eg - eo) <= 1e-6 * eo


def test_ho_full_size_properties(gpu_ctx):
    """32^3 hexes at p = 4 (2,146,689 DoFs): constants in the kernel of D + C, mass total = volume,
    linearity, the diffusion form symmetric, bitwise-reproducible Mult."""
    m = cdfem.box_mesh(3, 32, 4, perturb=0.1, with_coords=False)
    gpu_ctx.upload_mesh(m)
    one = np.ones(m.nl)
    gpu_ctx.pa_setup(kinds=3, kappa=0.1, alpha=1.0, conv=C3)
    assert np.abs(gpu_ctx.mult(one)).max() <= 1e-12
    gpu_ctx.pa_setup(kinds=4, mass=1.0)
    assert abs(one @ gpu_ctx.mult(one) - 1.0) <= 1e-11
    gpu_ctx.pa_setup(kinds=1, kappa=1.0)
    rng = np.random.default_rng(5)
    x, y = rng.uniform(-1, 1, m.nl), rng.uniform(-1, 1, m.nl)
    Kx, Ky = gpu_ctx.mult(x), gpu_ctx.mult(y)
    assert abs(x @ Ky - y @ Kx) <= 1e-11 * abs(x @ Ky)
    assert np.abs(gpu_ctx.mult(2.0 * x - 3.0 * y) - (2.0 * Kx - 3.0 * Ky)).max() <= 1e-12 * np.abs(Kx).max()
    np.testing.assert_array_equal(gpu_ctx.mult(x), Kx)


def test_ho_c3_full_size_fused_cg(gpu_ctx):
    """BASELINE config C3 at full size (128^3 hexes, p = 4, 135,005,697 DoFs, structured): the
    fused CG iteration's recursive residual (r, M^-1 r) after 30 iterations equals the residual
    recomputed from the returned iterate, with non-zero essential values."""
    n = 128
    m = cdfem.box_mesh(3, n, 4, with_coords=False)
    gpu_ctx.upload_mesh(m).set_structured(n, n, n)
    gpu_ctx.pa_setup(kinds=5, kappa=0.1, mass=1.0)
    rng = np.random.default_rng(128)
    u = np.zeros(m.nl)
    u[m.ess] = rng.uniform(-1, 1, len(m.ess))
    _, B = gpu_ctx.form_linear_system(u, rng.uniform(-1, 1, m.nl))
    del u
    X, info = gpu_ctx.solve(B, method="cg", rel_tol=0.0, abs_tol=0.0, max_iter=30)
    assert info["iterations"] == 30 and info["final_norm"] < info["initial_norm"]
    r = B - gpu_ctx.mult(X, constrained=True)
    del B, X
    d = gpu_ctx.diagonal()
    d[m.ess] = 1.0
    true = np.sqrt(r @ (r / d))
    assert abs(true - info["final_norm"]) <= 1e-6 * true



@pytest.mark.parametrize("n,p,pert,structured", [(2, 3, 0.1, False), (3, 3, 0.0, True), (3, 4, 0.15, False),
                                                 (4, 4, 0.0, True), (5, 4, 0.1, False)])
@pytest.mark.parametrize("kinds", [7, 5, 2])
@pytest.mark.parametrize("mf", [1, 3, 8, 9, 15])
def test_ho_mfma_stages_parity(gpu_ctx, n, p, pert, structured, kinds, mf):
    """set_option("ho_mfma", mf): the tile apply's LDS stages as block GEMMs on
    v_mfma_f64_16x16x4_f64 (1: stage x; 3: x and y; 15: x, y, y^T and x^T).  Mult and constrained
    Mult against the oracle (1e-13) and against the VALU stages (summation order only: 1e-14);
    includes a partly filled last block."""
    om = O.BoxMesh(3, n, p, perturb=pert)
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3, kinds=_kinds_o(kinds))
    x = np.random.default_rng(31).uniform(-1, 1, om.nl)
    xz = x.copy()
    xz[om.ess] = 0.0
    yo = A.mult(x)
    yc = A.mult(xz)
    yc[om.ess] = x[om.ess]
    out = {}
    try:
        for m in (0, mf):
            gpu_ctx.set_option("ho_mfma", m)
            gpu_ctx.upload_mesh(gm)
            if structured:
                gpu_ctx.set_structured(n, n, n)
            gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            out[m] = (gpu_ctx.mult(x), gpu_ctx.mult(x, constrained=True))
    finally:
        gpu_ctx.set_option("ho_mfma", 0)
    y, ycg = out[mf]
    assert np.abs(y - yo).max() <= 1e-13 * np.abs(yo).max()
    assert np.abs(ycg - yc).max() <= 1e-13 * np.abs(yc).max()
    assert np.abs(y - out[0][0]).max() <= 1e-14 * np.abs(yo).max()


@pytest.mark.parametrize("n,p", [(3, 4), (4, 3)])
@pytest.mark.parametrize("mf", [1, 9, 15])
def test_ho_mfma_fused_cg_parity(gpu_ctx, n, p, mf):
    """The fused high-order CG iteration with the MFMA stages: 50 fixed Jacobi-CG iterates with
    non-zero essential values against the oracle (1e-11)."""
    om = O.BoxMesh(3, n, p, perturb=0.1)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3, kinds=_kinds_o(5))
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    rng = np.random.default_rng(14)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    xo, io = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=50)
    try:
        gpu_ctx.set_option("ho_mfma", mf)
        gpu_ctx.upload_mesh(gm).set_structured(n, n, n)
        gpu_ctx.pa_setup(kinds=5, kappa=0.1, mass=1.0)
        _, B = gpu_ctx.form_linear_system(u, b)
        xg, ig = gpu_ctx.solve(B, method="cg", rel_tol=0.0, abs_tol=0.0, max_iter=50, check_every=7)
    finally:
        gpu_ctx.set_option("ho_mfma", 0)
    assert io["iterations"] == ig["iterations"] == 50
    assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)


@pytest.mark.parametrize("n,p,structured,kinds", [(3, 4, True, 7), (4, 3, True, 5), (3, 4, False, 7),
                                                  (5, 4, True, 6), (4, 3, False, 1), (3, 4, True, 2),
                                                  (4, 3, True, 3), (3, 4, True, 4)])
def test_ho_affine_factors(gpu_ctx, n, p, structured, kinds):
    """pa_affine on an affine box: 2 (default) runs the Kronecker-form tile (k_apply3d_ktile, 1D rule
    matrices, no quadrature-point stage), 1 the quadrature tile forming each point's data as
    W_q * g_e from one factor set per element.  Mult, constrained Mult, diagonal against the oracle
    (1e-13) and the per-point multilinear-map setup (pa_affine 0, rounding: 1e-13); 50 fused CG
    iterates against the oracle (1e-11); the byte count drops by the stream."""
    om = O.BoxMesh(3, n, p)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3, kinds=_kinds_o(kinds))
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    x = np.random.default_rng(41).uniform(-1, 1, om.nl)
    rng = np.random.default_rng(42)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    # pure convection (kinds 2): the Jacobi diagonal is zero off the boundary, so there is no oracle
    # solve to compare with (the GPU iterates are only checked for the iteration count)
    xo = None if kinds == 2 else O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=50)[0]
    out = {}
    try:
        for aff in (2, 1, 0):
            gpu_ctx.set_option("pa_affine", aff)
            gpu_ctx.upload_mesh(gm)
            if structured:
                gpu_ctx.set_structured(n, n, n)
            gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            _, B = gpu_ctx.form_linear_system(u, b)
            xg, ig = gpu_ctx.solve(B, method="cg", rel_tol=0.0, abs_tol=0.0, max_iter=50, check_every=7)
            gpu_ctx.set_option("ho_brick", 0)  # the tile apply's bytes (the block CG reports its own)
            nb = gpu_ctx.kernel_bytes(cdfem.K_APPLY)
            gpu_ctx.set_option("ho_brick", 1)
            out[aff] = dict(y=gpu_ctx.mult(x), yc=gpu_ctx.mult(x, constrained=True), dg=gpu_ctx.diagonal(),
                            bytes=nb, x=xg, it=ig["iterations"])
    finally:
        gpu_ctx.set_option("pa_affine", 2)
    yo = A.mult(x)
    for aff in (2, 1):
        assert out[aff]["bytes"] < out[0]["bytes"]
        assert np.abs(out[aff]["y"] - yo).max() <= 1e-13 * np.abs(yo).max()
        assert np.abs(out[aff]["dg"] - A.diag()).max() <= 1e-13 * np.abs(A.diag()).max()
        for k in ("y", "yc", "dg"):
            assert np.abs(out[aff][k] - out[0][k]).max() <= 1e-13 * np.abs(out[0][k]).max()
        assert out[aff]["it"] == 50
        if xo is not None:
            assert np.linalg.norm(out[aff]["x"] - xo) <= 1e-11 * np.linalg.norm(xo)




@pytest.mark.parametrize("shape,p,kinds", [((4, 4, 4), 4, 7), ((5, 3, 6), 4, 5), ((3, 4, 5), 3, 7), ((4, 5, 3), 3, 3),
                                           ((2, 2, 2), 4, 6), ((1, 3, 2), 4, 7)])
def test_ho_brick_cg_parity(gpu_ctx, shape, p, kinds):
    """ho_brick (default): the high-order CG on an affine structured box through k_hobrick_cg (the
    Kronecker tile core on 2^3-element blocks, the block's E->L in LDS, the patch buffer) and the brick
    update, instead of the tile apply's E-vector and the flat E->L update.  Boxes with partial blocks
    in every direction and non-zero essential values: 40 fixed Jacobi-CG iterates against the oracle
    (1e-11) and the tile path (1e-12); a converging SPD solve stops on the tile path's iteration with
    its solution (1e-10); bitwise repeatable; the byte count shows the block path ran."""
    om = O.BoxMesh(3, shape, p)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3, kinds=_kinds_o(kinds))
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    rng = np.random.default_rng(23)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    xo, _ = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=40)
    out, conv, nbytes = {}, {}, {}
    try:
        for hb in (1, 0):
            gpu_ctx.set_option("ho_brick", hb)
            gpu_ctx.upload_mesh(gm).set_structured(*shape)
            gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            nbytes[hb] = gpu_ctx.kernel_bytes(cdfem.K_UPDATE)
            _, B = gpu_ctx.form_linear_system(u, b)
            out[hb] = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=40, check_every=7)
            if hb:
                again = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=40)
                np.testing.assert_array_equal(again[0], out[hb][0])
            if kinds == 5:
                conv[hb] = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=1e-10, max_iter=2000, check_every=9)
    finally:
        gpu_ctx.set_option("ho_brick", 1)
    assert nbytes[1] != nbytes[0]
    for hb, (xg, ig) in out.items():
        assert ig["iterations"] == 40
        assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo), hb
    assert np.linalg.norm(out[1][0] - out[0][0]) <= 1e-12 * np.linalg.norm(out[0][0])
    if conv:
        assert conv[1][1]["converged"] and conv[1][1]["iterations"] == conv[0][1]["iterations"]
        assert np.linalg.norm(conv[1][0] - conv[0][0]) <= 1e-10 * np.linalg.norm(conv[0][0])


@pytest.mark.parametrize("shape,p,kinds", [((4, 4, 8), 4, 7), ((3, 5, 6), 4, 5), ((5, 3, 7), 3, 7), ((2, 3, 3), 4, 3),
                                           ((4, 2, 9), 3, 5)])
def test_ho_block_z4_parity(gpu_ctx, shape, p, kinds):
    """ho_block_z 4: the high-order brick CG on 2 x 2 x 4-element blocks (16 element tiles per block, an
    S x S x (4p + 1) patch; k_cg_update_faces with the patch's z side).  Boxes with partial blocks in z
    (6, 7, 3, 9 element layers) and in x / y, non-zero essential values: 40 fixed Jacobi-CG iterates
    against the oracle (1e-11) and against the 2^3 blocks (1e-12), bitwise repeatable; on the SPD operator
    a converging solve stops on the 2^3 blocks' iteration."""
    om = O.BoxMesh(3, shape, p)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3, kinds=_kinds_o(kinds))
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    rng = np.random.default_rng(41)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    xo, _ = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=40)
    out, conv = {}, {}
    try:
        for bz in (4, 2):
            gpu_ctx.set_option("ho_block_z", bz)
            gpu_ctx.upload_mesh(gm).set_structured(*shape)
            gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            assert gpu_ctx.kernel_name(cdfem.K_APPLY) == "k_hobrick_cg"
            _, B = gpu_ctx.form_linear_system(u, b)
            out[bz] = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=40, check_every=7)
            if bz == 4:
                again = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=40)
                np.testing.assert_array_equal(again[0], out[bz][0])
            if kinds == 5:
                conv[bz] = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=1e-10, max_iter=2000, check_every=9)
    finally:
        gpu_ctx.set_option("ho_block_z", 2)
    for bz, (xg, ig) in out.items():
        assert ig["iterations"] == 40
        assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo), bz
    assert np.linalg.norm(out[4][0] - out[2][0]) <= 1e-12 * np.linalg.norm(out[2][0])
    if conv:
        assert conv[4][1]["converged"] and conv[4][1]["iterations"] == conv[2][1]["iterations"]
        assert np.linalg.norm(conv[4][0] - conv[2][0]) <= 1e-10 * np.linalg.norm(conv[2][0])
    with pytest.raises(cdfem.CdfemError):
        gpu_ctx.set_option("ho_block_z", 3)


def test_ho_brick_c3_full_size_residual(gpu_ctx):
    """C3 itself (128^3 p = 4, 135 M DoFs) through the block CG: 20 Jacobi-CG iterations on the full
    operator, then the recomputed constrained residual equals the recursive one and the iterates
    equal the tile path's (the E->L sums differ in order only: 1e-12)."""
    n, p = 128, 4
    gm = cdfem.box_mesh(3, n, p, with_coords=False)
    b = np.random.default_rng(20261015).uniform(-1, 1, gm.nl)
    out, rec = {}, {}
    try:
        for hb in (1, 0):
            gpu_ctx.set_option("ho_brick", hb)
            gpu_ctx.upload_mesh(gm).set_structured(n, n, n)
            gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            _, B = gpu_ctx.form_linear_system(np.zeros(gm.nl), b)
            out[hb] = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=20)
            # the true constrained residual r = B - A_c x in the solver's norm sqrt(r . M^-1 r)
            dg = gpu_ctx.diagonal()
            ess = np.zeros(gm.nl, dtype=bool)
            ess[gm.ess] = True
            r = B - gpu_ctx.mult(out[hb][0], constrained=True)
            rec[hb] = np.sqrt(np.dot(r, np.where(ess, r, r / np.where(ess, 1.0, dg))))
            del dg, r, ess
    finally:
        gpu_ctx.set_option("ho_brick", 1)
    assert out[1][1]["iterations"] == out[0][1]["iterations"] == 20
    for hb in (1, 0):  # the recursive residual of the CG recursion equals the recomputed one
        assert abs(rec[hb] - out[hb][1]["final_norm"]) <= 1e-9 * out[hb][1]["initial_norm"], hb
    assert np.linalg.norm(out[1][0] - out[0][0]) <= 1e-12 * np.linalg.norm(out[0][0])
    assert abs(out[1][1]["final_norm"] - out[0][1]["final_norm"]) <= 1e-10 * out[0][1]["initial_norm"]


@pytest.mark.parametrize("shape,p", [((4, 4, 4), 4), ((3, 5, 4), 3), ((5, 3, 3), 4)])
def test_ho_brick_mfma_parity(gpu_ctx, shape, p):
    """ho_brick_mfma: the block CG's x stage as block GEMMs on v_mfma_f64_16x16x4_f64 (the north star's
    MFMA contraction), the full operator (kinds 7) with non-zero essential values: 40 fixed Jacobi-CG
    iterates against the oracle (1e-11) and against the VALU x stage (1e-12), bitwise repeatable."""
    om = O.BoxMesh(3, shape, p)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3, kinds=_kinds_o(7))
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    rng = np.random.default_rng(29)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    xo, _ = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=40)
    out = {}
    try:
        gpu_ctx.set_option("ho_brick", 1)
        for mf in (1, 0):
            gpu_ctx.set_option("ho_brick_mfma", mf)
            gpu_ctx.upload_mesh(gm).set_structured(*shape)
            gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            _, B = gpu_ctx.form_linear_system(u, b)
            out[mf] = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=40)
            if mf:
                again = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=40)
                np.testing.assert_array_equal(again[0], out[mf][0])
    finally:
        gpu_ctx.set_option("ho_brick_mfma", 0)
        gpu_ctx.set_option("ho_brick", 1)
    for mf, (xg, ig) in out.items():
        assert ig["iterations"] == 40
        assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo), mf
    assert np.linalg.norm(out[1][0] - out[0][0]) <= 1e-12 * np.linalg.norm(out[0][0])
