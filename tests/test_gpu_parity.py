"""GPU parity: the HIP path (through the C-ABI, libcdfem.so) against the CPU oracle.

Parity ladder, tolerances are for f64 arithmetic in a different summation order
(sum-factorized PA on the GPU vs assembled CSR on the CPU):
  1. Mult (constrained / unconstrained), diagonal, linear form: max|y_gpu - y_cpu| <= 1e-13 max|y_cpu|
  2. CG iterates after a fixed 50 iterations from x0 = 0: relative L2 <= 1e-11
  3. converged solutions (rel_tol 1e-13): relative L2 <= 1e-10   (north-star tolerance)
  4. MMS L2 error of the GPU solution equals the oracle's to 1e-6 relative
At the full BASELINE size (64^3, p = 2) the oracle CSR is too large for a seconds-long check, so
size-independent properties are used there: linearity, annihilation of constants, mass = volume,
symmetry of the SPD part, bitwise run-to-run reproducibility.
"""
import numpy as np
import pytest

import cdfem
from oracle import oracle as O

pytestmark = pytest.mark.gpu

MULT_TOL = 1e-13
C3 = (1.0, -2.0, 0.5)


def _mesh_pair(dim, n, p, perturb=0.0):
    om = O.BoxMesh(dim, n, p, perturb=perturb)
    gm = cdfem.Mesh(dim, p, om.verts, om.dofmap, om.nl, om.ess)
    return om, gm


def _ctx(gpu_ctx, gm, kinds, kappa=0.1, alpha=1.0, c=C3, s=1.0):
    gpu_ctx.upload_mesh(gm)
    gpu_ctx.pa_setup(kinds=kinds, kappa=kappa, alpha=alpha, conv=c[: gm.dim], mass=s)
    return gpu_ctx


def _kinds_to_oracle(k):
    return (O.DIFFUSION if k & 1 else 0) | (O.CONVECTION if k & 2 else 0) | (O.MASS if k & 4 else 0)


def _relmax(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


CASES = [(3, 3, 2, 0.0), (3, 3, 2, 0.25), (3, 5, 2, 0.1), (3, 4, 1, 0.2), (2, 9, 1, 0.0),
         (2, 5, 2, 0.2), (2, 4, 3, 0.15), (2, 3, 4, 0.1)]


@pytest.mark.parametrize("dim,n,p,pert", CASES)
@pytest.mark.parametrize("kinds", [7, 5, 1, 2, 4, 3])
def test_mult_parity(gpu_ctx, dim, n, p, pert, kinds):
    om, gm = _mesh_pair(dim, n, p, pert)
    c = C3[:dim]
    ctx = _ctx(gpu_ctx, gm, kinds, c=c)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=c, kinds=_kinds_to_oracle(kinds))
    x = np.random.default_rng(11).uniform(-1, 1, om.nl)
    y = ctx.mult(x)
    yo = A.mult(x)
    assert _relmax(y, yo) <= MULT_TOL
    # constrained operator: input ess zeroed, output ess = input
    xz = x.copy()
    xz[om.ess] = 0.0
    yco = A.mult(xz)
    yco[om.ess] = x[om.ess]
    assert _relmax(ctx.mult(x, constrained=True), yco) <= MULT_TOL


def test_mult_golden_vectors(gpu_ctx):
    """The committed oracle vectors (tests/golden/oracle_vectors.npz) on the GPU."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "oracle_vectors.npz"))
    for name, dim, p in (("h3p2", 3, 2), ("h3p2_pert", 3, 2), ("h3p1", 3, 1), ("q2p1", 2, 1),
                         ("q2p3_pert", 2, 3)):
        verts, dofmap = g[f"{name}_verts"], g[f"{name}_dofmap"]
        nl = int(dofmap.max()) + 1
        gm = cdfem.Mesh(dim, p, verts, dofmap, nl, np.zeros(0, dtype=np.int32))
        ctx = _ctx(gpu_ctx, gm, 7, c=C3[:dim])
        assert _relmax(ctx.mult(g[f"{name}_x"]), g[f"{name}_y"]) <= MULT_TOL
        assert _relmax(ctx.diagonal(), g[f"{name}_diag"]) <= MULT_TOL


@pytest.mark.parametrize("dim,n,p,pert", CASES[:6])
def test_diagonal_parity(gpu_ctx, dim, n, p, pert):
    om, gm = _mesh_pair(dim, n, p, pert)
    ctx = _ctx(gpu_ctx, gm, 7, c=C3[:dim])
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3[:dim])
    assert _relmax(ctx.diagonal(), A.diag()) <= MULT_TOL


def _mms_f_numpy(xyz, dim, kappa=0.1, s=1.0, c=C3, modes=(3, 3, 3)):
    k = np.pi * np.array(modes[:dim], dtype=float)
    sv, cv = np.sin(k * xyz), np.cos(k * xyz)
    u = np.prod(sv, axis=-1)
    conv = 0.0
    for d in range(dim):
        t = c[d] * k[d] * cv[..., d]
        for e in range(dim):
            if e != d:
                t = t * sv[..., e]
        conv = conv + t
    return kappa * np.sum(k * k) * u + conv + s * u


@pytest.mark.parametrize("dim,n,p,pert", [(3, 3, 2, 0.2), (2, 5, 1, 0.0), (2, 4, 3, 0.1)])
def test_linear_form_parity(gpu_ctx, dim, n, p, pert):
    om, gm = _mesh_pair(dim, n, p, pert)
    ctx = _ctx(gpu_ctx, gm, 7, c=C3[:dim])
    xq = ctx.quadrature_points(cdfem.RULE_LINEARFORM)
    fq = _mms_f_numpy(xq, dim, c=C3[:dim])
    b = ctx.lf_assemble(fq.reshape(-1))
    prm = O.mms_params(O.MMS_SIN, dim, kappa=0.1, s=1.0, c=C3[:dim], p=p)
    assert _relmax(b, O.lf_assemble(om, prm)) <= 1e-12


@pytest.mark.parametrize("dim,n,p", [(3, 4, 2), (2, 6, 2)])
def test_form_linear_system_parity(gpu_ctx, dim, n, p):
    om, gm = _mesh_pair(dim, n, p, 0.1)
    ctx = _ctx(gpu_ctx, gm, 7, c=C3[:dim])
    rng = np.random.default_rng(5)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    X, B = ctx.form_linear_system(u, b)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3[:dim])
    _, Bo = O.form_linear_system(A, om.bdr, u, b)
    np.testing.assert_array_equal(X, u)
    assert _relmax(B, Bo) <= MULT_TOL


def _spd_system(gpu_ctx, n=6, p=2, pert=0.15, seed=9):
    om, gm = _mesh_pair(3, n, p, pert)
    ctx = _ctx(gpu_ctx, gm, 5)                      # kappa K + s M (c = 0): SPD
    A = O.fa_assemble(om, kappa=0.1, s=1.0, kinds=O.DIFFUSION | O.MASS)
    rng = np.random.default_rng(seed)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    _, B = ctx.form_linear_system(u, b)
    return om, ctx, Ac, Bo, B


def test_cg_fixed_iterates_parity(gpu_ctx):
    om, ctx, Ac, Bo, B = _spd_system(gpu_ctx)
    dinv = 1.0 / Ac.diag()
    xo, io = O.cg(Ac, Bo, dinv=dinv, rel_tol=0.0, abs_tol=0.0, max_iter=50)
    xg, ig = ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=50, check_every=7)
    assert io["iterations"] == ig["iterations"] == 50
    assert not ig["converged"]
    assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)
    assert abs(ig["final_norm"] - io["final_norm"]) <= 1e-9 * io["final_norm"]


def test_cg_converged_parity_and_reproducible(gpu_ctx):
    om, ctx, Ac, Bo, B = _spd_system(gpu_ctx, n=8)
    dinv = 1.0 / Ac.diag()
    xo, io = O.cg(Ac, Bo, dinv=dinv, rel_tol=1e-13, max_iter=2000)
    xg, ig = ctx.solve(B, method="cg", rel_tol=1e-13, max_iter=2000)
    assert io["converged"] and ig["converged"]
    assert abs(ig["iterations"] - io["iterations"]) <= 2
    assert np.linalg.norm(xg - xo) <= 1e-10 * np.linalg.norm(xo)
    xg2, ig2 = ctx.solve(B, method="cg", rel_tol=1e-13, max_iter=2000)
    np.testing.assert_array_equal(xg, xg2)          # deterministic reductions, no atomics
    assert ig2["iterations"] == ig["iterations"]


def test_cg_unpreconditioned_and_early_exit(gpu_ctx):
    om, ctx, Ac, Bo, B = _spd_system(gpu_ctx, n=4)
    xo, io = O.cg(Ac, Bo, dinv=None, rel_tol=1e-12, max_iter=500)
    xg, ig = ctx.solve(B, method="cg", pc="none", rel_tol=1e-12, max_iter=500, check_every=3)
    assert io["converged"] and ig["converged"] and abs(io["iterations"] - ig["iterations"]) <= 1
    assert np.linalg.norm(xg - xo) <= 1e-10 * np.linalg.norm(xo)
    # zero right-hand side: converged at iteration 0 (nom = 0 <= r0)
    x0, i0 = ctx.solve(np.zeros(om.nl), method="cg", rel_tol=1e-12, max_iter=10)
    assert i0["converged"] and i0["iterations"] == 0 and not x0.any()


def test_cg_max_iter_reports_not_converged(gpu_ctx):
    om, ctx, Ac, Bo, B = _spd_system(gpu_ctx, n=6)
    with pytest.raises(cdfem.CdfemError) as ei:
        ctx.solve(B, method="cg", rel_tol=1e-14, max_iter=3, raise_on_fail=True)
    assert ei.value.code == cdfem.ERR_NOT_CONVERGED


def test_all_essential_single_element(gpu_ctx):
    """p=1 single hex: every dof is on the boundary -> X = boundary values after 1 iteration."""
    om, gm = _mesh_pair(3, 1, 1)
    ctx = _ctx(gpu_ctx, gm, 5)
    u = np.arange(1.0, om.nl + 1.0)
    X, B = ctx.form_linear_system(u, np.zeros(om.nl))
    np.testing.assert_array_equal(B, u)
    xs, info = ctx.solve(B, method="cg", rel_tol=1e-14, max_iter=10)
    assert info["converged"] and info["iterations"] <= 1
    np.testing.assert_allclose(xs, u, rtol=0, atol=1e-14 * u.max())


def test_mms_solution_error_matches_oracle(gpu_ctx):
    """diffusion-reaction MMS (c = 0, SPD, CG): the GPU solution's L2 error equals the oracle's."""
    dim, n, p = 3, 8, 2
    om, gm = _mesh_pair(dim, n, p)
    ctx = _ctx(gpu_ctx, gm, 5)
    xq = ctx.quadrature_points(cdfem.RULE_LINEARFORM)
    fq = _mms_f_numpy(xq, dim, c=(0.0, 0.0, 0.0))
    b = ctx.lf_assemble(fq.reshape(-1))
    prm = O.mms_params(O.MMS_SIN, dim, kappa=0.1, s=1.0, c=(0.0, 0.0, 0.0), p=p)
    u = np.zeros(om.nl)
    u[om.ess] = O.mms_u(prm, om.dof_coords()[om.ess])
    _, B = ctx.form_linear_system(u, b)
    xg, ig = ctx.solve(B, method="cg", rel_tol=1e-12, max_iter=2000)
    assert ig["converged"]
    eg = O.l2_error(om, xg, prm)
    A = O.fa_assemble(om, kappa=0.1, s=1.0, kinds=O.DIFFUSION | O.MASS)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, O.lf_assemble(om, prm))
    xo, io = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=1e-12, max_iter=2000)
    eo = O.l2_error(om, xo, prm)
    assert abs(eg - eo) <= 1e-6 * eo
    assert eo < 1e-2                     # 8^3 p=2: O(h^3) error of sin(3 pi x)...


def test_variable_coefficients(gpu_ctx):
    """kappa(x), s(x), c(x) sampled at quadrature points (host Coefficient::Eval) vs constant ones:
    a constant field passed per point equals the constant path bitwise."""
    om, gm = _mesh_pair(3, 3, 2, 0.1)
    ctx = gpu_ctx.upload_mesh(gm)
    nq = ctx.rule_size(cdfem.RULE_OPERATOR)
    x = np.random.default_rng(2).uniform(-1, 1, om.nl)
    ctx.pa_setup(kinds=7, kappa=0.3, alpha=1.0, conv=C3, mass=2.0)
    y_const = ctx.mult(x)
    ctx.pa_setup(kinds=7, kappa=0.0, alpha=1.0, conv=(0, 0, 0), mass=0.0,
                 kappa_q=np.full(om.ne * nq, 0.3), conv_q=np.tile(C3, om.ne * nq),
                 mass_q=np.full(om.ne * nq, 2.0))
    np.testing.assert_array_equal(ctx.mult(x), y_const)


# ---------------------------------------------------------------------------------------------
# BASELINE full size (64^3, p = 2): size-independent properties
# ---------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def full_size(gpu_ctx):
    gm = cdfem.box_mesh(3, 64, 2, with_coords=False)
    gpu_ctx.upload_mesh(gm)
    return gm


def test_full_size_properties(gpu_ctx, full_size):
    gm = full_size
    rng = np.random.default_rng(20261015)
    x, y = rng.uniform(-1, 1, gm.nl), rng.uniform(-1, 1, gm.nl)
    one = np.ones(gm.nl)
    # mass: 1^T M 1 = |Omega|
    gpu_ctx.pa_setup(kinds=cdfem.MASS, mass=1.0)
    assert abs(one @ gpu_ctx.mult(one) - 1.0) < 1e-12
    # diffusion + convection annihilate constants
    gpu_ctx.pa_setup(kinds=cdfem.DIFFUSION | cdfem.CONVECTION, kappa=0.1, conv=C3)
    assert np.abs(gpu_ctx.mult(one)).max() < 1e-11
    # SPD part symmetric, full operator linear
    gpu_ctx.pa_setup(kinds=5, kappa=0.1, mass=1.0)
    assert abs(x @ gpu_ctx.mult(y) - y @ gpu_ctx.mult(x)) <= 1e-12 * abs(x @ gpu_ctx.mult(y)) + 1e-12
    gpu_ctx.pa_setup(kinds=7, kappa=0.1, conv=C3, mass=1.0)
    a, b = 0.75, -1.25
    lhs = gpu_ctx.mult(a * x + b * y)
    rhs = a * gpu_ctx.mult(x) + b * gpu_ctx.mult(y)
    assert _relmax(lhs, rhs) <= 1e-13
    np.testing.assert_array_equal(gpu_ctx.mult(x), gpu_ctx.mult(x))


def test_full_size_cg_residual(gpu_ctx, full_size):
    """100 CG iterations at BASELINE size: the recomputed residual matches the recursive one."""
    gm = full_size
    gpu_ctx.pa_setup(kinds=5, kappa=0.1, mass=1.0)
    rng = np.random.default_rng(4)
    u = np.zeros(gm.nl)
    u[gm.ess] = rng.uniform(-1, 1, len(gm.ess))
    _, B = gpu_ctx.form_linear_system(u, rng.uniform(-1, 1, gm.nl))
    X, info = gpu_ctx.solve(B, method="cg", rel_tol=1e-8, max_iter=400)
    assert info["converged"]
    r = B - gpu_ctx.mult(X, constrained=True)
    d = gpu_ctx.diagonal()
    d[gm.ess] = 1.0
    rz = r @ (r / d)
    assert np.sqrt(rz) <= 2e-8 * info["initial_norm"]


# ---------------------------------------------------------------------------------------------
# structured brick fast path (cdfem_mesh_set_structured): same parity bar as the generic path
# ---------------------------------------------------------------------------------------------
def _brick_pair(n, p, perturb, kinds):
    om = O.BoxMesh(3, n, p, perturb=perturb)
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    return om, gm


@pytest.mark.parametrize("n,p,pert", [(4, 2, 0.0), (5, 2, 0.2), (3, 2, 0.1), (8, 2, 0.15), (6, 1, 0.2),
                                      (9, 1, 0.0)])
@pytest.mark.parametrize("kinds", [7, 5, 3])
def test_brick_mult_parity(gpu_ctx, n, p, pert, kinds):
    om, gm = _brick_pair(n, p, pert, kinds)
    gpu_ctx.upload_mesh(gm).set_structured(n, n, n)
    gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3, kinds=_kinds_to_oracle(kinds))
    x = np.random.default_rng(13).uniform(-1, 1, om.nl)
    assert _relmax(gpu_ctx.mult(x), A.mult(x)) <= MULT_TOL
    xz = x.copy()
    xz[om.ess] = 0.0
    yco = A.mult(xz)
    yco[om.ess] = x[om.ess]
    assert _relmax(gpu_ctx.mult(x, constrained=True), yco) <= MULT_TOL
    assert _relmax(gpu_ctx.diagonal(), A.diag()) <= MULT_TOL


def test_brick_anisotropic_box(gpu_ctx):
    """nx != ny != nz, none a multiple of the brick size."""
    nx, ny, nz, p = 6, 5, 7, 2
    om = O.BoxMesh(3, (nx, ny, nz), p, perturb=0.1)
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    gpu_ctx.upload_mesh(gm).set_structured(nx, ny, nz)
    gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3)
    x = np.random.default_rng(17).uniform(-1, 1, om.nl)
    assert _relmax(gpu_ctx.mult(x), A.mult(x)) <= MULT_TOL


def test_brick_rejects_non_lexicographic(gpu_ctx):
    om = O.BoxMesh(3, 4, 2)
    dm = om.dofmap.copy()
    dm[[0, 1]] = dm[[1, 0]]                           # swap two elements
    gm = cdfem.Mesh(3, 2, om.verts, dm, om.nl, om.ess)
    gpu_ctx.upload_mesh(gm)
    with pytest.raises(cdfem.CdfemError) as ei:
        gpu_ctx.set_structured(4, 4, 4)
    assert ei.value.code == cdfem.ERR_ARG


def test_brick_cg_parity(gpu_ctx):
    n, p = 8, 2
    om = O.BoxMesh(3, n, p, perturb=0.15)
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    gpu_ctx.upload_mesh(gm).set_structured(n, n, n)
    gpu_ctx.pa_setup(kinds=5, kappa=0.1, mass=1.0)
    A = O.fa_assemble(om, kappa=0.1, s=1.0, kinds=O.DIFFUSION | O.MASS)
    rng = np.random.default_rng(9)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    _, B = gpu_ctx.form_linear_system(u, b)
    assert _relmax(B, Bo) <= MULT_TOL
    dinv = 1.0 / Ac.diag()
    xo, io = O.cg(Ac, Bo, dinv=dinv, rel_tol=0.0, abs_tol=0.0, max_iter=50)
    xg, ig = gpu_ctx.solve(B, method="cg", rel_tol=0.0, abs_tol=0.0, max_iter=50, check_every=9)
    assert ig["iterations"] == 50
    assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)
    xo, io = O.cg(Ac, Bo, dinv=dinv, rel_tol=1e-13, max_iter=2000)
    xg, ig = gpu_ctx.solve(B, method="cg", rel_tol=1e-13, max_iter=2000)
    assert ig["converged"] and abs(ig["iterations"] - io["iterations"]) <= 2
    assert np.linalg.norm(xg - xo) <= 1e-10 * np.linalg.norm(xo)
    xg2, _ = gpu_ctx.solve(B, method="cg", rel_tol=1e-13, max_iter=2000)
    np.testing.assert_array_equal(xg, xg2)
    xn, inn = gpu_ctx.solve(B, method="cg", pc="none", rel_tol=1e-12, max_iter=2000)
    xon, ion = O.cg(Ac, Bo, dinv=None, rel_tol=1e-12, max_iter=2000)
    assert inn["converged"] and np.linalg.norm(xn - xon) <= 1e-10 * np.linalg.norm(xon)


@pytest.mark.parametrize("n,p", [(8, 2), (9, 1)])
def test_brick_cg_bench_operator_parity(gpu_ctx, n, p):
    """The bench's operator (D+C+M, kinds=7, c = (1, -2, 0.5)) through the fused brick CG: fixed
    Jacobi-CG iterates (tolerance 0, as bench.py times them) against the oracle's MFEM CGSolver
    restatement on the same eliminated matrix, and bitwise repeatable."""
    om = O.BoxMesh(3, n, p, perturb=0.1)
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    gpu_ctx.upload_mesh(gm).set_structured(n, n, n)
    gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3)
    b = np.random.default_rng(20261015).uniform(-1, 1, om.nl)
    u = np.zeros(om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    _, B = gpu_ctx.form_linear_system(u, b)
    assert _relmax(B, Bo) <= MULT_TOL
    xo, _ = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=30)
    xg, ig = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=30)
    assert ig["iterations"] == 30
    assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)
    xg2, _ = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=30)
    np.testing.assert_array_equal(xg, xg2)


@pytest.mark.parametrize("n,p,kinds", [(8, 2, 7), (6, 2, 3), (9, 1, 7), (5, 2, 4)])
def test_brick_affine_factors(gpu_ctx, n, p, kinds):
    """Affine box (pa_affine, default): the brick kernels form each point's data as W_q * g_e from
    one factor set per element instead of streaming the per-point qdata.  Against the oracle at the
    generic bar, against the per-point form (pa_affine 0) to rounding, and the byte count shows the
    factor form is in use (a perturbed mesh keeps the per-point stream)."""
    om = O.BoxMesh(3, n, p)
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3, kinds=_kinds_to_oracle(kinds))
    x = np.random.default_rng(31).uniform(-1, 1, om.nl)
    b = np.random.default_rng(32).uniform(-1, 1, om.nl)
    u = np.zeros(om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    xo, _ = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=30)
    out = {}
    try:
        for aff in (1, 0):
            gpu_ctx.set_option("pa_affine", aff)
            gpu_ctx.upload_mesh(gm).set_structured(n, n, n)
            gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            out[aff] = dict(y=gpu_ctx.mult(x), yc=gpu_ctx.mult(x, constrained=True), dg=gpu_ctx.diagonal(),
                            bytes=gpu_ctx.kernel_bytes(cdfem.K_APPLY))
            _, B = gpu_ctx.form_linear_system(u, b)
            out[aff]["x"], info = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0,
                                                max_iter=30)
            assert info["iterations"] == 30
    finally:
        gpu_ctx.set_option("pa_affine", 2)
    assert out[1]["bytes"] < out[0]["bytes"]
    assert _relmax(out[1]["y"], A.mult(x)) <= MULT_TOL
    assert _relmax(out[1]["dg"], A.diag()) <= MULT_TOL
    assert np.linalg.norm(out[1]["x"] - xo) <= 1e-11 * np.linalg.norm(xo)
    for k in ("y", "yc", "dg"):
        assert _relmax(out[1][k], out[0][k]) <= 1e-13
    assert np.linalg.norm(out[1]["x"] - out[0]["x"]) <= 1e-12 * np.linalg.norm(out[0]["x"])
    # a perturbed mesh is not affine: the per-point stream stays
    om2 = O.BoxMesh(3, n, p, perturb=0.1)
    gpu_ctx.upload_mesh(cdfem.Mesh(3, p, om2.verts, om2.dofmap, om2.nl, om2.ess)).set_structured(n, n, n)
    gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    assert gpu_ctx.kernel_bytes(cdfem.K_APPLY) == out[0]["bytes"]


def test_brick_full_size_matches_generic(gpu_ctx):
    """64^3 p=2: brick and generic paths agree (different E->L summation order only)."""
    gm = cdfem.box_mesh(3, 64, 2, with_coords=False)
    x = np.random.default_rng(21).uniform(-1, 1, gm.nl)
    gpu_ctx.upload_mesh(gm)
    gpu_ctx.pa_setup(kinds=7, kappa=0.1, conv=C3, mass=1.0)
    y_gen = gpu_ctx.mult(x, constrained=True)
    gpu_ctx.set_structured(64, 64, 64)
    gpu_ctx.pa_setup(kinds=7, kappa=0.1, conv=C3, mass=1.0)
    y_brk = gpu_ctx.mult(x, constrained=True)
    assert _relmax(y_brk, y_gen) <= 1e-14


def test_config_c1_reference_case(gpu_ctx):
    """BASELINE configs[0]: the reference's CPU-runnable case, 2D 64 x 64 quads, H1 order 1, the
    driver's MMS (linear_convection_diffusion_2D.cpp:159-215, Input/input_2d.yaml: kappa 0.1,
    s 1, c (1, -2), modes 3, 3).  The reference solves it with full assembly on the CPU; here the
    same system goes through the GPU path.  The SPD part (c = 0) under CG and the full operator
    under GMRES(30) + Jacobi (Input/petsc.opts) against the oracle's FA restatement: the same
    iteration counts (+-1), solutions to the stopping-tolerance bound and equal L2 errors."""
    n, p = 64, 1
    om, gm = _mesh_pair(2, n, p)
    for c, solver in (((0.0, 0.0), "cg"), ((1.0, -2.0), "gmres")):
        kinds = 5 if solver == "cg" else 7
        ctx = _ctx(gpu_ctx, gm, kinds, c=c)
        xq = ctx.quadrature_points(cdfem.RULE_LINEARFORM)
        b = ctx.lf_assemble(_mms_f_numpy(xq, 2, c=c).reshape(-1))
        prm = O.mms_params(O.MMS_SIN, 2, kappa=0.1, s=1.0, c=c, p=p)
        u = np.zeros(om.nl)
        u[om.ess] = O.mms_u(prm, om.dof_coords()[om.ess])
        _, B = ctx.form_linear_system(u, b)
        A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=c, kinds=_kinds_to_oracle(kinds))
        Ac, Bo = O.form_linear_system(A, om.bdr, u, O.lf_assemble(om, prm))
        assert np.abs(B - Bo).max() <= 1e-13 * np.abs(Bo).max()
        if solver == "cg":
            xg, ig = ctx.solve(B, method="cg", rel_tol=1e-12, max_iter=2000)
            xo, io = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=1e-12, max_iter=2000)
            tol = 1e-10
        else:
            xg, ig = ctx.solve(B, method="gmres", restart=30, rel_tol=1e-10, abs_tol=1e-12, max_iter=2000)
            xo, io = O.gmres(Ac, Bo, dinv=1.0 / Ac.diag(), restart=30, rtol=1e-10, atol=1e-12, max_it=2000)
            tol = 1e-8
        assert ig["converged"] and io["converged"] and abs(ig["iterations"] - io["iterations"]) <= 1
        assert np.linalg.norm(xg - xo) <= tol * np.linalg.norm(xo)
        eg, eo = O.l2_error(om, xg, prm), O.l2_error(om, xo, prm)
        assert abs(eg - eo) <= 1e-6 * eo and eo < 1e-2


@pytest.mark.parametrize("shape,kinds", [((8, 8, 8), 7), ((8, 8, 8), 5), ((9, 6, 7), 7), ((4, 4, 12), 1)])
def test_brick_cg_partial_bricks_parity(gpu_ctx, shape, kinds):
    """The brick CG kernel on cubes and on boxes with partial bricks, for several kinds masks: fixed
    Jacobi-CG iterates with essential values against the oracle (1e-11); bitwise repeatable."""
    nx, ny, nz = shape
    p = 2
    om = O.BoxMesh(3, shape, p, perturb=0.1)
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    gpu_ctx.upload_mesh(gm).set_structured(nx, ny, nz)
    gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    ko = (O.DIFFUSION if kinds & 1 else 0) | (O.CONVECTION if kinds & 2 else 0) | (O.MASS if kinds & 4 else 0)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3, kinds=ko)
    rng = np.random.default_rng(33)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    _, B = gpu_ctx.form_linear_system(u, b)
    xo, _ = O.cg(Ac, Bo, dinv=1.0 / Ac.diag(), rel_tol=0.0, abs_tol=0.0, max_iter=40)
    xg, ig = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=40, check_every=11)
    x2, _ = gpu_ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=40, check_every=11)
    assert ig["iterations"] == 40
    assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)
    np.testing.assert_array_equal(x2, xg)


@pytest.mark.parametrize("n,p,kinds", [(5, 2, 7), (4, 1, 5), (3, 2, 6)])
def test_generic_affine_factors(gpu_ctx, n, p, kinds):
    """The generic 3D element-block apply (no structured declaration) on affine factors: Mult,
    constrained Mult and fixed GMRES iterates against the oracle and against the per-point stream."""
    om = O.BoxMesh(3, n, p)
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=C3, kinds=_kinds_to_oracle(kinds))
    x = np.random.default_rng(51).uniform(-1, 1, om.nl)
    out = {}
    try:
        for aff in (1, 0):
            gpu_ctx.set_option("pa_affine", aff)
            gpu_ctx.upload_mesh(gm)
            gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            _, B = gpu_ctx.form_linear_system(np.zeros(om.nl), x)
            xg, _ = gpu_ctx.solve(B, method="gmres", restart=30, rel_tol=0.0, abs_tol=0.0, max_iter=40)
            out[aff] = dict(y=gpu_ctx.mult(x), yc=gpu_ctx.mult(x, constrained=True), x=xg,
                            bytes=gpu_ctx.kernel_bytes(cdfem.K_APPLY))
    finally:
        gpu_ctx.set_option("pa_affine", 2)
    assert out[1]["bytes"] < out[0]["bytes"]
    assert _relmax(out[1]["y"], A.mult(x)) <= MULT_TOL
    for k in ("y", "yc"):
        assert _relmax(out[1][k], out[0][k]) <= 1e-13
    assert np.linalg.norm(out[1]["x"] - out[0]["x"]) <= 1e-11 * np.linalg.norm(out[0]["x"])
