"""Pin the CPU oracle before trusting it (CPU only).

The reference holds no golden vectors for this path, so the oracle is pinned
against (a) closed-form known answers (tests/golden/analytic.json: Gauss rules, GLL nodes, exact
Q1/Q2 element matrices), (b) the reference's own verification method — manufactured solutions
(linear_convection_diffusion_2D.cpp:159-215, diffusion_mms.cpp:136-178) — turned into asserted
known answers: exact reproduction of FE-space polynomials, O(h^{p+1}) L2 rates, and (c) algebraic
identities of the three integrators.  Oracle regression vectors (oracle_vectors.npz) catch drift.
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def analytic():
    with open(os.path.join(GOLDEN, "analytic.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("n", [2, 3, 4])
def test_gauss_legendre_closed_form(analytic, n):
    x, w = O.gauss_legendre(n)
    ref = analytic["gauss_legendre"][str(n)]
    np.testing.assert_allclose(x, ref["x"], rtol=0, atol=1e-15)
    np.testing.assert_allclose(w, ref["w"], rtol=0, atol=1e-15)


@pytest.mark.parametrize("p", [1, 2, 4])
def test_gll_closed_form(analytic, p):
    np.testing.assert_allclose(O.gll_nodes(p), analytic["gll"][str(p)], rtol=0, atol=1e-15)


def test_rule_sizes_coincide():
    # Diffusion/Convection/Mass share n: p=1 quad 2, p=2 hex 4, p=4 hex 6
    for dim, p, n in ((2, 1, 2), (3, 2, 4), (3, 4, 6), (3, 1, 3), (2, 3, 4)):
        assert [O.rule_npts(k, dim, p) for k in range(3)] == [n, n, n]
    assert O.rule_npts(O.RULE_LF, 3, 2) == 3          # DomainLF order 2p
    assert O.rule_npts(O.RULE_L2, 2, 1) == 3          # driver's max(2, 2p+3)


@pytest.mark.parametrize("dim,p", [(2, 1), (3, 1), (2, 2), (3, 2)])
def test_element_matrices_exact(analytic, dim, p):
    """One unit element: FA matrices equal the exact rational ones (affine => rules exact)."""
    ref = analytic["elements"][f"dim{dim}_p{p}"]
    m = O.BoxMesh(dim, 1, p)
    c = ref["c"]
    for kinds, key, kw in ((O.MASS, "mass", dict(s=1.0)), (O.DIFFUSION, "stiffness", dict(kappa=1.0)),
                           (O.CONVECTION, "convection", dict(c=c, alpha=1.0))):
        A = O.fa_assemble(m, kinds=kinds, **kw).to_scipy().toarray()
        # single element: L-dof order == lexicographic local order
        R = np.array(ref[key])
        np.testing.assert_allclose(A, R, rtol=0, atol=2e-15 * max(1.0, np.abs(R).max()), err_msg=key)


@pytest.mark.parametrize("dim,p,pert", [(2, 2, 0.2), (3, 2, 0.25), (3, 1, 0.3)])
def test_integrator_identities(dim, p, pert):
    m = O.BoxMesh(dim, 3, p, perturb=pert)
    one = np.ones(m.nl)
    M = O.fa_assemble(m, kinds=O.MASS, s=1.0)
    K = O.fa_assemble(m, kinds=O.DIFFUSION, kappa=1.0)
    C = O.fa_assemble(m, kinds=O.CONVECTION, c=(1.0, -2.0, 0.5)[:dim])
    assert abs(one @ M.mult(one) - 1.0) < 1e-13            # |Omega| = 1 (boundary unperturbed)
    assert np.abs(K.mult(one)).max() < 1e-13                # K 1 = 0
    assert np.abs(C.mult(one)).max() < 1e-13                # C 1 = 0 (constant c)
    Ks, Ms = K.to_scipy(), M.to_scipy()
    assert abs(Ks - Ks.T).max() < 1e-15 and abs(Ms - Ms.T).max() < 1e-15
    # linear u: K u = boundary flux only -> (v, K u) for interior v equals 0
    xyz = m.dof_coords()
    u = xyz[:, 0] + 2 * xyz[:, 1]
    r = K.mult(u)
    assert np.abs(r[m.bdr == 0]).max() < 1e-12


@pytest.mark.parametrize("dim,p", [(2, 1), (2, 2), (3, 1), (3, 2)])
def test_polynomial_solution_reproduced(dim, p):
    """u in the FE space, exact quadrature on affine elements: the Galerkin solution IS u."""
    m = O.BoxMesh(dim, 3, p)
    c = (1.0, -2.0, 0.5)[:dim]
    prm = O.mms_params(O.MMS_POLY, dim, kappa=0.1, s=1.0, c=c, p=p)
    X, info, err = O.solve_mms(m, prm, 0.1, 1.0, c, tol=1e-14, atol=0.0)
    assert info["converged"]
    assert err < 1e-12
    np.testing.assert_allclose(X, O.mms_u(prm, m.dof_coords()), rtol=0, atol=1e-12)


@pytest.mark.parametrize("dim,p,ns", [(2, 1, (8, 16, 32)), (2, 2, (8, 16, 32)), (3, 1, (4, 8, 16)),
                                      (3, 2, (4, 8, 12))])
def test_mms_convergence_rate(dim, p, ns):
    """linear_convection_diffusion_2D.cpp problem (kappa .1, s 1, c (1,-2)), L2 rate p+1."""
    c = (1.0, -2.0, 0.5)[:dim]
    errs, hs = [], []
    for n in ns:
        m = O.BoxMesh(dim, n, p)
        prm = O.mms_params(O.MMS_SIN, dim, kappa=0.1, s=1.0, c=c, p=p)
        _, info, e = O.solve_mms(m, prm, 0.1, 1.0, c)
        assert info["converged"]
        errs.append(e)
        hs.append(1.0 / n)
    rates = np.diff(np.log(errs)) / np.diff(np.log(hs))
    assert rates[-1] > p + 1 - 0.15, rates


def test_gmres_and_cg_agree_on_spd():
    m = O.BoxMesh(3, 4, 2)
    A = O.fa_assemble(m, kappa=0.1, s=1.0, kinds=O.DIFFUSION | O.MASS)
    u = np.zeros(m.nl)
    rng = np.random.default_rng(1)
    b = rng.uniform(-1, 1, m.nl)
    Ac, B = O.form_linear_system(A, m.bdr, u, b)
    dinv = 1.0 / Ac.diag()
    x1, i1 = O.cg(Ac, B, dinv=dinv, rel_tol=1e-13, max_iter=1000)
    x2, i2 = O.gmres(Ac, B, dinv=dinv, rtol=1e-13, atol=0.0, max_it=1000)
    assert i1["converged"] and i2["converged"]
    np.testing.assert_allclose(x1, x2, rtol=0, atol=1e-10 * np.abs(x1).max())
    import scipy.sparse.linalg as spla
    xs = spla.spsolve(Ac.to_scipy().tocsc(), B)
    np.testing.assert_allclose(x1, xs, rtol=0, atol=1e-10 * np.abs(xs).max())


def test_gmres_restart_semantics():
    """PETSc GMRES(m) counts inner iterations.  Unrestarted GMRES minimises the residual over the
    whole Krylov space, so it needs no more iterations than any restarted variant, and every
    variant stops on the true preconditioned residual criterion."""
    m = O.BoxMesh(2, 16, 2)
    A = O.fa_assemble(m, kappa=0.1, s=1.0, c=(1.0, -2.0))
    b = np.random.default_rng(3).uniform(-1, 1, m.nl)
    Ac, B = O.form_linear_system(A, m.bdr, np.zeros(m.nl), b)
    dinv = 1.0 / Ac.diag()
    S = Ac.to_scipy()
    r0 = np.linalg.norm(dinv * B)
    xf, inf = O.gmres(Ac, B, dinv=dinv, restart=1000, rtol=1e-12, atol=0.0, max_it=1000)
    for restart in (5, 30):
        x, info = O.gmres(Ac, B, dinv=dinv, restart=restart, rtol=1e-12, atol=0.0, max_it=5000)
        assert info["converged"]
        assert info["iterations"] >= inf["iterations"]
        assert np.linalg.norm(dinv * (B - S @ x)) <= 1.01e-12 * r0
        np.testing.assert_allclose(x, xf, rtol=0, atol=1e-9 * np.abs(xf).max())


def test_ebe_matches_csr():
    m = O.BoxMesh(3, 3, 2, perturb=0.2)
    x = np.random.default_rng(7).uniform(-1, 1, m.nl)
    A = O.fa_assemble(m, kappa=0.1, s=1.0, c=(1.0, -2.0, 0.5))
    np.testing.assert_allclose(O.ebe_mult(m, x, kappa=0.1, s=1.0, c=(1.0, -2.0, 0.5)), A.mult(x),
                               rtol=0, atol=1e-14)


def test_oracle_regression_vectors():
    g = np.load(os.path.join(GOLDEN, "oracle_vectors.npz"))
    cases = [("h3p2", 3, 3, 2, 0.0), ("h3p2_pert", 3, 3, 2, 0.25), ("h3p1", 3, 4, 1, 0.0),
             ("q2p1", 2, 8, 1, 0.0), ("q2p3_pert", 2, 4, 3, 0.2)]
    for name, dim, n, p, pert in cases:
        m = O.BoxMesh(dim, n, p, perturb=pert)
        np.testing.assert_array_equal(m.verts, g[f"{name}_verts"])
        np.testing.assert_array_equal(m.dofmap, g[f"{name}_dofmap"])
        c = (1.0, -2.0, 0.5)[:dim]
        A = O.fa_assemble(m, kappa=0.1, alpha=1.0, s=1.0, c=c)
        y = A.mult(g[f"{name}_x"])
        np.testing.assert_allclose(y, g[f"{name}_y"], rtol=0, atol=1e-14 * np.abs(y).max())
        np.testing.assert_allclose(A.diag(), g[f"{name}_diag"], rtol=0, atol=1e-15)
        prm = O.mms_params(O.MMS_SIN, dim, kappa=0.1, s=1.0, c=c, p=p)
        np.testing.assert_allclose(O.lf_assemble(m, prm), g[f"{name}_b"], rtol=0, atol=1e-15)


@pytest.mark.parametrize("shape,p,pert,kinds", [((4, 3, 5), 2, 0.2, 7), ((3, 3, 3), 3, 0.1, 7), ((4, 4, 4), 1, 0.1, 5),
                                                ((3, 4, 3), 4, 0.0, 3), ((3, 3, 3), 2, 0.1, 4)])
def test_oracle_pa_matches_fa(shape, p, pert, kinds):
    """The host partial-assembly restatement (O.PA: MFEM's per-integrator point data and sum-factorised
    element loops, the CPU PA + CG baseline of bench.py) is the FA operator: Mult and the constrained
    Mult to 1e-13 of the assembled CSR, and CGSolver on it gives the CSR solve's 30 iterates (1e-12)."""
    om = O.BoxMesh(3, shape, p, perturb=pert)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=(1.0, -2.0, 0.5), kinds=kinds)
    pa = O.PA(om, kappa=0.1, alpha=1.0, s=1.0, c=(1.0, -2.0, 0.5), kinds=kinds)
    rng = np.random.default_rng(1)
    x, b = rng.uniform(-1, 1, om.nl), rng.uniform(-1, 1, om.nl)
    yo = A.mult(x)
    assert np.abs(pa.mult(x) - yo).max() <= 1e-13 * np.abs(yo).max()
    xz = x.copy()
    xz[om.ess] = 0.0
    yc = A.mult(xz)
    yc[om.ess] = x[om.ess]
    assert np.abs(pa.mult(x, constrained=True) - yc).max() <= 1e-13 * np.abs(yc).max()
    Ac, B = O.form_linear_system(A, om.bdr, np.zeros(om.nl), b)
    dinv = 1.0 / Ac.diag()
    x1, i1 = O.cg(Ac, B, dinv=dinv, rel_tol=0.0, abs_tol=0.0, max_iter=30)
    x2, i2 = pa.cg(B, dinv=dinv, rel_tol=0.0, abs_tol=0.0, max_iter=30)
    assert i1["iterations"] == i2["iterations"] == 30
    assert np.linalg.norm(x2 - x1) <= 1e-12 * np.linalg.norm(x1)


@pytest.mark.parametrize("shape,p,pert,kinds", [((3, 4, 2), 2, 0.2, 7), ((2, 3, 2), 4, 0.15, 7), ((3, 2, 2), 3, 0.1, 5),
                                                 ((2, 2, 3), 1, 0.2, 2), ((3, 3, 3), 2, 0.0, 4)])
def test_oracle_pa_diag_and_fls_match_fa(shape, p, pert, kinds):
    """orc_pa_diag (MFEM's AssembleDiagonal at the PA level: per-integrator sum-factorised element
    diagonals, E->L sum) is the assembled CSR's diagonal, and the PA FormLinearSystem (B = b - A X_e,
    B_ess = X_ess) the CSR elimination's B, both to 1e-13 on perturbed (non-affine) meshes.  These pin
    the host PA that checks the full-size C3 / C5 runs (tests/test_gpu_full_size.py)."""
    om = O.BoxMesh(3, shape, p, perturb=pert)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=(1.0, -2.0, 0.5), kinds=kinds)
    pa = O.PA(om, kappa=0.1, alpha=1.0, s=1.0, c=(1.0, -2.0, 0.5), kinds=kinds)
    do = A.diag()
    assert np.abs(pa.diag() - do).max() <= 1e-13 * np.abs(do).max()
    rng = np.random.default_rng(2)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    _, Bo = O.form_linear_system(A, om.bdr, u, b)
    assert np.abs(pa.form_linear_system(u, b) - Bo).max() <= 1e-13 * np.abs(Bo).max()


def test_oracle_cg_indefinite_preconditioner():
    """MFEM CGSolver stops unconverged when (r, M^-1 r) < 0: at iteration 0 (nom0 < 0) or at the
    iteration where betanom turns negative (kK + sM with s = -124: 210 negative Jacobi entries)."""
    om = O.BoxMesh(3, (6, 5, 7), 2)
    A = O.fa_assemble(om, kappa=0.1, s=-124.0, kinds=O.DIFFUSION | O.MASS)
    b = np.random.default_rng(3).uniform(-1, 1, om.nl)
    Ac, B = O.form_linear_system(A, om.bdr, np.zeros(om.nl), b)
    dg = Ac.diag()
    _, info = O.cg(Ac, B, dinv=1.0 / dg, rel_tol=1e-12, max_iter=200)
    assert not info["converged"] and info["iterations"] == 4
    Bn = np.where(dg < 0, B, 0.0)       # nom0 = sum B_i^2 / d_i over negative d_i < 0
    _, info = O.cg(Ac, Bn, dinv=1.0 / dg, rel_tol=1e-12, max_iter=200)
    assert not info["converged"] and info["iterations"] == 0


def test_oracle_stream_triad_probe():
    gbs = O.stream_triad_gbs(n=1 << 22, reps=2)
    assert 0.5 < gbs < 1e5
