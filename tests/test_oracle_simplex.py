"""CPU: the simplex (config C4) part of the oracle, pinned by closed forms and analysis.

There are no MFEM outputs to pin against (parity unpinned vs MFEM), so:
  * the collapsed Gauss rule is exact on monomials up to its degree (closed form a!b!c!/(a+b+c+3)!);
  * the P1 reference-tetrahedron stiffness and mass matrices equal their closed forms;
  * assembled operators satisfy the identities of the forms (constants in the kernel of
    diffusion + convection, mass total = volume, diffusion symmetric, convection skew on functions
    vanishing on the boundary when div c = 0);
  * the manufactured-solution error converges at rate p + 1 (P1: 2, P2: 3);
  * the product's Kuhn mesh generator (cdfem_kuhn_mesh, host code) reproduces the oracle's.
"""
import math
import os

import numpy as np
import pytest

from oracle import oracle as O


@pytest.mark.parametrize("dim,n", [(2, 3), (3, 3), (3, 4)])
def test_simplex_rule_exact_on_monomials(dim, n):
    xi, w = O.simplex_rule(dim, n)
    deg = 2 * n - dim
    for a in range(deg + 1):
        for b in range(deg + 1 - a):
            cs = range(deg + 1 - a - b) if dim == 3 else [0]
            for c in cs:
                f = xi[:, 0] ** a * xi[:, 1] ** b * (xi[:, 2] ** c if dim == 3 else 1.0)
                exact = math.factorial(a) * math.factorial(b) * math.factorial(c) / math.factorial(a + b + c + dim)
                assert abs((w * f).sum() - exact) <= 1e-15 * max(1.0, exact) + 1e-17


def _single_tet(p):
    class M:
        dim, ne, nv = 3, 1, 4
    m = M()
    m.p = p
    m.verts = np.array([[[0.0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1]]])
    m.nd = 4 if p == 1 else 10
    m.dofmap = np.arange(m.nd, dtype=np.int32)[None, :]
    m.nl = m.nd
    return m


def _dense(A):
    return A.to_scipy().toarray()


def test_p1_reference_tet_closed_forms():
    m = _single_tet(1)
    K = _dense(O.fa_assemble_simplex(m, kappa=1.0, kinds=O.DIFFUSION))
    Kx = np.array([[3, -1, -1, -1], [-1, 1, 0, 0], [-1, 0, 1, 0], [-1, 0, 0, 1]]) / 6.0
    np.testing.assert_allclose(K, Kx, rtol=0, atol=1e-15)
    M = _dense(O.fa_assemble_simplex(m, s=1.0, kinds=O.MASS))
    Mx = (np.ones((4, 4)) + np.eye(4)) / 120.0
    np.testing.assert_allclose(M, Mx, rtol=0, atol=1e-16)


def test_p2_reference_tet_mass_total_and_partition():
    m = _single_tet(2)
    M = _dense(O.fa_assemble_simplex(m, s=1.0, kinds=O.MASS))
    assert abs(M.sum() - 1.0 / 6.0) <= 1e-15
    # P2 vertex functions integrate to -vol/20, edge functions to vol/5
    row = M.sum(axis=1)
    np.testing.assert_allclose(row[:4], -1.0 / 120.0, atol=1e-16)
    np.testing.assert_allclose(row[4:], 1.0 / 30.0, atol=1e-16)


@pytest.mark.parametrize("dim,n,p", [(3, 3, 2), (3, 4, 1), (2, 5, 2)])
def test_simplex_operator_identities(dim, n, p):
    m = O.KuhnMesh(dim, n, p, perturb=0.15)
    c = (1.0, -2.0, 0.5)[:dim]
    one = np.ones(m.nl)
    DC = O.fa_assemble_simplex(m, kappa=0.3, c=c, kinds=O.DIFFUSION | O.CONVECTION)
    assert np.abs(DC.mult(one)).max() <= 1e-13
    M = O.fa_assemble_simplex(m, s=1.0, kinds=O.MASS)
    assert abs(one @ M.mult(one) - 1.0) <= 1e-13
    K = _dense(O.fa_assemble_simplex(m, kappa=1.0, kinds=O.DIFFUSION))
    np.testing.assert_allclose(K, K.T, rtol=0, atol=1e-13 * np.abs(K).max())
    Cm = _dense(O.fa_assemble_simplex(m, c=c, kinds=O.CONVECTION))
    inner = np.setdiff1d(np.arange(m.nl), m.ess)
    Ci = Cm[np.ix_(inner, inner)]
    np.testing.assert_allclose(Ci, -Ci.T, rtol=0, atol=1e-13 * np.abs(Cm).max())


@pytest.mark.parametrize("p", [1, 2])
def test_simplex_mms_rate(p):
    errs = []
    for n in (3, 6):
        m = O.KuhnMesh(3, n, p)
        prm = O.mms_params(O.MMS_SIN, 3, kappa=0.1, s=1.0, c=(1.0, -2.0, 0.5), modes=(1, 1, 1), p=p)
        _, info, e = O.solve_mms_simplex(m, prm, 0.1, 1.0, (1.0, -2.0, 0.5))
        assert info["converged"]
        errs.append(e)
    rate = math.log2(errs[0] / errs[1])
    assert rate >= p + 1 - 0.25, rate


@pytest.mark.parametrize("dim,n,p", [(3, 3, 2), (3, 2, 1), (2, 4, 2), (2, 3, 1)])
def test_product_kuhn_generator_matches_oracle(dim, n, p):
    import cdfem
    om = O.KuhnMesh(dim, n, p)
    gm = cdfem.kuhn_mesh(dim, n, p)
    assert gm.nl == om.nl and gm.ne == om.ne
    np.testing.assert_array_equal(gm.dofmap, om.dofmap)
    np.testing.assert_array_equal(gm.ess, om.ess)
    np.testing.assert_allclose(gm.verts, om.verts, rtol=0, atol=1e-15)
    np.testing.assert_allclose(gm.dof_xyz, O.dof_coords_simplex(om), rtol=0, atol=1e-15)


def test_kuhn_c4_sizes():
    """BASELINE config C4: 55^3 cubes x 6 = 998,250 tets; P2 = 1,367,631 dofs."""
    import ctypes as C

    import cdfem
    ne, nl, ness = C.c_int(), C.c_int64(), C.c_int()
    assert cdfem.lib().cdfem_kuhn_sizes(3, 55, 2, C.byref(ne), C.byref(nl), C.byref(ness)) == 0
    assert (ne.value, nl.value) == (998250, 1367631)
    assert ness.value == 111 ** 3 - 109 ** 3


def test_perturbed_kuhn_stays_valid():
    import cdfem
    m = cdfem.kuhn_mesh(3, 6, 2, perturb=0.2)
    V = m.verts
    J = np.stack([V[:, 1] - V[:, 0], V[:, 2] - V[:, 0], V[:, 3] - V[:, 0]], axis=-1)
    assert (np.linalg.det(J) > 0).all()


# ---- ILU(0) (PETSc PCILU, natural ordering: Input/petsc_circle.opts "-pc_type bjacobi
#      -sub_pc_type ilu", one block per rank) -------------------------------------------------------
def _ilu_lu(F):
    import scipy.sparse as sp
    M = F.to_scipy().tocsr()
    L = sp.tril(M, -1) + sp.identity(M.shape[0])
    U = sp.triu(M)
    return (L @ U).tocsr()


def test_ilu0_reproduces_a_on_its_pattern():
    """Defining property of ILU(0): (L U)_ij = a_ij for every (i, j) in the pattern of A."""
    m = O.KuhnMesh(2, 5, 2, perturb=0.1)
    A = O.fa_assemble_simplex(m, kappa=0.1, alpha=1.0, s=1.0, c=(1.0, -2.0))
    Ac, _ = O.form_linear_system(A, m.bdr, np.zeros(m.nl), np.zeros(m.nl))
    F = O.ilu0(Ac)
    S = Ac.to_scipy().tocsr()
    LU = _ilu_lu(F)
    rows = np.repeat(np.arange(S.shape[0]), np.diff(S.indptr))
    lu_on_pattern = np.asarray(LU[rows, S.indices]).ravel()
    assert np.abs(lu_on_pattern - S.data).max() <= 1e-12 * np.abs(S.data).max()
    # ... and it is not the exact factorisation (fill is dropped)
    assert np.abs((LU - S).toarray()).max() > 1e-6


def test_ilu0_gmres_converges_faster_than_jacobi():
    """ILU(0)-preconditioned GMRES solves the convection-diffusion system to the reference's
    tolerances in fewer steps than Jacobi, and the factor solve inverts L U."""
    m = O.KuhnMesh(2, 8, 2, perturb=0.1)
    A = O.fa_assemble_simplex(m, kappa=0.1, alpha=1.0, s=1.0, c=(1.0, -2.0))
    b = np.random.default_rng(3).uniform(-1, 1, m.nl)
    Ac, B = O.form_linear_system(A, m.bdr, np.zeros(m.nl), b)
    F = O.ilu0(Ac)
    xi, ii = O.gmres_ilu(Ac, B, F, restart=30, rtol=1e-10, atol=1e-12, max_it=500)
    xj, ij = O.gmres(Ac, B, dinv=1.0 / Ac.diag(), restart=30, rtol=1e-10, atol=1e-12, max_it=500)
    assert ii["converged"] and ij["converged"] and ii["iterations"] < ij["iterations"]
    assert np.linalg.norm(Ac.mult(xi) - B) <= 1e-8 * np.linalg.norm(B)
    assert np.linalg.norm(xi - xj) <= 1e-7 * np.linalg.norm(xj)
    # the factor solve is the inverse of L U
    r = np.random.default_rng(4).uniform(-1, 1, m.nl)
    z = O.ilu_solve(F, r)
    assert np.abs(_ilu_lu(F) @ z - r).max() <= 1e-11 * np.abs(r).max()


def test_radial_mms_on_synthetic_disk_converges():
    """Circle variant MMS (linear_convection_diffusion_2D_circle.cpp:140-215) through the oracle on the
    synthetic gmsh disk: the L2 error falls under refinement (P2 on a polygonal domain: the boundary
    approximation limits the rate to about 2) and the forcing matches a finite-difference restatement."""
    import sys
    import numpy as np
    sys.path.insert(0, os.path.dirname(__file__))
    import gmsh_synth
    import cdfem
    from oracle import oracle as O
    errs = []
    for nr in (6, 12):
        path = f"/tmp/cdfem_disk_{nr}.msh"
        gmsh_synth.write_circle(path, nr, perturb=0.0)
        m = cdfem.gmsh_mesh(path, 2)

        class OM:
            pass
        om = OM()
        om.dim, om.p, om.ne, om.nl, om.verts, om.dofmap, om.ess = 2, 2, m.ne, m.nl, m.verts, m.dofmap, m.ess
        om.bdr = np.zeros(m.nl, dtype=np.int32)
        om.bdr[m.ess] = 1
        prm = O.mms_params(O.MMS_RADIAL, 2, kappa=1.0, s=1.0, c=(1.0, 1.0), p=2)
        _, info, l2 = O.solve_mms_simplex(om, prm, 1.0, 1.0, (1.0, 1.0), max_it=2000)
        assert info["converged"]
        errs.append(l2)
    assert np.log2(errs[0] / errs[1]) >= 1.8, errs
    # forcing = -Lap u + c.grad u + u, checked by central differences at a few points
    prm = O.mms_params(O.MMS_RADIAL, 2, kappa=1.0, s=1.0, c=(1.0, 1.0), p=2)
    pts = np.array([[0.3, 0.1], [-0.5, 0.4], [0.05, -0.7], [0.0, 0.0]])
    h = 1e-4
    for x in pts:
        u = lambda p: O.mms_u(prm, np.array([p]))[0]  # noqa: E731
        ex, ey = np.array([h, 0.0]), np.array([0.0, h])
        lap = (u(x + ex) + u(x - ex) + u(x + ey) + u(x - ey) - 4 * u(x)) / h ** 2
        gx, gy = (u(x + ex) - u(x - ex)) / (2 * h), (u(x + ey) - u(x - ey)) / (2 * h)
        f = O.mms_f(prm, np.array([x]))[0]
        assert abs(f - (-lap + gx + gy + u(x))) <= 1e-4 * max(1.0, abs(f))


@pytest.mark.parametrize("dim,orders", [(2, range(0, 10)), (3, range(0, 7))])
def test_mfem_simplex_rules_exact_and_shared(dim, orders):
    """MFEM's tabulated simplex rules (tools/simplex_rules.py): the product's table
    (cdfem_simplex_rule_order) equals the oracle's, has MFEM's point counts, positive-or-documented
    weights, points inside the simplex, and integrates every monomial of the order exactly."""
    import ctypes as C
    import itertools
    import cdfem
    L = cdfem.lib()
    L.cdfem_simplex_rule_order.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    counts = {2: [1, 1, 3, 4, 6, 7, 12, 12, 16, 19], 3: [1, 1, 4, 5, 11, 14, 24]}
    for order in orders:
        xo, wo = O.simplex_rule_order(dim, order)
        n = L.cdfem_simplex_rule_order(dim, order, None, None)
        xi, w = np.zeros(n * dim), np.zeros(n)
        L.cdfem_simplex_rule_order(dim, order, xi.ctypes.data_as(C.POINTER(C.c_double)),
                                   w.ctypes.data_as(C.POINTER(C.c_double)))
        assert n == len(wo) == counts[dim][order]
        np.testing.assert_array_equal(xi.reshape(n, dim), xo)
        np.testing.assert_array_equal(w, wo)
        assert (xo >= -1e-15).all() and (xo.sum(axis=1) <= 1 + 1e-15).all()
        for tot in range(order + 1):
            for e in itertools.product(range(tot + 1), repeat=dim):
                if sum(e) != tot:
                    continue
                exact = math.prod(math.factorial(k) for k in e) / math.factorial(dim + tot)
                assert abs(np.sum(wo * np.prod(xo ** np.array(e), axis=1)) - exact) <= 1e-15


@pytest.mark.parametrize("dim,p", [(2, 1), (2, 2), (2, 3), (3, 1), (3, 2)])
def test_per_integrator_rules_are_mfems(dim, p):
    """MFEM's GetRule on affine simplices: diffusion on the tabulated rule of order 2p - 2,
    convection and mass on order 2p.  With per-point coefficients (the quantities that make the rule
    matter), one element's diffusion, convection and mass matrices from the oracle equal a direct
    restatement here: sum over those rules' points of w_q k_q (A grad phi_i).(A grad phi_j) / det J,
    w_q phi_i (c_q . A grad phi_j), w_q s_q det J phi_i phi_j, with the product's host basis and rules
    (cdfem_simplex_basis / cdfem_simplex_rule_order)."""
    import ctypes as C
    import cdfem
    L = cdfem.lib()
    dp = C.POINTER(C.c_double)
    L.cdfem_simplex_rule_order.argtypes = [C.c_int, C.c_int, dp, dp]
    L.cdfem_simplex_basis.argtypes = [C.c_int, C.c_int, C.c_int, dp, dp, dp]

    def rule(order):
        n = L.cdfem_simplex_rule_order(dim, order, None, None)
        xi, w = np.zeros(n * dim), np.zeros(n)
        L.cdfem_simplex_rule_order(dim, order, xi.ctypes.data_as(dp), w.ctypes.data_as(dp))
        return xi.reshape(n, dim), w
    nd = {(2, 1): 3, (2, 2): 6, (2, 3): 10, (3, 1): 4, (3, 2): 10}[(dim, p)]

    def basis(xi):
        phi, dphi = np.zeros(len(xi) * nd), np.zeros(len(xi) * nd * dim)
        L.cdfem_simplex_basis(dim, p, len(xi), np.ascontiguousarray(xi).ctypes.data_as(dp), phi.ctypes.data_as(dp),
                              dphi.ctypes.data_as(dp))
        return phi.reshape(len(xi), nd), dphi.reshape(len(xi), nd, dim)
    rng = np.random.default_rng(3)
    V = np.eye(dim + 1, dim, -1) * 1.0 + rng.uniform(-0.1, 0.1, (dim + 1, dim))   # a perturbed reference simplex
    J = (V[1:] - V[0]).T
    det = np.linalg.det(J)
    A = np.linalg.inv(J).T * det                                                     # adj(J)^T
    xd, wd = rule(max(2 * p - 2, 0))
    xc, wc = rule(2 * p)
    assert (len(wd), len(wc)) == {2: {1: (1, 3), 2: (3, 6), 3: (6, 12)}, 3: {1: (1, 4), 2: (4, 11)}}[dim][p]
    kq, cq, sq = rng.uniform(0.5, 2, len(wd)), rng.uniform(-1, 1, (len(wc), dim)), rng.uniform(0.5, 2, len(wc))
    pd, gd = basis(xd)
    pc, gc = basis(xc)
    Kd = np.einsum("q,qia,qja->ij", wd * kq / det, gd @ A.T, gd @ A.T)
    Cc = np.einsum("q,qi,qj->ij", wc, pc, np.einsum("qa,qja->qj", cq, gc @ A.T))
    Mm = np.einsum("q,qi,qj->ij", wc * sq * det, pc, pc)

    class M1:
        pass
    m = M1()
    m.dim, m.p, m.ne, m.nl = dim, p, 1, nd
    m.verts = V[None].copy()
    m.dofmap = np.arange(nd, dtype=np.int32)[None]
    for kinds, want, kw in ((O.DIFFUSION, Kd, dict(kappa_q=kq)), (O.CONVECTION, Cc, dict(c_q=cq.ravel())),
                            (O.MASS, Mm, dict(s_q=sq))):
        got = O.fa_assemble_q(m, kinds=kinds, simplex=True, **kw).to_scipy().toarray()
        assert np.abs(got - want).max() <= 1e-13 * np.abs(want).max(), kinds
