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
