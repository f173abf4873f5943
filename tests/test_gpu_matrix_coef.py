"""Variable coefficients incl. a MatrixCoefficient for the diffusion, and the ALE
operator it enables: Mass(J) + Diffusion(alpha dt / J cof cof^T) + Convection(phi_hat, -1) +
Mass(-div phi_hat) (diffusion_mms_ale.cpp:1017-1023), against the oracle's FA with the same per-point
coefficients (oracle.fa_assemble_q).

Tolerances: Mult / assembled values 1e-13 relative (sup norm), fixed GMRES iterates 1e-11.
"""
import numpy as np
import pytest

import cdfem
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _spd_tensors(rng, n, dim):
    """random symmetric positive definite tensors, xx,xy,yy / xx,xy,xz,yy,yz,zz"""
    L = rng.uniform(-0.5, 0.5, (n, dim, dim)) + np.eye(dim)[None] * 1.0
    K = np.einsum("nij,nkj->nik", L, L) * 0.2
    iu = np.triu_indices(dim)
    return K[:, iu[0], iu[1]].copy()


def _coeffs(ctx, m, rng):
    """random per-point coefficients, each at the points of its integrator's rule (on simplices MFEM's
    GetRule: diffusion 2p - 2, convection and mass 2p; on quads / hexes one shared rule)"""
    nd, nc, nm = (m.ne * ctx.rule_size(r) for r in (cdfem.RULE_DIFFUSION, cdfem.RULE_CONVECTION, cdfem.RULE_MASS))
    return dict(kappa=0.05, kappa_q=rng.uniform(0.01, 0.2, nd), kmat_q=_spd_tensors(rng, nd, m.dim),
                conv_q=rng.uniform(-1, 1, nc * m.dim), mass_q=rng.uniform(0.5, 2.0, nm), alpha=0.7)


TENSOR = [(2, 6, 2, 0.15, False), (3, 4, 2, 0.1, False), (3, 4, 2, 0.0, True), (3, 3, 4, 0.1, False),
          (3, 3, 4, 0.0, True), (2, 5, 3, 0.1, False)]


@pytest.mark.parametrize("dim,n,p,pert,structured", TENSOR)
def test_pa_matrix_coefficient_mult(gpu_ctx, dim, n, p, pert, structured):
    om = O.BoxMesh(dim, n, p, perturb=pert)
    gpu_ctx.upload_mesh(cdfem.Mesh(dim, p, om.verts, om.dofmap, om.nl, om.ess))
    if structured:
        gpu_ctx.set_structured(n, n, n)
    cf = _coeffs(gpu_ctx, om, np.random.default_rng(3))
    gpu_ctx.pa_setup(kinds=7, conv=None, mass=0.0, **cf)
    A = O.fa_assemble_q(om, kappa=cf["kappa"], kappa_q=cf["kappa_q"], kmat_q=cf["kmat_q"], alpha=cf["alpha"],
                        c_q=cf["conv_q"], s_q=cf["mass_q"])
    x = np.random.default_rng(4).uniform(-1, 1, om.nl)
    y, yo = gpu_ctx.mult(x), A.mult(x)
    assert np.abs(y - yo).max() <= 1e-13 * np.abs(yo).max()
    # diffusion alone: the tensor part is symmetric and has constants in its kernel
    gpu_ctx.pa_setup(kinds=1, kappa=0.0, kmat_q=cf["kmat_q"])
    one = np.ones(om.nl)
    assert np.abs(gpu_ctx.mult(one)).max() <= 1e-12 * np.abs(gpu_ctx.diagonal()).max()


@pytest.mark.parametrize("dim,p", [(2, 1), (2, 2), (2, 3), (3, 1), (3, 2)])
def test_fa_matrix_coefficient_csr(gpu_ctx, dim, p):
    om = O.KuhnMesh(dim, 4 if dim == 3 else 6, p, perturb=0.1)
    gm = cdfem.Mesh(dim, p, om.verts, om.dofmap, om.nl, om.ess, simplex=True)
    gpu_ctx.upload_mesh(gm)
    cf = _coeffs(gpu_ctx, om, np.random.default_rng(5))
    gpu_ctx.fa_setup(kinds=7, mass=0.0, **cf)
    A = O.fa_assemble_q(om, kappa=cf["kappa"], kappa_q=cf["kappa_q"], kmat_q=cf["kmat_q"], alpha=cf["alpha"],
                        c_q=cf["conv_q"], s_q=cf["mass_q"], simplex=True)
    rp, cols, vals = gpu_ctx.fa_csr()
    orp, ocol, oval = A.export()
    np.testing.assert_array_equal(rp, orp)
    np.testing.assert_array_equal(cols, ocol)
    assert np.abs(vals - oval).max() <= 1e-13 * np.abs(oval).max()


@pytest.mark.parametrize("kind", ["accuracy_a", "accuracy_b", "identity"])
@pytest.mark.parametrize("mesh", ["quad2", "tri2"])
def test_ale_operator(gpu_ctx, kind, mesh):
    """The ALE step operator on the reference square (one step t 0.3 -> 0.35, alpha 0.1, dt 0.05):
    Mult and fixed GMRES(30)+Jacobi iterates against the oracle; the identity map reduces it to
    M + alpha dt K, the diffusion_mms operator (diffusion_mms_ale_plan.tex identity check)."""
    alpha, dt, t0, t1 = 0.1, 0.05, 0.3, 0.35
    if mesh == "quad2":
        om = O.BoxMesh(2, 8, 2, perturb=0.1)
        gm = cdfem.Mesh(2, 2, om.verts, om.dofmap, om.nl, om.ess)
    else:
        om = O.KuhnMesh(2, 8, 2, perturb=0.1)
        gm = cdfem.Mesh(2, 2, om.verts, om.dofmap, om.nl, om.ess, simplex=True)
    gpu_ctx.upload_mesh(gm)
    # every coefficient at its integrator's rule (the three coincide on quads)
    pts = {r: gpu_ctx.quadrature_points(r).reshape(-1, 2)
           for r in (cdfem.RULE_DIFFUSION, cdfem.RULE_CONVECTION, cdfem.RULE_MASS)}
    metric = O.ale_coefficients(kind, pts[cdfem.RULE_DIFFUSION], t0, t1, alpha, dt)[1]
    phi = O.ale_coefficients(kind, pts[cdfem.RULE_CONVECTION], t0, t1, alpha, dt)[2]
    J, _, _, div = O.ale_coefficients(kind, pts[cdfem.RULE_MASS], t0, t1, alpha, dt)
    setup = gpu_ctx.fa_setup if gm.simplex else gpu_ctx.pa_setup
    # Mass(J) + Mass(-div phi) -> one mass coefficient; Convection(phi, -1) -> alpha = -1
    setup(kinds=7, kappa=0.0, kmat_q=metric, alpha=-1.0, conv_q=phi.ravel(), mass=0.0, mass_q=J - div)
    A = O.fa_assemble_q(om, kappa=0.0, kmat_q=metric, alpha=-1.0, c_q=phi.ravel(), s=0.0, s_q=J - div,
                        simplex=gm.simplex)
    x = np.random.default_rng(8).uniform(-1, 1, om.nl)
    y, yo = gpu_ctx.mult(x), A.mult(x)
    assert np.abs(y - yo).max() <= 1e-13 * np.abs(yo).max()
    rng = np.random.default_rng(9)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    _, B = gpu_ctx.form_linear_system(u, b)
    xo, _ = O.gmres(Ac, Bo, dinv=1.0 / Ac.diag(), restart=30, rtol=0.0, atol=0.0, max_it=40)
    xg, ig = gpu_ctx.solve(B, method="gmres", pc="jacobi", restart=30, rel_tol=0.0, abs_tol=0.0, max_iter=40)
    assert ig["iterations"] == 40
    assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)
    if kind == "identity":
        # J = 1, phi = 0: the operator is M + alpha dt K
        setup(kinds=5, kappa=alpha * dt, mass=1.0)
        np.testing.assert_allclose(gpu_ctx.mult(x), y, rtol=0, atol=1e-13 * np.abs(y).max())


def test_matrix_coefficient_rejects_bad_input(gpu_ctx):
    om = O.BoxMesh(2, 4, 1)
    gpu_ctx.upload_mesh(cdfem.Mesh(2, 1, om.verts, om.dofmap, om.nl, om.ess))
    with pytest.raises(cdfem.CdfemError):
        gpu_ctx.pa_setup(kinds=0, kmat_q=np.zeros(3 * om.ne * 4))
