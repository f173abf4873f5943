"""GPU GMRES(m) + Jacobi (PETSc KSPGMRES semantics, Input/petsc.opts:2-6) against the oracle's
restatement (oracle/cdfem_oracle.c:orc_gmres) on the same constrained systems.

Operator = the reference's full convection-diffusion-reaction form (non-symmetric:
linear_convection_diffusion_2D.cpp:335-338), so this is the solver the reference actually runs.
Tolerances (f64, PA on the GPU vs assembled CSR on the CPU):
  * fixed inner-step counts (rtol = atol = 0): iterate relative L2 <= 1e-11, residual estimates
    equal to 1e-9 relative;
  * converged (rtol 1e-10 / atol 1e-12, the reference's settings): same iteration count +-1,
    solution relative L2 <= 1e-8 (GMRES stops at a 1e-10 preconditioned residual, so the two
    solutions are only as close as the stopping tolerance times the conditioning allows);
  * repeated GPU solves bitwise identical.
"""
import numpy as np
import pytest

import cdfem
from oracle import oracle as O

pytestmark = pytest.mark.gpu
C3 = (1.0, -2.0, 0.5)


def _system(gpu_ctx, dim, n, p, pert, kinds=7, structured=False, seed=5):
    om = O.BoxMesh(dim, n, p, perturb=pert)
    gm = cdfem.Mesh(dim, p, om.verts, om.dofmap, om.nl, om.ess)
    gpu_ctx.upload_mesh(gm)
    if structured:
        gpu_ctx.set_structured(n, n, n)
    c = C3[:dim]
    gpu_ctx.pa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=c, mass=1.0)
    ok = (O.DIFFUSION if kinds & 1 else 0) | (O.CONVECTION if kinds & 2 else 0) | (O.MASS if kinds & 4 else 0)
    A = O.fa_assemble(om, kappa=0.1, alpha=1.0, s=1.0, c=c, kinds=ok)
    rng = np.random.default_rng(seed)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    _, B = gpu_ctx.form_linear_system(u, b)
    return om, Ac, Bo, B


CASES = [(2, 8, 2, 0.2, False), (3, 4, 2, 0.15, False), (3, 5, 1, 0.1, False), (3, 8, 2, 0.1, True)]


@pytest.mark.parametrize("dim,n,p,pert,structured", CASES)
@pytest.mark.parametrize("restart,steps", [(30, 20), (5, 23), (1, 4)])
def test_gmres_fixed_steps_parity(gpu_ctx, dim, n, p, pert, structured, restart, steps):
    om, Ac, Bo, B = _system(gpu_ctx, dim, n, p, pert, structured=structured)
    xo, io = O.gmres(Ac, Bo, dinv=1.0 / Ac.diag(), restart=restart, rtol=0.0, atol=0.0, max_it=steps)
    xg, ig = gpu_ctx.solve(B, method="gmres", pc="jacobi", restart=restart, rel_tol=0.0, abs_tol=0.0,
                           max_iter=steps)
    assert io["iterations"] == ig["iterations"] == steps
    assert not ig["converged"]
    assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)
    assert abs(ig["final_norm"] - io["final_norm"]) <= 1e-9 * io["final_norm"]


@pytest.mark.parametrize("dim,n,p,pert,structured", CASES)
def test_gmres_converged_parity(gpu_ctx, dim, n, p, pert, structured):
    om, Ac, Bo, B = _system(gpu_ctx, dim, n, p, pert, structured=structured)
    dinv = 1.0 / Ac.diag()
    xo, io = O.gmres(Ac, Bo, dinv=dinv, restart=30, rtol=1e-10, atol=1e-12, max_it=500)
    xg, ig = gpu_ctx.solve(B, method="gmres", pc="jacobi", restart=30, rel_tol=1e-10, abs_tol=1e-12,
                           max_iter=500)
    assert io["converged"] and ig["converged"]
    assert abs(ig["iterations"] - io["iterations"]) <= 1
    assert np.linalg.norm(xg - xo) <= 1e-8 * np.linalg.norm(xo)
    # the true preconditioned residual meets the PETSc test (up to the Givens estimate's drift)
    r = dinv * (Bo - Ac.mult(xg))
    r0 = np.linalg.norm(dinv * Bo)
    assert np.linalg.norm(r) <= 1e-9 * r0
    xg2, ig2 = gpu_ctx.solve(B, method="gmres", pc="jacobi", restart=30, rel_tol=1e-10, abs_tol=1e-12,
                             max_iter=500)
    np.testing.assert_array_equal(xg, xg2)
    assert ig2["iterations"] == ig["iterations"]


def test_gmres_unpreconditioned(gpu_ctx):
    om, Ac, Bo, B = _system(gpu_ctx, 2, 6, 2, 0.1)
    xo, io = O.gmres(Ac, Bo, dinv=None, restart=30, rtol=1e-10, atol=1e-12, max_it=500)
    xg, ig = gpu_ctx.solve(B, method="gmres", pc="none", restart=30, rel_tol=1e-10, abs_tol=1e-12,
                           max_iter=500)
    assert io["converged"] and ig["converged"] and abs(io["iterations"] - ig["iterations"]) <= 1
    assert np.linalg.norm(xg - xo) <= 1e-8 * np.linalg.norm(xo)


def test_gmres_edge_cases(gpu_ctx):
    om, Ac, Bo, B = _system(gpu_ctx, 2, 4, 1, 0.0)
    # zero right-hand side: converged before the first step (beta = 0)
    x0, i0 = gpu_ctx.solve(np.zeros(om.nl), method="gmres", max_iter=10)
    assert i0["converged"] and i0["iterations"] == 0 and not x0.any()
    # max_iter = 0: not converged, x = 0
    with pytest.raises(cdfem.CdfemError) as ei:
        gpu_ctx.solve(B, method="gmres", max_iter=0, raise_on_fail=True)
    assert ei.value.code == cdfem.ERR_NOT_CONVERGED
    # restart above the supported maximum is an argument error
    with pytest.raises(cdfem.CdfemError) as ei:
        gpu_ctx.solve(B, method="gmres", restart=65, max_iter=10)
    assert ei.value.code == cdfem.ERR_ARG


def test_gmres_all_essential(gpu_ctx):
    """single p=1 hex: every dof essential -> A_c = I; one step reaches the exact solution."""
    om = O.BoxMesh(3, 1, 1)
    gm = cdfem.Mesh(3, 1, om.verts, om.dofmap, om.nl, om.ess)
    gpu_ctx.upload_mesh(gm)
    gpu_ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    u = np.arange(1.0, om.nl + 1.0)
    _, B = gpu_ctx.form_linear_system(u, np.zeros(om.nl))
    xs, info = gpu_ctx.solve(B, method="gmres", rel_tol=1e-12, max_iter=10)
    assert info["converged"] and info["iterations"] == 1
    np.testing.assert_allclose(xs, u, rtol=0, atol=1e-14 * u.max())


TIGHT = [("hex p=2 brick", 3, 6, 2, 0.0, True), ("hex p=2 generic", 3, 4, 2, 0.15, False),
         ("hex p=4 structured", 3, 3, 4, 0.0, True), ("hex p=4 generic", 3, 3, 4, 0.1, False),
         ("quad p=3", 2, 6, 3, 0.15, False)]


@pytest.mark.parametrize("name,dim,n,p,pert,structured", TIGHT)
def test_gmres_tight_solution_parity_pa(gpu_ctx, name, dim, n, p, pert, structured):
    """SURVEY §8d ladder step 3 for the reference's own solver: GMRES(30) + Jacobi on the full
    nonsymmetric D+C+M operator, GPU and oracle both solved to rtol 1e-13: solutions within 1e-10
    relative L2 (north-star tolerance)."""
    om, Ac, Bo, B = _system(gpu_ctx, dim, n, p, pert, structured=structured)
    dinv = 1.0 / Ac.diag()
    xo, io = O.gmres(Ac, Bo, dinv=dinv, restart=30, rtol=1e-13, atol=0.0, max_it=5000)
    xg, ig = gpu_ctx.solve(B, method="gmres", pc="jacobi", restart=30, rel_tol=1e-13, abs_tol=0.0,
                           max_iter=5000)
    assert io["converged"] and ig["converged"], (io, ig)
    assert np.linalg.norm(xg - xo) <= 1e-10 * np.linalg.norm(xo)


def test_gmres_tight_solution_parity_fa_tets(gpu_ctx):
    """The same bar on the assembled path (C4's FA CSR on Kuhn tets, P2)."""
    om = O.KuhnMesh(3, 4, 2, perturb=0.1)
    gm = cdfem.Mesh(3, 2, om.verts, om.dofmap, om.nl, om.ess, simplex=True)
    gpu_ctx.upload_mesh(gm)
    gpu_ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    A = O.fa_assemble_simplex(om, kappa=0.1, alpha=1.0, s=1.0, c=C3)
    rng = np.random.default_rng(9)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    _, B = gpu_ctx.form_linear_system(u, b)
    xo, io = O.gmres(Ac, Bo, dinv=1.0 / Ac.diag(), restart=30, rtol=1e-13, atol=0.0, max_it=5000)
    xg, ig = gpu_ctx.solve(B, method="gmres", pc="jacobi", restart=30, rel_tol=1e-13, abs_tol=0.0,
                           max_iter=5000)
    assert io["converged"] and ig["converged"], (io, ig)
    assert np.linalg.norm(xg - xo) <= 1e-10 * np.linalg.norm(xo)


@pytest.mark.parametrize("n,p,kinds", [(8, 2, 7), (6, 2, 5), (7, 1, 7), (9, 2, 3)])
def test_gmres_patch_buffer_pass_bitwise(gpu_ctx, n, p, kinds):
    """gm_pb: on the structured patch-buffer Mult, the first orthogonalisation pass sums each row's
    patch entries itself (essential rows: the basis vector) instead of reading the Mult's row-sum
    kernel output.  Same sums in the same order: 35 GMRES(10) iterates (three restarts, so the
    cycle-start Mult through the row-sum kernel is exercised too) bitwise equal to gm_pb 0, and
    1e-11 of the oracle; partial bricks (n not a multiple of 4) included."""
    om, Ac, Bo, B = _system(gpu_ctx, 3, n, p, 0.1, kinds=kinds, structured=True)
    xo, _ = O.gmres(Ac, Bo, dinv=1.0 / Ac.diag(), restart=10, rtol=0.0, atol=0.0, max_it=35)
    out = {}
    try:
        for pb in (0, 1):
            gpu_ctx.set_option("gm_pb", pb)
            out[pb] = gpu_ctx.solve(B, method="gmres", pc="jacobi", restart=10, rel_tol=0.0, abs_tol=0.0,
                                    max_iter=35)
    finally:
        gpu_ctx.set_option("gm_pb", 1)
    (x0, i0), (x1, i1) = out[0], out[1]
    assert i0["iterations"] == i1["iterations"] == 35
    np.testing.assert_array_equal(x1, x0)
    assert i1["final_norm"] == i0["final_norm"]
    assert np.linalg.norm(x1 - xo) <= 1e-11 * np.linalg.norm(xo)


@pytest.mark.parametrize("structured,restart", [(True, 30), (True, 7), (False, 10)])
def test_gmres_poll_interval_bitwise(gpu_ctx, structured, restart):
    """gm_poll k (default 4): the host records an event and checks the device state every k inner steps
    instead of after every step.  Steps it queued past the converged step exit at their first check (their
    Mult runs and writes scratch only), so the solution, the iteration count and the final residual are
    bitwise those of checking every step, for converging solves (the stop inside a poll interval) and
    for fixed step counts across restarts; on the structured patch-buffer path and the generic one."""
    om, Ac, Bo, B = _system(gpu_ctx, 3, 6, 2, 0.0 if structured else 0.1, structured=structured, seed=19)
    xo, io = O.gmres(Ac, Bo, dinv=1.0 / Ac.diag(), restart=restart, rtol=1e-10, atol=1e-12, max_it=500)
    out = {}
    try:
        for k in (1, 4, 7):
            gpu_ctx.set_option("gm_poll", k)
            out[k] = (gpu_ctx.solve(B, method="gmres", pc="jacobi", restart=restart, rel_tol=1e-10, abs_tol=1e-12,
                                    max_iter=500),
                      gpu_ctx.solve(B, method="gmres", pc="jacobi", restart=restart, rel_tol=0.0, abs_tol=0.0,
                                    max_iter=2 * restart + 3))
    finally:
        gpu_ctx.set_option("gm_poll", 4)
    (x1, i1), (f1, j1) = out[1]
    assert i1["converged"] and abs(i1["iterations"] - io["iterations"]) <= 1
    assert np.linalg.norm(x1 - xo) <= 1e-8 * np.linalg.norm(xo)
    assert j1["iterations"] == 2 * restart + 3
    for k in (4, 7):
        (xk, ik), (fk, jk) = out[k]
        np.testing.assert_array_equal(xk, x1)
        assert ik["iterations"] == i1["iterations"] and ik["converged"] and ik["final_norm"] == i1["final_norm"]
        np.testing.assert_array_equal(fk, f1)
        assert jk["iterations"] == j1["iterations"]
    with pytest.raises(cdfem.CdfemError):
        gpu_ctx.set_option("gm_poll", 0)
