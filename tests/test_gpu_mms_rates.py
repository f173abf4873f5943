"""Analytic pin of the GPU discretisation: L2 convergence rates of the manufactured solution.

The reference holds no golden vectors, so besides the oracle restatement the GPU
path is pinned to the mathematics the reference's MMS drivers rely on
(linear_convection_diffusion_2D.cpp:159-215, ComputeL2Error at :383-392): an H1 order-p solution
on a refined hex mesh must converge in L2 at rate p + 1.  Solved through the production kernels:
the structured brick CG at p = 2 (the BASELINE C2 path) and the fused high-order CG at p = 4 (the
C3 path), κ∇²-plus-reaction operator (c = 0, CG needs SPD), rel_tol 1e-13.  The L2 error is
measured by the oracle's quadrature (test infrastructure).
"""
import math

import numpy as np
import pytest

import cdfem
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _mms_error(gpu_ctx, n, p):
    om = O.BoxMesh(3, n, p)
    prm = O.mms_params(O.MMS_SIN, 3, kappa=0.1, s=1.0, c=(0.0, 0.0, 0.0), modes=(1, 1, 1), p=p)
    gm = cdfem.Mesh(3, p, om.verts, om.dofmap, om.nl, om.ess)
    gpu_ctx.upload_mesh(gm).set_structured(n, n, n)
    gpu_ctx.pa_setup(kinds=cdfem.DIFFUSION | cdfem.MASS, kappa=0.1, mass=1.0)
    xyz = gpu_ctx.quadrature_points(cdfem.RULE_LINEARFORM)
    b = gpu_ctx.lf_assemble(O.mms_f(prm, xyz).reshape(-1))
    u = np.zeros(om.nl)
    u[om.ess] = O.mms_u(prm, om.dof_coords()[om.ess])
    _, B = gpu_ctx.form_linear_system(u, b)
    X, info = gpu_ctx.solve(B, method="cg", rel_tol=1e-13, abs_tol=0.0, max_iter=5000)
    assert info["converged"]
    return O.l2_error(om, X, prm)


@pytest.mark.parametrize("p,ns,min_rate", [(2, (4, 8, 16), 2.8), (4, (2, 4, 8), 4.6)])
def test_mms_l2_rate(gpu_ctx, p, ns, min_rate):
    errs = [_mms_error(gpu_ctx, n, p) for n in ns]
    rates = [math.log2(errs[k] / errs[k + 1]) for k in range(len(errs) - 1)]
    print(f"p={p} n={ns} L2={errs} rates={rates}")
    assert all(e > 0 for e in errs)
    assert rates[-1] >= min_rate, (errs, rates)


def test_mms_l2_rate_tets_p2_gmres():
    """C4 path (Kuhn tets, P2, GPU full assembly + FormLinearSystem + GMRES(30)/Jacobi on the full
    convection-diffusion-reaction operator): L2 rate 3 under refinement."""
    import cdfem as cd
    C3 = (1.0, -2.0, 0.5)
    errs = []
    with cd.Context(0) as ctx:
        for n in (4, 8):
            gm = cd.kuhn_mesh(3, n, 2)
            om = O.KuhnMesh(3, n, 2)
            prm = O.mms_params(O.MMS_SIN, 3, kappa=0.1, s=1.0, c=C3, modes=(1, 1, 1), p=2)
            b = O.lf_assemble_simplex(om, prm)
            u = np.zeros(om.nl)
            u[om.ess] = O.mms_u(prm, gm.dof_xyz[om.ess])
            ctx.upload_mesh(gm)
            ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            _, B = ctx.form_linear_system(u, b)
            X, info = ctx.solve(B, method="gmres", restart=30, rel_tol=1e-12, abs_tol=0.0, max_iter=3000)
            assert info["converged"]
            errs.append(O.l2_error_simplex(om, X, prm))
    rate = math.log2(errs[0] / errs[1])
    print(f"tets P2 n=(4, 8) L2={errs} rate={rate}")
    assert rate >= 2.7, errs
