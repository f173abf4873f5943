"""gmsh v2.2 reader (cdfem_gmsh_*: the reference's mesh input, linear_convection_diffusion_2D.cpp:290)
and P1-P3 triangles, on synthetic meshes written by tests/gmsh_synth.py.

CPU: the reader against an independent parse, and the oracle's P3 basis against closed forms and
convergence rates. GPU: FA / DomainLF / the GMRES(30)+Jacobi MMS solve against the oracle.
"""
import math
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
import gmsh_synth  # noqa: E402

import cdfem  # noqa: E402
from oracle import oracle as O  # noqa: E402

C2 = (1.0, -2.0)


def _msh(tmp_path, n=5, perturb=0.2, seed=0):
    p = str(tmp_path / f"sq{n}_{seed}.msh")
    info = gmsh_synth.write_square(p, n, perturb=perturb, seed=seed)
    return p, info


class _OM:
    """oracle view of a product mesh (same arrays)"""

    def __init__(self, m):
        self.dim, self.p, self.ne, self.nl = m.dim, m.order, m.ne, m.nl
        self.verts, self.dofmap, self.ess = m.verts, m.dofmap, m.ess
        self.bdr = np.zeros(m.nl, dtype=np.int32)
        self.bdr[m.ess] = 1


@pytest.mark.parametrize("order", [1, 2, 3])
def test_reader_counts_geometry_orientation(tmp_path, order):
    n = 5
    path, info = _msh(tmp_path, n)
    m = cdfem.gmsh_mesh(path, order)
    nv, ntri = info["n_nodes"], info["n_tri"]
    nedges = 3 * n * n + 2 * n
    assert m.dim == 2 and m.ne == ntri
    assert m.nl == nv + (order - 1) * nedges + (ntri if order == 3 else 0)
    nodes, tris = gmsh_synth.read_triangles(path)
    want = sorted(tuple(sorted((round(nodes[v][0], 14), round(nodes[v][1], 14)) for v in t)) for t in tris)
    got = sorted(tuple(sorted((round(x, 14), round(y, 14)) for x, y in tv)) for tv in m.verts)
    assert got == want
    V = m.verts
    det = (V[:, 1, 0] - V[:, 0, 0]) * (V[:, 2, 1] - V[:, 0, 1]) - (V[:, 1, 1] - V[:, 0, 1]) * (V[:, 2, 0] - V[:, 0, 0])
    assert (det > 0).all()                       # the clockwise triangles were re-oriented
    # every dof's coordinate as the oracle places it from each element (consistent edge orientation)
    np.testing.assert_allclose(O.dof_coords_simplex(_OM(m)), m.dof_xyz, rtol=0, atol=1e-15)
    # dof multiplicity: edge and interior dofs in 1 or 2 elements
    cnt = np.bincount(m.dofmap.ravel(), minlength=m.nl)
    assert (cnt[nv:] >= 1).all() and (cnt[nv:] <= 2).all()


def test_reader_boundary_attributes(tmp_path):
    path, _ = _msh(tmp_path, 4)
    m = cdfem.gmsh_mesh(path, 3)
    x, y, mask = m.dof_xyz[:, 0], m.dof_xyz[:, 1], m.bdr_mask
    for bit, on in ((0, y == 0.0), (1, x == 1.0), (2, y == 1.0), (3, x == 0.0)):
        np.testing.assert_array_equal((mask >> bit) & 1 == 1, on)
    only_left = cdfem.gmsh_mesh(path, 3, ess_attrs=[4])
    np.testing.assert_array_equal(np.sort(only_left.ess), np.nonzero(x == 0.0)[0])
    assert len(m.ess) == np.count_nonzero((x == 0) | (x == 1) | (y == 0) | (y == 1))


def test_reader_rejects_bad_input(tmp_path):
    bad = tmp_path / "bad.msh"
    bad.write_text("$MeshFormat\n4.1 0 8\n$EndMeshFormat\n")
    with pytest.raises(cdfem.CdfemError):
        cdfem.gmsh_mesh(str(bad), 1)
    path, _ = _msh(tmp_path, 2)
    with pytest.raises(cdfem.CdfemError):
        cdfem.gmsh_mesh(path, 4)                  # triangles: order <= 3
    with pytest.raises(cdfem.CdfemError):
        cdfem.gmsh_mesh(str(tmp_path / "missing.msh"), 1)


def test_oracle_p3_exactness_and_identities(tmp_path):
    path, _ = _msh(tmp_path, 4)
    om = _OM(cdfem.gmsh_mesh(path, 3))
    one = np.ones(om.nl)
    M = O.fa_assemble_simplex(om, s=1.0, kinds=O.MASS)
    assert abs(one @ M.mult(one) - 1.0) <= 1e-13
    DC = O.fa_assemble_simplex(om, kappa=0.7, c=C2, kinds=O.DIFFUSION | O.CONVECTION)
    assert np.abs(DC.mult(one)).max() <= 1e-12
    # a total-degree-2 polynomial (MMS_POLY with p = 1: g(x) g(y), g linear) is interpolated exactly
    prm = O.mms_params(O.MMS_POLY, 2, modes=(1, 1, 1), p=1)
    u = O.mms_u(prm, O.dof_coords_simplex(om))
    assert O.l2_error_simplex(om, u, prm) <= 1e-13


def test_oracle_p3_mms_rate(tmp_path):
    errs = []
    for n in (4, 8):
        path, _ = _msh(tmp_path, n, perturb=0.0)
        om = _OM(cdfem.gmsh_mesh(path, 3))
        prm = O.mms_params(O.MMS_SIN, 2, kappa=0.1, s=1.0, c=C2, modes=(1, 1, 1), p=3)
        _, info, e = O.solve_mms_simplex(om, prm, 0.1, 1.0, C2)
        assert info["converged"]
        errs.append(e)
    assert math.log2(errs[0] / errs[1]) >= 3.6


# ---------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("order", [1, 2, 3])
def test_gpu_fa_and_lf_on_gmsh(gpu_ctx, tmp_path, order):
    path, _ = _msh(tmp_path, 6, seed=order)
    m = cdfem.gmsh_mesh(path, order)
    om = _OM(m)
    gpu_ctx.upload_mesh(m)
    gpu_ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C2, mass=1.0)
    A = O.fa_assemble_simplex(om, kappa=0.1, alpha=1.0, s=1.0, c=C2)
    rp, cols, vals = gpu_ctx.fa_csr()
    orp, ocol, oval = A.export()
    np.testing.assert_array_equal(rp, orp)
    np.testing.assert_array_equal(cols, ocol)
    assert np.abs(vals - oval).max() <= 1e-13 * np.abs(oval).max()
    prm = O.mms_params(O.MMS_SIN, 2, kappa=0.1, s=1.0, c=C2, modes=(3, 3, 3), p=order)
    xq = gpu_ctx.quadrature_points(cdfem.RULE_LINEARFORM)
    b = gpu_ctx.lf_assemble(O.mms_f(prm, xq).reshape(-1))
    bo = O.lf_assemble_simplex(om, prm)
    assert np.abs(b - bo).max() <= 1e-12 * np.abs(bo).max()


@pytest.mark.gpu
def test_gpu_lf_on_tets(gpu_ctx):
    gm = cdfem.kuhn_mesh(3, 3, 2, perturb=0.1)
    om = O.KuhnMesh(3, 3, 2)
    om.verts, om.dofmap = gm.verts, gm.dofmap
    gpu_ctx.upload_mesh(gm)
    prm = O.mms_params(O.MMS_SIN, 3, kappa=0.1, s=1.0, c=(1.0, -2.0, 0.5), modes=(1, 1, 1), p=2)
    xq = gpu_ctx.quadrature_points(cdfem.RULE_LINEARFORM)
    b = gpu_ctx.lf_assemble(O.mms_f(prm, xq).reshape(-1))
    bo = O.lf_assemble_simplex(om, prm)
    assert np.abs(b - bo).max() <= 1e-12 * np.abs(bo).max()


@pytest.mark.gpu
def test_gpu_reference_input_sequence_p3(gpu_ctx, tmp_path):
    """The reference's default run (Input/input_2d.yaml: order 3, kappa 0.1, s 1, c (1,-2), modes
    3,3; GMRES(30)+Jacobi, rtol 1e-10, atol 1e-12) on a synthetic gmsh square, GPU vs oracle."""
    path, _ = _msh(tmp_path, 12, perturb=0.25, seed=3)
    m = cdfem.gmsh_mesh(path, 3)
    om = _OM(m)
    prm = O.mms_params(O.MMS_SIN, 2, kappa=0.1, s=1.0, c=C2, modes=(3, 3, 3), p=3)
    Xo, io, eo = O.solve_mms_simplex(om, prm, 0.1, 1.0, C2)
    gpu_ctx.upload_mesh(m)
    gpu_ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C2, mass=1.0)
    b = gpu_ctx.lf_assemble(O.mms_f(prm, gpu_ctx.quadrature_points(cdfem.RULE_LINEARFORM)).reshape(-1))
    u = np.zeros(m.nl)
    u[m.ess] = O.mms_u(prm, m.dof_xyz[m.ess])
    _, B = gpu_ctx.form_linear_system(u, b)
    X, ig = gpu_ctx.solve(B, method="gmres", restart=30, rel_tol=1e-10, abs_tol=1e-12, max_iter=500)
    assert io["converged"] and ig["converged"] and abs(ig["iterations"] - io["iterations"]) <= 1
    eg = O.l2_error_simplex(om, X, prm)
    assert abs(eg - eo) <= 1e-6 * eo
