"""The reference's own inputs through the product: Mesh/unit_square.msh and Mesh/unit_circle.msh
(fixture tests/golden/reference_meshes.npz, made by tests/golden/make_reference_meshes.py) with the
reference's two default configurations:

  square  Input/input_2d.yaml:1-16        order 3, kappa 0.1, s 1, c (1,-2), modes (3,3), Input/petsc.opts
          (GMRES(30) + Jacobi, rtol 1e-10, atol 1e-12, max_it 500); linear_convection_diffusion_2D.cpp:
          290-305 (mesh, space), 319-343 (ess, forms), 349-377 (FormLinearSystem, PETSc solve, recover)
  circle  Input/input_2d_circle.yaml:1-13 order 3, kappa 1, s 1, c (1,1), radial MMS
          (linear_convection_diffusion_2D_circle.cpp:140-215), Input/petsc_circle.opts (GMRES(30) +
          bjacobi/ILU(0), rtol 1e-10, atol 1e-12, max_it 2000); :294-304, 372

CPU: the fixture equals the reference files as the product reader sees them (when /root/reference
exists), the sizes (938 / 510 / 80 and 3056 / 1593 / 128), and the dof numbering equals an
independent restatement of MFEM's (Mesh(file, 1, 1) finalize + first-met edge order), which PETSc's
ILU(0) depends on.
GPU: both configurations end to end against the oracle (iterations +-1, MMS L2 to 1e-6 relative,
solutions to 1e-10 relative L2 when both sides solve to rtol 1e-13), through the Python C-ABI
binding and through the MFEM-shaped C++ driver, plus `mpiexec -n 2` of both against one rank.
Parity is against the oracle (MFEM/PETSc are absent: parity unpinned beyond the oracle).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
import reference_meshes as R  # noqa: E402

import cdfem  # noqa: E402
from oracle import oracle as O  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "continuum-mechanics-mfem_amd", "lib", "convection_diffusion")
MPIEXEC = "/opt/conda/bin/mpiexec"
PETSC_OPTS = "-ksp_type gmres\n-ksp_rtol 1.0e-10\n-ksp_atol 1.0e-12\n-ksp_max_it 500\n-pc_type jacobi\n"
CIRCLE_OPTS = ("-ksp_type gmres\n-ksp_rtol 1.0e-10\n-ksp_atol 1.0e-12\n-ksp_max_it 2000\n"
               "-pc_type bjacobi\n-sub_ksp_type preonly\n-sub_pc_type ilu\n")
# (kappa, s, c, mms kind, options text, pc, max_it) of the two default configurations
CONFIGS = {
    "square": (0.1, 1.0, (1.0, -2.0), O.MMS_SIN, PETSC_OPTS, "jacobi", 500),
    "circle": (1.0, 1.0, (1.0, 1.0), O.MMS_RADIAL, CIRCLE_OPTS, "ilu", 2000),
}
ORDER = 3


@pytest.fixture(scope="module")
def msh(tmp_path_factory):
    d = tmp_path_factory.mktemp("refmesh")
    return {n: R.write_msh(n, str(d / R.REF_FILES[n])) for n in R.REF_FILES}


def _topology(path):
    import ctypes as C
    L = cdfem.lib()
    dim, nv, ne, nbe = C.c_int(), C.c_int64(), C.c_int(), C.c_int()
    assert L.cdfem_gmsh_topology_sizes(os.fsencode(path), C.byref(dim), C.byref(nv), C.byref(ne), C.byref(nbe)) == 0
    d = dim.value
    vxyz = np.zeros((nv.value, d))
    ev = np.zeros((ne.value, d + 1), dtype=np.int32)
    bv = np.zeros((nbe.value, d), dtype=np.int32)
    ba = np.zeros(nbe.value, dtype=np.int32)
    ip = C.POINTER(C.c_int32)
    assert L.cdfem_gmsh_topology(os.fsencode(path), vxyz.ctypes.data_as(C.POINTER(C.c_double)),
                                 ev.ctypes.data_as(ip), bv.ctypes.data_as(ip), ba.ctypes.data_as(ip)) == 0
    return vxyz, ev, bv, ba


def _om(m):
    class OM:
        pass
    om = OM()
    om.dim, om.p, om.ne, om.nl, om.verts, om.dofmap, om.ess = m.dim, m.order, m.ne, m.nl, m.verts, m.dofmap, m.ess
    om.bdr = np.zeros(m.nl, dtype=np.int32)
    om.bdr[m.ess] = 1
    return om


# ---- CPU --------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["square", "circle"])
def test_fixture_is_the_reference_mesh(msh, name):
    """The product reader gives bitwise the same topology and order-3 space from the fixture's file
    as from the reference's own file (skipped where /root/reference is absent, e.g. the GPU box)."""
    ref = R.reference_file(name)
    if ref is None:
        pytest.skip("/root/reference not present")
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_reference_meshes as MK
    raw = MK.parse_msh(ref)
    fx = R.load(name)
    for k in ("node_id", "node_xyz", "elem_id", "elem_type", "elem_phys", "elem_geom", "elem_nodes"):
        np.testing.assert_array_equal(fx[k], raw[k])
    assert fx["physical"] == raw["physical"]
    for a, b in zip(_topology(ref), _topology(msh[name])):
        np.testing.assert_array_equal(a, b)
    m0, m1 = cdfem.gmsh_mesh(ref, ORDER), cdfem.gmsh_mesh(msh[name], ORDER)
    for k in ("verts", "dofmap", "ess", "dof_xyz", "bdr_mask"):
        np.testing.assert_array_equal(getattr(m0, k), getattr(m1, k))


@pytest.mark.parametrize("name", ["square", "circle"])
def test_reference_mesh_sizes(msh, name):
    ntri, nvert, nbdr = R.SIZES[name]
    vxyz, ev, bv, ba = _topology(msh[name])
    assert (len(ev), len(vxyz), len(bv)) == (ntri, nvert, nbdr)
    want_attrs = {1, 2, 3, 4} if name == "square" else {1}
    assert set(ba.tolist()) == want_attrs
    nedge = nvert + ntri - 1          # Euler, simply connected planar triangulation
    m = cdfem.gmsh_mesh(msh[name], ORDER)
    assert m.ne == ntri and m.nl == nvert + 2 * nedge + ntri
    # every boundary dof lies on the boundary curve, and the count is 3 per boundary edge (P3)
    xy = m.dof_xyz[m.ess]
    if name == "square":
        on = (np.abs(xy) < 1e-14) | (np.abs(xy - 1.0) < 1e-14)
        assert on.any(axis=1).all()
    else:
        assert np.abs(np.hypot(xy[:, 0], xy[:, 1]) - 1.0).max() < 2e-3   # P3 nodes on straight chords
    assert len(m.ess) == 3 * nbdr


def _mfem_numbering(node_xyz, tris, order):
    """Independent restatement of MFEM's H1 numbering of a triangle mesh read from a file:
    Mesh(file, 1, 1) -> Finalize -> CheckElementOrientation (clockwise: swap vertices 0, 1) ->
    MarkTriMeshForRefinement (Triangle::MarkEdge: longest edge first); FiniteElementSpace: vertex
    dofs, then (order-1) dofs per edge, edges numbered as GetElementToEdgeTable's DSTable first meets
    them, element by element, local edges (0,1),(1,2),(2,0), each edge's dofs along increasing vertex
    index; then element interiors.  Returns the product's dofmap layout (local order: vertices, edges
    (0,1),(0,2),(1,2), interior) for comparison."""
    P = node_xyz[:, :2]
    rot = []
    for t in tris:
        v = list(t)
        a, b, c = P[v[0]], P[v[1]], P[v[2]]
        if (b[0] - a[0]) * (c[1] - a[1]) - (b[1] - a[1]) * (c[0] - a[0]) < 0:
            v[0], v[1] = v[1], v[0]
        p0, p1, p2 = P[v[0]], P[v[1]], P[v[2]]
        d0 = (p1[0] - p0[0]) * (p1[0] - p0[0]) + (p1[1] - p0[1]) * (p1[1] - p0[1])
        d1 = (p2[0] - p1[0]) * (p2[0] - p1[0]) + (p2[1] - p1[1]) * (p2[1] - p1[1])
        d2 = (p2[0] - p0[0]) * (p2[0] - p0[0]) + (p2[1] - p0[1]) * (p2[1] - p0[1])
        if d0 >= d1 and d0 >= d2:
            pass
        elif d0 >= d1 or d1 < d2:
            v = [v[2], v[0], v[1]]
        else:
            v = [v[1], v[2], v[0]]
        rot.append(v)
    edges = {}
    for v in rot:
        for i, j in ((0, 1), (1, 2), (2, 0)):
            edges.setdefault((min(v[i], v[j]), max(v[i], v[j])), len(edges))
    nv, k = len(P), order - 1
    out = []
    for e, v in enumerate(rot):
        row = list(v)
        for i, j in ((0, 1), (0, 2), (1, 2)):
            a, b = v[i], v[j]
            base = nv + edges[(min(a, b), max(a, b))] * k
            row += [base + (q if a < b else k - 1 - q) for q in range(k)]
        if order == 3:
            row.append(nv + len(edges) * k + e)
        out.append(row)
    return np.array(out, dtype=np.int32)


@pytest.mark.parametrize("name", ["square", "circle"])
@pytest.mark.parametrize("order", [2, 3])
def test_dof_numbering_is_mfems(msh, name, order):
    fx = R.load(name)
    idx = {int(n): i for i, n in enumerate(fx["node_id"])}
    tris = [[idx[int(n)] for n in row] for row, t in zip(fx["elem_nodes"], fx["elem_type"]) if t == 2]
    want = _mfem_numbering(fx["node_xyz"], tris, order)
    m = cdfem.gmsh_mesh(msh[name], order)
    np.testing.assert_array_equal(m.dofmap, want)
    # the rotation is not the identity on these meshes (the test would not see a missing one)
    assert (want[:, :3] != np.array(tris)).any()


def test_reader_rejects_large_boundary_tags(tmp_path):
    """A boundary physical tag above 31 is an error, not a silently dropped boundary."""
    import gmsh_synth
    p = str(tmp_path / "sq.msh")
    gmsh_synth.write_square(p, 3)
    txt = open(p).read().replace("\n1 1 2 1 1 ", "\n1 1 2 100 100 ", 1)
    assert txt != open(p).read()
    bad = tmp_path / "tag100.msh"
    bad.write_text(txt)
    with pytest.raises(cdfem.CdfemError):
        cdfem.gmsh_mesh(str(bad), 1)


# ---- GPU --------------------------------------------------------------------------------------
def _gpu_system(ctx, m, name):
    kappa, s, c, kind, _, _, _ = CONFIGS[name]
    prm = O.mms_params(kind, 2, kappa=kappa, s=s, c=c, modes=(3, 3, 3), p=ORDER)
    ctx.upload_mesh(m)
    ctx.fa_setup(kinds=7, kappa=kappa, alpha=1.0, conv=c, mass=s)
    b = ctx.lf_assemble(O.mms_f(prm, ctx.quadrature_points(cdfem.RULE_LINEARFORM)).reshape(-1))
    u = np.zeros(m.nl)
    u[m.ess] = O.mms_u(prm, m.dof_xyz[m.ess])
    _, B = ctx.form_linear_system(u, b)
    return prm, B


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["square", "circle"])
def test_gpu_reference_default_configuration(gpu_ctx, msh, name):
    """The default run on the reference's mesh: iterations +-1 and MMS L2 error to 1e-6 relative
    against the oracle at the reference's tolerances; then both solved to rtol 1e-13: solutions
    within 1e-10 relative L2."""
    kappa, s, c, _, _, pc, max_it = CONFIGS[name]
    m = cdfem.gmsh_mesh(msh[name], ORDER)
    om = _om(m)
    prm, B = _gpu_system(gpu_ctx, m, name)
    Xo, io, eo = O.solve_mms_simplex(om, prm, kappa, s, c, max_it=max_it, pc=pc)
    X, ig = gpu_ctx.solve(B, method="gmres", pc=pc, restart=30, rel_tol=1e-10, abs_tol=1e-12, max_iter=max_it)
    assert io["converged"] and ig["converged"], (io, ig)
    assert abs(ig["iterations"] - io["iterations"]) <= 1, (ig, io)
    eg = O.l2_error_simplex(om, X, prm)
    assert abs(eg - eo) <= 1e-6 * eo, (eg, eo)
    # tight: both to rtol 1e-13
    Xt, it = gpu_ctx.solve(B, method="gmres", pc=pc, restart=30, rel_tol=1e-13, abs_tol=0.0, max_iter=20000)
    Xot, iot = O.solve_mms_simplex(om, prm, kappa, s, c, tol=1e-13, atol=0.0, max_it=20000, pc=pc)[:2]
    assert it["converged"] and iot["converged"], (it, iot)
    assert np.linalg.norm(Xt - Xot) <= 1e-10 * np.linalg.norm(Xot)


def _run_driver(args, opts_text, tmp_path, np_ranks=0):
    opts = tmp_path / "petsc.opts"
    opts.write_text(opts_text)
    cmd = [EXE, *args, "-opts", str(opts)]
    if np_ranks:
        cmd = [MPIEXEC, "-n", str(np_ranks), *cmd]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    return {k: float(v) for k, v in (ln.split() for ln in r.stdout.splitlines())}


def _driver_args(name, path):
    kappa, s, c, _, _, _, _ = CONFIGS[name]
    a = ["-d", "2", "-mesh", path, "-p", str(ORDER), "-k", repr(kappa), "-s", repr(s),
         "-c", f"{c[0]!r},{c[1]!r},0", "-m", "3,3,3"]
    return a + (["-mms", "radial"] if name == "circle" else [])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["square", "circle"])
def test_gpu_reference_driver_one_rank(msh, tmp_path, name):
    """The MFEM-shaped C++ driver (cpp/convection_diffusion.cpp, the reference driver's hot-path text)
    on the reference mesh with the reference's options file, against the oracle."""
    kappa, s, c, _, opts, pc, max_it = CONFIGS[name]
    out = _run_driver(_driver_args(name, msh[name]), opts, tmp_path)
    m = cdfem.gmsh_mesh(msh[name], ORDER)
    om = _om(m)
    prm = O.mms_params(CONFIGS[name][3], 2, kappa=kappa, s=s, c=c, modes=(3, 3, 3), p=ORDER)
    _, io, eo = O.solve_mms_simplex(om, prm, kappa, s, c, max_it=max_it, pc=pc)
    assert int(out["dofs"]) == m.nl and int(out["ranks"]) == 1
    assert out["converged"] == 1 and abs(out["iterations"] - io["iterations"]) <= 1, (out, io)
    assert abs(out["l2_abs"] - eo) <= 1e-6 * eo


@pytest.mark.gpu
def test_gpu_reference_square_mpi2(msh, tmp_path):
    """`mpiexec -n 2` of the square's default run (ParMesh(MPI_COMM_WORLD, *mesh) partition, shared
    dofs summed across ranks) against one rank: same dofs, iterations +-2, L2 to 1e-7."""
    args = _driver_args("square", msh["square"])
    one = _run_driver(args, PETSC_OPTS, tmp_path)
    two = _run_driver(args, PETSC_OPTS, tmp_path, np_ranks=2)
    assert int(two["ranks"]) == 2 and two["dofs"] == one["dofs"]
    assert two["converged"] == 1 and abs(two["iterations"] - one["iterations"]) <= 2
    assert abs(two["l2_abs"] - one["l2_abs"]) <= 1e-7 * one["l2_abs"]


@pytest.mark.gpu
def test_gpu_reference_circle_mpi2_block_jacobi(msh, tmp_path):
    """`mpiexec -n 2` of the circle's default run with its own options file (Input/petsc_circle.opts:
    bjacobi, one ILU(0) block per rank) against the oracle's block-Jacobi restatement on the same
    partition (ParMesh's recursive coordinate bisection, the owned dofs of each rank in its local
    order): iterations +-1, MMS L2 error to 1e-6 relative."""
    kappa, s, c, kind, opts, _, max_it = CONFIGS["circle"]
    two = _run_driver(_driver_args("circle", msh["circle"]), opts, tmp_path, np_ranks=2)
    m = cdfem.gmsh_mesh(msh["circle"], ORDER)
    part = cdfem.partition_rcb(m, 2)
    blocks = []
    for r in range(2):
        ls = cdfem.local_space(m, part, r)
        blocks.append(ls.l2g[ls.n_not_owned:])
    prm = O.mms_params(kind, 2, kappa=kappa, s=s, c=c, modes=(3, 3, 3), p=ORDER)
    _, io, eo = O.solve_mms_simplex(_om(m), prm, kappa, s, c, max_it=max_it, pc="ilu", blocks=blocks)
    assert int(two["ranks"]) == 2 and int(two["dofs"]) == m.nl
    assert two["converged"] == 1 and abs(two["iterations"] - io["iterations"]) <= 1, (two, io)
    assert abs(two["l2_abs"] - eo) <= 1e-6 * eo


# ---- the reference's transient configurations on its own mesh -------------------------------------
# Input/input_diffusion_mms.yaml:6-14 (diffusion_mms.cpp) and Input/input.yaml:1-8
# (linear_convection_diffusion_1D.cpp) both read Mesh/unit_square.msh with Input/petsc.opts.
LIB = os.path.join(ROOT, "continuum-mechanics-mfem_amd", "lib")


def _refine(vxyz, ev, bv, ba):
    """One Mesh::UniformRefinement of a triangle mesh: a vertex at every edge midpoint, four children
    per triangle (orientation kept), two per boundary edge (attribute kept).  The numbering differs
    from MFEM's; Jacobi-GMRES iterations and L2 errors do not depend on it beyond rounding."""
    nv = len(vxyz)
    edges = {}

    def mid(a, b):
        return edges.setdefault((min(a, b), max(a, b)), nv + len(edges))
    tris = []
    for a, b, c in ev:
        ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
        tris += [(a, ab, ca), (ab, b, bc), (ca, bc, c), (ab, bc, ca)]
    bes, bas = [], []
    for (a, b), t in zip(bv, ba):
        m_ = mid(a, b)
        bes += [(a, m_), (m_, b)]
        bas += [t, t]
    out = np.zeros((nv + len(edges), vxyz.shape[1]))
    out[:nv] = vxyz
    for (a, b), i in edges.items():
        out[i] = 0.5 * (vxyz[a] + vxyz[b])
    return out, np.array(tris, dtype=np.int32), np.array(bes, dtype=np.int32), np.array(bas, dtype=np.int32)


def _space(vxyz, ev, bv, ba, order):
    """cdfem_simplex_space on a topology: the oracle's mesh container, essential dofs on every
    boundary attribute."""
    import ctypes as C
    L = cdfem.lib()
    dim, ne, nbe = vxyz.shape[1], len(ev), len(bv)
    dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
    vx = np.ascontiguousarray(vxyz, dtype=np.float64)
    e, b, a = (np.ascontiguousarray(z, dtype=np.int32) for z in (ev, bv, ba))
    nl = C.c_int64()
    assert L.cdfem_simplex_space_sizes(dim, len(vx), vx.ctypes.data_as(dp), ne, e.ctypes.data_as(ip), order,
                                       C.byref(nl)) == 0
    nd = (order + 1) * (order + 2) // 2
    verts = np.zeros((ne, dim + 1, dim))
    dofs = np.zeros((ne, nd), dtype=np.int32)
    mask = np.zeros(nl.value, dtype=np.int32)
    xyz = np.zeros((nl.value, dim))
    assert L.cdfem_simplex_space(dim, len(vx), vx.ctypes.data_as(dp), ne, e.ctypes.data_as(ip), nbe,
                                 b.ctypes.data_as(ip), a.ctypes.data_as(ip), order, verts.ctypes.data_as(dp),
                                 dofs.ctypes.data_as(ip), mask.ctypes.data_as(ip), xyz.ctypes.data_as(dp)) == 0

    class OM:
        pass
    om = OM()
    om.dim, om.p, om.ne, om.nl, om.verts, om.dofmap = dim, order, ne, nl.value, verts, dofs
    om.ess = np.nonzero(mask)[0].astype(np.int32)
    om.bdr = (mask != 0).astype(np.int32)
    return om


@pytest.mark.gpu
def test_gpu_reference_diffusion_mms_configuration(msh, tmp_path):
    """Input/input_diffusion_mms.yaml end to end: Mesh/unit_square.msh refined once
    (serial_ref_levels 1: 3,752 triangles), order 1, alpha 0.1, dt 0.05, t_final 2.0 (40 backward-
    Euler steps of diffusion_mms.cpp:425-463), Input/petsc.opts.  The C++ driver on the GPU against the
    oracle's time loop on the same refined mesh: GMRES iterations within one per step, final L2
    error to 1e-6 relative."""
    sys.path.insert(0, os.path.dirname(__file__))
    from test_cpp_driver import _oracle_diffusion_mms
    opts = tmp_path / "petsc.opts"
    opts.write_text(PETSC_OPTS)
    r = subprocess.run([os.path.join(LIB, "diffusion_mms"), "-mesh", msh["square"], "-p", "1", "-rs", "1",
                        "-a", "0.1", "-dt", "0.05", "-T", "2.0", "-opts", str(opts)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    out = {k: float(v) for k, v in (ln.split() for ln in r.stdout.splitlines())}
    om = _space(*_refine(*_topology(msh["square"])), 1)
    assert om.ne == 4 * 938 and int(out["dofs"]) == om.nl
    l2, its, nsteps = _oracle_diffusion_mms(om, True, 0.1, 0.05, 2.0)
    assert int(out["steps"]) == nsteps == 40
    assert abs(out["gmres_iterations"] - its) <= nsteps, (out, its)
    assert abs(out["final_l2"] - l2) <= 1e-6 * l2, (out, l2)


@pytest.mark.gpu
def test_gpu_reference_three_peclet_configuration(msh, tmp_path):
    """Input/input.yaml end to end: Mesh/unit_square.msh, order 3, dt 1e-3, t_final 1.0 (1000 steps
    of three backward-Euler systems, Pe = 1, 10, 100; linear_convection_diffusion_1D.cpp:375-400,
    537-576), Input/petsc.opts.  The C++ driver on the GPU against the oracle's loop
    (oracle.transient_three_peclet) on the same mesh: per block final absolute and relative L2 errors
    to 1e-6, GMRES iterations within one per step and block."""
    opts = tmp_path / "petsc.opts"
    opts.write_text(PETSC_OPTS)
    r = subprocess.run([os.path.join(LIB, "convection_diffusion_1d"), "-mesh", msh["square"], "-p", "3",
                        "-dt", "1e-3", "-T", "1.0", "-opts", str(opts)],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr
    out = {k: float(v) for k, v in (ln.split() for ln in r.stdout.splitlines())}
    m = cdfem.gmsh_mesh(msh["square"], 3)
    errs, its, nsteps, _ = O.transient_three_peclet(_om(m), 1e-3, 1.0, simplex=True)
    assert int(out["steps"]) == nsteps == 1000 and int(out["dofs"]) == m.nl
    for k in range(3):
        a, rel = errs[k]
        assert abs(out[f"abs_l2_pe{k + 1}"] - a) <= 1e-6 * a, (k, out, errs)
        assert abs(out[f"rel_l2_pe{k + 1}"] - rel) <= 1e-6 * rel
    assert abs(out["gmres_iterations"] - sum(its)) <= 3 * nsteps, (out, its)
