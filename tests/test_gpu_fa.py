"""GPU full assembly on simplices (BASELINE config C4) against the oracle.

The GPU assembles the CSR itself (cdfem_fa_setup), with element matrices, a deterministic gather
and the elimination all running on the device. Checks:
  * the CSR pattern (row pointers, sorted columns) equals the oracle's exactly;
  * the values agree to 1e-13 of max|A|, for both A and the FormLinearSystem matrix;
  * Mult, the constrained Mult, the diagonal and FormLinearSystem on the CSR operator agree to 1e-13;
  * GMRES(30)+Jacobi (the reference's solver) and CG agree with the oracle's solvers on the same
    systems, at the tolerances of tests/test_gpu_gmres.py;
  * the MMS solve through the GPU path has the oracle's L2 error;
  * repeated assembly is bitwise identical;
  * at the full C4 size (55^3 x 6 tets, P2, 1.37 M DoFs), size-independent properties hold.
"""
import numpy as np
import pytest

import cdfem
from oracle import oracle as O

pytestmark = pytest.mark.gpu
C3 = (1.0, -2.0, 0.5)


def _kinds_o(k):
    return (O.DIFFUSION if k & 1 else 0) | (O.CONVECTION if k & 2 else 0) | (O.MASS if k & 4 else 0)


def _setup(gpu_ctx, dim, n, p, pert, kinds=7):
    gm = cdfem.kuhn_mesh(dim, n, p, perturb=pert)
    om = O.KuhnMesh(dim, n, p)                 # container for the same arrays
    om.verts, om.dofmap = gm.verts, gm.dofmap
    gpu_ctx.upload_mesh(gm)
    c = C3[:dim]
    gpu_ctx.fa_setup(kinds=kinds, kappa=0.1, alpha=1.0, conv=c, mass=1.0)
    A = O.fa_assemble_simplex(om, kappa=0.1, alpha=1.0, s=1.0, c=c, kinds=_kinds_o(kinds))
    return gm, om, A


CASES = [(3, 3, 2, 0.15), (3, 4, 1, 0.1), (2, 6, 2, 0.2), (2, 5, 1, 0.0), (3, 2, 2, 0.0)]


@pytest.mark.parametrize("dim,n,p,pert", CASES)
@pytest.mark.parametrize("kinds", [7, 5, 2])
def test_fa_csr_parity(gpu_ctx, dim, n, p, pert, kinds):
    gm, om, A = _setup(gpu_ctx, dim, n, p, pert, kinds)
    rp, cols, vals = gpu_ctx.fa_csr()
    orp, ocol, oval = A.export()
    np.testing.assert_array_equal(rp, orp)
    np.testing.assert_array_equal(cols, ocol)
    assert np.abs(vals - oval).max() <= 1e-13 * np.abs(oval).max()
    Ac, _ = O.form_linear_system(A, om.bdr, np.zeros(om.nl), np.zeros(om.nl))
    _, _, cvals = gpu_ctx.fa_csr(constrained=True)
    _, _, ocv = Ac.export()
    assert np.abs(cvals - ocv).max() <= 1e-13 * np.abs(ocv).max()


@pytest.mark.parametrize("dim,n,p,pert", CASES[:3])
def test_fa_operator_parity(gpu_ctx, dim, n, p, pert):
    gm, om, A = _setup(gpu_ctx, dim, n, p, pert)
    rng = np.random.default_rng(3)
    x = rng.uniform(-1, 1, om.nl)
    yo = A.mult(x)
    assert np.abs(gpu_ctx.mult(x) - yo).max() <= 1e-13 * np.abs(yo).max()
    xz = x.copy()
    xz[om.ess] = 0.0
    yc = A.mult(xz)
    yc[om.ess] = x[om.ess]
    assert np.abs(gpu_ctx.mult(x, constrained=True) - yc).max() <= 1e-13 * np.abs(yc).max()
    d = gpu_ctx.diagonal()
    assert np.abs(d - A.diag()).max() <= 1e-13 * np.abs(A.diag()).max()
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    _, Bo = O.form_linear_system(A, om.bdr, u, b)
    _, B = gpu_ctx.form_linear_system(u, b)
    assert np.abs(B - Bo).max() <= 1e-13 * np.abs(Bo).max()


@pytest.mark.parametrize("dim,n,p,pert", [(3, 4, 2, 0.1), (2, 8, 1, 0.15)])
def test_fa_gmres_parity(gpu_ctx, dim, n, p, pert):
    gm, om, A = _setup(gpu_ctx, dim, n, p, pert)
    rng = np.random.default_rng(8)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    _, B = gpu_ctx.form_linear_system(u, b)
    dinv = 1.0 / Ac.diag()
    # fixed steps across restarts
    xo, io = O.gmres(Ac, Bo, dinv=dinv, restart=7, rtol=0.0, atol=0.0, max_it=25)
    xg, ig = gpu_ctx.solve(B, method="gmres", restart=7, rel_tol=0.0, abs_tol=0.0, max_iter=25)
    assert io["iterations"] == ig["iterations"] == 25
    assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)
    # the reference's settings (Input/petsc.opts)
    xo, io = O.gmres(Ac, Bo, dinv=dinv, restart=30, rtol=1e-10, atol=1e-12, max_it=500)
    xg, ig = gpu_ctx.solve(B, method="gmres", restart=30, rel_tol=1e-10, abs_tol=1e-12, max_iter=500)
    assert io["converged"] and ig["converged"] and abs(io["iterations"] - ig["iterations"]) <= 1
    assert np.linalg.norm(xg - xo) <= 1e-8 * np.linalg.norm(xo)


class _DelaunayOM:
    """Oracle container for a product simplex Mesh (the Delaunay mesh of cdfem.delaunay_cube)."""

    def __init__(self, m):
        self.dim, self.p, self.ne, self.nl = m.dim, m.order, m.ne, m.nl
        self.verts, self.dofmap, self.ess = m.verts, m.dofmap, m.ess
        self.bdr = np.zeros(m.nl, dtype=np.int32)
        self.bdr[m.ess] = 1


@pytest.mark.parametrize("order", [1, 2])
def test_fa_delaunay_parity(order):
    """BASELINE configs[3] on genuinely unstructured connectivity (the c4u bench mesh family): a
    Delaunay tetrahedralisation of random points in the unit cube (cdfem.delaunay_cube, 3000 points,
    ~16.6 K tets), in Qhull's unbanded point order, so the FA setup picks the geometric SpMV order
    and the Krylov solve runs permuted.  Against the oracle: the CSR pattern exact, values and the
    constrained Mult to 1e-13, 25 fixed GMRES(7) iterates to 1e-11, the reference's GMRES settings
    (iterations +-1, solutions to 1e-8) and both solved to rtol 1e-13 to 1e-10."""
    gm = cdfem.simplex_space(*cdfem.delaunay_cube(3000, seed=5), order)
    om = _DelaunayOM(gm)
    A = O.fa_assemble_simplex(om, kappa=0.1, alpha=1.0, s=1.0, c=C3)
    with cdfem.Context(0) as ctx:
        ctx.upload_mesh(gm)
        ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
        rp, cols, vals = ctx.fa_csr()
        orp, ocol, oval = A.export()
        np.testing.assert_array_equal(rp, orp)
        np.testing.assert_array_equal(cols, ocol)
        assert np.abs(vals - oval).max() <= 1e-13 * np.abs(oval).max()
        rng = np.random.default_rng(9)
        x = rng.uniform(-1, 1, om.nl)
        xz = x.copy()
        xz[om.ess] = 0.0
        yc = A.mult(xz)
        yc[om.ess] = x[om.ess]
        assert np.abs(ctx.mult(x, constrained=True) - yc).max() <= 1e-13 * np.abs(yc).max()
        u = np.zeros(om.nl)
        u[om.ess] = rng.uniform(-1, 1, len(om.ess))
        b = rng.uniform(-1, 1, om.nl)
        Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
        _, B = ctx.form_linear_system(u, b)
        assert np.abs(B - Bo).max() <= 1e-13 * np.abs(Bo).max()
        dinv = 1.0 / Ac.diag()
        xo, io = O.gmres(Ac, Bo, dinv=dinv, restart=7, rtol=0.0, atol=0.0, max_it=25)
        xg, ig = ctx.solve(B, method="gmres", restart=7, rel_tol=0.0, abs_tol=0.0, max_iter=25)
        assert io["iterations"] == ig["iterations"] == 25
        assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)
        xo, io = O.gmres(Ac, Bo, dinv=dinv, restart=30, rtol=1e-10, atol=1e-12, max_it=2000)
        xg, ig = ctx.solve(B, method="gmres", restart=30, rel_tol=1e-10, abs_tol=1e-12, max_iter=2000)
        assert io["converged"] and ig["converged"] and abs(io["iterations"] - ig["iterations"]) <= 1
        assert np.linalg.norm(xg - xo) <= 1e-8 * np.linalg.norm(xo)
        xo, io = O.gmres(Ac, Bo, dinv=dinv, restart=30, rtol=1e-13, atol=0.0, max_it=4000)
        xg, ig = ctx.solve(B, method="gmres", restart=30, rel_tol=1e-13, abs_tol=0.0, max_iter=4000)
        assert io["converged"] and ig["converged"]
        assert np.linalg.norm(xg - xo) <= 1e-10 * np.linalg.norm(xo)


def test_fa_cg_parity(gpu_ctx):
    gm, om, A = _setup(gpu_ctx, 3, 4, 2, 0.1, kinds=5)   # kappa K + s M: SPD
    rng = np.random.default_rng(4)
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, np.zeros(om.nl), b)
    _, B = gpu_ctx.form_linear_system(np.zeros(om.nl), b)
    dinv = 1.0 / Ac.diag()
    xo, io = O.cg(Ac, Bo, dinv=dinv, rel_tol=0.0, abs_tol=0.0, max_iter=40)
    xg, ig = gpu_ctx.solve(B, method="cg", rel_tol=0.0, abs_tol=0.0, max_iter=40, check_every=9)
    assert io["iterations"] == ig["iterations"] == 40
    assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)
    xo, io = O.cg(Ac, Bo, dinv=dinv, rel_tol=1e-13, max_iter=2000)
    xg, ig = gpu_ctx.solve(B, method="cg", rel_tol=1e-13, max_iter=2000)
    assert io["converged"] and ig["converged"] and abs(io["iterations"] - ig["iterations"]) <= 2
    assert np.linalg.norm(xg - xo) <= 1e-10 * np.linalg.norm(xo)


def test_fa_mms_matches_oracle(gpu_ctx):
    """C4 driver sequence on the GPU (FA + FormLinearSystem + GMRES/Jacobi) vs the oracle's."""
    dim, n, p = 3, 5, 2
    gm = cdfem.kuhn_mesh(dim, n, p)
    om = O.KuhnMesh(dim, n, p)
    prm = O.mms_params(O.MMS_SIN, 3, kappa=0.1, s=1.0, c=C3, modes=(1, 1, 1), p=p)
    Xo, io, eo = O.solve_mms_simplex(om, prm, 0.1, 1.0, C3)
    b = O.lf_assemble_simplex(om, prm)         # the linear form is not on the GPU path for simplices
    u = np.zeros(om.nl)
    u[om.ess] = O.mms_u(prm, gm.dof_xyz[om.ess])
    gpu_ctx.upload_mesh(gm)
    gpu_ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    _, B = gpu_ctx.form_linear_system(u, b)
    X, ig = gpu_ctx.solve(B, method="gmres", restart=30, rel_tol=1e-10, abs_tol=1e-12, max_iter=500)
    assert ig["converged"] and abs(ig["iterations"] - io["iterations"]) <= 1
    eg = O.l2_error_simplex(om, X, prm)
    assert abs(eg - eo) <= 1e-6 * eo


def test_fa_reproducible_and_coefficient_arrays(gpu_ctx):
    gm, om, A = _setup(gpu_ctx, 3, 3, 2, 0.1)
    _, _, v1 = gpu_ctx.fa_csr()
    gpu_ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    _, _, v2 = gpu_ctx.fa_csr()
    np.testing.assert_array_equal(v1, v2)
    # MFEM's per-integrator rules on P2 tets: diffusion order 2 (4 points), convection / mass order 4
    # (11 points); the operator rule of the tensor elements does not exist here
    nqd, nqc, nqm = (gpu_ctx.rule_size(r) for r in (cdfem.RULE_DIFFUSION, cdfem.RULE_CONVECTION, cdfem.RULE_MASS))
    assert (nqd, nqc, nqm) == (4, 11, 11)
    with pytest.raises(cdfem.CdfemError):
        gpu_ctx.rule_size(cdfem.RULE_OPERATOR)
    xyz = gpu_ctx.quadrature_points(cdfem.RULE_DIFFUSION)
    assert xyz.shape == (gm.ne, nqd, 3)
    gpu_ctx.fa_setup(kinds=7, kappa=0.0, kappa_q=np.full(gm.ne * nqd, 0.1), alpha=1.0,
                     conv_q=np.tile(np.array(C3), gm.ne * nqc), mass=0.0, mass_q=np.full(gm.ne * nqm, 1.0))
    _, _, v3 = gpu_ctx.fa_csr()
    assert np.abs(v3 - v1).max() <= 1e-14 * np.abs(v1).max()
    # a variable kappa(x) = 1 + x: x^T K 1 = 0 still (constants in the kernel), K symmetric
    kq = 1.0 + xyz[..., 0].ravel()
    gpu_ctx.fa_setup(kinds=1, kappa=0.0, kappa_q=kq)
    rng = np.random.default_rng(0)
    x, y = rng.uniform(-1, 1, gm.nl), rng.uniform(-1, 1, gm.nl)
    assert np.abs(gpu_ctx.mult(np.ones(gm.nl))).max() <= 1e-13
    assert abs(x @ gpu_ctx.mult(y) - y @ gpu_ctx.mult(x)) <= 1e-12 * np.abs(x @ gpu_ctx.mult(y))


def test_fa_pa_setup_rejected_on_simplex(gpu_ctx):
    gm = cdfem.kuhn_mesh(3, 2, 2)
    gpu_ctx.upload_mesh(gm)
    with pytest.raises(cdfem.CdfemError) as ei:
        gpu_ctx.pa_setup(kinds=7, kappa=0.1, conv=C3, mass=1.0)
    assert ei.value.code == cdfem.ERR_UNSUPPORTED


def test_fa_c4_full_size_properties(gpu_ctx):
    """55^3 x 6 tets, P2 (1,367,631 DoFs): kernel of D+C, mass = volume, D symmetric, GMRES runs."""
    gm = cdfem.kuhn_mesh(3, 55, 2, perturb=0.1, with_coords=False)
    gpu_ctx.upload_mesh(gm)
    one = np.ones(gm.nl)
    gpu_ctx.fa_setup(kinds=3, kappa=0.1, alpha=1.0, conv=C3)
    assert np.abs(gpu_ctx.mult(one)).max() <= 1e-12
    gpu_ctx.fa_setup(kinds=4, mass=1.0)
    assert abs(one @ gpu_ctx.mult(one) - 1.0) <= 1e-11
    gpu_ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
    rp, cols, vals = gpu_ctx.fa_csr()
    assert rp[-1] == len(cols) and (np.diff(rp) > 0).all()
    b = np.random.default_rng(1).uniform(-1, 1, gm.nl)
    _, B = gpu_ctx.form_linear_system(np.zeros(gm.nl), b)
    # 10 full GMRES(30) cycles: the Givens residual estimate must be the true preconditioned
    # residual of the returned iterate (size-independent consistency of the whole solver path)
    X, info = gpu_ctx.solve(B, method="gmres", restart=30, rel_tol=0.0, abs_tol=0.0, max_iter=300)
    assert info["iterations"] == 300
    r = B - gpu_ctx.mult(X, constrained=True)
    d = gpu_ctx.diagonal()
    dinv = np.where(np.isin(np.arange(gm.nl), gm.ess), 1.0, 1.0 / d)
    true = np.linalg.norm(dinv * r)
    assert abs(true - info["final_norm"]) <= 1e-6 * true
    assert info["final_norm"] <= 1e-3 * info["initial_norm"]


def test_fa_spmv_mixed_columns_bitwise():
    """Mixed SELL columns: slices whose rows reach a column beyond 16 bits of their own row (an
    unstructured mesh's far neighbours) stream 32-bit columns, the rest 16-bit deltas.  A Kuhn P2
    numbering with 3 far-apart dof pairs swapped (69 K dofs, natural SpMV order) makes a few slices
    wide: Mult, the constrained Mult and 40 GMRES iterates are bitwise the all-32-bit ones, and the
    SpMV's byte count lies strictly between the all-16-bit and all-32-bit counts."""
    gm = cdfem.kuhn_mesh(3, 20, 2, perturb=0.05)
    rng = np.random.default_rng(12)
    lab = np.arange(gm.nl, dtype=np.int32)
    for _ in range(3):
        i = int(rng.integers(0, gm.nl // 4))
        j = int(rng.integers(3 * gm.nl // 4, gm.nl))
        lab[i], lab[j] = lab[j], lab[i]
    m = cdfem.Mesh(gm.dim, gm.order, gm.verts, lab[gm.dofmap], gm.nl, np.sort(lab[gm.ess]), None, simplex=True)
    x = rng.uniform(-1, 1, m.nl)
    b = rng.uniform(-1, 1, m.nl)
    res = {}
    for idx16 in (1, 0):
        with cdfem.Context(0) as ctx:
            ctx.set_option("sell_order", 0)          # natural order: the swapped labels stay far
            ctx.set_option("spmv_index16", idx16)
            ctx.upload_mesh(m)
            ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            _, B = ctx.form_linear_system(np.zeros(m.nl), b)
            X, _ = ctx.solve(B, method="gmres", restart=30, rel_tol=0.0, abs_tol=0.0, max_iter=40)
            nnz = len(ctx.fa_csr()[1])
            res[idx16] = (ctx.mult(x), ctx.mult(x, constrained=True), X, ctx.kernel_bytes(cdfem.K_APPLY))
    for a, c in zip(res[1][:3], res[0][:3]):
        np.testing.assert_array_equal(a, c)
    assert res[0][3] - 2.0 * nnz < res[1][3] < res[0][3]


@pytest.mark.parametrize("mesh,order", [("kuhn", 1), ("delaunay", 2), ("delaunay", 6)])
def test_fa_spmv_lds_windows_bitwise(mesh, order):
    """LDS-staged SpMV windows (set_option "spmv_lds": each workgroup stages its window's distinct
    columns in LDS and the entries read x there through 16-bit window positions) give the windowed
    layout's row sums bit for bit: Mult, the constrained Mult and 40 GMRES iterates are bitwise those
    of the same windowed layout without LDS, on the Kuhn lattice (natural windows) and on an
    unstructured Delaunay mesh (RCM and Morton windows), at two window sizes.  The FA CG's den sums
    its per-workgroup partials, whose grouping follows the launch, so its 30 iterates agree to 1e-12."""
    if mesh == "kuhn":
        m = cdfem.kuhn_mesh(3, 14, 2, perturb=0.1)
    else:
        m = cdfem.simplex_space(*cdfem.delaunay_cube(6000, seed=4), 2)
    rng = np.random.default_rng(17)
    x = rng.uniform(-1, 1, m.nl)
    b = rng.uniform(-1, 1, m.nl)
    for win in (512, 1024):
        res = {}
        for lds in (0, win):
            with cdfem.Context(0) as ctx:
                ctx.set_option("sell_order", order)
                ctx.set_option("sell_window", win)
                ctx.set_option("spmv_lds", lds)
                ctx.upload_mesh(m)
                ctx.fa_setup(kinds=5, kappa=0.1, mass=1.0)
                _, Bs = ctx.form_linear_system(np.zeros(m.nl), b)
                Xc, _ = ctx.solve(Bs, method="cg", rel_tol=0.0, abs_tol=0.0, max_iter=30)
                ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
                _, B = ctx.form_linear_system(np.zeros(m.nl), b)
                X, _ = ctx.solve(B, method="gmres", restart=30, rel_tol=0.0, abs_tol=0.0, max_iter=40)
                res[lds] = (ctx.mult(x), ctx.mult(x, constrained=True), X, Xc)
        for k, name in enumerate(("mult", "constrained mult", "gmres")):
            np.testing.assert_array_equal(res[0][k], res[win][k], err_msg=name)
        assert np.linalg.norm(res[win][3] - res[0][3]) <= 1e-12 * np.linalg.norm(res[0][3])


@pytest.mark.parametrize("order", [6, 2])
def test_fa_spmv_lanes_per_row(order):
    """LDS-staged layouts with 2 or 4 lanes per row (set_option "spmv_lpr": each lane sums a contiguous
    part of its row, the parts combined in a fixed order) on an unstructured Delaunay mesh (Morton and
    RCM windows): Mult and the constrained Mult agree with the oracle's CSR to 1e-13 and with one lane
    per row to 1e-14, 40 GMRES iterates with one lane per row to 1e-11, and repeated products are
    bitwise equal."""
    m = cdfem.simplex_space(*cdfem.delaunay_cube(6000, seed=8), 2)
    om = _DelaunayOM(m)
    A = O.fa_assemble_simplex(om, kappa=0.1, alpha=1.0, s=1.0, c=C3)
    rng = np.random.default_rng(19)
    x = rng.uniform(-1, 1, m.nl)
    b = rng.uniform(-1, 1, m.nl)
    yo = A.mult(x)
    res = {}
    for lpr in (1, 2, 4):
        with cdfem.Context(0) as ctx:
            ctx.set_option("sell_order", order)
            ctx.set_option("sell_window", 512)
            ctx.set_option("spmv_lds", 512)
            ctx.set_option("spmv_lpr", lpr)
            ctx.upload_mesh(m)
            ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            assert ctx.kernel_name(cdfem.K_APPLY) == "k_sell_spmv_lds"
            y = ctx.mult(x)
            np.testing.assert_array_equal(y, ctx.mult(x))
            _, B = ctx.form_linear_system(np.zeros(m.nl), b)
            X, _ = ctx.solve(B, method="gmres", restart=30, rel_tol=0.0, abs_tol=0.0, max_iter=40)
            res[lpr] = (y, ctx.mult(x, constrained=True), X)
        assert np.abs(y - yo).max() <= 1e-13 * np.abs(yo).max()
    for lpr in (2, 4):
        for k in (0, 1):
            assert np.abs(res[lpr][k] - res[1][k]).max() <= 1e-14 * np.abs(res[1][k]).max()
        assert np.linalg.norm(res[lpr][2] - res[1][2]) <= 1e-11 * np.linalg.norm(res[1][2])


def test_fa_spmv_index16_matches_int32(gpu_ctx):
    """The SpMV's 16-bit column deltas (set_option "spmv_index16", the default) give the same bits
    as 32-bit columns, for Mult, the constrained Mult and a CG solve.  A random DoF numbering
    (bandwidth > 2^15) falls back to 32-bit columns when the SpMV keeps the mesh's base order
    (sell_order 1) and is brought back into 16 bits by the reverse Cuthill-McKee order (sell_order 3,
    the auto order without LDS staging); both give the permuted result."""
    gm = cdfem.kuhn_mesh(3, 16, 2, perturb=0.1)      # 35,937 DoFs, lattice bandwidth 2,180
    rng = np.random.default_rng(16)
    x = rng.uniform(-1, 1, gm.nl)
    b = rng.uniform(-1, 1, gm.nl)
    res = {}
    gpu_ctx.set_option("sell_order", 3)              # the SELL paths that stream column deltas
    try:
        for flag in (1, 0):
            gpu_ctx.set_option("spmv_index16", flag)
            gpu_ctx.upload_mesh(gm)
            gpu_ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            _, B = gpu_ctx.form_linear_system(np.zeros(gm.nl), b)
            X, info = gpu_ctx.solve(B, method="gmres", restart=30, rel_tol=0.0, abs_tol=0.0, max_iter=40)
            res[flag] = (gpu_ctx.mult(x), gpu_ctx.mult(x, constrained=True), X,
                         gpu_ctx.kernel_bytes(cdfem.K_APPLY))
        for a, c in zip(res[1][:3], res[0][:3]):
            np.testing.assert_array_equal(a, c)
        nnz = len(gpu_ctx.fa_csr()[1])
        assert res[0][3] - res[1][3] == 2.0 * nnz       # 10 instead of 12 bytes per entry
        # random numbering
        gpu_ctx.set_option("spmv_index16", 1)
        perm = rng.permutation(gm.nl).astype(np.int32)
        xyzp = np.empty_like(gm.dof_xyz)
        xyzp[perm] = gm.dof_xyz
        gp = cdfem.Mesh(gm.dim, gm.order, gm.verts, perm[gm.dofmap], gm.nl, perm[gm.ess], xyzp,
                        simplex=True)
        xp = np.empty_like(x)
        xp[perm] = x
        y = res[1][0]
        # natural base order: the shuffled numbering puts some columns beyond 16 bits of their row ->
        # those slices stream 32-bit columns (mixed layout: between the two byte counts); auto
        # (default): the reverse Cuthill-McKee base order brings every delta back into 16 bits
        for order in (1, 3):
            gpu_ctx.set_option("sell_order", order)
            gpu_ctx.upload_mesh(gp)
            gpu_ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            nb = gpu_ctx.kernel_bytes(cdfem.K_APPLY)
            if order == 1:
                assert res[1][3] < nb < res[0][3]
            else:
                assert nb == res[1][3]
            yp = gpu_ctx.mult(xp)
            assert np.abs(yp[perm] - y).max() <= 1e-13 * np.abs(y).max()
    finally:
        gpu_ctx.set_option("spmv_index16", 1)
        gpu_ctx.set_option("sell_order", 8)


@pytest.mark.parametrize("dim,n,p,pert", [(2, 8, 2, 0.15), (3, 4, 2, 0.1), (2, 10, 1, 0.1)])
def test_fa_gmres_ilu_parity(gpu_ctx, dim, n, p, pert):
    """GMRES left-preconditioned with ILU(0) (Input/petsc_circle.opts: bjacobi + ilu, one block per
    rank) against the oracle's ILU(0) GMRES: fixed steps across restarts to 1e-11, converged to the
    reference's tolerances with the same iteration count (+-1); ILU needs fewer steps than Jacobi."""
    gm, om, A = _setup(gpu_ctx, dim, n, p, pert)
    rng = np.random.default_rng(11)
    u = np.zeros(om.nl)
    u[om.ess] = rng.uniform(-1, 1, len(om.ess))
    b = rng.uniform(-1, 1, om.nl)
    Ac, Bo = O.form_linear_system(A, om.bdr, u, b)
    _, B = gpu_ctx.form_linear_system(u, b)
    F = O.ilu0(Ac)
    xo, io = O.gmres_ilu(Ac, Bo, F, restart=7, rtol=0.0, atol=0.0, max_it=25)
    xg, ig = gpu_ctx.solve(B, method="gmres", pc="ilu", restart=7, rel_tol=0.0, abs_tol=0.0, max_iter=25)
    assert io["iterations"] == ig["iterations"] == 25
    assert np.linalg.norm(xg - xo) <= 1e-11 * np.linalg.norm(xo)
    xo, io = O.gmres_ilu(Ac, Bo, F, restart=30, rtol=1e-10, atol=1e-12, max_it=2000)
    xg, ig = gpu_ctx.solve(B, method="gmres", pc="ilu", restart=30, rel_tol=1e-10, abs_tol=1e-12, max_iter=2000)
    assert io["converged"] and ig["converged"] and abs(io["iterations"] - ig["iterations"]) <= 1
    assert np.linalg.norm(xg - xo) <= 1e-8 * np.linalg.norm(xo)
    _, ij = gpu_ctx.solve(B, method="gmres", pc="jacobi", restart=30, rel_tol=1e-10, abs_tol=1e-12, max_iter=2000)
    assert ig["iterations"] < ij["iterations"]
    # repeated solves reuse the factors and the captured sweep graph: bitwise identical
    xg2, _ = gpu_ctx.solve(B, method="gmres", pc="ilu", restart=30, rel_tol=1e-10, abs_tol=1e-12, max_iter=2000)
    np.testing.assert_array_equal(xg, xg2)


def test_ilu_rejected_for_cg_and_pa(gpu_ctx):
    gm, om, A = _setup(gpu_ctx, 2, 3, 1, 0.0)
    B = np.ones(om.nl)
    with pytest.raises(cdfem.CdfemError):
        gpu_ctx.solve(B, method="cg", pc="ilu")
    m = cdfem.box_mesh(2, 3, 1)
    gpu_ctx.upload_mesh(m)
    gpu_ctx.pa_setup(kinds=5, kappa=0.1, mass=1.0)
    with pytest.raises(cdfem.CdfemError):
        gpu_ctx.solve(np.ones(m.nl), method="gmres", pc="ilu")


@pytest.mark.parametrize("order", [2, 3, 4, 5, 1, 6, 8])
def test_fa_reordered_space_solves(gpu_ctx, order):
    """The SpMV order (sell_order: 1 natural + windows, 2 RCM + windows, 3 auto = geometric + global
    on a shuffled numbering, 4 RCM + global, 5 geometric + global, 6 Morton + windows, 8 = the
    default, Morton windows staged in LDS with 2 lanes per row) on a randomly relabelled Kuhn P2
    mesh: Krylov solves run in
    the permuted space (B in / X out permuted once per solve).  Against the mesh-order SpMV
    (sell_order 0) on the same shuffled mesh: Mult and constrained Mult to 1e-14 (a row sums its
    entries in space-column order instead of CSR order), Jacobi GMRES and CG iterates to 1e-12 (the
    dot products run in the space order), ILU(0) GMRES (mesh-order factors, the permuted SpMV around
    each apply) to 1e-12."""
    gm = cdfem.kuhn_mesh(3, 8, 2, perturb=0.1)
    rng = np.random.default_rng(31)
    g = rng.permutation(gm.nl).astype(np.int32)
    xyz = np.empty_like(gm.dof_xyz)
    xyz[g] = gm.dof_xyz
    sm = cdfem.Mesh(gm.dim, gm.order, gm.verts, g[gm.dofmap], gm.nl, np.sort(g[gm.ess]), xyz, simplex=True)
    x = rng.uniform(-1, 1, sm.nl)
    b = rng.uniform(-1, 1, sm.nl)
    res = {}
    try:
        for so in (0, order):
            gpu_ctx.set_option("sell_order", so)
            gpu_ctx.upload_mesh(sm)
            gpu_ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=C3, mass=1.0)
            _, B = gpu_ctx.form_linear_system(np.zeros(sm.nl), b)
            r = [gpu_ctx.mult(x), gpu_ctx.mult(x, constrained=True)]
            r.append(gpu_ctx.solve(B, method="gmres", pc="jacobi", restart=10, rel_tol=0.0, abs_tol=0.0,
                                   max_iter=25)[0])
            r.append(gpu_ctx.solve(B, method="gmres", pc="ilu", restart=10, rel_tol=0.0, abs_tol=0.0,
                                   max_iter=15)[0])
            gpu_ctx.fa_setup(kinds=5, kappa=0.1, mass=1.0)       # SPD: CG (den fused into the SpMV)
            _, B2 = gpu_ctx.form_linear_system(np.zeros(sm.nl), b)
            r.append(gpu_ctx.solve(B2, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=30)[0])
            xc, info = gpu_ctx.solve(B2, method="cg", pc="jacobi", rel_tol=1e-10, abs_tol=0.0, max_iter=500)
            assert info["converged"]
            r.append(xc)
            res[so] = r
        base, new = res[0], res[order]
        for k in (0, 1):
            assert np.abs(new[k] - base[k]).max() <= 1e-14 * np.abs(base[k]).max(), k
        for k in (2, 3, 4, 5):
            assert np.abs(new[k] - base[k]).max() <= 1e-12 * np.abs(base[k]).max(), k
    finally:
        gpu_ctx.set_option("sell_order", 8)


def test_lds_spmv_grid_bound(gpu_ctx):
    """the LDS-staged SpMV launches one workgroup per window and its CG form writes one
    partial per workgroup, so the window count must fit the partial slots (kSpmvMaxBlocks = 65536).
    With 64-row windows (spmv_lds 64, one lane per row) a P2 Kuhn mesh of 82^3 cubes has
    165^3 = 4.49 M rows = 70.2 K windows: an explicit choice is refused with a message (no write past
    the partial buffer), and the automatic layout on the same mesh sets up and applies normally."""
    m = cdfem.kuhn_mesh(3, 82, 2, with_coords=True)
    assert m.nl > 64 * 65536
    try:
        gpu_ctx.set_option("spmv_lds", 64)
        gpu_ctx.set_option("spmv_lpr", 1)
        gpu_ctx.upload_mesh(m)
        with pytest.raises(cdfem.CdfemError, match="exceed the SpMV grid"):
            gpu_ctx.fa_setup(kinds=cdfem.DIFFUSION | cdfem.MASS, kappa=0.1, mass=1.0)
    finally:
        gpu_ctx.set_option("spmv_lds", -1)
        gpu_ctx.set_option("spmv_lpr", 0)
    gpu_ctx.upload_mesh(m)
    gpu_ctx.fa_setup(kinds=cdfem.DIFFUSION | cdfem.MASS, kappa=0.1, mass=1.0)
    x = np.ones(m.nl)
    y = gpu_ctx.mult(x)
    assert np.isfinite(y).all()
