"""CPU oracle bindings — TEST INFRASTRUCTURE ONLY.

Thin ctypes/numpy wrapper over ``oracle/_build/liborc.so`` (built from ``oracle/cdfem_oracle.c``).
Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` import this
module, and only as the checker.  The product (``continuum-mechanics-mfem_amd/``) never imports it.

See the header of ``cdfem_oracle.c`` for what is restated from the reference and how the oracle is
pinned (manufactured-solution known answers; bit parity with an MFEM run is unpinned).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liborc.so")

DIFFUSION, CONVECTION, MASS = 1, 2, 4
RULE_DIFFUSION, RULE_CONVECTION, RULE_MASS, RULE_LF, RULE_L2 = 0, 1, 2, 3, 4

_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH) or (
        os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "cdfem_oracle.c"))
    ):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        dp, ip, lp = C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(C.c_int64)
        L.orc_gauss_legendre.argtypes = [C.c_int, dp, dp]
        L.orc_gll_nodes.argtypes = [C.c_int, dp]
        L.orc_lagrange.argtypes = [C.c_int, dp, C.c_double, dp, dp]
        L.orc_rule_npts.argtypes = [C.c_int, C.c_int, C.c_int]
        L.orc_mesh_box.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, dp, ip, ip]
        L.orc_fa_assemble.restype = C.c_void_p
        L.orc_fa_assemble.argtypes = [C.c_int, C.c_int, C.c_int, dp, ip, C.c_int64, C.c_double,
                                      C.c_double, C.c_double, dp, C.c_int]
        for nm in ("orc_fa_assemble_q", "orc_fa_assemble_simplex_q"):
            f = getattr(L, nm)
            f.restype = C.c_void_p
            f.argtypes = [C.c_int, C.c_int, C.c_int, dp, ip, C.c_int64, C.c_double, dp, dp, C.c_double, dp, dp,
                          C.c_double, dp, C.c_int]
        L.orc_csr_free.argtypes = [C.c_void_p]
        L.orc_csr_n.argtypes = [C.c_void_p]
        L.orc_csr_n.restype = C.c_int64
        L.orc_csr_nnz.argtypes = [C.c_void_p]
        L.orc_csr_nnz.restype = C.c_int64
        L.orc_csr_export.argtypes = [C.c_void_p, lp, C.POINTER(C.c_int32), dp]
        L.orc_csr_spmv.argtypes = [C.c_void_p, dp, dp]
        L.orc_csr_import.restype = C.c_void_p
        L.orc_csr_import.argtypes = [C.c_int64, lp, C.POINTER(C.c_int32), dp]
        L.orc_form_linear_system.restype = C.c_void_p
        L.orc_form_linear_system.argtypes = [C.c_void_p, ip, dp, dp, dp]
        L.orc_csr_diag.argtypes = [C.c_void_p, dp]
        L.orc_cg.argtypes = [C.c_void_p, dp, dp, dp, C.c_double, C.c_double, C.c_int, ip, dp]
        L.orc_gmres.argtypes = [C.c_void_p, dp, dp, dp, C.c_int, C.c_double, C.c_double, C.c_int, ip, dp]
        L.orc_ilu0.restype = C.c_void_p
        L.orc_ilu0.argtypes = [C.c_void_p]
        L.orc_ilu_solve.argtypes = [C.c_void_p, dp, dp]
        L.orc_gmres_ilu.argtypes = [C.c_void_p, C.c_void_p, dp, dp, C.c_int, C.c_double, C.c_double, C.c_int,
                                    ip, dp]
        L.orc_pa_setup.restype = C.c_void_p
        L.orc_pa_setup.argtypes = [C.c_int, C.c_int, dp, ip, C.c_int64, C.c_double, C.c_double, C.c_double, dp,
                                   C.c_int]
        L.orc_pa_free.argtypes = [C.c_void_p]
        L.orc_pa_mult.argtypes = [C.c_void_p, ip, dp, dp]
        L.orc_pa_diag.argtypes = [C.c_void_p, dp]
        L.orc_pa_cg.argtypes = [C.c_void_p, ip, dp, dp, dp, C.c_double, C.c_double, C.c_int, ip, dp]
        L.orc_stream_triad.argtypes = [C.c_int64, C.c_int]
        L.orc_stream_triad.restype = C.c_double
        L.orc_mms_u.argtypes = [dp, dp]
        L.orc_mms_u.restype = C.c_double
        L.orc_mms_f.argtypes = [dp, dp]
        L.orc_mms_f.restype = C.c_double
        L.orc_lf_assemble.argtypes = [C.c_int, C.c_int, C.c_int, dp, ip, C.c_int64, dp, dp]
        L.orc_dof_coords.argtypes = [C.c_int, C.c_int, C.c_int, dp, ip, dp]
        L.orc_l2_error.argtypes = [C.c_int, C.c_int, C.c_int, dp, ip, dp, dp, C.c_int]
        L.orc_l2_error.restype = C.c_double
        L.orc_ebe_mult.argtypes = [C.c_int, C.c_int, C.c_int, dp, ip, C.c_int64, C.c_double,
                                   C.c_double, C.c_double, dp, C.c_int, dp, dp]
        L.orc_simplex_nd.argtypes = [C.c_int, C.c_int]
        L.orc_simplex_rule.argtypes = [C.c_int, C.c_int, dp, dp]
        L.orc_simplex_rule_order.argtypes = [C.c_int, C.c_int, dp, dp]
        L.orc_mesh_kuhn_sizes.argtypes = [C.c_int, C.c_int, C.c_int, ip, lp]
        L.orc_mesh_kuhn.argtypes = [C.c_int, C.c_int, C.c_int, C.c_double, dp, ip, ip]
        L.orc_fa_assemble_simplex.restype = C.c_void_p
        L.orc_fa_assemble_simplex.argtypes = [C.c_int, C.c_int, C.c_int, dp, ip, C.c_int64, C.c_double,
                                              C.c_double, C.c_double, dp, C.c_int]
        L.orc_lf_assemble_simplex.argtypes = [C.c_int, C.c_int, C.c_int, dp, ip, C.c_int64, dp, dp]
        L.orc_l2_error_simplex.argtypes = [C.c_int, C.c_int, C.c_int, dp, ip, dp, dp]
        L.orc_l2_error_simplex.restype = C.c_double
        L.orc_dof_coords_simplex.argtypes = [C.c_int, C.c_int, C.c_int, dp, ip, dp]
        L.orc_num_threads.restype = C.c_int
        L.orc_set_num_threads.argtypes = [C.c_int]
        L.orc_pin_threads.argtypes = [C.POINTER(C.c_int), C.c_int]
        L.orc_pin_threads.restype = C.c_int
        _lib = L
    return _lib


def _d(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _i(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


def gauss_legendre(n):
    x, w = np.zeros(n), np.zeros(n)
    lib().orc_gauss_legendre(n, _d(x), _d(w))
    return x, w


def gll_nodes(p):
    x = np.zeros(p + 1)
    lib().orc_gll_nodes(p, _d(x))
    return x


def basis_tables(p, n):
    """B[q, d] = phi_d(xi_q), G[q, d] = phi_d'(xi_q) at n Gauss points on [0,1]."""
    nodes = gll_nodes(p)
    pts, _ = gauss_legendre(n)
    B, G = np.zeros((n, p + 1)), np.zeros((n, p + 1))
    for q in range(n):
        phi, dphi = np.zeros(p + 1), np.zeros(p + 1)
        lib().orc_lagrange(p, _d(nodes), float(pts[q]), _d(phi), _d(dphi))
        B[q], G[q] = phi, dphi
    return B, G


def rule_npts(which, dim, p):
    return lib().orc_rule_npts(which, dim, p)


class BoxMesh:
    """Structured [0,1]^dim box mesh (see orc_mesh_box for numbering conventions)."""

    def __init__(self, dim, n, p, perturb=0.0):
        nx, ny, nz = (n, n, n) if np.isscalar(n) else tuple(n) + ((1,) if len(n) == 2 else ())
        if dim == 2:
            nz = 1
        self.dim, self.p, self.n = dim, p, (nx, ny, nz)
        self.ne = nx * ny * nz
        self.nv = 8 if dim == 3 else 4
        self.nd = (p + 1) ** dim
        self.nl = (p * nx + 1) * (p * ny + 1) * ((p * nz + 1) if dim == 3 else 1)
        self.verts = np.zeros((self.ne, self.nv, dim))
        self.dofmap = np.zeros((self.ne, self.nd), dtype=np.int32)
        self.bdr = np.zeros(self.nl, dtype=np.int32)
        lib().orc_mesh_box(dim, nx, ny, nz, p, float(perturb), _d(self.verts), _i(self.dofmap),
                           _i(self.bdr))
        self.ess = np.nonzero(self.bdr)[0].astype(np.int32)

    def dof_coords(self):
        xyz = np.zeros((self.nl, self.dim))
        lib().orc_dof_coords(self.dim, self.p, self.ne, _d(self.verts), _i(self.dofmap), _d(xyz))
        return xyz


class KuhnMesh:
    """Kuhn simplex mesh of [0,1]^dim, P1/P2 (see orc_mesh_kuhn for the conventions; config C4)."""

    def __init__(self, dim, n, p, perturb=0.0):
        L = lib()
        ne, nl = C.c_int(), C.c_int64()
        L.orc_mesh_kuhn_sizes(dim, n, p, C.byref(ne), C.byref(nl))
        self.dim, self.p, self.n = dim, p, n
        self.ne, self.nl = ne.value, nl.value
        self.nv = dim + 1
        self.nd = L.orc_simplex_nd(dim, p)
        self.verts = np.zeros((self.ne, self.nv, dim))
        self.dofmap = np.zeros((self.ne, self.nd), dtype=np.int32)
        self.bdr = np.zeros(self.nl, dtype=np.int32)
        if L.orc_mesh_kuhn(dim, n, p, float(perturb), _d(self.verts), _i(self.dofmap), _i(self.bdr)):
            raise RuntimeError("orc_mesh_kuhn: inverted element")
        self.ess = np.nonzero(self.bdr)[0].astype(np.int32)


def _simplex_arrays(mesh):
    return (np.ascontiguousarray(mesh.verts, dtype=np.float64), np.ascontiguousarray(mesh.dofmap, dtype=np.int32))


def lf_assemble_simplex(mesh, prm):
    v, d = _simplex_arrays(mesh)
    b = np.zeros(mesh.nl)
    lib().orc_lf_assemble_simplex(mesh.dim, mesh.p, mesh.ne, _d(v), _i(d), mesh.nl, _d(prm), _d(b))
    return b


def l2_error_simplex(mesh, u, prm):
    v, d = _simplex_arrays(mesh)
    u = np.ascontiguousarray(u, dtype=np.float64)
    return lib().orc_l2_error_simplex(mesh.dim, mesh.p, mesh.ne, _d(v), _i(d), _d(u), _d(prm))


def dof_coords_simplex(mesh):
    v, d = _simplex_arrays(mesh)
    xyz = np.zeros((mesh.nl, mesh.dim))
    lib().orc_dof_coords_simplex(mesh.dim, mesh.p, mesh.ne, _d(v), _i(d), _d(xyz))
    return xyz


def solve_mms_simplex(mesh, prm, kappa, s, c, alpha=1.0, tol=1e-10, atol=1e-12, max_it=500, pc="jacobi",
                      blocks=None):
    """C4 driver sequence on the oracle: FA CSR, FormLinearSystem, GMRES(30) + Jacobi (Input/petsc.opts)
    or + ILU(0) (pc="ilu": Input/petsc_circle.opts on one rank; with blocks, the per-rank owned dof
    lists: block-Jacobi ILU(0), the same options under mpirun -np N), L2 error."""
    A = fa_assemble_simplex(mesh, kappa=kappa, alpha=alpha, s=s, c=c)
    b = lf_assemble_simplex(mesh, prm)
    u = np.zeros(mesh.nl)
    xyz = dof_coords_simplex(mesh)
    u[mesh.ess] = mms_u(prm, xyz[mesh.ess])
    Ac, B = form_linear_system(A, mesh.bdr, u, b)
    if pc == "ilu" and blocks is not None:
        X, info = gmres_bjacobi_ilu(Ac, B, blocks, rtol=tol, atol=atol, max_it=max_it)
    elif pc == "ilu":
        X, info = gmres_ilu(Ac, B, ilu0(Ac), rtol=tol, atol=atol, max_it=max_it)
    else:
        X, info = gmres(Ac, B, dinv=1.0 / Ac.diag(), rtol=tol, atol=atol, max_it=max_it)
    return X, info, l2_error_simplex(mesh, X, prm)


def simplex_rule_order(dim, order):
    """MFEM's IntRules.Get(simplex, order) (tabulated; collapsed Gauss beyond the tables)."""
    xi, w = np.zeros(64 * dim), np.zeros(64)
    nq = lib().orc_simplex_rule_order(dim, order, _d(xi), _d(w))
    return xi[: nq * dim].reshape(nq, dim), w[:nq]


def simplex_rule(dim, n):
    xi, w = np.zeros(n ** dim * dim), np.zeros(n ** dim)
    nq = lib().orc_simplex_rule(dim, n, _d(xi), _d(w))
    return xi.reshape(nq, dim), w


class CSR:
    def __init__(self, handle):
        self.h = handle
        L = lib()
        self.n, self.nnz = L.orc_csr_n(handle), L.orc_csr_nnz(handle)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_csr_free(self.h)
            self.h = None

    def export(self):
        rp = np.zeros(self.n + 1, dtype=np.int64)
        col = np.zeros(self.nnz, dtype=np.int32)
        val = np.zeros(self.nnz)
        lib().orc_csr_export(self.h, rp.ctypes.data_as(C.POINTER(C.c_int64)),
                             col.ctypes.data_as(C.POINTER(C.c_int32)), _d(val))
        return rp, col, val

    def to_scipy(self):
        import scipy.sparse as sp
        rp, col, val = self.export()
        return sp.csr_matrix((val, col, rp), shape=(self.n, self.n))

    def mult(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(self.n)
        lib().orc_csr_spmv(self.h, _d(x), _d(y))
        return y

    def diag(self):
        d = np.zeros(self.n)
        lib().orc_csr_diag(self.h, _d(d))
        return d


def _conv(c, dim):
    cc = np.zeros(3)
    if c is not None:
        cc[: len(c)] = c
    return cc


def _opt(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float64)


def fa_assemble_q(mesh, kappa=0.0, kappa_q=None, kmat_q=None, alpha=1.0, c=None, c_q=None, s=0.0, s_q=None,
                  kinds=DIFFUSION | CONVECTION | MASS, simplex=False):
    """FA CSR with per-quadrature-point coefficients (arrays element-major in the operator rule's point
    order; None: the constant).  kmat_q: the symmetric MatrixCoefficient of DiffusionIntegrator,
    K = kappa I + K_q, components xx,xy,yy (2D) / xx,xy,xz,yy,yz,zz (3D)."""
    cc = _conv(c, mesh.dim)
    arrs = [_opt(a) for a in (kappa_q, kmat_q, c_q, s_q)]
    ptr = [None if a is None else _d(a) for a in arrs]
    verts = np.ascontiguousarray(mesh.verts, dtype=np.float64)
    dofmap = np.ascontiguousarray(mesh.dofmap, dtype=np.int32)
    f = lib().orc_fa_assemble_simplex_q if simplex else lib().orc_fa_assemble_q
    h = f(mesh.dim, mesh.p, mesh.ne, _d(verts), _i(dofmap), mesh.nl, float(kappa), ptr[0], ptr[1], float(alpha),
          _d(cc), ptr[2], float(s), ptr[3], kinds)
    if not h:
        raise RuntimeError("orc_fa_assemble_q: unsupported element / rule")
    return CSR(h)


def fa_assemble(mesh: BoxMesh, kappa=1.0, alpha=1.0, s=1.0, c=None, kinds=DIFFUSION | CONVECTION | MASS):
    cc = _conv(c, mesh.dim)
    h = lib().orc_fa_assemble(mesh.dim, mesh.p, mesh.ne, _d(mesh.verts), _i(mesh.dofmap), mesh.nl,
                              kappa, alpha, s, _d(cc), kinds)
    if not h:
        raise RuntimeError("orc_fa_assemble: integrator rules do not coincide")
    return CSR(h)


def fa_assemble_simplex(mesh, kappa=1.0, alpha=1.0, s=1.0, c=None, kinds=DIFFUSION | CONVECTION | MASS):
    """FA CSR on P1/P2 simplices (mesh: KuhnMesh or any object with dim/p/ne/verts/dofmap/nl)."""
    cc = _conv(c, mesh.dim)
    verts = np.ascontiguousarray(mesh.verts, dtype=np.float64)
    dofmap = np.ascontiguousarray(mesh.dofmap, dtype=np.int32)
    h = lib().orc_fa_assemble_simplex(mesh.dim, mesh.p, mesh.ne, _d(verts), _i(dofmap), mesh.nl,
                                      kappa, alpha, s, _d(cc), kinds)
    if not h:
        raise RuntimeError("orc_fa_assemble_simplex: unsupported order")
    return CSR(h)


def ebe_mult(mesh: BoxMesh, x, kappa=1.0, alpha=1.0, s=1.0, c=None, kinds=DIFFUSION | CONVECTION | MASS):
    cc = _conv(c, mesh.dim)
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.zeros(mesh.nl)
    lib().orc_ebe_mult(mesh.dim, mesh.p, mesh.ne, _d(mesh.verts), _i(mesh.dofmap), mesh.nl, kappa,
                       alpha, s, _d(cc), kinds, _d(x), _d(y))
    return y


class PA:
    """MFEM's host partial assembly of the 3D hex operator (orc_pa_*: per-integrator point data, L->E,
    one sum-factorised element loop per integrator, E->L): the CPU PA + CG baseline of bench.py."""

    def __init__(self, mesh: BoxMesh, kappa=1.0, alpha=1.0, s=1.0, c=None, kinds=DIFFUSION | CONVECTION | MASS):
        if mesh.dim != 3:
            raise ValueError("PA restatement: 3D hexes")
        self.nl, self.bdr = mesh.nl, np.ascontiguousarray(mesh.bdr, dtype=np.int32)
        self.h = lib().orc_pa_setup(mesh.p, mesh.ne, _d(mesh.verts), _i(mesh.dofmap), mesh.nl, kappa, alpha, s,
                                    _d(_conv(c, 3)), kinds)
        if not self.h:
            raise RuntimeError("orc_pa_setup: unsupported order")

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_pa_free(self.h)
            self.h = None

    def mult(self, x, constrained=False):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.empty(self.nl)
        lib().orc_pa_mult(self.h, _i(self.bdr) if constrained else None, _d(x), _d(y))
        return y

    def diag(self):
        """AssembleDiagonal at the PA level (orc_pa_diag: per-integrator sum-factorised element
        diagonals, then the E->L sum); unconstrained, as the FA CSR's diagonal."""
        y = np.empty(self.nl)
        lib().orc_pa_diag(self.h, _d(y))
        return y

    def form_linear_system(self, X, b):
        """FormLinearSystem on the PA operator (ConstrainedOperator::EliminateRHS, DIAG_ONE): B = b - A X_e
        with X_e = X on the essential dofs and 0 elsewhere, then B_ess = X_ess."""
        ess = self.bdr != 0
        xe = np.where(ess, X, 0.0)
        B = np.asarray(b, dtype=np.float64) - self.mult(xe)
        B[ess] = X[ess]
        return B

    def cg(self, b, dinv=None, rel_tol=1e-12, abs_tol=0.0, max_iter=500):
        """CGSolver on the constrained operator (b: FormLinearSystem's B, dinv: 1 / diag with ess 1)."""
        b = np.ascontiguousarray(b, dtype=np.float64)
        x = np.zeros(self.nl)
        it, fn = C.c_int(0), C.c_double(0.0)
        di = None if dinv is None else _d(np.ascontiguousarray(dinv, dtype=np.float64))
        conv = lib().orc_pa_cg(self.h, _i(self.bdr), di, _d(b), _d(x), rel_tol, abs_tol, max_iter,
                               C.byref(it), C.byref(fn))
        return x, {"converged": bool(conv), "iterations": it.value, "final_norm": fn.value}


def stream_triad_gbs(n=1 << 26, reps=5):
    """Host STREAM triad GB/s (24 B per index) on the current OpenMP threads."""
    return lib().orc_stream_triad(n, reps)


def form_linear_system(A: CSR, ess_marker, X, b):
    B = np.zeros(A.n)
    ess_marker = np.ascontiguousarray(ess_marker, dtype=np.int32)
    X = np.ascontiguousarray(X, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    h = lib().orc_form_linear_system(A.h, _i(ess_marker), _d(X), _d(b), _d(B))
    return CSR(h), B


def cg(A: CSR, b, dinv=None, rel_tol=1e-12, abs_tol=0.0, max_iter=500):
    b = np.ascontiguousarray(b, dtype=np.float64)
    x = np.zeros(A.n)
    it, fn = C.c_int(0), C.c_double(0)
    di = None if dinv is None else _d(np.ascontiguousarray(dinv, dtype=np.float64))
    conv = lib().orc_cg(A.h, di, _d(b), _d(x), rel_tol, abs_tol, max_iter, C.byref(it), C.byref(fn))
    return x, dict(converged=bool(conv), iterations=it.value, final_norm=fn.value)


def gmres(A: CSR, b, dinv=None, restart=30, rtol=1e-10, atol=1e-12, max_it=500):
    b = np.ascontiguousarray(b, dtype=np.float64)
    x = np.zeros(A.n)
    it, fn = C.c_int(0), C.c_double(0)
    di = None if dinv is None else _d(np.ascontiguousarray(dinv, dtype=np.float64))
    conv = lib().orc_gmres(A.h, di, _d(b), _d(x), restart, rtol, atol, max_it, C.byref(it), C.byref(fn))
    return x, dict(converged=bool(conv), iterations=it.value, final_norm=fn.value)


def csr_from_scipy(S) -> CSR:
    """An oracle CSR of a scipy matrix (columns sorted per row; explicit zeros kept)."""
    S = S.tocsr()
    S.sort_indices()
    rp = np.ascontiguousarray(S.indptr, dtype=np.int64)
    col = np.ascontiguousarray(S.indices, dtype=np.int32)
    val = np.ascontiguousarray(S.data, dtype=np.float64)
    return CSR(lib().orc_csr_import(len(rp) - 1, rp.ctypes.data_as(C.POINTER(C.c_int64)),
                                    col.ctypes.data_as(C.POINTER(C.c_int32)), _d(val)))


def gmres_bjacobi_ilu(Ac: CSR, b, blocks, restart=30, rtol=1e-10, atol=1e-12, max_it=500):
    """PETSc KSPGMRES + PCBJACOBI with one ILU(0) block per rank (Input/petsc_circle.opts:6-8 under
    mpirun -np N).  blocks: per rank, the global dofs it owns in its local (natural) order.  The
    system is renumbered rank by rank (PETSc's global order: rank-contiguous rows), the
    preconditioner is ILU(0) of the block-diagonal part (entries coupling two ranks dropped: ILU(0)
    of a block-diagonal matrix is the per-block ILU(0)), GMRES runs on the renumbered system and the
    solution is numbered back."""
    import scipy.sparse as sp
    perm = np.concatenate([np.asarray(bl, dtype=np.int64) for bl in blocks])
    assert len(perm) == Ac.n and len(np.unique(perm)) == Ac.n
    S = Ac.to_scipy()[perm][:, perm].tocoo()
    owner = np.repeat(np.arange(len(blocks)), [len(bl) for bl in blocks])
    keep = owner[S.row] == owner[S.col]
    Ap = csr_from_scipy(S.tocsr())
    Bd = csr_from_scipy(sp.csr_matrix((S.data[keep], (S.row[keep], S.col[keep])), shape=S.shape))
    xp, info = gmres_ilu(Ap, np.asarray(b)[perm], ilu0(Bd), restart=restart, rtol=rtol, atol=atol, max_it=max_it)
    x = np.zeros(Ac.n)
    x[perm] = xp
    return x, info


def ilu0(A: CSR) -> CSR:
    """ILU(0) factors in A's pattern (unit-lower L and U packed), PETSc PCILU semantics."""
    return CSR(lib().orc_ilu0(A.h))


def ilu_solve(F: CSR, r):
    r = np.ascontiguousarray(r, dtype=np.float64)
    z = np.zeros(F.n)
    lib().orc_ilu_solve(F.h, _d(r), _d(z))
    return z


def gmres_ilu(A: CSR, b, F: CSR, restart=30, rtol=1e-10, atol=1e-12, max_it=500):
    """GMRES(m) left-preconditioned with ILU(0) factors F (Input/petsc_circle.opts)."""
    b = np.ascontiguousarray(b, dtype=np.float64)
    x = np.zeros(A.n)
    it, fn = C.c_int(0), C.c_double(0)
    conv = lib().orc_gmres_ilu(A.h, F.h, _d(b), _d(x), restart, rtol, atol, max_it, C.byref(it), C.byref(fn))
    return x, dict(converged=bool(conv), iterations=it.value, final_norm=fn.value)


MMS_SIN, MMS_POLY, MMS_DIFFUSION_T, MMS_RADIAL, MMS_ERFC = 1, 2, 3, 4, 5


def mms_params(kind, dim, kappa=0.1, s=1.0, alpha=1.0, c=(1.0, -2.0, 0.5), modes=(3, 3, 3), t=0.0, p=1):
    cc = _conv(c, dim)
    return np.array([kind, kappa, s, alpha, cc[0], cc[1], cc[2], modes[0], modes[1], modes[2], t, p, dim],
                    dtype=np.float64)


def mms_u(prm, xyz):
    xyz = np.atleast_2d(xyz)
    out = np.zeros(len(xyz))
    L = lib()
    for i, x in enumerate(xyz):
        xx = np.zeros(3)
        xx[: len(x)] = x
        out[i] = L.orc_mms_u(_d(prm), _d(xx))
    return out


def mms_f(prm, xyz):
    """Forcing of the manufactured solution at points (orc_mms_f), shape (..., dim) -> (...)."""
    xyz = np.asarray(xyz, dtype=np.float64)
    pts = xyz.reshape(-1, xyz.shape[-1])
    out = np.zeros(len(pts))
    L = lib()
    for i, x in enumerate(pts):
        xx = np.zeros(3)
        xx[: len(x)] = x
        out[i] = L.orc_mms_f(_d(prm), _d(xx))
    return out.reshape(xyz.shape[:-1])


def lf_assemble(mesh: BoxMesh, prm):
    b = np.zeros(mesh.nl)
    lib().orc_lf_assemble(mesh.dim, mesh.p, mesh.ne, _d(mesh.verts), _i(mesh.dofmap), mesh.nl,
                          _d(np.ascontiguousarray(prm)), _d(b))
    return b


def l2_error(mesh: BoxMesh, u, prm=None):
    u = np.ascontiguousarray(u, dtype=np.float64)
    if prm is None:
        return lib().orc_l2_error(mesh.dim, mesh.p, mesh.ne, _d(mesh.verts), _i(mesh.dofmap), _d(u),
                                  _d(np.zeros(13)), 1)
    return lib().orc_l2_error(mesh.dim, mesh.p, mesh.ne, _d(mesh.verts), _i(mesh.dofmap), _d(u),
                              _d(np.ascontiguousarray(prm)), 0)


def solve_mms(mesh: BoxMesh, prm, kappa, s, c, alpha=1.0, solver="gmres", tol=1e-10, atol=1e-12,
              max_it=500):
    """The driver sequence of linear_convection_diffusion_2D.cpp:319-377 on the CPU oracle.

    Returns (u, info, l2_error).
    """
    A = fa_assemble(mesh, kappa=kappa, alpha=alpha, s=s, c=c)
    b = lf_assemble(mesh, prm)
    u = np.zeros(mesh.nl)
    xyz = mesh.dof_coords()
    u[mesh.ess] = mms_u(prm, xyz[mesh.ess])                # ProjectBdrCoefficient
    Ac, B = form_linear_system(A, mesh.bdr, u, b)           # FormLinearSystem
    dinv = 1.0 / Ac.diag()
    if solver == "gmres":
        X, info = gmres(Ac, B, dinv=dinv, rtol=tol, atol=atol, max_it=max_it)
    else:
        X, info = cg(Ac, B, dinv=dinv, rel_tol=tol, abs_tol=0.0, max_iter=max_it)
    return X, info, l2_error(mesh, X, prm)                  # RecoverFEMSolution (P = I) + L2 error


def set_threads(n):
    lib().orc_set_num_threads(int(n))


def pin_threads(cpus):
    """Pin OpenMP thread t to cpus[t] (and the calling thread to cpus[0]); returns threads pinned."""
    a = np.ascontiguousarray(cpus, dtype=np.int32)
    return lib().orc_pin_threads(a.ctypes.data_as(C.POINTER(C.c_int)), len(a))


def num_threads():
    return lib().orc_num_threads()


# ---- ALE diffusion MMS coefficients (diffusion_mms_ale.cpp:213-440, 455-558) -------------------------
# Restated from the reference's AleMap: A(xhat, t) maps the reference square onto Omega(t); the
# driver assembles on the reference mesh  Mass(J) + Diffusion(alpha dt / J cof cof^T)
# + Convection(phi_hat, -1) + Mass(-div phi_hat)  (:1017-1023).
ALE_MAPS = ("identity", "accuracy_a", "accuracy_b")


def _ale_amp(kind, t):
    return 0.5 * np.sin(np.pi * t) if kind == "accuracy_a" else np.sin(np.pi * t)   # :411-414, :436-439


def _ale_g(z):      # AccuracyAShape_, :417-421
    h = ((-z + 1.5) * z - 0.5) * z
    return np.sin(np.pi * h)


def _ale_gp(z):     # AccuracyAShapeD1_, :422-427
    h = ((-z + 1.5) * z - 0.5) * z
    hp = (-3.0 * z + 3.0) * z - 0.5
    return np.pi * np.cos(np.pi * h) * hp


def ale_gradient(kind, xy, t):
    """G = dA/dxhat (MapGradient, :252-287) at points xy (n, 2): (n, 2, 2)."""
    x, y = xy[:, 0], xy[:, 1]
    G = np.zeros((len(xy), 2, 2))
    if kind == "identity":
        G[:, 0, 0] = G[:, 1, 1] = 1.0
    elif kind == "accuracy_a":
        a = _ale_amp(kind, t)
        G[:, 0, 0] = 1.0 + a * _ale_gp(x)
        G[:, 1, 1] = 1.0 + a * _ale_gp(y)
    else:
        a = _ale_amp(kind, t)
        ax, ay, dax, day = x * (1 - x), y * (1 - y), 1 - 2 * x, 1 - 2 * y
        G[:, 0, 0] = 1.0 + a * dax * ay
        G[:, 0, 1] = a * ax * day
        G[:, 1, 0] = a * dax * ay
        G[:, 1, 1] = 1.0 + a * ax * day
    return G


def ale_coefficients(kind, xy, t_old, t_new, alpha, dt):
    """Per-point coefficients of the ALE left-hand side at t_new: J (AleJacobianCoefficient, :455-469),
    the metric alpha dt / J cof(G) cof(G)^T as xx,xy,yy (AleMetricTensorCoefficient, :474-502), the
    integrated grid flux phi_hat and its divergence (IntegratedMappedGridFlux, :338-407)."""
    G = ale_gradient(kind, xy, t_new)
    J = G[:, 0, 0] * G[:, 1, 1] - G[:, 0, 1] * G[:, 1, 0]
    Cf = np.zeros_like(G)                       # MapCofactor, :290-299
    Cf[:, 0, 0], Cf[:, 0, 1], Cf[:, 1, 0], Cf[:, 1, 1] = G[:, 1, 1], -G[:, 0, 1], -G[:, 1, 0], G[:, 0, 0]
    M = np.einsum("nij,nkj->nik", Cf, Cf) * (alpha * dt / J)[:, None, None]
    metric = np.stack([M[:, 0, 0], M[:, 0, 1], M[:, 1, 1]], axis=1)
    x, y = xy[:, 0], xy[:, 1]
    phi = np.zeros((len(xy), 2))
    div = np.zeros(len(xy))
    if kind == "accuracy_a":
        a0, a1 = _ale_amp(kind, t_old), _ale_amp(kind, t_new)
        i1, i2 = a1 - a0, 0.5 * (a1 * a1 - a0 * a0)
        gx, gxp, gy, gyp = _ale_g(x), _ale_gp(x), _ale_g(y), _ale_gp(y)
        phi[:, 0] = gx * (i1 + i2 * gyp)
        phi[:, 1] = gy * (i1 + i2 * gxp)
        div = i1 * (gxp + gyp) + 2.0 * i2 * gxp * gyp
    elif kind == "accuracy_b":
        i1 = _ale_amp(kind, t_new) - _ale_amp(kind, t_old)
        ax, ay, dax, day = x * (1 - x), y * (1 - y), 1 - 2 * x, 1 - 2 * y
        q = ax * ay
        phi[:, 0] = phi[:, 1] = i1 * q
        div = i1 * (dax * ay + ax * day)
    return J, metric, phi, div


def transient_three_peclet(mesh, dt, t_final, peclet=(1.0, 10.0, 100.0), simplex=False, rtol=1e-10, atol=1e-12,
                           max_it=500):
    """linear_convection_diffusion_1D.cpp:375-400,537-576 on the oracle: three uncoupled backward-Euler
    systems (M + dt C(beta = (1, 0)) + (dt / Pe) K) c_k^{n+1} = M c_k^n on the unit square, Dirichlet
    on x = 0 and x = 1 (BuildXDirichletBoundaryMarker, :219-266) set to the erfc solution (MMS_ERFC,
    :128-166) at t^{n+1}, GMRES(30) + Jacobi per block (Input/petsc.opts).  Returns, per block, the
    final absolute and relative L2 errors (order max(2, 2p + 3), :483-510) and the GMRES iterations."""
    p = mesh.p
    if simplex:
        xyz = dof_coords_simplex(mesh)
        asm = fa_assemble_simplex
        err = l2_error_simplex
    else:
        xyz = mesh.dof_coords()
        asm = fa_assemble
        err = l2_error
    ess = (np.abs(xyz[:, 0]) <= 1e-8) | (np.abs(xyz[:, 0] - 1.0) <= 1e-8)
    marker = ess.astype(np.int32)
    M = asm(mesh, s=1.0, kinds=MASS)
    A = [asm(mesh, kappa=dt / pe, alpha=dt, s=1.0, c=(1.0, 0.0), kinds=DIFFUSION | CONVECTION | MASS) for pe in peclet]
    c = [np.zeros(mesh.nl) for _ in peclet]
    nsteps = int(np.ceil(t_final / dt - 1e-12))
    its = [0, 0, 0]
    for step in range(1, nsteps + 1):
        t = step * dt
        for k, pe in enumerate(peclet):
            rhs = M.mult(c[k])
            u = c[k].copy()
            u[ess] = mms_u(mms_params(MMS_ERFC, 2, kappa=pe, t=t, p=p), xyz[ess])
            Ac, B = form_linear_system(A[k], marker, u, rhs)
            c[k], info = gmres(Ac, B, dinv=1.0 / Ac.diag(), rtol=rtol, atol=atol, max_it=max_it)
            assert info["converged"]
            its[k] += info["iterations"]
    t = nsteps * dt
    out = []
    for k, pe in enumerate(peclet):
        prm = mms_params(MMS_ERFC, 2, kappa=pe, t=t, p=p)
        a = err(mesh, c[k], prm)
        nrm = err(mesh, np.zeros(mesh.nl), prm)
        out.append((a, a / nrm if nrm > 1e-14 else 0.0))
    return out, its, nsteps, c
