"""Python binding of libcdfem.so (the C-ABI in include/cdfem.h) via ctypes.

This is plumbing for tests, the benchmark and Python callers: every numerical operation runs in
the HIP kernels of the library.  There is NO CPU fallback — if the shared library or a GPU is
missing, the calls raise (``CdfemError``), they never compute on the host.

The classes mirror the reference's operator interface on the hot path
(linear_convection_diffusion_2D.cpp:335-377):

    ParBilinearForm-like  -> Context.pa_setup(...)   (Diffusion/Convection/Mass integrators + Assemble)
    Operator::Mult        -> Context.mult(x)          (constrained=True: the FormLinearSystem operator)
    FormLinearSystem      -> Context.form_linear_system(x, b)
    Krylov Mult(B, X)     -> Context.solve(B, method="cg"|"gmres", ...)
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_PKG_ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
LIB_PATH = os.path.join(_PKG_ROOT, "lib", "libcdfem.so")
HEADER_PATH = os.path.abspath(os.path.join(_PKG_ROOT, "..", "include", "cdfem.h"))

DIFFUSION, CONVECTION, MASS = 1, 2, 4
HOST, DEVICE = 0, 1
CG, GMRES = 0, 1
PC_NONE, PC_JACOBI, PC_ILU = 0, 1, 2
_PCS = {"none": PC_NONE, "jacobi": PC_JACOBI, "ilu": PC_ILU}
RULE_OPERATOR, RULE_LINEARFORM, RULE_ERROR, RULE_DIFFUSION, RULE_CONVECTION, RULE_MASS = 0, 1, 2, 3, 4, 5
K_APPLY, K_E2L, K_UPDATE, K_DIRECTION, K_ORTH = 0, 1, 2, 3, 4

OK, ERR_ARG, ERR_HIP, ERR_STATE, ERR_UNSUPPORTED, ERR_NOT_CONVERGED, ERR_COMM = range(7)


class CdfemError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"cdfem error {code}: {msg}")
        self.code = code


class SolverParams(C.Structure):
    _fields_ = [("method", C.c_int), ("pc", C.c_int), ("max_iter", C.c_int), ("restart", C.c_int),
                ("rel_tol", C.c_double), ("abs_tol", C.c_double), ("check_every", C.c_int),
                ("print_level", C.c_int)]


class SolverResult(C.Structure):
    _fields_ = [("converged", C.c_int), ("iterations", C.c_int), ("final_norm", C.c_double),
                ("initial_norm", C.c_double), ("seconds", C.c_double)]


class FormCoeffs(C.Structure):
    _fields_ = [("kinds", C.c_uint), ("kappa", C.c_double), ("kappa_q", C.POINTER(C.c_double)),
                ("kappa_mat_q", C.POINTER(C.c_double)), ("alpha", C.c_double), ("conv", C.POINTER(C.c_double)),
                ("conv_q", C.POINTER(C.c_double)), ("mass", C.c_double), ("mass_q", C.POINTER(C.c_double))]


ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_int, C.c_void_p)
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double),
                          C.POINTER(C.c_double), C.c_int64, C.c_void_p)
NBR_EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_double),
                              C.POINTER(C.c_double), C.c_void_p)

_lib = None
_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


def _declare(L):
    vp, i64 = C.c_void_p, C.c_int64
    sig = {
        "cdfem_abi_version": (C.c_int, []),
        "cdfem_device_count": (C.c_int, []),
        "cdfem_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
        "cdfem_destroy": (None, [vp]),
        "cdfem_last_error": (C.c_char_p, [vp]),
        "cdfem_synchronize": (C.c_int, [vp]),
        "cdfem_alloc": (C.c_int, [vp, C.c_size_t, C.POINTER(vp)]),
        "cdfem_free": (C.c_int, [vp, vp]),
        "cdfem_memcpy": (C.c_int, [vp, vp, C.c_int, vp, C.c_int, C.c_size_t]),
        "cdfem_mesh_upload": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, _dp, i64, _ip, C.c_int, _ip]),
        "cdfem_mesh_set_structured": (C.c_int, [vp, C.c_int, C.c_int, C.c_int]),
        "cdfem_rule_size": (C.c_int, [vp, C.c_int, C.POINTER(C.c_int)]),
        "cdfem_quadrature_points": (C.c_int, [vp, C.c_int, _dp, C.c_int]),
        "cdfem_pa_setup": (C.c_int, [vp, C.c_uint, C.c_double, _dp, C.c_double, _dp, _dp, C.c_double, _dp]),
        "cdfem_pa_mult": (C.c_int, [vp, vp, vp, C.c_int, C.c_int]),
        "cdfem_pa_setup_form": (C.c_int, [vp, C.POINTER(FormCoeffs)]),
        "cdfem_fa_setup_form": (C.c_int, [vp, C.POINTER(FormCoeffs)]),
        "cdfem_comm_share": (C.c_int, [vp, vp]),
        "cdfem_gmsh_topology_sizes": (C.c_int, [C.c_char_p, C.POINTER(C.c_int), C.POINTER(i64), C.POINTER(C.c_int),
                                                C.POINTER(C.c_int)]),
        "cdfem_gmsh_topology": (C.c_int, [C.c_char_p, _dp, _ip, _ip, _ip]),
        "cdfem_simplex_space_sizes": (C.c_int, [C.c_int, i64, _dp, C.c_int, _ip, C.c_int, C.POINTER(i64)]),
        "cdfem_simplex_space": (C.c_int, [C.c_int, i64, _dp, C.c_int, _ip, C.c_int, _ip, _ip, C.c_int, _dp, _ip, _ip,
                                          _dp]),
        "cdfem_pa_diagonal": (C.c_int, [vp, vp, C.c_int]),
        "cdfem_lf_assemble": (C.c_int, [vp, vp, vp, C.c_int]),
        "cdfem_form_linear_system": (C.c_int, [vp, vp, vp, vp, vp, C.c_int]),
        "cdfem_solve": (C.c_int, [vp, C.POINTER(SolverParams), vp, vp, C.c_int, C.POINTER(SolverResult)]),
        "cdfem_set_option": (C.c_int, [vp, C.c_char_p, C.c_int]),
        "cdfem_stream_bench": (C.c_int, [vp, C.c_int, C.c_size_t, C.c_int, _dp]),
        "cdfem_fp64_bench": (C.c_int, [vp, C.c_int, C.c_int, _dp]),
        "cdfem_profile_enable": (C.c_int, [vp, C.c_int]),
        "cdfem_profile_reset": (C.c_int, [vp]),
        "cdfem_profile_read": (C.c_int, [vp, C.c_int, _dp, C.POINTER(i64)]),
        "cdfem_kernel_bytes": (C.c_int, [vp, C.c_int, _dp]),
        "cdfem_kernel_flops": (C.c_int, [vp, C.c_int, _dp]),
        "cdfem_kernel_name": (C.c_int, [vp, C.c_int, C.c_char_p, C.c_size_t]),
        "cdfem_profile_launches": (C.c_int, [vp, C.c_int, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]),
        "cdfem_comm_unique_id": (C.c_int, [C.c_char_p]),
        "cdfem_comm_init_rccl": (C.c_int, [vp, C.c_int, C.c_int, C.c_char_p]),
        "cdfem_comm_init_host": (C.c_int, [vp, C.c_int, C.c_int, ALLREDUCE_FN, EXCHANGE_FN, vp]),
        "cdfem_set_slab": (C.c_int, [vp, C.c_int, C.c_int]),
        "cdfem_set_shared": (C.c_int, [vp, C.c_int, _ip, C.POINTER(i64), _ip]),
        "cdfem_check_shared": (C.c_int, [vp, C.POINTER(i64)]),
        "cdfem_comm_set_host_nbr_exchange": (C.c_int, [vp, NBR_EXCHANGE_FN, vp]),
        "cdfem_true_size": (C.c_int, [vp, C.POINTER(i64), C.POINTER(i64)]),
        "cdfem_prolongate": (C.c_int, [vp, vp, vp, C.c_int]),
        "cdfem_comm_info": (C.c_int, [vp, C.c_char_p, C.c_size_t]),
        "cdfem_partition_rcb": (C.c_int, [C.c_int, C.c_int, C.c_int, _dp, C.c_int, _ip]),
        "cdfem_sell_plan": (C.c_int, [i64, _ip, _ip, C.c_int, C.c_int, _dp, _ip, C.POINTER(i64)]),
        "cdfem_local_space_sizes": (C.c_int, [C.c_int, C.c_int, i64, _ip, _ip, C.c_int, C.POINTER(C.c_int),
                                              C.POINTER(i64), C.POINTER(C.c_int), C.POINTER(i64), C.POINTER(i64)]),
        "cdfem_local_space": (C.c_int, [C.c_int, C.c_int, i64, _ip, _ip, C.c_int, _ip, _ip, C.POINTER(i64), _ip,
                                        C.POINTER(i64), _ip]),
        "cdfem_box_sizes": (C.c_int, [C.c_int] * 7 + [C.POINTER(C.c_int), C.POINTER(i64), C.POINTER(C.c_int)]),
        "cdfem_box_mesh": (C.c_int, [C.c_int] * 7 + [C.c_double, _dp, _ip, _ip, _dp]),
        "cdfem_mesh_upload_simplex": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, _dp, i64, _ip, C.c_int, _ip]),
        "cdfem_fa_setup": (C.c_int, [vp, C.c_uint, C.c_double, _dp, C.c_double, _dp, _dp, C.c_double, _dp]),
        "cdfem_fa_csr": (C.c_int, [vp, C.c_int, C.POINTER(i64), _ip, _ip, _dp]),
        "cdfem_kuhn_sizes": (C.c_int, [C.c_int] * 3 + [C.POINTER(C.c_int), C.POINTER(i64), C.POINTER(C.c_int)]),
        "cdfem_kuhn_mesh": (C.c_int, [C.c_int] * 3 + [C.c_double, _dp, _ip, _ip, _dp]),
        "cdfem_gmsh_sizes": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(i64)]),
        "cdfem_gmsh_mesh": (C.c_int, [C.c_char_p, C.c_int, _dp, _ip, _ip, _dp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


def lib():
    """Load libcdfem.so; raises if it has not been built (no fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CdfemError(ERR_STATE, f"{LIB_PATH} not built: run __graft_entry__.build() or make")
        _lib = _declare(C.CDLL(LIB_PATH))
    return _lib


def exported_symbols_from_header(path=HEADER_PATH):
    """Function names declared in include/cdfem.h (used by the ABI export test)."""
    import re
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(cdfem_[a-z0-9_]+)\s*\(", txt)))


def device_count():
    return lib().cdfem_device_count()


def comm_unique_id() -> bytes:
    """RCCL unique id (128 bytes) created on rank 0 and broadcast to the other ranks."""
    buf = C.create_string_buffer(128)
    rc = lib().cdfem_comm_unique_id(buf)
    if rc:
        raise CdfemError(rc, "ncclGetUniqueId failed")
    return buf.raw


def comm_info(ctx=None) -> dict:
    """Backend, RCCL version and the librccl file libcdfem.so is bound to in this process."""
    buf = C.create_string_buffer(4096)
    rc = lib().cdfem_comm_info(ctx.h if ctx is not None else None, buf, len(buf))
    if rc:
        raise CdfemError(rc, "cdfem_comm_info failed")
    return dict(kv.split("=", 1) for kv in buf.value.decode().split(" "))


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _p(a):
    return None if a is None else a.ctypes.data_as(_dp)


@dataclass
class Mesh:
    dim: int
    order: int
    verts: np.ndarray      # (ne, 2^dim, dim) tensor / (ne, dim+1, dim) simplex
    dofmap: np.ndarray     # (ne, nd) int32
    nl: int
    ess: np.ndarray        # int32
    dof_xyz: np.ndarray | None = None
    simplex: bool = False

    @property
    def ne(self):
        return self.dofmap.shape[0]


def box_mesh(dim, n, order, z_range=None, perturb=0.0, with_coords=True) -> Mesh:
    """Structured [0,1]^dim mesh (or a z-slab [z0,z1) of it) generated by the library."""
    nx, ny, nz = (n, n, n) if np.isscalar(n) else (tuple(n) + (1,))[:3]
    z0, z1 = z_range if z_range is not None else (0, 0)
    L = lib()
    ne, nl, ness = C.c_int(), C.c_int64(), C.c_int()
    rc = L.cdfem_box_sizes(dim, nx, ny, nz, order, z0, z1, C.byref(ne), C.byref(nl), C.byref(ness))
    if rc:
        raise CdfemError(rc, "bad box mesh arguments")
    nv, nd = 2 ** dim, (order + 1) ** dim
    verts = np.zeros((ne.value, nv, dim))
    dofmap = np.zeros((ne.value, nd), dtype=np.int32)
    ess = np.zeros(ness.value, dtype=np.int32)
    xyz = np.zeros((nl.value, dim)) if with_coords else None
    rc = L.cdfem_box_mesh(dim, nx, ny, nz, order, z0, z1, float(perturb), _p(verts),
                          dofmap.ctypes.data_as(_ip), ess.ctypes.data_as(_ip), _p(xyz))
    if rc:
        raise CdfemError(rc, "box mesh generation failed")
    return Mesh(dim, order, verts, dofmap, nl.value, ess, xyz)


def kuhn_mesh(dim, n, order, perturb=0.0, with_coords=True) -> Mesh:
    """Kuhn simplex mesh of [0,1]^dim (n^dim cubes x dim! simplices, P1/P2; config C4)."""
    L = lib()
    ne, nl, ness = C.c_int(), C.c_int64(), C.c_int()
    rc = L.cdfem_kuhn_sizes(dim, n, order, C.byref(ne), C.byref(nl), C.byref(ness))
    if rc:
        raise CdfemError(rc, "bad Kuhn mesh arguments")
    nd = dim + 1 if order == 1 else (dim + 1) * (dim + 2) // 2
    verts = np.zeros((ne.value, dim + 1, dim))
    dofmap = np.zeros((ne.value, nd), dtype=np.int32)
    ess = np.zeros(ness.value, dtype=np.int32)
    xyz = np.zeros((nl.value, dim)) if with_coords else None
    rc = L.cdfem_kuhn_mesh(dim, n, order, float(perturb), _p(verts), dofmap.ctypes.data_as(_ip),
                           ess.ctypes.data_as(_ip), _p(xyz))
    if rc:
        raise CdfemError(rc, "Kuhn mesh generation failed (inverted element?)")
    return Mesh(dim, order, verts, dofmap, nl.value, ess, xyz, simplex=True)


def simplex_space(vxyz, elem_v, bdr_v, bdr_attr, order) -> Mesh:
    """H1 space of the given order on a simplex topology (cdfem_simplex_space): vertex coordinates
    (nv, dim), elements (ne, dim + 1) and boundary facets (nbe, dim) with their attributes; essential
    dofs on every boundary attribute."""
    L = lib()
    vx = np.ascontiguousarray(vxyz, dtype=np.float64)
    dim = vx.shape[1]
    ev, bv, ba = _i32(elem_v), _i32(bdr_v), _i32(bdr_attr)
    nl = C.c_int64()
    rc = L.cdfem_simplex_space_sizes(dim, len(vx), _p(vx), len(ev), ev.ctypes.data_as(_ip), order, C.byref(nl))
    if rc:
        raise CdfemError(rc, "bad simplex topology")
    nd = dim + 1 if order == 1 else (dim + 1) * (dim + 2) // 2 if order == 2 else 10
    verts = np.zeros((len(ev), dim + 1, dim))
    dofmap = np.zeros((len(ev), nd), dtype=np.int32)
    mask = np.zeros(nl.value, dtype=np.int32)
    xyz = np.zeros((nl.value, dim))
    rc = L.cdfem_simplex_space(dim, len(vx), _p(vx), len(ev), ev.ctypes.data_as(_ip), len(bv), bv.ctypes.data_as(_ip),
                               ba.ctypes.data_as(_ip), order, _p(verts), dofmap.ctypes.data_as(_ip),
                               mask.ctypes.data_as(_ip), _p(xyz))
    if rc:
        raise CdfemError(rc, "simplex space construction failed")
    m = Mesh(dim, order, verts, dofmap, nl.value, np.nonzero(mask)[0].astype(np.int32), xyz, simplex=True)
    m.bdr_mask = mask
    return m


def delaunay_cube(npts, seed=0):
    """A genuinely unstructured tetrahedral mesh of [0,1]^3 (BASELINE configs[3], "unstructured tet
    mesh"): the Delaunay tetrahedralisation (scipy.spatial, Qhull) of about npts random points — the 8
    corners, uniform points on the 12 edges and the 6 faces (k - 2, (k - 2)^2 each, k = npts^(1/3))
    and uniform interior points — so that no four points are coplanar except on a cube face.  The flat
    tetrahedra Qhull returns for coplanar points of one face (volume exactly 0, all four vertices in
    the face plane) are dropped, which leaves the mesh conforming; the boundary facets are the faces
    held by one tetrahedron (attribute 1).  Returns (vxyz, tets, facets, attrs) in Qhull's point
    order (unbanded: the FA setup chooses the SpMV order)."""
    from scipy.spatial import Delaunay  # host-side mesh generation only
    rng = np.random.default_rng(seed)
    k = max(3, int(round(npts ** (1.0 / 3.0))))
    parts = [np.array([[i, j, l] for i in (0.0, 1.0) for j in (0.0, 1.0) for l in (0.0, 1.0)])]
    for a in range(3):  # 4 edges along axis a
        for b0 in (0.0, 1.0):
            for b1 in (0.0, 1.0):
                e = np.empty((k - 2, 3))
                e[:, a] = rng.uniform(0.0, 1.0, k - 2)
                e[:, (a + 1) % 3], e[:, (a + 2) % 3] = b0, b1
                parts.append(e)
    for a in range(3):  # 2 faces normal to axis a
        for c in (0.0, 1.0):
            f = rng.uniform(0.0, 1.0, ((k - 2) ** 2, 3))
            f[:, a] = c
            parts.append(f)
    nb = sum(len(q) for q in parts)
    parts.append(rng.uniform(0.0, 1.0, (max(npts - nb, 1), 3)))
    pts = np.concatenate(parts)
    tets = Delaunay(pts).simplices.astype(np.int32)
    v = pts[tets]
    vol = np.einsum("ij,ij->i", np.cross(v[:, 1] - v[:, 0], v[:, 2] - v[:, 0]), v[:, 3] - v[:, 0])
    flat = np.abs(vol) <= 1e-14 * max(np.abs(vol).max(), 1e-300)
    on_face = np.zeros(len(tets), dtype=bool)
    for a in range(3):
        for c in (0.0, 1.0):
            on_face |= np.all(v[:, :, a] == c, axis=1)
    if np.any(flat & ~on_face):
        raise RuntimeError("Delaunay returned a flat tetrahedron off the cube faces (degenerate input)")
    tets = tets[~flat]
    faces = np.sort(np.concatenate([tets[:, [1, 2, 3]], tets[:, [0, 2, 3]], tets[:, [0, 1, 3]], tets[:, [0, 1, 2]]]), 1)
    uniq, cnt = np.unique(faces, axis=0, return_counts=True)
    facets = uniq[cnt == 1].astype(np.int32)
    return pts, tets, facets, np.ones(len(facets), dtype=np.int32)


def gmsh_mesh(path, order, ess_attrs=None) -> Mesh:
    """A gmsh v2.2 simplex mesh (e.g. the reference's Mesh/unit_square.msh) with an H1 space of the
    given order; essential dofs on the boundary attributes ess_attrs (None: all)."""
    L = lib()
    dim, ne, nl = C.c_int(), C.c_int(), C.c_int64()
    bpath = os.fsencode(path)
    rc = L.cdfem_gmsh_sizes(bpath, order, C.byref(dim), C.byref(ne), C.byref(nl))
    if rc:
        raise CdfemError(rc, f"cannot read gmsh mesh {path} at order {order}")
    d = dim.value
    nd = d + 1 if order == 1 else (d + 1) * (d + 2) // 2 if order == 2 else 10
    verts = np.zeros((ne.value, d + 1, d))
    dofmap = np.zeros((ne.value, nd), dtype=np.int32)
    mask = np.zeros(nl.value, dtype=np.int32)
    xyz = np.zeros((nl.value, d))
    rc = L.cdfem_gmsh_mesh(bpath, order, _p(verts), dofmap.ctypes.data_as(_ip), mask.ctypes.data_as(_ip), _p(xyz))
    if rc:
        raise CdfemError(rc, f"cannot read gmsh mesh {path}")
    sel = mask != 0 if ess_attrs is None else (mask & sum(1 << (a - 1) for a in ess_attrs)) != 0
    m = Mesh(d, order, verts, dofmap, nl.value, np.nonzero(sel)[0].astype(np.int32), xyz, simplex=True)
    m.bdr_mask = mask
    return m


def partition_rcb(mesh: Mesh, nranks) -> np.ndarray:
    """Element -> rank (recursive coordinate bisection of the element centroids; ParMesh's partition)."""
    verts = _f64(mesh.verts)
    part = np.zeros(mesh.ne, dtype=np.int32)
    rc = lib().cdfem_partition_rcb(mesh.dim, mesh.ne, verts.shape[1], _p(verts), int(nranks), part.ctypes.data_as(_ip))
    if rc:
        raise CdfemError(rc, "cdfem_partition_rcb failed")
    return part


SELL_ORDER = {"legacy": 0, "natural": 1, "rcm": 2, "auto": 3, "rcm_global": 4, "geometric": 5, "morton": 6,
              "morton_global": 7, "morton_lds": 8}


def sell_plan(rowptr, cols, mode="auto", xyz=None):
    """Order of the FA SpMV (host only; sell_plan.cpp): returns (perm, info) with perm[space row] =
    mesh row and info = {base (1 natural, 2 RCM, 3 geometric), window (0: global length sort),
    max_delta, bw_natural, bw_rcm, padding, bw_geometric} (base 4: Morton); xyz = (nl, dim) dof coordinates or None."""
    rp, cl = _i32(rowptr), _i32(cols)
    nl = len(rp) - 1
    perm = np.zeros(nl, dtype=np.int32)
    info = np.zeros(7, dtype=np.int64)
    X = None if xyz is None else _f64(xyz)
    rc = lib().cdfem_sell_plan(nl, rp.ctypes.data_as(_ip), cl.ctypes.data_as(_ip),
                               SELL_ORDER.get(mode, mode), 0 if X is None else X.shape[1], _p(X),
                               perm.ctypes.data_as(_ip), info.ctypes.data_as(C.POINTER(C.c_int64)))
    if rc:
        raise CdfemError(rc, "cdfem_sell_plan failed")
    keys = ("base", "window", "max_delta", "bw_natural", "bw_rcm")
    d = {k: int(v) for k, v in zip(keys, info[:5])}
    d["padding"] = info[5] / 1e6
    d["bw_geometric"] = int(info[6])
    return perm, d


@dataclass
class LocalSpace:
    """The rank-local piece of a partitioned mesh (cdfem_local_space): a Mesh in local numbering
    (dofs owned by lower ranks first), its global element / dof ids and the shared-dof lists."""
    mesh: Mesh
    elems: np.ndarray
    l2g: np.ndarray
    nbr_ranks: np.ndarray
    nbr_off: np.ndarray
    nbr_idx: np.ndarray
    n_not_owned: int


def local_space(mesh: Mesh, part, rank) -> LocalSpace:
    L = lib()
    dm = _i32(mesh.dofmap)
    part = _i32(part)
    ne_loc, nl_loc, n_nbr, n_sh, n_no = C.c_int(), C.c_int64(), C.c_int(), C.c_int64(), C.c_int64()
    args = (mesh.ne, dm.shape[1], int(mesh.nl), dm.ctypes.data_as(_ip), part.ctypes.data_as(_ip), int(rank))
    rc = L.cdfem_local_space_sizes(*args, C.byref(ne_loc), C.byref(nl_loc), C.byref(n_nbr), C.byref(n_sh), C.byref(n_no))
    if rc:
        raise CdfemError(rc, f"cdfem_local_space_sizes failed for rank {rank}")
    elems = np.zeros(ne_loc.value, dtype=np.int32)
    loc = np.zeros((ne_loc.value, dm.shape[1]), dtype=np.int32)
    l2g = np.zeros(nl_loc.value, dtype=np.int64)
    nr = np.zeros(n_nbr.value, dtype=np.int32)
    no = np.zeros(n_nbr.value + 1, dtype=np.int64)
    ni = np.zeros(max(n_sh.value, 1), dtype=np.int32)
    rc = L.cdfem_local_space(*args, elems.ctypes.data_as(_ip), loc.ctypes.data_as(_ip),
                             l2g.ctypes.data_as(C.POINTER(C.c_int64)), nr.ctypes.data_as(_ip),
                             no.ctypes.data_as(C.POINTER(C.c_int64)), ni.ctypes.data_as(_ip))
    if rc:
        raise CdfemError(rc, f"cdfem_local_space failed for rank {rank}")
    g2l = np.full(mesh.nl, -1, dtype=np.int64)
    g2l[l2g] = np.arange(len(l2g))
    ess = g2l[mesh.ess]
    ess = np.sort(ess[ess >= 0]).astype(np.int32)
    xyz = mesh.dof_xyz[l2g] if mesh.dof_xyz is not None else None
    m = Mesh(mesh.dim, mesh.order, np.ascontiguousarray(mesh.verts[elems]), loc, len(l2g), ess, xyz,
             simplex=mesh.simplex)
    return LocalSpace(m, elems, l2g, nr, no, ni[: n_sh.value], int(n_no.value))


class Context:
    """One GPU context (cdfem_ctx): mesh + H1 space + fused PA operator + Krylov solvers."""

    def __init__(self, device=0):
        L = lib()
        h = C.c_void_p()
        rc = L.cdfem_create(int(device), C.byref(h))
        if rc:
            raise CdfemError(rc, f"cdfem_create(device={device}) failed "
                                 f"({L.cdfem_device_count()} HIP devices visible)")
        self.h = h
        self.L = L
        self.mesh = None

    def close(self):
        if getattr(self, "h", None):
            self.L.cdfem_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _chk(self, rc, allow=()):
        if rc and rc not in allow:
            raise CdfemError(rc, self.L.cdfem_last_error(self.h).decode())
        return rc

    # -- space ---------------------------------------------------------------------------------
    def upload_mesh(self, mesh: Mesh):
        verts = _f64(mesh.verts)
        dofmap = _i32(mesh.dofmap)
        ess = _i32(mesh.ess)
        up = self.L.cdfem_mesh_upload_simplex if mesh.simplex else self.L.cdfem_mesh_upload
        self._chk(up(self.h, mesh.dim, mesh.order, dofmap.shape[0], _p(verts), int(mesh.nl),
                     dofmap.ctypes.data_as(_ip), len(ess), ess.ctypes.data_as(_ip)))
        self.mesh = mesh
        self.nl = int(mesh.nl)
        return self

    def set_structured(self, nx, ny, nz):
        """Enable the structured brick fast path (mesh must be the lexicographic box numbering)."""
        self._chk(self.L.cdfem_mesh_set_structured(self.h, int(nx), int(ny), int(nz)))
        return self

    def rule_size(self, rule):
        n = C.c_int()
        self._chk(self.L.cdfem_rule_size(self.h, rule, C.byref(n)))
        return n.value

    def quadrature_points(self, rule):
        nq = self.rule_size(rule)
        xyz = np.zeros((self.mesh.ne, nq, self.mesh.dim))
        self._chk(self.L.cdfem_quadrature_points(self.h, rule, _p(xyz), HOST))
        return xyz

    # -- operator ------------------------------------------------------------------------------
    def _form(self, kinds, kappa, alpha, conv, mass, kappa_q, kmat_q, conv_q, mass_q):
        cv = None
        if conv is not None:
            cv = np.zeros(3)
            cv[: len(conv)] = conv
        keep = [cv] + [_f64(a) if a is not None else None for a in (kappa_q, kmat_q, conv_q, mass_q)]
        f = FormCoeffs(int(kinds), float(kappa), _p(keep[1]), _p(keep[2]), float(alpha), _p(keep[0]), _p(keep[3]),
                       float(mass), _p(keep[4]))
        return f, keep

    def pa_setup(self, kinds=DIFFUSION | CONVECTION | MASS, kappa=1.0, alpha=1.0, conv=None, mass=1.0,
                 kappa_q=None, conv_q=None, mass_q=None, kmat_q=None):
        """Partial assembly of the Diffusion (+ optional symmetric MatrixCoefficient kmat_q, components
        xx,xy,yy / xx,xy,xz,yy,yz,zz per point: K = kappa I + K_q), Convection and Mass integrators."""
        f, keep = self._form(kinds, kappa, alpha, conv, mass, kappa_q, kmat_q, conv_q, mass_q)
        self._chk(self.L.cdfem_pa_setup_form(self.h, C.byref(f)))
        return self

    def fa_setup(self, kinds=DIFFUSION | CONVECTION | MASS, kappa=1.0, alpha=1.0, conv=None, mass=1.0,
                 kappa_q=None, conv_q=None, mass_q=None, kmat_q=None):
        """Full assembly (CSR on the GPU) of the same form; simplex meshes."""
        f, keep = self._form(kinds, kappa, alpha, conv, mass, kappa_q, kmat_q, conv_q, mass_q)
        self._chk(self.L.cdfem_fa_setup_form(self.h, C.byref(f)))
        return self

    def fa_csr(self, constrained=False):
        """(rowptr, cols, vals) of the assembled matrix (constrained: the FormLinearSystem one)."""
        nnz = C.c_int64()
        self._chk(self.L.cdfem_fa_csr(self.h, int(constrained), C.byref(nnz), None, None, None))
        rp = np.zeros(self.nl + 1, dtype=np.int32)
        cols = np.zeros(nnz.value, dtype=np.int32)
        vals = np.zeros(nnz.value)
        self._chk(self.L.cdfem_fa_csr(self.h, int(constrained), C.byref(nnz), rp.ctypes.data_as(_ip),
                                      cols.ctypes.data_as(_ip), _p(vals)))
        return rp, cols, vals

    def mult(self, x, constrained=False):
        x = _f64(x)
        y = np.zeros(self.nl)
        self._chk(self.L.cdfem_pa_mult(self.h, x.ctypes.data, y.ctypes.data, int(constrained), HOST))
        return y

    def diagonal(self):
        d = np.zeros(self.nl)
        self._chk(self.L.cdfem_pa_diagonal(self.h, d.ctypes.data, HOST))
        return d

    def lf_assemble(self, f_q):
        f_q = _f64(f_q)
        b = np.zeros(self.nl)
        self._chk(self.L.cdfem_lf_assemble(self.h, f_q.ctypes.data, b.ctypes.data, HOST))
        return b

    def form_linear_system(self, x, b):
        x, b = _f64(x), _f64(b)
        X, B = np.zeros(self.nl), np.zeros(self.nl)
        self._chk(self.L.cdfem_form_linear_system(self.h, x.ctypes.data, b.ctypes.data, X.ctypes.data,
                                                  B.ctypes.data, HOST))
        return X, B

    def solve(self, B, method="cg", pc="jacobi", rel_tol=1e-12, abs_tol=0.0, max_iter=500, restart=30,
              check_every=16, raise_on_fail=False):
        prm = SolverParams(CG if method == "cg" else GMRES, _PCS[pc],
                           int(max_iter), int(restart), float(rel_tol), float(abs_tol), int(check_every), 0)
        res = SolverResult()
        B = _f64(B)
        X = np.zeros(self.nl)
        rc = self.L.cdfem_solve(self.h, C.byref(prm), B.ctypes.data, X.ctypes.data, HOST, C.byref(res))
        self._chk(rc, allow=() if raise_on_fail else (ERR_NOT_CONVERGED,))
        return X, dict(converged=bool(res.converged), iterations=res.iterations,
                       final_norm=res.final_norm, initial_norm=res.initial_norm, seconds=res.seconds)

    # -- multi-GPU (z-slab element partition) ----------------------------------------------------
    def comm_init_rccl(self, rank, nranks, uid: bytes):
        """RCCL communicator from a 128-byte unique id (rank 0: comm_unique_id(), broadcast it)."""
        self._chk(self.L.cdfem_comm_init_rccl(self.h, int(rank), int(nranks), uid))

    def comm_init_torch(self, group=None):
        """Host-callback communicator over torch.distributed (any backend, e.g. gloo)."""
        import torch
        import torch.distributed as dist
        import time
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        # host seconds spent inside the callbacks (rehearsal timing: bench.py --comm host)
        self.comm_stats = {"allreduce_s": 0.0, "allreduce_calls": 0, "exchange_s": 0.0, "exchange_calls": 0}
        st = self.comm_stats

        def allreduce(buf, n, _user):
            t0 = time.perf_counter()
            try:
                a = np.ctypeslib.as_array(buf, shape=(n,))
                t = torch.from_numpy(a.copy())
                dist.all_reduce(t, group=group)
                a[:] = t.numpy()
                return 0
            except Exception:  # errors must not unwind through C
                return 1
            finally:
                st["allreduce_s"] += time.perf_counter() - t0
                st["allreduce_calls"] += 1

        def exchange(send_lo, recv_lo, send_hi, recv_hi, n, _user):
            t0 = time.perf_counter()
            try:
                reqs, outs = [], []
                if bool(send_lo):
                    reqs.append(dist.isend(torch.from_numpy(np.ctypeslib.as_array(send_lo, (n,)).copy()),
                                           rank - 1, group=group))
                    t = torch.empty(n, dtype=torch.float64)
                    reqs.append(dist.irecv(t, rank - 1, group=group))
                    outs.append((recv_lo, t))
                if bool(send_hi):
                    reqs.append(dist.isend(torch.from_numpy(np.ctypeslib.as_array(send_hi, (n,)).copy()),
                                           rank + 1, group=group))
                    t = torch.empty(n, dtype=torch.float64)
                    reqs.append(dist.irecv(t, rank + 1, group=group))
                    outs.append((recv_hi, t))
                for r in reqs:
                    r.wait()
                for ptr, t in outs:
                    np.ctypeslib.as_array(ptr, (n,))[:] = t.numpy()
                return 0
            except Exception:
                return 1
            finally:
                st["exchange_s"] += time.perf_counter() - t0
                st["exchange_calls"] += 1

        def nbr_exchange(n_nbr, ranks, off, send, recv, _user):
            try:
                reqs, outs = [], []
                tot = off[n_nbr]
                sa = np.ctypeslib.as_array(send, (tot,)).copy()
                for k in range(n_nbr):
                    a, b, r = off[k], off[k + 1], ranks[k]
                    reqs.append(dist.isend(torch.from_numpy(sa[a:b].copy()), r, group=group))
                    t = torch.empty(b - a, dtype=torch.float64)
                    reqs.append(dist.irecv(t, r, group=group))
                    outs.append((a, b, t))
                for q in reqs:
                    q.wait()
                ra = np.ctypeslib.as_array(recv, (tot,))
                for a, b, t in outs:
                    ra[a:b] = t.numpy()
                return 0
            except Exception:
                return 1

        self._cb = (ALLREDUCE_FN(allreduce), EXCHANGE_FN(exchange), NBR_EXCHANGE_FN(nbr_exchange))  # keep alive
        self._chk(self.L.cdfem_comm_init_host(self.h, rank, world, self._cb[0], self._cb[1], None))
        self._chk(self.L.cdfem_comm_set_host_nbr_exchange(self.h, self._cb[2], None))

    def comm_init_host(self, rank, world, allreduce, exchange):
        """Host-callback communicator from two Python functions (numpy views of the staging buffers):
        allreduce(a) sums the 1-D array a over the ranks in place; exchange(send_lo, recv_lo, send_hi,
        recv_hi) swaps interface planes with the ranks below / above (None where there is no neighbour).
        Used to run several ranks as threads of one process (tools/mr_kernel_list.py)."""
        def ar(buf, n, _user):
            try:
                allreduce(np.ctypeslib.as_array(buf, shape=(n,)))
                return 0
            except Exception:  # errors must not unwind through C
                return 1

        def ex(send_lo, recv_lo, send_hi, recv_hi, n, _user):
            try:
                v = [np.ctypeslib.as_array(q, (n,)) if bool(q) else None for q in (send_lo, recv_lo, send_hi, recv_hi)]
                exchange(*v)
                return 0
            except Exception:
                return 1
        self._cb = (ALLREDUCE_FN(ar), EXCHANGE_FN(ex))  # keep alive
        self._chk(self.L.cdfem_comm_init_host(self.h, int(rank), int(world), self._cb[0], self._cb[1], None))

    def set_slab(self, zlo_shared, zhi_shared):
        self._chk(self.L.cdfem_set_slab(self.h, int(bool(zlo_shared)), int(bool(zhi_shared))))

    def set_shared(self, ls: LocalSpace, check=True):
        """General partition: the shared-dof lists of this rank's LocalSpace (checked against the
        neighbours' lists by global id unless check=False; the check is collective)."""
        nr, no, ni = _i32(ls.nbr_ranks), np.ascontiguousarray(ls.nbr_off, dtype=np.int64), _i32(ls.nbr_idx)
        if len(ni) == 0:
            ni = np.zeros(1, dtype=np.int32)
        self._chk(self.L.cdfem_set_shared(self.h, len(nr), nr.ctypes.data_as(_ip),
                                          no.ctypes.data_as(C.POINTER(C.c_int64)), ni.ctypes.data_as(_ip)))
        if check:  # collective with the neighbours: the lists must pair entries by global id
            self.check_shared(ls.l2g)

    def check_shared(self, l2g):
        """cdfem_check_shared: every shared entry's global id equals the neighbour's at its position."""
        g = np.ascontiguousarray(l2g, dtype=np.int64)
        self._chk(self.L.cdfem_check_shared(self.h, g.ctypes.data_as(C.POINTER(C.c_int64))))

    def true_size(self):
        """(number of true dofs, first owned L-dof): the T-vector is the L-vector suffix."""
        nt, f = C.c_int64(), C.c_int64()
        self._chk(self.L.cdfem_true_size(self.h, C.byref(nt), C.byref(f)))
        return nt.value, f.value

    def prolongate(self, X):
        """x = P X (owned entries from X, the other shared entries from their owner rank)."""
        X = _f64(X)
        x = np.zeros(self.nl)
        self._chk(self.L.cdfem_prolongate(self.h, X.ctypes.data, x.ctypes.data, HOST))
        return x

    # -- device-resident variants (benchmarks) ------------------------------------------------------
    def alloc(self, nbytes):
        p = C.c_void_p()
        self._chk(self.L.cdfem_alloc(self.h, int(nbytes), C.byref(p)))
        return p.value

    def free(self, ptr):
        self._chk(self.L.cdfem_free(self.h, C.c_void_p(ptr)))

    def to_device(self, a):
        a = _f64(a)
        p = self.alloc(a.nbytes)
        self._chk(self.L.cdfem_memcpy(self.h, C.c_void_p(p), DEVICE, a.ctypes.data, HOST, a.nbytes))
        return p

    def from_device(self, ptr, n):
        out = np.zeros(n)
        self._chk(self.L.cdfem_memcpy(self.h, out.ctypes.data, HOST, C.c_void_p(ptr), DEVICE, out.nbytes))
        return out

    def solve_device(self, dB, dX, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=100,
                     restart=30, check_every=0):
        prm = SolverParams(CG if method == "cg" else GMRES, _PCS[pc],
                           int(max_iter), int(restart), float(rel_tol), float(abs_tol),
                           int(check_every if check_every else max_iter), 0)
        res = SolverResult()
        rc = self.L.cdfem_solve(self.h, C.byref(prm), C.c_void_p(dB), C.c_void_p(dX), DEVICE, C.byref(res))
        self._chk(rc, allow=(ERR_NOT_CONVERGED,))
        return dict(converged=bool(res.converged), iterations=res.iterations, final_norm=res.final_norm,
                    initial_norm=res.initial_norm, seconds=res.seconds)

    def mult_device(self, dx, dy, constrained=False):
        self._chk(self.L.cdfem_pa_mult(self.h, C.c_void_p(dx), C.c_void_p(dy), int(constrained), DEVICE))

    def synchronize(self):
        self._chk(self.L.cdfem_synchronize(self.h))

    def stream_bench(self, mode=0, nbytes=2 << 30, reps=10):
        """Measured HBM bandwidth (GB/s): mode 0 read 16 B/lane, 1 read 8 B/lane, 2 copy."""
        g = C.c_double()
        self._chk(self.L.cdfem_stream_bench(self.h, int(mode), int(nbytes), int(reps), C.byref(g)))
        return g.value

    def fp64_bench(self, mode=0, reps=10):
        """Achieved f64 TFLOP/s of a compute probe: mode 0 VALU v_fma_f64, 1 v_mfma_f64_16x16x4_f64."""
        t = C.c_double()
        self._chk(self.L.cdfem_fp64_bench(self.h, int(mode), int(reps), C.byref(t)))
        return t.value

    def set_option(self, key, value):
        self._chk(self.L.cdfem_set_option(self.h, key.encode(), int(value)))

    # -- profiling -----------------------------------------------------------------------------------
    def profile(self, on=True):
        self._chk(self.L.cdfem_profile_enable(self.h, int(on)))
        self._chk(self.L.cdfem_profile_reset(self.h))

    def profile_read(self, kernel):
        ms, n = C.c_double(), C.c_int64()
        self._chk(self.L.cdfem_profile_read(self.h, kernel, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def profile_launches(self, kernel):
        """Per-launch milliseconds of kernel id since the last reset (launch order)."""
        n = C.c_int64()
        self._chk(self.L.cdfem_profile_launches(self.h, kernel, None, 0, C.byref(n)))
        out = np.zeros(n.value)
        self._chk(self.L.cdfem_profile_launches(self.h, kernel, out.ctypes.data, n.value, C.byref(n)))
        return out

    def kernel_name(self, kernel):
        """HIP kernel name of kernel id in the current configuration (assembled-operator apply)."""
        buf = C.create_string_buffer(128)
        self._chk(self.L.cdfem_kernel_name(self.h, kernel, buf, 128))
        return buf.value.decode()

    def kernel_flops(self, kernel):
        """Algorithmic f64 flops of one launch of the 3D PA apply (FMA = 2)."""
        f = C.c_double()
        self._chk(self.L.cdfem_kernel_flops(self.h, kernel, C.byref(f)))
        return f.value

    def kernel_bytes(self, kernel):
        b = C.c_double()
        self._chk(self.L.cdfem_kernel_bytes(self.h, kernel, C.byref(b)))
        return b.value
