"""The unstructured tetrahedral mesh family of the c4u bench config (cdfem.delaunay_cube: Delaunay
tetrahedralisation of random points in the unit cube, scipy/Qhull on the host) and the product's
H1 space on it (cdfem_simplex_space).  CPU only: the mesh must be a conforming, positively oriented
tetrahedralisation of exactly the cube, with its boundary on the cube's faces, before any GPU parity
test (tests/test_gpu_fa.py::test_fa_delaunay_parity) or bench line uses it."""
import numpy as np
import pytest

import cdfem


@pytest.mark.parametrize("npts,seed", [(500, 0), (4000, 3)])
def test_delaunay_cube_is_a_conforming_mesh_of_the_cube(npts, seed):
    pts, tets, facets, attrs = cdfem.delaunay_cube(npts, seed=seed)
    assert len(pts) == npts and tets.shape[1] == 4 and facets.shape[1] == 3
    v = pts[tets]
    vol = np.abs(np.einsum("ij,ij->i", np.cross(v[:, 1] - v[:, 0], v[:, 2] - v[:, 0]), v[:, 3] - v[:, 0])) / 6
    assert vol.min() > 0.0 and abs(vol.sum() - 1.0) <= 1e-12
    # conforming: every face is held by one tetrahedron (the boundary) or two
    faces = np.sort(np.concatenate([tets[:, [1, 2, 3]], tets[:, [0, 2, 3]], tets[:, [0, 1, 3]], tets[:, [0, 1, 2]]]), 1)
    _, cnt = np.unique(faces, axis=0, return_counts=True)
    assert set(np.unique(cnt)) <= {1, 2} and (cnt == 1).sum() == len(facets)
    # the boundary facets tile the six faces: each lies in one face plane, total area 6
    fx = pts[facets]
    plane = np.zeros(len(facets), dtype=bool)
    for a in range(3):
        for c in (0.0, 1.0):
            plane |= np.all(fx[:, :, a] == c, axis=1)
    assert plane.all()
    area = 0.5 * np.linalg.norm(np.cross(fx[:, 1] - fx[:, 0], fx[:, 2] - fx[:, 0]), axis=1).sum()
    assert abs(area - 6.0) <= 1e-12
    assert np.all(attrs == 1)
    # deterministic for a seed
    again = cdfem.delaunay_cube(npts, seed=seed)
    np.testing.assert_array_equal(again[1], tets)


@pytest.mark.parametrize("order", [1, 2])
def test_simplex_space_on_the_delaunay_mesh(order):
    pts, tets, facets, attrs = cdfem.delaunay_cube(2000, seed=1)
    m = cdfem.simplex_space(pts, tets, facets, attrs, order)
    v = m.verts
    vol = np.einsum("ij,ij->i", np.cross(v[:, 1] - v[:, 0], v[:, 2] - v[:, 0]), v[:, 3] - v[:, 0]) / 6
    assert vol.min() > 0.0                      # re-oriented to det J > 0
    edges = np.unique(np.sort(tets[:, [[0, 1], [0, 2], [0, 3], [1, 2], [1, 3], [2, 3]]].reshape(-1, 2), 1), axis=0)
    assert m.nl == len(pts) + (order == 2) * len(edges)
    # essential dofs = the dofs on the cube's surface
    on = np.abs(m.dof_xyz - 0.5).max(1) >= 0.5 - 1e-12
    np.testing.assert_array_equal(np.sort(m.ess), np.nonzero(on)[0])
