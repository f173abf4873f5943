"""Synthetic gmsh v2.2 ASCII meshes for the reader tests (test infrastructure, no reference files).

Written in the format the reference's inputs use (Mesh/*.msh, read at
linear_convection_diffusion_2D.cpp:290):
  * $MeshFormat 2.2 0 8, $PhysicalNames, $Nodes, $Elements;
  * domain triangles (type 2, physical tag 1);
  * boundary lines (type 1) with physical tags 1 bottom, 2 right, 3 top, 4 left, following
    Mesh/unit_square.geo's convention.
To exercise the reader, the writer also:
  * uses non-contiguous node ids;
  * perturbs interior nodes;
  * flips the orientation of every third triangle (clockwise as written);
  * adds an unused node and a type-15 point element.
"""
import numpy as np


def write_square(path, n, perturb=0.2, seed=0, shift_ids=1000):
    rng = np.random.default_rng(seed)
    h = 1.0 / n
    ids, xy = {}, []
    for j in range(n + 1):
        for i in range(n + 1):
            x, y = i * h, j * h
            if 0 < i < n and 0 < j < n:
                x += perturb * h * rng.uniform(-0.5, 0.5)
                y += perturb * h * rng.uniform(-0.5, 0.5)
            ids[(i, j)] = shift_ids + 3 * (j * (n + 1) + i)  # non-contiguous ids
            xy.append((ids[(i, j)], x, y))
    unused = shift_ids + 3 * (n + 1) ** 2 + 7
    els = []
    # boundary lines: bottom (1), right (2), top (3), left (4)
    for i in range(n):
        els.append((1, 1, ids[(i, 0)], ids[(i + 1, 0)]))
        els.append((1, 2, ids[(n, i)], ids[(n, i + 1)]))
        els.append((1, 3, ids[(i + 1, n)], ids[(i, n)]))
        els.append((1, 4, ids[(0, i + 1)], ids[(0, i)]))
    els.append((15, 1, ids[(0, 0)]))
    k = 0
    for j in range(n):
        for i in range(n):
            a, b, c, d = ids[(i, j)], ids[(i + 1, j)], ids[(i + 1, j + 1)], ids[(i, j + 1)]
            for tri in ((a, b, c), (a, c, d)) if (i + j) % 2 == 0 else ((a, b, d), (b, c, d)):
                if k % 3 == 2:
                    tri = (tri[0], tri[2], tri[1])  # clockwise as written
                els.append((2, 1) + tri)
                k += 1
    with open(path, "w") as f:
        f.write("$MeshFormat\n2.2 0 8\n$EndMeshFormat\n")
        f.write('$PhysicalNames\n5\n1 1 "bottom"\n1 2 "right"\n1 3 "top"\n1 4 "left"\n2 1 "domain"\n'
                "$EndPhysicalNames\n")
        f.write(f"$Nodes\n{len(xy) + 1}\n")
        for nid, x, y in xy:
            f.write(f"{nid} {x!r} {y!r} 0\n")
        f.write(f"{unused} 0.5 0.5 0\n$EndNodes\n")
        f.write(f"$Elements\n{len(els)}\n")
        for e, el in enumerate(els, start=1):
            typ, tag, *nodes = el
            f.write(f"{e} {typ} 2 {tag} {tag} " + " ".join(str(v) for v in nodes) + "\n")
        f.write("$EndElements\n")
    return {"n_nodes": (n + 1) ** 2, "n_tri": 2 * n * n, "n_bdr_edges": 4 * n}


def read_triangles(path):
    """Minimal independent parse: node coordinates and domain triangles (for cross-checks)."""
    nodes, tris = {}, []
    with open(path) as f:
        lines = f.read().splitlines()
    i = 0
    while i < len(lines):
        if lines[i] == "$Nodes":
            m = int(lines[i + 1])
            for ln in lines[i + 2:i + 2 + m]:
                t = ln.split()
                nodes[int(t[0])] = (float(t[1]), float(t[2]))
            i += m + 2
        elif lines[i] == "$Elements":
            m = int(lines[i + 1])
            for ln in lines[i + 2:i + 2 + m]:
                t = ln.split()
                if t[1] == "2":
                    nt = int(t[2])
                    tris.append(tuple(int(v) for v in t[3 + nt:]))
            i += m + 2
        else:
            i += 1
    return nodes, tris


def write_circle(path, nr, perturb=0.15, seed=0, shift_ids=500):
    """Unit disk as the reference's Mesh/unit_circle.geo describes it (centre (0,0), radius 1, one
    boundary curve with physical tag 1, domain tag 1): nr concentric rings of 6k vertices, the outer
    ring exactly on r = 1, annuli triangulated by merging the two rings by angle (6 nr^2 triangles).
    Interior vertices are jittered; every fourth triangle is written clockwise."""
    rng = np.random.default_rng(seed)
    rings = [[(0.0, 0.0)]]
    for k in range(1, nr + 1):
        n = 6 * k
        off = 0.5 * (k % 2) * 2 * np.pi / n
        ring = []
        for j in range(n):
            a = off + 2 * np.pi * j / n
            r = k / nr
            if k < nr:
                r += perturb / nr * rng.uniform(-0.5, 0.5)
                a += perturb * np.pi / n * rng.uniform(-0.5, 0.5)
            ring.append((float(r * np.cos(a)), float(r * np.sin(a))))
        rings.append(ring)
    ids, xy = [], []
    for k, ring in enumerate(rings):
        ids.append([])
        for j, (x, y) in enumerate(ring):
            nid = shift_ids + 2 * len(xy)
            ids[k].append(nid)
            xy.append((nid, x, y))

    def ang(p):
        return np.arctan2(p[1], p[0]) % (2 * np.pi)

    tris = []
    for j in range(6):  # fan around the centre
        tris.append((ids[0][0], ids[1][j], ids[1][(j + 1) % 6]))
    for k in range(2, nr + 1):
        inner, outer = rings[k - 1], rings[k]
        m, n = len(inner), len(outer)
        ai = [ang(p) for p in inner]
        bo = [ang(p) for p in outer]
        # start both walks at the smallest angle of each ring
        i0, j0 = int(np.argmin(ai)), int(np.argmin(bo))
        a_un = [ai[(i0 + t) % m] + (2 * np.pi if (i0 + t) % m < i0 else 0.0) for t in range(m + 1)]
        a_un[m] = a_un[0] + 2 * np.pi
        b_un = [bo[(j0 + t) % n] + (2 * np.pi if (j0 + t) % n < j0 else 0.0) for t in range(n + 1)]
        b_un[n] = b_un[0] + 2 * np.pi
        i = j = 0
        while i < m or j < n:
            I, I1 = ids[k - 1][(i0 + i) % m], ids[k - 1][(i0 + i + 1) % m]
            J, J1 = ids[k][(j0 + j) % n], ids[k][(j0 + j + 1) % n]
            if j < n and (i == m or b_un[j + 1] <= a_un[i + 1]):
                tris.append((I, J, J1))
                j += 1
            else:
                tris.append((I, J, I1))
                i += 1
    els = []
    outer_ids = ids[nr]
    for j in range(len(outer_ids)):
        els.append((1, 1, outer_ids[j], outer_ids[(j + 1) % len(outer_ids)]))
    for t, tri in enumerate(tris):
        if t % 4 == 3:
            tri = (tri[0], tri[2], tri[1])
        els.append((2, 1) + tuple(tri))
    with open(path, "w") as f:
        f.write("$MeshFormat\n2.2 0 8\n$EndMeshFormat\n")
        f.write('$PhysicalNames\n2\n1 1 "boundary"\n2 1 "domain"\n$EndPhysicalNames\n')
        f.write(f"$Nodes\n{len(xy)}\n")
        for nid, x, y in xy:
            f.write(f"{nid} {x!r} {y!r} 0\n")
        f.write("$EndNodes\n")
        f.write(f"$Elements\n{len(els)}\n")
        for e, el in enumerate(els, start=1):
            typ, tag, *nodes = el
            f.write(f"{e} {typ} 2 {tag} {tag} " + " ".join(str(v) for v in nodes) + "\n")
        f.write("$EndElements\n")
    return {"n_nodes": len(xy), "n_tri": len(tris), "n_bdr_edges": len(outer_ids)}
