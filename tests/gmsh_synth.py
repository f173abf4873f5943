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
