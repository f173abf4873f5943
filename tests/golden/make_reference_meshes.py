#!/usr/bin/env python3
"""Make tests/golden/reference_meshes.npz: the reference's two default meshes as data fixtures.

Test infrastructure.  Input (this container only): the reference's own gmsh v2.2 files
  /root/reference/myapps/convection_diffusion/Mesh/unit_square.msh  (Input/input_2d.yaml:1)
  /root/reference/myapps/convection_diffusion/Mesh/unit_circle.msh  (Input/input_2d_circle.yaml:1)
read with an independent minimal parser (below).  Output, per mesh <name> in {square, circle}:
  <name>_node_id    int64 (N,)    gmsh node ids, file order
  <name>_node_xyz   float64 (N,3) coordinates (the file's decimal text parsed to the nearest double)
  <name>_elem_id    int64 (E,)    gmsh element ids, file order
  <name>_elem_type  int32 (E,)    1 = 2-node line, 2 = 3-node triangle
  <name>_elem_phys  int32 (E,)    physical tag (first tag)
  <name>_elem_geom  int32 (E,)    elementary tag (second tag)
  <name>_elem_nodes int64 (E,3)   node ids (-1 padded for lines)
  <name>_physical   str           the $PhysicalNames block as JSON [[dim, tag, name], ...]
tests/reference_meshes.py writes the same gmsh v2.2 file back from these arrays, so the GPU box
(where /root/reference does not exist) feeds the product reader the reference's mesh.

usage: python tests/golden/make_reference_meshes.py [REFERENCE_MESH_DIR]
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_MESH_DIR = "/root/reference/myapps/convection_diffusion/Mesh"
FILES = {"square": "unit_square.msh", "circle": "unit_circle.msh"}


def parse_msh(path):
    """Independent parse of a gmsh v2.2 ASCII file: nodes, elements (lines, triangles) and names."""
    with open(path) as f:
        lines = f.read().splitlines()
    out = {"physical": []}
    i = 0
    while i < len(lines):
        tag = lines[i].strip()
        if tag == "$MeshFormat":
            ver = lines[i + 1].split()
            assert ver[0].startswith("2.") and ver[1] == "0", ver
            i += 2
        elif tag == "$PhysicalNames":
            n = int(lines[i + 1])
            for ln in lines[i + 2:i + 2 + n]:
                d, t, name = ln.split(maxsplit=2)
                out["physical"].append([int(d), int(t), name.strip('"')])
            i += n + 2
        elif tag == "$Nodes":
            n = int(lines[i + 1])
            rows = [ln.split() for ln in lines[i + 2:i + 2 + n]]
            out["node_id"] = np.array([int(r[0]) for r in rows], dtype=np.int64)
            out["node_xyz"] = np.array([[float(v) for v in r[1:4]] for r in rows], dtype=np.float64)
            i += n + 2
        elif tag == "$Elements":
            n = int(lines[i + 1])
            eid, typ, phys, geom, nodes = [], [], [], [], []
            for ln in lines[i + 2:i + 2 + n]:
                t = [int(v) for v in ln.split()]
                ntag = t[2]
                vs = t[3 + ntag:]
                assert t[1] in (1, 2) and len(vs) == (2 if t[1] == 1 else 3), ln
                eid.append(t[0])
                typ.append(t[1])
                phys.append(t[3])
                geom.append(t[4] if ntag > 1 else t[3])
                nodes.append(vs + [-1] * (3 - len(vs)))
            out.update(elem_id=np.array(eid, dtype=np.int64), elem_type=np.array(typ, dtype=np.int32),
                       elem_phys=np.array(phys, dtype=np.int32), elem_geom=np.array(geom, dtype=np.int32),
                       elem_nodes=np.array(nodes, dtype=np.int64))
            i += n + 2
        else:
            i += 1
    return out


def main(ref_dir=REF_MESH_DIR):
    arrays = {}
    for name, fn in FILES.items():
        m = parse_msh(os.path.join(ref_dir, fn))
        for k, v in m.items():
            arrays[f"{name}_{k}"] = np.array(json.dumps(v)) if k == "physical" else v
        ntri = int((m["elem_type"] == 2).sum())
        nlin = int((m["elem_type"] == 1).sum())
        print(f"{fn}: {len(m['node_id'])} nodes, {ntri} triangles, {nlin} boundary lines")
    out = os.path.join(HERE, "reference_meshes.npz")
    np.savez_compressed(out, **arrays)
    print("wrote", out)


if __name__ == "__main__":
    main(*sys.argv[1:])
