"""The reference's default meshes (Mesh/unit_square.msh, Mesh/unit_circle.msh) from the committed
fixture tests/golden/reference_meshes.npz (made by tests/golden/make_reference_meshes.py).

write_msh(name, path) writes the gmsh v2.2 ASCII file back: node coordinates as the shortest decimal
that round-trips the stored double (the file's own text parses to that same double), so the product
reader sees the reference mesh bit for bit on the GPU box, where /root/reference does not exist.
Test infrastructure.
"""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "reference_meshes.npz")
REF_MESH_DIR = "/root/reference/myapps/convection_diffusion/Mesh"
REF_FILES = {"square": "unit_square.msh", "circle": "unit_circle.msh"}
# (triangles, vertices, boundary edges) of the two files
SIZES = {"square": (938, 510, 80), "circle": (3056, 1593, 128)}


def load(name):
    with np.load(FIXTURE, allow_pickle=False) as z:
        d = {k[len(name) + 1:]: z[k] for k in z.files if k.startswith(name + "_")}
    d["physical"] = json.loads(str(d["physical"]))
    return d


def write_msh(name, path):
    m = load(name)
    with open(path, "w") as f:
        f.write("$MeshFormat\n2.2 0 8\n$EndMeshFormat\n")
        f.write(f"$PhysicalNames\n{len(m['physical'])}\n")
        for d, t, nm in m["physical"]:
            f.write(f'{d} {t} "{nm}"\n')
        f.write("$EndPhysicalNames\n")
        f.write(f"$Nodes\n{len(m['node_id'])}\n")
        for nid, (x, y, z) in zip(m["node_id"], m["node_xyz"]):
            f.write(f"{nid} {float(x)!r} {float(y)!r} {float(z)!r}\n")
        f.write("$EndNodes\n")
        f.write(f"$Elements\n{len(m['elem_id'])}\n")
        for eid, typ, ph, ge, nodes in zip(m["elem_id"], m["elem_type"], m["elem_phys"], m["elem_geom"],
                                          m["elem_nodes"]):
            vs = " ".join(str(int(v)) for v in nodes if v >= 0)
            f.write(f"{eid} {typ} 2 {ph} {ge} {vs}\n")
        f.write("$EndElements\n")
    return path


def reference_file(name):
    """Path of the reference's own file when /root/reference is present (this container), else None."""
    p = os.path.join(REF_MESH_DIR, REF_FILES[name])
    return p if os.path.exists(p) else None
