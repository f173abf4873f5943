"""Wall time per GMRES(30)+Jacobi iteration on the small problems the reference's drivers actually
run (launch- and latency-bound, not bandwidth-bound), GPU box only.

Problems (fixed iteration count, tolerances 0):
  square  the reference's Mesh/unit_square.msh (fixture), P3 triangles, FA: 4,295 dofs
  q64     64 x 64 quads p = 2, PA (diffusion_mms-sized): 16,641 dofs
  q128    128 x 128 quads p = 2, PA: 66,049 dofs
  t16     16^3 x 6 Kuhn tets P2, FA: 35,937 dofs
Each variant (set_option key=value, or none) gets its own context per problem; rounds interleave.

    python tools/small_solve.py [--iters 300] [--rounds 5] [--variants "base:,graph:gm_graph=1"]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "continuum-mechanics-mfem_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import cdfem  # noqa: E402
import reference_meshes as R  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=300)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--problems", default="square,q64,q128,t16")
ap.add_argument("--variants", default="base:")
ap.add_argument("--method", default="gmres")
args = ap.parse_args()


def problem(name):
    if name == "square":
        d = tempfile.mkdtemp()
        path = R.write_msh("square", os.path.join(d, "unit_square.msh"))
        m = cdfem.gmsh_mesh(path, 3)
        return m, "fa", (0.1, 1.0, (1.0, -2.0))
    if name.startswith("q"):
        n = int(name[1:])
        return cdfem.box_mesh(2, (n, n), 2, with_coords=False), "pa", (0.1, 1.0, (1.0, -2.0))
    if name.startswith("t"):
        n = int(name[1:])
        return cdfem.kuhn_mesh(3, n, 2, with_coords=False), "fa", (0.1, 1.0, (1.0, -2.0, 0.5))
    raise SystemExit(f"unknown problem {name}")


variants = []
for spec in args.variants.split(","):
    label, opts = spec.split(":")
    variants.append((label, [kv.split("=") for kv in filter(None, opts.split("+"))]))

out = {}
for pname in args.problems.split(","):
    m, asm, (kappa, s, c) = problem(pname)
    b = np.random.default_rng(5).uniform(-1, 1, m.nl)
    runs = []
    for label, opts in variants:
        ctx = cdfem.Context(0)
        for k, v in opts:
            ctx.set_option(k, int(v))
        ctx.upload_mesh(m)
        setup = ctx.fa_setup if asm == "fa" else ctx.pa_setup
        setup(kinds=7, kappa=kappa, alpha=1.0, conv=c, mass=s)
        _, B = ctx.form_linear_system(np.zeros(m.nl), b)
        runs.append(dict(label=label, ctx=ctx, dB=ctx.to_device(B), dX=ctx.alloc(8 * m.nl), t=[]))
    ref = None
    for rnd in range(args.rounds + 1):
        for r in runs:
            ctx = r["ctx"]
            ctx.synchronize()
            t0 = time.perf_counter()
            info = ctx.solve_device(r["dB"], r["dX"], method=args.method, pc="jacobi", rel_tol=0.0, abs_tol=0.0,
                                    max_iter=args.iters, restart=30)
            ctx.synchronize()
            dt = time.perf_counter() - t0
            x = ctx.from_device(r["dX"], m.nl)
            if ref is None:
                ref = x
            r["err"] = float(np.abs(x - ref).max() / max(np.abs(ref).max(), 1e-300))
            if rnd:
                r["t"].append(dt / max(info["iterations"], 1) * 1e6)
    out[pname] = {"dofs": m.nl, **{r["label"]: {"us_per_iter": float(np.median(r["t"])),
                                                 "min": float(np.min(r["t"])), "max_rel_diff": r["err"]}
                                   for r in runs}}
    for r in runs:
        r["ctx"].free(r["dB"])
        r["ctx"].free(r["dX"])
        r["ctx"].close()
    print(json.dumps({pname: out[pname]}), flush=True)
print(json.dumps(out, indent=1))
