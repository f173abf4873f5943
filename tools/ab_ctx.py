"""Context-to-context spread of the C2 brick CG (GPU box only): K contexts of the same 64^3 p=2
workload, each with its own allocations, solved interleaved; prints the median microseconds per
CG iteration of each context.  Separates buffer-placement effects from code effects.

Usage: python tools/ab_ctx.py [--contexts K] [--rounds R] [--iters N]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "continuum-mechanics-mfem_amd", "python"))
import cdfem  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--contexts", type=int, default=4)
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--iters", type=int, default=200)
ap.add_argument("--n", type=int, default=64)
args = ap.parse_args()

n = args.n
mesh = cdfem.box_mesh(3, n, 2, with_coords=False)
b = np.random.default_rng(1).uniform(-1, 1, mesh.nl)
ctxs = []
for k in range(args.contexts):
    ctx = cdfem.Context(0)
    ctx.upload_mesh(mesh).set_structured(n, n, n)
    ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=(1.0, -2.0, 0.5), mass=1.0)
    _, B = ctx.form_linear_system(np.zeros(mesh.nl), b)
    ctxs.append(dict(ctx=ctx, dB=ctx.to_device(B), dX=ctx.alloc(8 * mesh.nl), us=[]))
for rnd in range(args.rounds + 1):
    for c in ctxs:
        c["ctx"].synchronize()
        t0 = time.perf_counter()
        info = c["ctx"].solve_device(c["dB"], c["dX"], method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0,
                                     max_iter=args.iters, check_every=args.iters)
        dt = time.perf_counter() - t0
        if rnd:
            c["us"].append(dt / info["iterations"] * 1e6)
print(json.dumps({f"ctx{k}": round(float(np.median(c["us"])), 2) for k, c in enumerate(ctxs)}, indent=1))
