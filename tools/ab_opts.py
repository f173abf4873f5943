"""Interleaved in-process A/B of context options on a brick CG workload (default C2: 64^3 hex p = 2,
D + C + M), GPU box only.  Each variant is its own context with the given set_option values (set
before upload and setup); per round every variant runs one fixed Jacobi-CG solve uninstrumented
(us per iteration, host clock) and one with profiling events (apply / update kernel averages).

    python tools/ab_opts.py --variant "cg_xfold=0" --variant "cg_xfold=1" [--rounds 5] [--iters 100]
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
ap.add_argument("--variant", action="append", required=True)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=100)
ap.add_argument("--n", type=int, default=64)
ap.add_argument("--p", type=int, default=2)
ap.add_argument("--kinds", type=int, default=7)
args = ap.parse_args()

n = args.n
mesh = cdfem.box_mesh(3, n, args.p, with_coords=False)
b = np.random.default_rng(1).uniform(-1, 1, mesh.nl)
runs = []
for v in args.variant:
    ctx = cdfem.Context(0)
    opts = {}
    for kv in filter(None, v.split(",")):
        k, val = kv.split("=")
        opts[k] = int(val)
        ctx.set_option(k, int(val))
    ctx.upload_mesh(mesh).set_structured(n, n, n)
    ctx.pa_setup(kinds=args.kinds, kappa=0.1, conv=(1.0, -2.0, 0.5), mass=1.0)
    _, B = ctx.form_linear_system(np.zeros(mesh.nl), b)
    runs.append(dict(label=v, ctx=ctx, dB=ctx.to_device(B), dX=ctx.alloc(8 * mesh.nl), it_us=[], apply_us=[],
                     upd_us=[], e2l_us=[]))
for rnd in range(args.rounds + 1):
    for r in runs:
        ctx = r["ctx"]
        ctx.synchronize()
        t0 = time.perf_counter()
        info = ctx.solve_device(r["dB"], r["dX"], method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0,
                                max_iter=args.iters, check_every=args.iters)
        ctx.synchronize()
        dt = time.perf_counter() - t0
        r["x"] = ctx.from_device(r["dX"], mesh.nl)
        ctx.profile(True)
        ctx.solve_device(r["dB"], r["dX"], method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0,
                         max_iter=args.iters, check_every=args.iters)
        ctx.synchronize()
        a = ctx.profile_read(cdfem.K_APPLY)
        u = ctx.profile_read(cdfem.K_UPDATE)
        e = ctx.profile_read(cdfem.K_E2L)
        ctx.profile(False)
        if rnd:
            r["it_us"].append(dt / info["iterations"] * 1e6)
            r["apply_us"].append(a[0] / max(a[1], 1) * 1e3)
            r["upd_us"].append(u[0] / max(u[1], 1) * 1e3)
            r["e2l_us"].append(e[0] / max(e[1], 1) * 1e3)
out = {"dofs": mesh.nl, "cg_iters": args.iters, "rounds": args.rounds}
x0 = runs[0]["x"]
for r in runs:
    med = {k: float(np.median(r[k])) for k in ("it_us", "apply_us", "upd_us", "e2l_us")}
    med["dof_iter_per_s"] = mesh.nl / (med["it_us"] * 1e-6)
    med["rel_diff_vs_first"] = float(np.linalg.norm(r["x"] - x0) / np.linalg.norm(x0))
    med["bitwise_first"] = bool(np.array_equal(r["x"], x0))
    med["it_us_all"] = [round(t, 2) for t in r["it_us"]]
    out[r["label"]] = med
print(json.dumps(out, indent=1))
