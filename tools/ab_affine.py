"""Interleaved in-process A/B of the affine-factor brick applies (pa_affine 2 Kronecker form, 1 point
data from the factors) against the per-point qdata stream (pa_affine 0) on the C2 workload (64^3
hex p = 2, D + C + M), GPU box only.

Two contexts (pa_affine is read by pa_setup); per round each runs a fixed Jacobi-CG solve (apply
launch time from the profiling events) and a fixed GMRES(30) solve.  Prints medians and the
relative difference of the two contexts' iterates.

    python tools/ab_affine.py [--rounds 5] [--iters 100] [--n 64] [--forms 2,1,0]
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
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=100)
ap.add_argument("--gmres-iters", type=int, default=60)
ap.add_argument("--n", type=int, default=64)
ap.add_argument("--p", type=int, default=2)
ap.add_argument("--forms", default="2,1,0")
args = ap.parse_args()

n = args.n
mesh = cdfem.box_mesh(3, n, args.p, with_coords=False)
b = np.random.default_rng(1).uniform(-1, 1, mesh.nl)
runs = []
for aff in [int(f) for f in args.forms.split(",")]:
    ctx = cdfem.Context(0)
    ctx.set_option("pa_affine", aff)
    ctx.upload_mesh(mesh).set_structured(n, n, n)
    ctx.pa_setup(kinds=7, kappa=0.1, conv=(1.0, -2.0, 0.5), mass=1.0)
    _, B = ctx.form_linear_system(np.zeros(mesh.nl), b)
    runs.append(dict(label=f"pa_affine={aff}", ctx=ctx, dB=ctx.to_device(B), dX=ctx.alloc(8 * mesh.nl),
                     bytes=ctx.kernel_bytes(cdfem.K_APPLY), cg_us=[], apply_us=[], upd_us=[], gm_us=[]))
for rnd in range(args.rounds + 1):
    for r in runs:
        ctx = r["ctx"]
        ctx.profile(True)
        ctx.synchronize()
        t0 = time.perf_counter()
        info = ctx.solve_device(r["dB"], r["dX"], method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0,
                                max_iter=args.iters)
        ctx.synchronize()
        dt = time.perf_counter() - t0
        a = ctx.profile_read(cdfem.K_APPLY)
        u = ctx.profile_read(cdfem.K_UPDATE)
        ctx.profile(False)
        r["x_cg"] = ctx.from_device(r["dX"], mesh.nl)
        ctx.synchronize()
        t1 = time.perf_counter()
        ig = ctx.solve_device(r["dB"], r["dX"], method="gmres", pc="jacobi", rel_tol=0.0, abs_tol=0.0,
                              max_iter=args.gmres_iters, restart=30)
        ctx.synchronize()
        dg = time.perf_counter() - t1
        r["x_gm"] = ctx.from_device(r["dX"], mesh.nl)
        if rnd:
            r["cg_us"].append(dt / info["iterations"] * 1e6)
            r["apply_us"].append(a[0] / max(a[1], 1) * 1e3)
            r["upd_us"].append(u[0] / max(u[1], 1) * 1e3)
            r["gm_us"].append(dg / ig["iterations"] * 1e6)


def rel(a, c):
    return float(np.linalg.norm(a - c) / np.linalg.norm(c))


out = {"dofs": mesh.nl, "cg_iters": args.iters, "gmres_iters": args.gmres_iters,
       "rel_diff_cg_vs_last": [rel(r["x_cg"], runs[-1]["x_cg"]) for r in runs],
       "rel_diff_gmres_vs_last": [rel(r["x_gm"], runs[-1]["x_gm"]) for r in runs]}
for r in runs:
    med = {k: float(np.median(r[k])) for k in ("cg_us", "apply_us", "upd_us", "gm_us")}
    med["apply_bytes"] = r["bytes"]
    med["cg_dof_iter_per_s"] = mesh.nl / (med["cg_us"] * 1e-6)
    med["gmres_dof_iter_per_s"] = mesh.nl / (med["gm_us"] * 1e-6)
    out[r["label"]] = med
print(json.dumps(out, indent=1))
