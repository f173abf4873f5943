"""Interleaved in-process A/B of run-time options on the C2 GMRES(30) + Jacobi leg (64^3 hex p=2,
D+C+M; the reference's solver, Input/petsc.opts), GPU box only.  One context; options are set
before each solve.  Prints per variant the median operator-apply and orthogonalisation times per
inner step (HIP events) and the wall time per step.

    python tools/ab_gmres.py [--rounds R] [--iters K] [--variants "gm_dpp=0/brick_mult_pb=0,gm_dpp=1/brick_mult_pb=0"]
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
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--iters", type=int, default=60)
ap.add_argument("--n", type=int, default=64)
ap.add_argument("--variants", default="gm_ept=4,gm_ept=5")
ap.add_argument("--no-prof", action="store_true", help="no HIP events around the kernels: wall time only")
args = ap.parse_args()

n = args.n
mesh = cdfem.box_mesh(3, n, 2, with_coords=False)
ctx = cdfem.Context(0)
ctx.upload_mesh(mesh).set_structured(n, n, n)
ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=(1.0, -2.0, 0.5), mass=1.0)
b = np.random.default_rng(20261015).uniform(-1, 1, mesh.nl)
_, B = ctx.form_linear_system(np.zeros(mesh.nl), b)
dB, dX = ctx.to_device(B), ctx.alloc(8 * mesh.nl)
# a variant is one or more k=v settings joined by '/', all set before its solve (options persist on
# the context, so every variant should name every key the list varies)
variants = [(v, [kv.split("=") for kv in v.split("/")]) for v in args.variants.split(",")]
res = {name: {"apply_us": [], "orth_us": [], "step_us": []} for name, _ in variants}
ref = None
for rnd in range(args.rounds + 1):
    for name, kvs in variants:
        for k, v in kvs:
            ctx.set_option(k, int(v))
        ctx.set_option("profile_mask", (1 << cdfem.K_APPLY) | (1 << cdfem.K_ORTH))
        ctx.profile(not args.no_prof)
        ctx.synchronize()
        t0 = time.perf_counter()
        info = ctx.solve_device(dB, dX, method="gmres", pc="jacobi", rel_tol=0.0, abs_tol=0.0,
                                max_iter=args.iters, restart=30)
        ctx.synchronize()
        dt = time.perf_counter() - t0
        a = ctx.profile_read(cdfem.K_APPLY)
        o = ctx.profile_read(cdfem.K_ORTH)
        ctx.profile(False)
        x = ctx.from_device(dX, mesh.nl)
        if ref is None:
            ref = x
        assert np.abs(x - ref).max() <= 1e-9 * np.abs(ref).max()
        if rnd == 0:
            continue
        r = res[name]
        r["apply_us"].append(a[0] / max(a[1], 1) * 1e3)
        r["orth_us"].append(o[0] / max(o[1], 1) * 1e3)
        r["step_us"].append(dt / info["iterations"] * 1e6)
print(json.dumps({k: {m: round(float(np.median(v)), 2) for m, v in r.items()} for k, r in res.items()}, indent=1))
