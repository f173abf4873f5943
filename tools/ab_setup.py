"""Interleaved in-process A/B of setup-time options on the PA CG workloads (GPU box only).

Each variant is its own context, with its options set before cdfem_pa_setup (e.g. mass_from_d):
    python tools/ab_setup.py [--n 64 --p 2 | --n 128 --p 4] [--iters K] [--rounds R]
                             [--variants "label:opt=v+opt=v,..."]
Prints per variant the median wall time per CG iteration (uninstrumented solves), the apply
kernel's HIP-event time from a separate profiled solve, and the max relative difference of the
iterate against the first variant's.
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
ap.add_argument("--n", type=int, default=64)
ap.add_argument("--p", type=int, default=2)
ap.add_argument("--kinds", type=int, default=7)
ap.add_argument("--iters", type=int, default=100)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--variants", default="stored:mass_from_d=0,derived:mass_from_d=1")
args = ap.parse_args()

mesh = cdfem.box_mesh(3, args.n, args.p, with_coords=False)
b = np.random.default_rng(1).uniform(-1, 1, mesh.nl)
vs = []
for spec in args.variants.split(","):
    label, opts = spec.split(":")
    ctx = cdfem.Context(0)
    for kv in filter(None, opts.split("+")):
        k, v = kv.split("=")
        ctx.set_option(k, int(v))
    ctx.upload_mesh(mesh).set_structured(args.n, args.n, args.n)
    ctx.pa_setup(kinds=args.kinds, kappa=0.1, conv=(1.0, -2.0, 0.5), mass=1.0)
    _, B = ctx.form_linear_system(np.zeros(mesh.nl), b)
    vs.append(dict(label=label, ctx=ctx, dB=ctx.to_device(B), dX=ctx.alloc(8 * mesh.nl), it=[], ap=[],
                   bytes=ctx.kernel_bytes(cdfem.K_APPLY)))
ref = None
for rnd in range(args.rounds + 1):
    for v in vs:
        ctx = v["ctx"]
        ctx.synchronize()
        t0 = time.perf_counter()
        info = ctx.solve_device(v["dB"], v["dX"], max_iter=args.iters)
        ctx.synchronize()
        dt = time.perf_counter() - t0
        ctx.set_option("profile_mask", 1 << cdfem.K_APPLY)
        ctx.profile(True)
        ctx.solve_device(v["dB"], v["dX"], max_iter=args.iters)
        a = ctx.profile_read(cdfem.K_APPLY)
        ctx.profile(False)
        x = ctx.from_device(v["dX"], mesh.nl)
        if ref is None:
            ref = x
        v["diff"] = float(np.abs(x - ref).max() / np.abs(ref).max())
        if rnd == 0:
            continue
        v["it"].append(dt / info["iterations"] * 1e6)
        v["ap"].append(a[0] / max(a[1], 1) * 1e3)
out = {}
for v in vs:
    ap_us = float(np.median(v["ap"]))
    out[v["label"]] = {"iter_us": float(np.median(v["it"])), "apply_us": ap_us, "apply_bytes": v["bytes"],
                       "apply_GBs": v["bytes"] / (ap_us * 1e-6) / 1e9, "max_rel_diff_vs_first": v["diff"]}
print(json.dumps(out, indent=1))
for v in vs:
    v["ctx"].free(v["dB"])
    v["ctx"].free(v["dX"])
    v["ctx"].close()
