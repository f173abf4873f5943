"""Interleaved in-process A/B of SpMV variants on the C4 workload (Kuhn tets, P2, FA CSR + GMRES),
GPU box only.

Usage: python tools/ab_c4.py [--rounds R] [--iters K] [--n N] [--variants spmv_variant=0,spmv_variant=1]
Prints per-variant median SpMV launch time (HIP events), GMRES orthogonalisation time and the
achieved algorithmic GB/s of the SpMV.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "continuum-mechanics-mfem_amd", "python"))
import cdfem  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=60)
ap.add_argument("--n", type=int, default=55)
ap.add_argument("--variants", default="spmv_variant=0,spmv_variant=1")
args = ap.parse_args()

mesh = cdfem.kuhn_mesh(3, args.n, 2, with_coords=False)
ctx = cdfem.Context(0)
ctx.upload_mesh(mesh)
ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=(1.0, -2.0, 0.5), mass=1.0)
b = np.random.default_rng(20261015).uniform(-1, 1, mesh.nl)
_, B = ctx.form_linear_system(np.zeros(mesh.nl), b)
dB, dX = ctx.to_device(B), ctx.alloc(8 * mesh.nl)
variants = [v.split("=") for v in args.variants.split(",")]
res = {f"{k}={v}": {"spmv_us": [], "orth_us": []} for k, v in variants}
ref = None
for rnd in range(args.rounds + 1):
    for k, v in variants:
        ctx.set_option(k, int(v))
        ctx.set_option("profile_mask", (1 << cdfem.K_APPLY) | (1 << cdfem.K_ORTH))
        ctx.profile(True)
        ctx.synchronize()
        ctx.solve_device(dB, dX, method="gmres", pc="jacobi", rel_tol=0.0, abs_tol=0.0,
                         max_iter=args.iters, restart=30)
        a = ctx.profile_read(cdfem.K_APPLY)
        o = ctx.profile_read(cdfem.K_ORTH)
        ctx.profile(False)
        x = ctx.from_device(dX, mesh.nl)
        if ref is None:
            ref = x
        assert np.abs(x - ref).max() <= 1e-10 * np.abs(ref).max()
        if rnd == 0:
            continue  # warm-up round
        r = res[f"{k}={v}"]
        r["spmv_us"].append(a[0] / max(a[1], 1) * 1e3)
        r["orth_us"].append(o[0] / max(o[1], 1) * 1e3)
bytes_spmv = ctx.kernel_bytes(cdfem.K_APPLY)
out = {}
for name, r in res.items():
    med = {k: float(np.median(v)) for k, v in r.items()}
    med["spmv_GBs"] = bytes_spmv / (med["spmv_us"] * 1e-6) / 1e9
    out[name] = med
print(json.dumps(out, indent=1))
ctx.free(dB)
ctx.free(dX)
ctx.close()
