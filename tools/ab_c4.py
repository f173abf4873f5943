"""Interleaved in-process A/B of FA SpMV layouts on the C4 workload (Kuhn tets, P2, FA CSR +
GMRES(30)/Jacobi), GPU box only.

Each variant is its own context (the SpMV layout is fixed when the FA pattern is built):
    label:mesh:opt=val+opt=val...     mesh = natural | shuffled (random dof relabelling); options
                                      set before the mesh upload (sell_order, spmv_xcd, spmv_variant)
Prints per variant the median SpMV launch time (HIP events), the GMRES orthogonalisation time, the
wall time per solve and the algorithmic GB/s of the SpMV; checks every variant's GMRES iterate
against the first variant's (mapped through the relabelling).

    python tools/ab_c4.py [--rounds R] [--iters K] [--n N] [--variants ...]
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
ap.add_argument("--iters", type=int, default=60)
ap.add_argument("--n", type=int, default=55)
ap.add_argument("--points", type=int, default=170000, help="delaunay: random points (cdfem.delaunay_cube)")
ap.add_argument("--variants", default="legacy:natural:sell_order=0+spmv_xcd=0,auto:natural:sell_order=3,"
                                      "shuf_legacy:shuffled:sell_order=0+spmv_xcd=0,shuf_auto:shuffled:sell_order=3")
args = ap.parse_args()

base = cdfem.kuhn_mesh(3, args.n, 2, with_coords=False)
delaunay = None
if "delaunay" in args.variants:
    delaunay = cdfem.simplex_space(*cdfem.delaunay_cube(args.points, seed=20261017), 2)
g = np.random.default_rng(7).permutation(base.nl).astype(np.int32)   # shuffled label of mesh dof i
shuffled = cdfem.Mesh(base.dim, base.order, base.verts, g[base.dofmap], base.nl, np.sort(g[base.ess]),
                      None, simplex=True)
b_nat = np.random.default_rng(20261015).uniform(-1, 1, base.nl)
b_shuf = np.empty_like(b_nat)
b_shuf[g] = b_nat

variants = []
for spec in args.variants.split(","):
    label, mesh, opts = spec.split(":")
    m = {"natural": base, "shuffled": shuffled, "delaunay": delaunay}[mesh]
    ctx = cdfem.Context(0)
    for kv in filter(None, opts.split("+")):
        k, val = kv.split("=")
        ctx.set_option(k, int(val))
    t0 = time.perf_counter()
    ctx.upload_mesh(m)
    ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=(1.0, -2.0, 0.5), mass=1.0)
    setup_s = time.perf_counter() - t0
    b = b_shuf if mesh == "shuffled" else b_nat if mesh == "natural" else \
        np.random.default_rng(20261015).uniform(-1, 1, m.nl)
    _, B = ctx.form_linear_system(np.zeros(m.nl), b)
    variants.append(dict(label=label, mesh=mesh, ctx=ctx, dB=ctx.to_device(B), dX=ctx.alloc(8 * m.nl),
                         spmv_us=[], orth_us=[], solve_ms=[], setup_s=setup_s))
    print(f"# {label}: setup {setup_s:.2f} s", flush=True)

refs = {}
for rnd in range(args.rounds + 1):
    for v in variants:
        ctx = v["ctx"]
        ctx.set_option("profile_mask", (1 << cdfem.K_APPLY) | (1 << cdfem.K_ORTH))
        ctx.profile(True)
        ctx.synchronize()
        t0 = time.perf_counter()
        ctx.solve_device(v["dB"], v["dX"], method="gmres", pc="jacobi", rel_tol=0.0, abs_tol=0.0,
                         max_iter=args.iters, restart=30)
        ctx.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        a = ctx.profile_read(cdfem.K_APPLY)
        o = ctx.profile_read(cdfem.K_ORTH)
        ctx.profile(False)
        nl_v = delaunay.nl if v["mesh"] == "delaunay" else base.nl
        x = ctx.from_device(v["dX"], nl_v)
        if v["mesh"] == "shuffled":
            x = x[g]                          # back to the natural labels
        key = "delaunay" if v["mesh"] == "delaunay" else "kuhn"
        if key not in refs:
            refs[key] = x
        ref = refs[key]
        err = float(np.abs(x - ref).max() / np.abs(ref).max())
        assert err <= 1e-9, (v["label"], err)
        if rnd == 0:
            continue  # warm-up round
        v["spmv_us"].append(a[0] / max(a[1], 1) * 1e3)
        v["orth_us"].append(o[0] / max(o[1], 1) * 1e3)
        v["solve_ms"].append(wall)
        v["err"] = err
out = {}
for v in variants:
    nbytes = v["ctx"].kernel_bytes(cdfem.K_APPLY)
    med = {k: float(np.median(v[k])) for k in ("spmv_us", "orth_us", "solve_ms")}
    med["spmv_GBs"] = nbytes / (med["spmv_us"] * 1e-6) / 1e9
    med["setup_s"] = v["setup_s"]
    med["max_rel_diff_vs_first"] = v.get("err", 0.0)
    out[v["label"]] = med
print(json.dumps(out, indent=1))
for v in variants:
    v["ctx"].free(v["dB"])
    v["ctx"].free(v["dX"])
    v["ctx"].close()
