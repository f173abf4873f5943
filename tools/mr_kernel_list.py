#!/usr/bin/env python3
"""Kernel launches per CG iteration of the slab brick CG, one configuration per run: one rank, or N
ranks run as threads of this one process (each its own context on device 0, a host communicator over
thread barriers), with the multi-rank folds (cg_mr_fold 1) or without.  Run it under rocprofv3
--kernel-trace (one process, no launcher) and summarise the trace with --summary:

    rocprofv3 --kernel-trace -d OUT -o run --output-format csv -- python3 tools/mr_kernel_list.py --world 2 --fold 1
    python3 tools/mr_kernel_list.py --summary OUT --world 2 --iters 100

The summary divides every kernel's launches by ranks x iterations and keeps those launched at least
once per iteration: the one-rank loop is k_brick_cg + k_cg_update_faces; the folded N-rank loop adds
k_pack_qplanes only."""
import argparse
import glob
import json
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "continuum-mechanics-mfem_amd", "python"))

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=16)
ap.add_argument("--per", type=int, default=16, help="element layers per rank")
ap.add_argument("--world", type=int, default=1)
ap.add_argument("--fold", type=int, default=1)
ap.add_argument("--overlap", type=int, default=0, help="mr_overlap (0: one apply launch per iteration)")
ap.add_argument("--iters", type=int, default=100)
ap.add_argument("--summary", default=None)
args = ap.parse_args()

if args.summary:
    import csv
    f = glob.glob(os.path.join(args.summary, "**", "*kernel_trace.csv"), recursive=True)[0]
    cnt = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("cdfem::", "").strip()
        cnt[k] = cnt.get(k, 0) + 1
    its = args.world * args.iters
    json.dump({"ranks": args.world, "iters": args.iters, "fold": args.fold,
               "per_rank_per_iteration": {k: round(v / its, 3) for k, v in sorted(cnt.items(), key=lambda kv: -kv[1])
                                          if v / its >= 0.5}}, sys.stdout)
    print()
    sys.exit(0)

import cdfem  # noqa: E402

world, n, per, p = args.world, args.n, args.per, 2
bar = threading.Barrier(world)
slots, planes, out = [None] * world, {}, [None] * world


def rank_main(r):
    def allreduce(a):
        slots[r] = a.copy()
        bar.wait()
        tot = slots[0].copy()
        for k in range(1, world):
            tot += slots[k]
        bar.wait()
        a[:] = tot

    def exchange(s_lo, r_lo, s_hi, r_hi):
        if s_lo is not None:
            planes[(r, r - 1)] = s_lo.copy()
        if s_hi is not None:
            planes[(r, r + 1)] = s_hi.copy()
        bar.wait()
        if r_lo is not None:
            r_lo[:] = planes[(r - 1, r)]
        if r_hi is not None:
            r_hi[:] = planes[(r + 1, r)]
        bar.wait()

    m = cdfem.box_mesh(3, (n, n, per * world), p, z_range=(r * per, (r + 1) * per), with_coords=False)
    ctx = cdfem.Context(0)
    ctx.set_option("cg_mr_fold", args.fold)
    ctx.set_option("mr_overlap", args.overlap)
    ctx.upload_mesh(m).set_structured(n, n, per)
    if world > 1:
        ctx.comm_init_host(r, world, allreduce, exchange)
        ctx.set_slab(r > 0, r < world - 1)
    ctx.pa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=(1.0, -2.0, 0.5), mass=1.0)
    b = np.random.default_rng(300 + r).uniform(-1, 1, m.nl)
    _, B = ctx.form_linear_system(np.zeros(m.nl), b)
    X, info = ctx.solve(B, method="cg", rel_tol=0.0, abs_tol=0.0, max_iter=args.iters, check_every=args.iters)
    out[r] = info["iterations"]
    ctx.close()


th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
for t in th:
    t.start()
for t in th:
    t.join()
print(json.dumps({"ranks": world, "fold": args.fold, "iterations": out}))
