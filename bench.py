#!/usr/bin/env python3
"""Benchmark: DoF-iter/s of the MI355X PA + CG hot path (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 3D 64^3 hex mesh of [0,1]^3, H1 order 2 (2,146,689 DoFs),
convection-diffusion-reaction operator kappa=0.1, c=(1,-2,0.5), s=1 (Input/input_2d.yaml:7-10 with
the 3D extension of SURVEY.md §8d), Dirichlet on the whole boundary, matrix-free partial assembly,
Jacobi-preconditioned CG (MFEM CGSolver semantics).

A "step" = one CG solve of --cg-iters iterations (tolerances 0, so the iteration count is fixed)
from x0 = 0 on a synthetic right-hand side resident in HBM.
value = (true DoFs summed over ranks) x iterations x steps / max-over-ranks wall time.

Multi-GPU (torchrun, one rank per GPU): each rank owns a 64^3-element slab of a 64 x 64 x (64 N)
mesh; weak scaling.  The data-path exchange (interface DoF sum, Krylov scalars) is done by the
library over RCCL when it is built with the partitioned solver; torch.distributed (gloo) only
carries the barrier, the id broadcast and the max-over-ranks timing.

Extra fields on the JSON line: roofline (dominant kernel = fused PA apply, HIP events at its dispatch
start / end on the library stream, in a profiled pass of the same steps right after the uninstrumented
timed region), cpu_baseline (the oracle's FA-CSR + Jacobi-CG restatement of
the reference CPU path, timed on this host, rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "continuum-mechanics-mfem_amd", "python"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# MI355X dense f64 peak, the same on the VALU (v_fma_f64) and the matrix cores (v_mfma_f64): 78.6
# TFLOP/s spec; measured here 62.8 / 75.0 (profiles/r01c_fp64_probe.json)
F64_PEAK_TFLOPS = 78.6


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--elems", dest="n", type=int, default=None, help="elements per direction (per-rank slab depth); "
                    "default 64 (c2) / 128 (c3)")
    ap.add_argument("--order", type=int, default=None, help="default 2 (c2) / 4 (c3)")
    ap.add_argument("--cg-iters", type=int, default=None, help="default 100 (c2) / 20 (c3)")
    ap.add_argument("--kinds", type=int, default=7, help="1 diffusion | 2 convection | 4 mass")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--spd-steps", type=int, default=2,
                    help="informational CG line on the symmetric kK+sM operator (steps of 200 it); 0 = skip")
    ap.add_argument("--per-point-steps", type=int, default=2,
                    help="informational: the CG line with the per-point qdata stream (pa_affine 0); 0 = skip")
    ap.add_argument("--gmres-iters", type=int, default=60,
                    help="informational GMRES(30)+Jacobi line (the reference's solver); 0 = skip")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="target length of the timed CPU-baseline sample (iterations scaled to it)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="per-launch HBM bytes of the apply kernel from a rocprofv3 --pmc pass")
    ap.add_argument("--sq-json", default=os.path.join(ROOT, "profiles", "sq_counters.json"),
                    help="SQ counter record of the apply kernel (tools/sq_record.py): roofline.limiter")
    ap.add_argument("--rocprof-json", default=os.path.join(ROOT, "profiles", "rocprof_kernels.json"),
                    help="rocprofv3 kernel-trace averages of the apply kernel (tools/rocprof_avg.py): "
                         "roofline.rocprof_avg_us and its source CSV")
    ap.add_argument("--no-profile-events", action="store_true")
    ap.add_argument("--no-kron-form", action="store_true",
                    help="skip the informational Kronecker-form leg (profiles: its k_brick_cg launches share the name)")
    ap.add_argument("--path", choices=["brick", "generic"], default=None,
                    help="brick: structured fast path (fused E->L, fused CG direction); generic: any mesh")
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c4s", "c4u", "c5", "c5w"], default="c2",
                    help="c2: 64^3 hex p=2 PA + CG (BASELINE metric config; N>1: weak scaling, a 64^3 slab "
                         "per rank); c3: 128^3 hex p=4 PA + CG (configs[2]); c4: Kuhn 55^3 x 6 tets P2, FA CSR "
                         "+ GMRES(30)/Jacobi (configs[3]); c4u: the same on a Delaunay mesh of random points "
                         "(~1M tets, unstructured connectivity); c5: 256^3 hex p=2 PA + CG split into N z-slabs "
                         "(configs[4] at N=8: 256 x 256 x 32 per rank); c5w: SURVEY 8e's weak series, a "
                         "256 x 256 x 32 slab per rank (N=8: the C5 mesh)")
    ap.add_argument("--tet-n", type=int, default=55, help="c4: cubes per direction (6 tets each)")
    ap.add_argument("--tet-points", type=int, default=170000,
                    help="c4u: Delaunay points (about 6 tets per point: 170000 -> ~1.03M tets)")
    ap.add_argument("--comm", choices=["rccl", "host"], default="rccl",
                    help="N>1 data-path communicator: rccl (production, one GPU per rank) or host "
                         "(gloo callbacks; rehearses the N>1 flow with several ranks on one GPU)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=INT",
                    help="cdfem_set_option before the mesh upload (repeatable; A/B runs, e.g. ho_brick=0). "
                         "The options in effect are echoed in config.options")
    a = ap.parse_args()
    a.set = dict((k, int(v)) for k, v in (kv.split("=") for kv in a.set))
    c3 = a.config == "c3"
    a.n = a.n or (128 if c3 else 256 if a.config in ("c5", "c5w") else 64)
    a.order = a.order or (4 if c3 else 2)
    a.cg_iters = a.cg_iters or (20 if c3 else 100)
    a.path = a.path or ("brick" if a.order <= 2 else "generic")
    return a


def kernel_label(name, affine):
    """The roofline kernel (cdfem_kernel_name: rocprof's name first) with what it does."""
    what = {
        "k_brick_cg": "brick patch gather + fused CG direction + D/C/M PA apply" +
                      (", Kronecker form of the affine factors, x += alpha d folded in" if affine else "") +
                      " + in-LDS E->L + d.Ad",
        "k_hobrick_cg": "2^3-element blocks: patch gather + CG direction, D1 x D1 thread tile per element in the "
                        "Kronecker form, in-LDS E->L, x += alpha d folded in",
        "k_apply3d_ktile": "D1 x D1 thread tile per element, Kronecker form of the affine factors, CG direction folded in",
        "k_apply3d_tile": "Q1 x Q1 thread tile per element, z planes in registers",
        "k_apply3d": "fused L->E gather + D/C/M PA apply"}
    return f"{name} ({what.get(name, 'PA apply')})"


def kinds_label(kinds):
    """Integrator set of a kinds bit mask: 1 Diffusion, 2 Convection, 4 Mass (e.g. 7 -> D+C+M)."""
    return "+".join(n for b, n in ((1, "D"), (2, "C"), (4, "M")) if kinds & b)


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # libcdfem.so (and through it the /opt/rocm librccl it links) is loaded BEFORE torch: torch
    # bundles its own librccl with the same soname, which would otherwise be the one libcdfem
    # binds to.  config.comm records the library actually used (cdfem_comm_info).
    import cdfem
    cdfem.lib()
    pg = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pg = dist
    return world, rank, local, pg


def barrier(pg):
    if pg is not None:
        pg.barrier()


def allmax(pg, v):
    if pg is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def host_cores(args):
    """Threads for the CPU baseline and a description of the host.  The job's CPU share is the
    scheduler affinity mask, further capped by OMP_NUM_THREADS when the harness sets it (the GPU
    box reports the whole machine in nproc but grants each one-GPU job 16 threads)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    share = min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff
    model = "?"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return (args.cpu_threads or share), {"host_nproc": os.cpu_count(), "affinity_cpus": aff,
                                         "omp_num_threads": omp, "cpu_model": model}


CPU_SAMPLES = 5  # median of >= 5 timed samples after one warm-up


def _cpu_idle(window=0.5):
    """Idle fraction of every CPU over a short window (/proc/stat), {} when unreadable."""
    def snap():
        out = {}
        for line in open("/proc/stat"):
            if line.startswith("cpu") and line[3].isdigit():
                f = line.split()
                vals = [int(v) for v in f[1:]]
                out[int(f[0][3:])] = (vals[3] + (vals[4] if len(vals) > 4 else 0), sum(vals))
        return out
    try:
        a = snap()
        time.sleep(window)
        b = snap()
    except (OSError, ValueError, IndexError):
        return {}
    return {c: (b[c][0] - a[c][0]) / max(b[c][1] - a[c][1], 1) for c in b if c in a}


def pick_cpus(n):
    """n CPUs of this job's affinity mask for the CPU baseline, one per physical core, on one
    package: the package with the most idle time, and in it the most idle cores over a 0.5 s
    window (other jobs share the host's cores).  Falls back to the lowest allowed CPUs when the
    topology is unreadable."""
    allowed = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))

    def topo(c, f):
        try:
            return int(open(f"/sys/devices/system/cpu/cpu{c}/topology/{f}").read())
        except (OSError, ValueError):
            return None
    idle = _cpu_idle()
    cores = {}  # (package, core) -> [cpus]
    for c in allowed:
        cores.setdefault((topo(c, "physical_package_id"), topo(c, "core_id")), []).append(c)
    # a core's idleness: its least idle hardware thread (a busy sibling slows the core)
    score = {k: min(idle.get(c, 1.0) for c in v) for k, v in cores.items()}
    pkgs = {}
    for k, sc in score.items():
        pkgs[k[0]] = pkgs.get(k[0], 0.0) + sc
    order = sorted(cores, key=lambda k: (-pkgs[k[0]], k[0], -score[k], cores[k][0]))
    out = [cores[k][0] for k in order][:n]
    for c in allowed:  # fewer physical cores than threads: SMT siblings too
        if len(out) >= n:
            break
        if c not in out:
            out.append(c)
    return out


class PinnedThreads:
    """Pin the oracle's OpenMP threads to pick_cpus(n) for the CPU baseline (timing stability on
    a shared host: the r02 unpinned samples varied 1.8x between runs) and restore the calling
    thread's affinity afterwards (the GPU runtime's threads keep theirs)."""

    def __init__(self, O, n):
        self.O, self.n = O, n

    def __enter__(self):
        self.saved = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None
        self.cpus = pick_cpus(self.n)
        self.pinned = self.O.pin_threads(self.cpus)
        return self

    def __exit__(self, *exc):
        if self.saved is not None:
            os.sched_setaffinity(0, self.saved)
        return False

    def record(self):
        return {"pinned_cpus": f"{len(self.cpus)} cores: " + ",".join(str(c) for c in sorted(self.cpus)),
                "threads_pinned": self.pinned}


def cpu_samples(run, dofs, seconds, max_it, min_it=10, calib_it=5):
    """Time an oracle solver leg: calibrate on calib_it iterations, one untimed warm-up sample, then
    CPU_SAMPLES timed samples of about seconds / CPU_SAMPLES each.  run(k) runs k iterations and
    returns the iterations done.  Returns the median DoF-iter/s and the sample record."""
    t0 = time.perf_counter()
    run(calib_it)
    per_it = (time.perf_counter() - t0) / calib_it
    k = int(min(max_it, max(min_it, seconds / CPU_SAMPLES / per_it)))
    run(k)  # warm-up sample
    rates, total_t, total_it = [], 0.0, 0
    for _ in range(CPU_SAMPLES):
        t0 = time.perf_counter()
        its = run(k)
        dt = time.perf_counter() - t0
        rates.append(dofs * its / dt)
        total_t += dt
        total_it += its
    med = float(np.median(rates))
    rec = {"samples": [round(r, 1) for r in rates], "median": med, "min": float(min(rates)),
           "max": float(max(rates)), "spread": round((max(rates) - min(rates)) / med, 4),
           "iterations_per_sample": k}
    return med, rec, total_it, total_t


def cpu_baseline(args, n, p, kinds):
    """Oracle (C restatement of the reference's CPU FA path) timed on this host's cores: Jacobi-CG
    (like-for-like with the GPU metric) and, on the same assembled matrix, GMRES(30)+Jacobi (the
    reference's solver, Input/petsc.opts:2-6).  Each leg: median of CPU_SAMPLES samples after a
    warm-up (cpu_samples).  For p >= 3 the FA matrix of the full mesh is out of reach of the CPU
    (729-wide rows at p = 4), so the sample is a 12^3 mesh of the same order (throughput per
    DoF-iteration is the reported unit)."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    threads, host = host_cores(args)
    O.set_threads(threads)
    with PinnedThreads(O, threads) as pin:
        out = _cpu_baseline_box(args, O, n, p, kinds, threads, host)
    out.update(pin.record())
    return out


def _cpu_baseline_box(args, O, n, p, kinds, threads, host):
    if p >= 3:
        n = min(n, 12)
    m = O.BoxMesh(3, n, p)
    t0 = time.perf_counter()
    ok = (O.DIFFUSION if kinds & 1 else 0) | (O.CONVECTION if kinds & 2 else 0) | (O.MASS if kinds & 4 else 0)
    A = O.fa_assemble(m, kappa=0.1, alpha=1.0, s=1.0, c=(1.0, -2.0, 0.5), kinds=ok)
    rng = np.random.default_rng(20261015)
    b = rng.uniform(-1, 1, m.nl)
    Ac, B = O.form_linear_system(A, m.bdr, np.zeros(m.nl), b)
    del A
    dinv = 1.0 / Ac.diag()
    t_asm = time.perf_counter() - t0

    host_bw = host_bandwidth(O, Ac, m.nl)

    def cg(k):
        return O.cg(Ac, B, dinv=dinv, rel_tol=0.0, abs_tol=0.0, max_iter=k)[1]["iterations"]

    def gmres(k):  # the reference's solver on the same matrix: GMRES(30) + Jacobi, fixed inner steps
        return O.gmres(Ac, B, dinv=dinv, restart=30, rtol=0.0, atol=0.0, max_it=k)[1]["iterations"]
    v, rec, its, dt = cpu_samples(cg, m.nl, args.cpu_seconds, 20000, calib_it=10)
    gv, grec, gits, gdt = cpu_samples(gmres, m.nl, 0.5 * args.cpu_seconds, 3000)
    # SURVEY 8d's like-for-like leg: MFEM's host partial assembly (per-integrator point data, one
    # sum-factorised element loop per integrator, L->E / E->L) under CGSolver, same matrix-free operator
    t0 = time.perf_counter()
    pa = O.PA(m, kappa=0.1, alpha=1.0, s=1.0, c=(1.0, -2.0, 0.5), kinds=ok)
    t_pa = time.perf_counter() - t0

    def pacg(k):
        return pa.cg(B, dinv=dinv, rel_tol=0.0, abs_tol=0.0, max_iter=k)[1]["iterations"]
    pv, prec, pits, pdt = cpu_samples(pacg, m.nl, 0.5 * args.cpu_seconds, 3000, calib_it=3)
    del pa
    return {"value": v, "unit": "DoF-iter/s", "cores": threads, "kind": "port",
            "sample": f"oracle FA-CSR Jacobi-CG, {n}^3 hex p={p} ({m.nl} DoFs, nnz={Ac.nnz}): median of "
                      f"{CPU_SAMPLES} samples of {rec['iterations_per_sample']} iterations after a warm-up "
                      f"({its} iterations, {dt:.2f} s timed); assembly+FormLinearSystem {t_asm:.1f} s untimed",
            **rec, **host_bw,
            "gmres": {"value": gv, "unit": "DoF-iter/s",
                      "sample": f"oracle FA-CSR GMRES(30)+Jacobi on the same matrix: median of {CPU_SAMPLES} "
                                f"samples of {grec['iterations_per_sample']} inner steps ({gits} steps, "
                                f"{gdt:.2f} s timed)", **grec},
            "pa_cg": {"value": pv, "unit": "DoF-iter/s",
                      "sample": f"oracle host PA (MFEM's AssemblyLevel::PARTIAL on the CPU: per-integrator point "
                                f"data, sum-factorised element loops, L->E / E->L) + Jacobi-CG on the same mesh and "
                                f"operator: median of {CPU_SAMPLES} samples of {prec['iterations_per_sample']} "
                                f"iterations ({pits} iterations, {pdt:.2f} s timed); PA setup {t_pa:.1f} s untimed",
                      **prec},
            **host}


def host_bandwidth(O, A, nl, reps=10):
    """What the CPU baseline's pinned cores get from memory: a STREAM triad (orc_stream_triad, 3 x 512 MB,
    best of 5) and the oracle's CSR SpMV on the baseline's matrix (median of reps, SURVEY 8d bytes
    12 nnz + 4 (n + 1) + 16 n).  A host-to-host swing of the baseline follows these numbers."""
    triad = O.stream_triad_gbs(1 << 26, 5)
    x = np.random.default_rng(5).uniform(-1, 1, nl)
    A.mult(x)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        A.mult(x)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    sb = 12.0 * A.nnz + 4.0 * (nl + 1) + 16.0 * nl
    return {"host_stream_gbs": round(triad, 1), "spmv_gbs": round(sb / t / 1e9, 1),
            "spmv_frac_of_stream": round(sb / t / 1e9 / triad, 3) if triad > 0 else None,
            "spmv_ms": round(t * 1e3, 2)}


def cpu_baseline_c4(args, n, p, mesh=None):
    """Oracle FA-CSR GMRES(30)/Jacobi on the same Kuhn mesh, or on `mesh` (c4u: the same Delaunay
    mesh; bounded sample, median of CPU_SAMPLES samples after a warm-up)."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    threads, host = host_cores(args)
    O.set_threads(threads)
    with PinnedThreads(O, threads) as pin:
        out = _cpu_baseline_kuhn(args, O, n, p, threads, host, mesh)
    out.update(pin.record())
    return out


class _OracleMesh:
    """The oracle's mesh container for a product simplex Mesh (verts, dofmap, boundary marker)."""

    def __init__(self, m):
        self.dim, self.p, self.ne, self.nl = m.dim, m.order, m.ne, m.nl
        self.verts, self.dofmap, self.ess = m.verts, m.dofmap, m.ess
        self.bdr = np.zeros(m.nl, dtype=np.int32)
        self.bdr[m.ess] = 1


def _cpu_baseline_kuhn(args, O, n, p, threads, host, mesh=None):
    m = O.KuhnMesh(3, n, p) if mesh is None else _OracleMesh(mesh)
    t0 = time.perf_counter()
    A = O.fa_assemble_simplex(m, kappa=0.1, alpha=1.0, s=1.0, c=(1.0, -2.0, 0.5))
    b = np.random.default_rng(20261015).uniform(-1, 1, m.nl)
    Ac, B = O.form_linear_system(A, m.bdr, np.zeros(m.nl), b)
    del A
    dinv = 1.0 / Ac.diag()
    t_asm = time.perf_counter() - t0

    def gmres(k):
        return O.gmres(Ac, B, dinv=dinv, restart=30, rtol=0.0, atol=0.0, max_it=k)[1]["iterations"]
    host_bw = host_bandwidth(O, Ac, m.nl)
    v, rec, its, dt = cpu_samples(gmres, m.nl, args.cpu_seconds, 3000)
    what = f"Kuhn {n}^3x6 tets" if mesh is None else f"the same Delaunay mesh ({m.ne} tets)"
    return {"value": v, "unit": "DoF-iter/s", "cores": threads, "kind": "port",
            "sample": f"oracle FA-CSR GMRES(30)/Jacobi, {what} P{p} ({m.nl} DoFs, nnz={Ac.nnz}): median "
                      f"of {CPU_SAMPLES} samples of {rec['iterations_per_sample']} iterations after a warm-up "
                      f"({its} iterations, {dt:.2f} s timed); assembly+FormLinearSystem {t_asm:.1f} s untimed",
            **rec, **host_bw, **host}


def main_c4(args):
    """BASELINE configs[3]: unstructured-path tets, FA CSR SpMV + GMRES(30)/Jacobi on 1 GPU."""
    import cdfem
    n, p = args.tet_n, 2
    unstructured = args.config == "c4u"
    t_mesh = 0.0
    if unstructured:
        # c4u: unstructured connectivity (Delaunay of random points, scipy/Qhull on the host, untimed)
        t0 = time.perf_counter()
        mesh = cdfem.simplex_space(*cdfem.delaunay_cube(args.tet_points, seed=20261017), p)
        t_mesh = time.perf_counter() - t0
    else:
        mesh = cdfem.kuhn_mesh(3, n, p, with_coords=False)
    shuffled = args.config == "c4s"
    if shuffled:
        # c4s: the same mesh with a random dof numbering (what a gmsh file without bandwidth
        # reduction gives): the FA setup's SpMV order (sell_order auto) recovers the locality with
        # reverse Cuthill-McKee and the Krylov solve runs in that order (sell_plan.cpp)
        g = np.random.default_rng(7).permutation(mesh.nl).astype(np.int32)
        mesh = cdfem.Mesh(mesh.dim, mesh.order, mesh.verts, g[mesh.dofmap], mesh.nl, np.sort(g[mesh.ess]),
                          None, simplex=True)
    ctx = cdfem.Context(0)
    for k, v in args.set.items():
        ctx.set_option(k, v)
    ctx.upload_mesh(mesh)
    t0 = time.perf_counter()
    ctx.fa_setup(kinds=7, kappa=0.1, alpha=1.0, conv=(1.0, -2.0, 0.5), mass=1.0)
    t_setup = time.perf_counter() - t0
    b = np.random.default_rng(20261015).uniform(-1, 1, mesh.nl)
    _, B = ctx.form_linear_system(np.zeros(mesh.nl), b)
    dB, dX = ctx.to_device(B), ctx.alloc(8 * mesh.nl)
    iters_per_step = args.gmres_iters or 60

    def step():
        return ctx.solve_device(dB, dX, method="gmres", pc="jacobi", rel_tol=0.0, abs_tol=0.0,
                                max_iter=iters_per_step, restart=30)

    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    # timed region: the production path, no instrumentation
    t0 = time.perf_counter()
    iters = 0
    for _ in range(args.steps):
        iters += step()["iterations"]
    ctx.synchronize()
    dt = time.perf_counter() - t0
    roof = None
    if not args.no_profile_events:
        # profiled pass of the same steps: HIP events around the SpMV (dispatch start / end) and the
        # orthogonalisation.  Events carry completion fences, so they stay out of the timed region.
        ctx.set_option("profile_mask", (1 << cdfem.K_APPLY) | (1 << cdfem.K_ORTH))
        ctx.profile(True)
        for _ in range(args.steps):
            step()
        ctx.synchronize()
        ms, cnt = ctx.profile_read(cdfem.K_APPLY)
        o_ms, o_cnt = ctx.profile_read(cdfem.K_ORTH)
        ctx.profile(False)
        if cnt:
            per = ms / cnt * 1e-3
            bytes_ = ctx.kernel_bytes(cdfem.K_APPLY)
            traffic = None
            if os.path.exists(args.traffic_json):
                try:
                    key = f"{args.config}_n{n}_p{p}" if not unstructured else f"c4u_pts{args.tet_points}_p{p}"
                    traffic = json.load(open(args.traffic_json)).get(key, {}).get("hbm_bytes_per_launch")
                except Exception:
                    traffic = None
            roof = {"bound": "hbm", "achieved": round(bytes_ / per / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(bytes_ / per / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "kernel": (f"{ctx.kernel_name(cdfem.K_APPLY)} (SELL-64 SpMV on the eliminated FA matrix"
                               f"{', LDS-staged windows' if ctx.kernel_name(cdfem.K_APPLY).endswith('_lds') else ''})"),
                    "algorithmic_bytes_per_launch": bytes_, "avg_launch_us": round(per * 1e6, 2), "launches": cnt,
                    "other_kernels_avg_us": {"gmres_orth": round(o_ms / max(o_cnt, 1) * 1e3, 2)}}
    rp, _, _ = ctx.fa_csr()
    nnz = int(rp[-1])
    if roof is not None:
        # SURVEY.md 8(d) prices the SpMV at 12 B per nonzero (32-bit columns); the kernel streams
        # 16-bit column deltas, so the bytes it must move (algorithmic_bytes_per_launch) are fewer
        sb = 12.0 * nnz + 4.0 * (mesh.nl + 1) + 16.0 * mesh.nl
        roof["survey_bytes_per_launch"] = sb
        roof["survey_frac"] = round(sb / (roof["avg_launch_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
    cpu = None
    if not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline_c4(args, n, p, mesh if unstructured else None)
        except Exception as e:
            cpu = {"error": repr(e)}
    out = {"metric": "DoF-iter/s (CG, 3D p=2 hex convection-diffusion) + achieved HBM GB/s",
           "value": mesh.nl * iters / dt, "unit": "DoF-iter/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": {"workload": (f"C4u: Delaunay tets of {args.tet_points} random points in the unit cube "
                                   f"({mesh.ne} tets) P2" if unstructured else
                                   f"{'C4s' if shuffled else 'C4'}: Kuhn {n}^3x6 tets P2"
                                   f"{', shuffled dof numbering (RCM SpMV order)' if shuffled else ''}")
                                  + f", FA CSR (GPU-assembled) + GMRES(30)/Jacobi {iters_per_step} it/step",
                      **({"mesh_generation_s": round(t_mesh, 1)} if unstructured else {}),
                      "dofs": mesh.nl, "elements": mesh.ne, "nnz": nnz,
                      "fa_setup_s": round(t_setup, 3), "parallelism": "single"},
           "roofline": roof, "cpu_baseline": cpu}
    print(json.dumps(out), flush=True)
    ctx.free(dB)
    ctx.free(dX)
    ctx.close()


def main():
    args = parse()
    if args.config in ("c4", "c4s", "c4u"):
        return main_c4(args)
    world, rank, local, pg = dist_setup(args)
    import cdfem

    n, p = args.n, args.order
    if args.config == "c5":
        # configs[4]: one n^3 mesh split into `world` z-slabs (n x n x n/world elements per rank)
        if n % world:
            raise SystemExit(f"c5: {n} element layers do not split over {world} ranks")
        nzr, nz = n // world, n
    elif args.config == "c5w":
        # SURVEY 8e weak series: an n x n x n/8 slab per rank (256 x 256 x 32), N = 8 is C5's 256^3
        nzr, nz = n // 8, (n // 8) * world
    else:
        # weak scaling: rank r owns elements iz in [r n, (r+1) n) of an n x n x (world n) mesh
        nzr, nz = n, n * world
    mesh = cdfem.box_mesh(3, (n, n, nz), p, z_range=(rank * nzr, (rank + 1) * nzr), with_coords=False)
    ndev = cdfem.device_count()
    ctx = cdfem.Context(local % ndev)  # one rank per GPU on a node; ranks share a GPU only in rehearsals
    for k, v in args.set.items():
        ctx.set_option(k, v)
    ctx.upload_mesh(mesh)
    if args.path == "brick" or p >= 3:
        ctx.set_structured(n, n, nzr)  # p >= 3: structured E->L (no position arrays)
    if world > 1:
        if args.comm == "rccl":
            # RCCL communicator over xGMI; the id travels over the gloo control group.  Every rank
            # reports whether its init succeeded; if any failed, every rank exits non-zero: a
            # scaling number is never measured on a silent host fallback (the host-callback
            # communicator is opt-in, --comm host, for rehearsals with several ranks on one GPU)
            obj = [cdfem.comm_unique_id() if rank == 0 else None]
            pg.broadcast_object_list(obj, src=0)
            err = None
            try:
                ctx.comm_init_rccl(rank, world, obj[0])
            except cdfem.CdfemError as e:
                err = str(e)
            if allmax(pg, 1.0 if err else 0.0) > 0.0:
                print(f"rank {rank}: RCCL communicator unavailable ({err or 'failed on another rank'}) on "
                      f"device {local % ndev} of {ndev}; refusing to run the N>1 bench on the host "
                      "fallback (use --comm host to rehearse with several ranks on one GPU)",
                      file=sys.stderr, flush=True)
                ctx.close()
                pg.destroy_process_group()
                raise SystemExit(3)
        else:
            ctx.comm_init_torch()
        ctx.set_slab(rank > 0, rank < world - 1)
    comm_lib = cdfem.comm_info(ctx)
    comm_ranks = None
    if world > 1:
        # per rank: its device and the communicator library it bound (gathered to rank 0)
        mine = {"rank": rank, "device": local % ndev, "comm": comm_lib}
        comm_ranks = [None] * world
        pg.all_gather_object(comm_ranks, mine)
    c = (1.0, -2.0, 0.5)
    ctx.pa_setup(kinds=args.kinds, kappa=0.1, alpha=1.0, conv=c, mass=1.0)
    # pa_affine (default): on this parallelepiped mesh the brick kernels form the point data from
    # per-element factors; the byte count tells which form the context took
    nq = (p + 2) ** 3
    ncomp = (6 if args.kinds & 1 else 0) + (3 if args.kinds & 2 else 0) + (1 if args.kinds & 4 else 0)
    affine = ctx.kernel_bytes(cdfem.K_APPLY) < 8.0 * ncomp * nq * mesh.ne
    # pa_uniform (default): on this uniformly refined box every element has the same factors, and the
    # brick CG applies the one 27 x 27 element matrix on the matrix cores; the byte count (no factor
    # stream) tells whether the context took that form
    uni_opt = int(args.set.get("pa_uniform", 1))
    uni_bytes = ctx.kernel_bytes(cdfem.K_APPLY)
    ctx.set_option("pa_uniform", 0)
    uniform = uni_opt != 0 and ctx.kernel_bytes(cdfem.K_APPLY) != uni_bytes
    ctx.set_option("pa_uniform", uni_opt)

    # synthetic RHS resident in HBM: B = FormLinearSystem(u_bc = 0, b ~ U[-1,1))
    rng = np.random.default_rng(20261015 + rank)
    b = rng.uniform(-1, 1, mesh.nl)
    _, B = ctx.form_linear_system(np.zeros(mesh.nl), b)
    dB = ctx.to_device(B)
    dX = ctx.alloc(8 * mesh.nl)

    def step():
        return ctx.solve_device(dB, dX, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0,
                                max_iter=args.cg_iters, check_every=args.cg_iters)

    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    host_comm = world > 1 and args.comm == "host"
    if host_comm:  # rehearsal: host seconds inside the communicator callbacks over the timed steps
        for k in ctx.comm_stats:
            ctx.comm_stats[k] = 0 if k.endswith("calls") else 0.0
    # timed region: the production path, no instrumentation
    barrier(pg)
    ctx.synchronize()
    t0 = time.perf_counter()
    iters = 0
    for _ in range(args.steps):
        info = step()
        iters += info["iterations"]
    ctx.synchronize()
    barrier(pg)
    dt = time.perf_counter() - t0
    dt_max = allmax(pg, dt)
    comm_timing = None
    if host_comm:
        cs = dict(ctx.comm_stats)
        mine = {"rank": rank, "s_total": dt, "iters": iters,
                "allreduce_us_per_iter": cs["allreduce_s"] / max(iters, 1) * 1e6,
                "allreduce_calls_per_iter": cs["allreduce_calls"] / max(iters, 1),
                "exchange_us_per_iter": cs["exchange_s"] / max(iters, 1) * 1e6,
                "exchange_calls_per_iter": cs["exchange_calls"] / max(iters, 1),
                "comm_share": (cs["allreduce_s"] + cs["exchange_s"]) / dt}
        comm_timing = [None] * world
        pg.all_gather_object(comm_timing, mine)

    # roofline of the dominant kernel (fused PA apply): a profiled pass of the same steps with HIP
    # events at the kernel's dispatch start / end on the library stream.  Event-bracketed launches
    # carry completion fences (measured ~8 % of a C2 iteration), so they stay out of the timed region.
    roof = None
    if not args.no_profile_events:
        ctx.set_option("profile_mask", 1 << cdfem.K_APPLY)
        ctx.profile(True)
        for _ in range(args.steps):
            step()
        ctx.synchronize()
        ms, cnt = ctx.profile_read(cdfem.K_APPLY)
        each = ctx.profile_launches(cdfem.K_APPLY)
        # the other kernels: one extra (untimed) step with events around every kernel
        ctx.profile(False)
        ctx.set_option("profile_mask", -1)
        ctx.profile(True)
        step()
        ctx.synchronize()
        e_ms, e_cnt = ctx.profile_read(cdfem.K_E2L)
        u_ms, u_cnt = ctx.profile_read(cdfem.K_UPDATE)
        d_ms, d_cnt = ctx.profile_read(cdfem.K_DIRECTION)
        ctx.profile(False)
        if cnt:
            # every solve ends with an apply that returns at its first check (the update before it set
            # `done`, or its betanom step stops the solve): a launch with no work.  The roofline
            # divides the launch's bytes by the FULL launches' average (>= half the median: the
            # early-return ones take a few us); the all-launch average is kept beside it
            full = each[each >= 0.5 * np.median(each)] if len(each) else each
            per_all = ms / cnt * 1e-3
            per = float(full.mean()) * 1e-3 if len(full) else per_all
            bytes_ = ctx.kernel_bytes(cdfem.K_APPLY)
            achieved = bytes_ / per / 1e9
            traffic = None
            key = f"n{n}_p{p}_k{args.kinds}" + ("_aff" if affine else "")
            if os.path.exists(args.traffic_json):
                try:
                    tj = json.load(open(args.traffic_json))
                    traffic = tj.get(key, {}).get("hbm_bytes_per_launch")
                except Exception:
                    traffic = None
            limiter = None
            if os.path.exists(args.sq_json):
                try:
                    limiter = json.load(open(args.sq_json)).get(key)
                except Exception:
                    limiter = None
            hbm_view = {"achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic}
            if affine:
                # affine factors: the apply reads ~10 doubles per element instead of the point stream,
                # so its f64 arithmetic (VALU v_fma_f64; no MFMA in this kernel) is the other roofline.
                # bound = whichever view the kernel sits closer to; both are kept
                flops = ctx.kernel_flops(cdfem.K_APPLY)
                tf = flops / per / 1e12
                valu_view = {"achieved": round(tf, 2), "peak": F64_PEAK_TFLOPS, "unit": "TFLOP/s",
                             "frac": round(tf / F64_PEAK_TFLOPS, 4), "traffic": traffic,
                             "compute_unit": "VALU v_fma_f64 (78.6 TFLOP/s f64 dense peak)",
                             "algorithmic_flops_per_launch": flops}
                if valu_view["frac"] >= hbm_view["frac"]:
                    roof = {"bound": "f64-valu", **valu_view, "hbm_view": hbm_view}
                else:
                    roof = {"bound": "hbm", **hbm_view, "valu_view": valu_view}
            else:
                roof = {"bound": "hbm", **hbm_view}
            rp = None
            if os.path.exists(args.rocprof_json):
                try:
                    rp = json.load(open(args.rocprof_json)).get(key)
                except Exception:
                    rp = None
            roof.update({
                    "kernel": kernel_label(ctx.kernel_name(cdfem.K_APPLY), affine),
                    "algorithmic_bytes_per_launch": bytes_, "avg_launch_us": round(per * 1e6, 2),
                    "avg_launch_us_all": round(per_all * 1e6, 2),
                    "launches": cnt, "full_launches": int(len(full)),
                    "avg_note": "avg_launch_us: the full launches (each solve's last apply returns at its first check "
                                "and is left out: avg_launch_us_all keeps it); achieved/frac use avg_launch_us",
                    # the same kernel in a rocprofv3 --kernel-trace of the bench (full launches), and the CSV of its
                    # per-launch durations the figure is recomputed from (tools/rocprof_avg.py)
                    "rocprof_avg_us": rp.get("avg_us_full") if rp else None,
                    "rocprof_avg_all_us": rp.get("avg_us_all") if rp else None,
                    "rocprof_source": rp.get("source") if rp else None,
                    "rocprof_frac_hbm": (round(bytes_ / (rp["avg_us_full"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
                                         if rp and rp.get("avg_us_full") else None),
                    # what binds the kernel per its SQ counters (issue / memory / LDS), beside the closer roofline
                    "limiter": limiter["limiter"] if limiter else None,
                    "limiter_counters": limiter,
                    "events_note": "avg_launch_us is event-bracketed: the completion fences add a few percent per "
                                   "kernel against the uninstrumented ms_per_step",
                    "other_kernels_avg_us": {
                        "e2l": round(e_ms / max(e_cnt, 1) * 1e3, 2),
                        "cg_update": round(u_ms / max(u_cnt, 1) * 1e3, 2),
                        "cg_direction": round(d_ms / max(d_cnt, 1) * 1e3, 2)}})

    # informational: the same steps with the Kronecker form of the per-element factors (pa_uniform 0,
    # the form any affine box takes), when the uniform element matrix ran above
    kron = None
    if world == 1 and uniform and not args.no_kron_form:
        ctx.set_option("pa_uniform", 0)
        step()
        ctx.synchronize()
        t0 = time.perf_counter()
        kits = sum(step()["iterations"] for _ in range(args.steps))
        ctx.synchronize()
        kdt = time.perf_counter() - t0
        ctx.set_option("pa_uniform", uni_opt)
        kron = {"value": mesh.nl * kits / kdt, "unit": "DoF-iter/s", "ms_per_step": kdt / args.steps * 1e3,
                "qdata": "the Kronecker form of the per-element factors on the VALU (pa_uniform 0)"}

    # host-boundary (PCIe-inclusive) rate: one solve with B and X in host memory (not `value`)
    host_rate = None
    if world == 1:
        t0 = time.perf_counter()
        _, hinfo = ctx.solve(B, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0,
                             max_iter=args.cg_iters, check_every=args.cg_iters)
        host_rate = mesh.nl * hinfo["iterations"] / (time.perf_counter() - t0)

    # informational: GMRES(30) + Jacobi (Input/petsc.opts) on the same operator, fixed inner steps
    gm = None
    if world == 1 and args.gmres_iters > 0:
        def gstep():
            return ctx.solve_device(dB, dX, method="gmres", pc="jacobi", rel_tol=0.0, abs_tol=0.0,
                                    max_iter=args.gmres_iters, restart=30)
        gstep()
        ctx.synchronize()
        t0 = time.perf_counter()
        ginfo = gstep()
        ctx.synchronize()
        gdt = time.perf_counter() - t0
        # breakdown from a profiled pass of the same solve, after the timed one: the events bracketing the
        # apply and the CGS passes cost the GPU ~10 us each per step (profiles/r06/ab_gmres_events)
        ctx.set_option("profile_mask", (1 << cdfem.K_APPLY) | (1 << cdfem.K_ORTH))
        ctx.profile(True)
        gstep()
        ctx.synchronize()
        o_ms, o_cnt = ctx.profile_read(cdfem.K_ORTH)
        a_ms, a_cnt = ctx.profile_read(cdfem.K_APPLY)
        ctx.profile(False)
        its = ginfo["iterations"]
        # CGS passes at inner step j move 8 N (2 j + 7) bytes (gmres.hip header)
        js = [k % 30 for k in range(its)]
        orth_bytes = sum(8.0 * mesh.nl * (2 * j + 7) for j in js) / max(len(js), 1)
        gm = {"value": mesh.nl * its / gdt, "unit": "DoF-iter/s", "iterations": its, "restart": 30,
              "ms_per_iter": gdt / max(its, 1) * 1e3,
              "apply_avg_us": round(a_ms / max(a_cnt, 1) * 1e3, 2),
              "orth_avg_us": round(o_ms / max(o_cnt, 1) * 1e3, 2),
              "orth_achieved_gbs": round(orth_bytes / (o_ms / max(o_cnt, 1) * 1e-3) / 1e9, 1) if o_cnt else None}

    # informational: SURVEY §8d's symmetric CG operator kK + sM (c = 0), where CG is a convergent
    # method; fixed 200 iterations per solve, same mesh
    spd = None
    if world == 1 and args.kinds == 7 and args.spd_steps > 0:
        ctx.pa_setup(kinds=5, kappa=0.1, mass=1.0)
        _, B5 = ctx.form_linear_system(np.zeros(mesh.nl), b)
        dB5 = ctx.to_device(B5)

        def sstep():
            return ctx.solve_device(dB5, dX, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0, max_iter=200,
                                    check_every=200)
        sstep()
        ctx.synchronize()
        t0 = time.perf_counter()
        sits = sum(sstep()["iterations"] for _ in range(args.spd_steps))
        ctx.synchronize()
        sdt = time.perf_counter() - t0
        ctx.set_option("profile_mask", 1 << cdfem.K_APPLY)
        ctx.profile(True)
        sstep()
        ctx.synchronize()
        a_ms, a_cnt = ctx.profile_read(cdfem.K_APPLY)
        ctx.profile(False)
        sb = ctx.kernel_bytes(cdfem.K_APPLY)
        s_us = a_ms / max(a_cnt, 1) * 1e3
        spd = {"value": mesh.nl * sits / sdt, "unit": "DoF-iter/s", "operator": "kK+sM (kinds=5, c=0)",
               "cg_iters_per_step": 200, "steps": args.spd_steps, "apply_avg_us": round(s_us, 2),
               "apply_frac": (round(ctx.kernel_flops(cdfem.K_APPLY) / (s_us * 1e-6) / 1e12 / F64_PEAK_TFLOPS, 4)
                              if affine else round(sb / (s_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)) if a_cnt else None,
               "apply_frac_of": "f64 78.6 TFLOP/s" if affine else "HBM 8 TB/s"}
        ctx.free(dB5)

    # informational: the same CG steps with MFEM's per-point qdata stream (pa_affine 0), so the line
    # shows both forms of the operator on one box
    per_point = None
    if world == 1 and affine and args.per_point_steps > 0 and args.config in ("c2", "c3"):
        c2 = cdfem.Context(local % ndev)
        for k, v in args.set.items():
            c2.set_option(k, v)
        c2.set_option("pa_affine", 0)
        c2.upload_mesh(mesh)
        if args.path == "brick" or p >= 3:
            c2.set_structured(n, n, nzr)
        c2.pa_setup(kinds=args.kinds, kappa=0.1, alpha=1.0, conv=c, mass=1.0)
        dB2, dX2 = c2.to_device(B), c2.alloc(8 * mesh.nl)

        def pstep():
            return c2.solve_device(dB2, dX2, method="cg", pc="jacobi", rel_tol=0.0, abs_tol=0.0,
                                   max_iter=args.cg_iters, check_every=args.cg_iters)
        pstep()
        c2.synchronize()
        t0 = time.perf_counter()
        pits = sum(pstep()["iterations"] for _ in range(args.per_point_steps))
        c2.synchronize()
        pdt = time.perf_counter() - t0
        c2.set_option("profile_mask", 1 << cdfem.K_APPLY)
        c2.profile(True)
        pstep()
        c2.synchronize()
        a_ms, a_cnt = c2.profile_read(cdfem.K_APPLY)
        c2.profile(False)
        p_us = a_ms / max(a_cnt, 1) * 1e3
        pb = c2.kernel_bytes(cdfem.K_APPLY)
        per_point = {"value": mesh.nl * pits / pdt, "unit": "DoF-iter/s", "steps": args.per_point_steps,
                     "qdata": "per-point stream (pa_affine 0, MFEM's PA layout)", "apply_avg_us": round(p_us, 2),
                     "apply_hbm_frac": round(pb / (p_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4) if a_cnt else None,
                     "algorithmic_bytes_per_launch": pb}
        c2.free(dB2)
        c2.free(dX2)
        c2.close()

    ntrue = mesh.nl  # per rank (slab L-vector); interface planes counted once below
    total_dofs = (p * n + 1) ** 2 * (p * nz + 1) if world > 1 else ntrue
    value = total_dofs * iters / dt_max
    out = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                # c5: the 256^3 FA matrix is out of the host's reach; per-DoF rate on the 64^3 mesh
                cpu = cpu_baseline(args, min(n, 64), p, args.kinds)
            except Exception as e:  # reported, never fatal for the GPU number
                cpu = {"error": repr(e)}
        out = {
            "metric": "DoF-iter/s (CG, 3D p=2 hex convection-diffusion) + achieved HBM GB/s",
            "value": value, "unit": "DoF-iter/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt_max / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong" if args.config == "c5" else "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"{n}x{n}x{nz} hex, H1 p={p}, PA {kinds_label(args.kinds)} (kinds={args.kinds}), "
                                   f"Jacobi-CG {args.cg_iters} it/step",
                       "operator_note": ("fixed-iteration Jacobi-CG on the BASELINE metric's convection-diffusion "
                                         "operator: a bandwidth figure of the operator + CG vector work (CG has no "
                                         "convergence meaning on the nonsymmetric D+C+M); solver-faithful lines are "
                                         "'gmres' (the reference's GMRES(30)+Jacobi, same operator) and 'spd_cg' "
                                         "(CG on the symmetric kK+sM, SURVEY 8d)") if args.kinds & 2 else
                                        "fixed-iteration Jacobi-CG on a symmetric operator",
                       "dofs": total_dofs, "elements": n * n * nz, "cg_iters_per_step": args.cg_iters,
                       "parallelism": f"slab{world}" if world > 1 else "single",
                       "path": {"k_brick_cg": "brick", "k_hobrick_cg": "ho_brick"}.get(
                           ctx.kernel_name(cdfem.K_APPLY), args.path),
                       **({"options": args.set} if args.set else {}),
                       "qdata": ("uniform box: every element's factors equal, so the apply runs the one 27 x 27 "
                                 "element matrix as a GEMM on the matrix cores (pa_uniform 1, 56 "
                                 "v_mfma_f64_16x16x4_f64 per 64 elements); the operator equals the Kronecker and "
                                 "per-point forms to rounding (tests/test_gpu_uniform.py); the Kronecker form's "
                                 "rate is the 'kronecker_form' line" if uniform else
                                 "affine: 10 factors per element applied in their Kronecker form (pa_affine 2, 1D rule "
                                 "matrices per axis); the operator equals the per-point form to rounding (1e-13 "
                                 "relative, tests/test_gpu_affine.py)" if affine
                                 else "per-point stream (MFEM's PA layout)"),
                       "series": "strong: fixed n^3 split into z-slabs" if args.config == "c5"
                                 else "weak: an n x n x n/8 slab per rank (SURVEY 8e)" if args.config == "c5w"
                                 else "weak: an n^3 slab per rank",
                       **({"comm": args.comm, "comm_lib": comm_lib, "comm_ranks": comm_ranks} if world > 1 else {}),
                       **({"comm_host_timing": comm_timing} if comm_timing else {})},
            "roofline": roof, "cpu_baseline": cpu,
        }
        if kron is not None:
            out["kronecker_form"] = kron
        if gm is not None:
            out["gmres"] = gm
        if spd is not None:
            out["spd_cg"] = spd
        if per_point is not None:
            out["per_point_qdata"] = per_point
        if host_rate is not None:
            out["host_boundary_rate"] = {"value": host_rate, "unit": "DoF-iter/s",
                                         "note": "one solve with B/X in host memory (PCIe copies included)"}
        print(json.dumps(out), flush=True)
    ctx.free(dB)
    ctx.free(dX)
    ctx.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
