"""RCCL runtime check on a one-GPU box.

The slab CG/GMRES exchange (`csrc/comm.hip`: `ncclSend/ncclRecv` of the interface planes, 8-byte
`ncclAllReduce`s) runs only when ranks sit on different GPUs, i.e. in the driver's multi-GPU
bench; RCCL refuses two ranks on one device, so the multi-rank GPU tests use the host-callback
communicator.  This test runs the same RCCL calls on a one-rank communicator
(`cpp/rccl_selftest.cpp`, built by the package Makefile against the librccl that `libcdfem.so`
links): the bootstrap, a device-buffer all-reduce on a non-default stream and a grouped self
send/recv of one p = 2 interface plane.  It pins that RCCL works on the box image before the N > 1
runs depend on it.  It runs as a child process so that its communicator and proxy threads end
with it.
"""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
EXE = os.path.join(ROOT, "continuum-mechanics-mfem_amd", "lib", "rccl_selftest")


def test_rccl_comm_init_in_process(gpu_ctx):
    import cdfem
    uid = cdfem.comm_unique_id()  # the bytes bench.py broadcasts from rank 0
    assert len(uid) == 128 and any(uid)
    # ncclCommInitRank inside this process, beside live contexts (the N > 1 bench order); a
    # re-init destroys the first communicator, close() the second
    ctx = cdfem.Context(0)
    try:
        ctx.comm_init_rccl(0, 1, uid)
        ctx.comm_init_rccl(0, 1, cdfem.comm_unique_id())
    finally:
        ctx.close()


def test_rccl_one_rank_allreduce_and_self_exchange():
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} missing: run __graft_entry__.build() first")
    out = subprocess.run([EXE], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "RCCL SELFTEST OK" in out.stdout, out.stdout + out.stderr
    assert "allreduce 3.25, mismatches 0" in out.stdout


def test_bench_refuses_host_fallback(tmp_path):
    """`bench.py --gpus 2` (default --comm rccl) with both ranks on the box's one GPU: RCCL refuses
    two ranks on one device, and the bench must exit non-zero instead of producing an N > 1 number
    on the host-callback fallback; `--comm host` is the explicit rehearsal mode and runs."""
    import socket
    import sys

    def port():
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            return s.getsockname()[1]
    base = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
            "--master-addr", "127.0.0.1"]
    args = ["bench.py", "--gpus", "2", "--elems", "8", "--steps", "1", "--warmup", "0", "--cg-iters", "5",
            "--no-cpu-baseline", "--spd-steps", "0", "--gmres-iters", "0", "--no-profile-events"]
    r = subprocess.run(base + ["--master-port", str(port())] + args, capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    assert r.returncode != 0, r.stdout[-2000:]
    assert "refusing to run the N>1 bench on the host fallback" in r.stderr, r.stderr[-3000:]
    assert '"metric"' not in r.stdout
    r = subprocess.run(base + ["--master-port", str(port())] + args + ["--comm", "host"], capture_output=True,
                       text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    import json
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["config"]["comm"] == "host"
    assert [d["rank"] for d in out["config"]["comm_ranks"]] == [0, 1]
