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
