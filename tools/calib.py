"""Run the HBM stream probes once (for FETCH_SIZE calibration under rocprofv3 --pmc)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "continuum-mechanics-mfem_amd", "python"))
import cdfem  # noqa: E402

with cdfem.Context(0) as ctx:
    for mode in (0, 1, 2):
        print(mode, ctx.stream_bench(mode, 1 << 30, 3))
