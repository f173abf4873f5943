"""f64 compute-rate probe on the GPU box: VALU v_fma_f64 vs v_mfma_f64_16x16x4_f64 (TFLOP/s).
Backs DESIGN.md 4.2 (why the high-order contractions stay on VALU)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "continuum-mechanics-mfem_amd", "python"))
import cdfem  # noqa: E402

with cdfem.Context(0) as ctx:
    out = {"valu_fma_f64_tflops": ctx.fp64_bench(0, 20), "mfma_f64_16x16x4_tflops": ctx.fp64_bench(1, 20)}
    # 4 MFMA (8192 flop per wave) interleaved with nv VALU FMAs per lane (128 nv flop per wave) per trip:
    # sum-of-rates if the two pipes overlap, single rate if they share one
    for mode, nv in ((2, 16), (3, 32), (4, 64)):
        out[f"mixed_4mfma_{nv}fma_tflops"] = ctx.fp64_bench(mode, 20)
print(json.dumps(out))
