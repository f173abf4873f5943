import os, sys, json
sys.path.insert(0, os.path.join("continuum-mechanics-mfem_amd", "python"))
import cdfem
with cdfem.Context(0) as ctx:
    out = {m: round(ctx.stream_bench(m, 2 << 30, 10), 1) for m in (0, 1, 3, 4, 5, 6, 7, 8, 9)}
print(json.dumps(out))
