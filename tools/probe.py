"""HBM probes on the GPU box: grid-stride streams and per-wave private chunks (brick pattern)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "continuum-mechanics-mfem_amd", "python"))
import cdfem  # noqa: E402

names = ["read16_gridstride", "read8_gridstride", "copy16", "chunk_U8_1wave", "chunk_U16_1wave",
         "chunk_U8_free", "chunk_U4_1wave", "chunk_U32_1wave", "ileave_U8_1wave", "ileave_U4_1wave",
         "chunk_U8_1wave_skew256B", "chunk_U8_1wave_skew512B", "chunk_U8_1wave_skew1K", "chunk_U8_1wave_skew4K",
         "wgchunk4_U8_1wave", "wgchunk2_U8", "gridstride_64thr_1wave_1024wg", "gridstride_64thr_1wave_4096wg"]
with cdfem.Context(0) as ctx:
    print(json.dumps({nm: round(ctx.stream_bench(m, 2 << 30, 10), 1) for m, nm in enumerate(names)}, indent=1))
