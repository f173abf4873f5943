#!/usr/bin/env python3
"""Per-kernel averages (per dispatch) of the SQ counter passes written by tools/pmc_sq.sh.
usage: python tools/pmc_sq_summary.py OUTDIR [kernel-substring] > summary.json"""
import collections
import csv
import glob
import json
import os
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
res = collections.defaultdict(dict)
for f in sorted(glob.glob(os.path.join(src, "sq_*", "**", "*counter_collection.csv"), recursive=True)):
    per = collections.defaultdict(float)
    name = {}
    for r in csv.DictReader(open(f)):
        k = (r["Dispatch_Id"], r["Counter_Name"])
        per[k] += float(r["Counter_Value"])
        name[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
    by = collections.defaultdict(list)
    for (d, cn), v in per.items():
        by[(name[d], cn)].append(v)
    for (kn, cn), vs in by.items():
        if pat and pat not in kn:
            continue
        big = [x for x in vs if x > 0.01 * max(vs)] if max(vs) > 0 else vs
        res[kn][cn] = {"avg": sum(big) / len(big), "dispatches": len(big)}
out = {}
for kn, d in res.items():
    o = {k: v["avg"] for k, v in sorted(d.items())}
    w = o.get("SQ_WAVE_CYCLES")
    if w:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS"):
            if k in o:
                o["frac_" + k] = o[k] / w
    if o.get("SQ_WAVES"):
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM"):
            if k in o:
                o["per_wave_" + k] = o[k] / o["SQ_WAVES"]
    out[kn] = o
json.dump(out, sys.stdout, indent=1)
