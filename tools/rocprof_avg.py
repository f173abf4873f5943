#!/usr/bin/env python3
"""Per-launch durations of one kernel from a rocprofv3 --kernel-trace CSV, and the averages bench.py
quotes beside its event timing (roofline.rocprof_avg_us / rocprof_source).

    rocprofv3 --kernel-trace --stats -d OUT -o run --output-format csv -- python3 bench.py ...
    python3 tools/rocprof_avg.py --trace OUT --kernel k_brick_cg --key n64_p2_k7_aff \
        --csv profiles/r06/r06b_c2_k_brick_cg_launches.csv

Writes the kernel's launches (start-ordered durations in ns) to --csv and updates --json[key] with
avg_us_all (every launch), avg_us_full (launches of at least half the median: each CG solve's last
apply returns at its first check and takes a few us) and the CSV path, so the bench line's roofline
fraction can be recomputed from a committed file.
"""
import argparse
import csv
import glob
import json
import os
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("--trace", required=True, help="rocprofv3 output directory (searched for *kernel_trace.csv)")
ap.add_argument("--kernel", required=True)
ap.add_argument("--key", required=True, help="bench.py's roofline key, e.g. n64_p2_k7_aff")
ap.add_argument("--csv", required=True, help="where to write this kernel's per-launch durations")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap.add_argument("--json", default=os.path.join(ROOT, "profiles", "rocprof_kernels.json"))
ap.add_argument("--skip", type=int, default=0, help="leading launches to drop (warm-up solves)")
a = ap.parse_args()

files = glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True)
if not files:
    raise SystemExit(f"no kernel_trace.csv under {a.trace}")
rows = []
for f in files:
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("cdfem::", "").strip()
        if name == a.kernel:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
rows.sort()
rows = rows[a.skip:]
if not rows:
    raise SystemExit(f"no launches of {a.kernel}")
dur = [d for _, d in rows]
med = statistics.median(dur)
full = [d for d in dur if d >= 0.5 * med]
os.makedirs(os.path.dirname(os.path.abspath(a.csv)), exist_ok=True)
with open(a.csv, "w") as fo:
    fo.write("launch,duration_ns\n")
    for i, d in enumerate(dur):
        fo.write(f"{i},{d}\n")
rec = {"kernel": a.kernel, "launches": len(dur), "full_launches": len(full),
       "avg_us_all": round(sum(dur) / len(dur) / 1e3, 3), "avg_us_full": round(sum(full) / len(full) / 1e3, 3),
       "median_us": round(med / 1e3, 3), "source": os.path.relpath(os.path.abspath(a.csv), ROOT)}
db = json.load(open(a.json)) if os.path.exists(a.json) else {}
db[a.key] = rec
with open(a.json, "w") as fo:
    json.dump(db, fo, indent=1, sort_keys=True)
print(json.dumps({a.key: rec}))
