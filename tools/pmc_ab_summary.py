"""Per-kernel-instantiation PMC summary of tools/pmc_ab.sh (corrected HBM bytes per launch)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            name[r["Dispatch_Id"]] = r["Kernel_Name"]
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for k, cs in agg.items():
        for c, v in cs.items():
            out[name[k]][c].append(v)
    return out


cal = load(os.path.join(d, "calib"))
fc = next((1 << 20) / (sum(v["FETCH_SIZE"]) / len(v["FETCH_SIZE"])) for k, v in cal.items() if "k_stream_read" in k)
res = collections.defaultdict(dict)
for p in sorted(glob.glob(os.path.join(d, "p*"))):
    if not os.path.isdir(p):
        continue
    for k, cs in load(p).items():
        for c, v in cs.items():
            big = [x for x in v if x > 0.01 * max(v)] if max(v) > 0 else v
            res[k][c] = sum(big) / len(big)
print(f"fetch correction {fc:.3f}")
for k in sorted(res):
    if "spmv" not in k and "perm" not in k:
        continue
    r = res[k]
    f = r.get("FETCH_SIZE", 0) * 1024 * fc / 1e6
    w = r.get("WRITE_SIZE", 0) * 1024 / 1e6
    h, m = r.get("TCC_HIT_sum", 0), r.get("TCC_MISS_sum", 0)
    print(f"{k[:110]:110s} read {f:8.1f} MB write {w:7.1f} MB  L2 hit {h / max(h + m, 1):.3f}")
