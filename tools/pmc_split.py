"""Per-launch PMC counter of one kernel, split into consecutive groups of launches (the variants an
in-process A/B ran in order, e.g. tools/ab.py --rounds 0 --variants a,b):

    python tools/pmc_split.py <counter_collection.csv> <kernel substring> <groups> [scale]

Prints, per group, the launches and the mean counter value per launch times scale (FETCH_SIZE is
in KiB and gfx950 reports half the bytes read: scale = 2048 gives bytes; WRITE_SIZE: 1024).
"""
import collections
import csv
import sys

path, sub, groups = sys.argv[1], sys.argv[2], int(sys.argv[3])
scale = float(sys.argv[4]) if len(sys.argv) > 4 else 1.0
per = collections.OrderedDict()
for r in csv.DictReader(open(path)):
    if sub in r["Kernel_Name"]:
        d = int(r["Dispatch_Id"])
        per[d] = per.get(d, 0.0) + float(r["Counter_Value"])
ids = sorted(per)
n = len(ids) // groups
for g in range(groups):
    vals = [per[i] for i in ids[g * n:(g + 1) * n]]
    print(f"group {g}: {len(vals)} launches, mean {sum(vals) / max(len(vals), 1) * scale:.6g}")
