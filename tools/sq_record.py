#!/usr/bin/env python3
"""Record one kernel's SQ counter summary (tools/pmc_sq.sh passes) in profiles/sq_counters.json under a
bench key (the keys of profiles/pmc_traffic.json), with the limiter the counters name.

usage: python tools/sq_record.py OUTDIR KEY KERNEL WAVES_PER_SIMD ROUND

Per wave-cycle fractions (SQ_* / SQ_WAVE_CYCLES) are what one wave sees; with W waves sharing a SIMD,
W x the VALU fraction is the share of the SIMD's cycles its VALU issues.  The limiter:
  issue   (VALU)  when the SIMD's VALU is busy >= 50 % of the kernel (f64 FMAs and bookkeeping),
  memory          when waves wait on memory (SQ_WAIT_ANY) >= 40 % of their cycles,
  LDS             when LDS instructions + waits take >= 25 %,
  latency / occupancy otherwise (none of the pipes busy: too few waves to hide the dependencies).
bench.py copies the record into roofline.limiter beside roofline.bound."""
import json
import os
import subprocess
import sys

out_dir, key, kernel, waves, rnd = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5]
here = os.path.dirname(os.path.abspath(__file__))
summ = json.loads(subprocess.check_output([sys.executable, os.path.join(here, "pmc_sq_summary.py"), out_dir, kernel]))
e = summ[kernel]
w = e["SQ_WAVE_CYCLES"]
valu = e["SQ_ACTIVE_INST_VALU"] / w
mem = e["SQ_WAIT_ANY"] / w
lds = (e.get("SQ_ACTIVE_INST_LDS", 0.0) + e.get("SQ_WAIT_INST_LDS", 0.0)) / w
simd_valu = min(1.0, waves * valu)
if simd_valu >= 0.5:
    lim = "issue (VALU)"
elif mem >= 0.4:
    lim = "memory"
elif lds >= 0.25:
    lim = "LDS"
else:
    lim = "latency / occupancy"
rec = {"kernel": kernel, "round": rnd, "source": out_dir, "waves_per_simd": waves, "limiter": lim,
       "simd_valu_busy": round(simd_valu, 3), "wave_valu": round(valu, 3), "wave_wait_mem": round(mem, 3),
       "wave_wait_issue": round(e.get("SQ_WAIT_INST_ANY", 0.0) / w, 3), "wave_lds": round(lds, 3),
       "lds_bank_conflict_per_lds_inst": round(e.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(e.get("SQ_INSTS_LDS", 1.0), 1.0), 2),
       "per_wave": {k[len("per_wave_"):]: round(v, 1) for k, v in e.items() if k.startswith("per_wave_")}}
path = os.path.join(here, "..", "profiles", "sq_counters.json")
db = json.load(open(path)) if os.path.exists(path) else {}
db[key] = rec
json.dump(db, open(path, "w"), indent=1, sort_keys=True)
print(json.dumps(rec))
