"""HBM/fabric traffic per launch of one kernel from rocprofv3 --pmc passes
(separate runs: FETCH_SIZE, WRITE_SIZE, TCC_HIT_sum/TCC_MISS_sum), with the
gfx950 correction measured by scripts/ubench/fetch_calib.hip
(profiles/r02/c4/fetch_calibration.json): FETCH_SIZE counts 64 B per 128-B
line fetched for every access width, so fetched bytes = 2 x FETCH_SIZE KB x
1024; WRITE_SIZE is taken as bytes (exact for coalesced stores per the guide).
Usage: python scripts/pmc_traffic.py CONFIG KERNEL_SUBSTR OUT.json dir1 [dir2 ...]
KERNEL_SUBSTR "step:N[:EXCL,...]": the sum over every engine kernel (k_*, minus
names containing an EXCL) of a run of N bench steps, divided by N
(multi-kernel steps: C3/C4/C5)."""
import csv
import glob
import json
import statistics
import sys

import os

cfg, pat, out_path, dirs = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4:]
ROUTE = os.environ.get("IBM_ROUTE")  # the ibm route the passes ran (bench.py checks it before using the file)
if pat.startswith("step:"):
    parts = pat.split(":")
    n_steps = int(parts[1])
    excl = [x for x in (parts[2].split(",") if len(parts) > 2 else []) if x]
    tot, disp = {}, {}
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "")
                    if "k_" not in name or "rocclr" in name or any(x in name for x in excl):
                        continue
                    c = row["Counter_Name"]
                    tot[c] = tot.get(c, 0.0) + float(row["Counter_Value"])
                    disp.setdefault(c, set()).add((d, row.get("Dispatch_Id", "")))
    per_step = {c: v / n_steps for c, v in tot.items()}
    fetch = per_step.get("FETCH_SIZE", 0.0) * 1024 * 2
    write = per_step.get("WRITE_SIZE", 0.0) * 1024
    res = {"config": cfg, "kernel": "every engine kernel of a step", "steps": n_steps,
           "dispatches": {c: len(v) for c, v in disp.items()}, "per_step": per_step,
           "fetch_bytes_corrected": fetch, "write_bytes": write, "traffic_bytes_per_launch": fetch + write,
           "traffic_unit": "bytes per step (bench's roofline for multi-kernel steps is per step)",
           "ibm_route": ROUTE,
           "l2_hit_rate": (per_step["TCC_HIT_sum"] / (per_step["TCC_HIT_sum"] + per_step["TCC_MISS_sum"]))
           if "TCC_HIT_sum" in per_step else None,
           "traffic_note": "fetched = 2 x FETCH_SIZE (profiles/r02/c4/fetch_calibration.json) + WRITE_SIZE, "
                           "summed over the step's kernels; separate rocprofv3 --pmc passes with --kernel-trace only"}
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res, indent=1))
    sys.exit(0)
vals = {}
kname = None
for d in dirs:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if pat not in row.get("Kernel_Name", ""):
                    continue
                kname = row["Kernel_Name"]
                key = (row["Counter_Name"], d, row.get("Dispatch_Id", ""))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
per = {}
for (name, _d, _disp), v in vals.items():
    per.setdefault(name, []).append(v)
med = {k: statistics.median(v) for k, v in per.items()}
fetch = med.get("FETCH_SIZE", 0.0) * 1024 * 2
write = med.get("WRITE_SIZE", 0.0) * 1024
res = {"config": cfg, "kernel": kname, "launches_sampled": {k: len(v) for k, v in per.items()},
       "median_per_launch": med, "fetch_bytes_corrected": fetch, "write_bytes": write,
       "traffic_bytes_per_launch": fetch + write,
       "l2_hit_rate": (med["TCC_HIT_sum"] / (med["TCC_HIT_sum"] + med["TCC_MISS_sum"]))
       if "TCC_HIT_sum" in med else None,
       "traffic_note": "fetched = 2 x FETCH_SIZE (64 B counted per 128-B line for 2/4/8/16-B accesses alike, "
                       "profiles/r02/c4/fetch_calibration.json) + WRITE_SIZE; medians over the profiled launches; "
                       "separate rocprofv3 --pmc passes with --kernel-trace only"}
json.dump(res, open(out_path, "w"), indent=1)
print(json.dumps(res, indent=1))
