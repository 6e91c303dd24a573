"""Summarise rocprofv3 --pmc counter CSVs: per kernel (substring match) and
counter, the median per-dispatch value. Usage:
python scripts/pmc_summary.py KERNEL_SUBSTR dir1 [dir2 ...] > summary.json"""
import csv
import glob
import json
import statistics
import sys

pat = sys.argv[1]
vals = {}
for d in sys.argv[2:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if pat not in row.get("Kernel_Name", ""):
                    continue
                key = (row["Counter_Name"], row.get("Dispatch_Id", ""))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
per = {}
for (name, _disp), v in vals.items():
    per.setdefault(name, []).append(v)
print(json.dumps({"kernel": pat, "dispatches": {k: len(v) for k, v in per.items()},
                  "median": {k: statistics.median(v) for k, v in per.items()}}, indent=1))
