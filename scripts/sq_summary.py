"""Per-kernel SQ counter ratios from one rocprofv3 --pmc pass (gpu_session.sh
step pmcsq): the share of wave cycles waiting on anything / on LDS
instructions, LDS bank-conflict cycles per LDS-array cycle, LDS and vector
memory read instructions per wave. Usage: python scripts/sq_summary.py DIR"""
import csv
import glob
import re
import sys

tot = {}
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            n = row.get("Kernel_Name", "")
            m = re.search(r"(k_\w+(<[^()]*>)?)", n)
            if not m:
                continue
            d = tot.setdefault(m.group(1), {})
            d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
print(f"{'kernel':44s} {'waves':>9s} {'wait/cyc':>8s} {'ldswait/cyc':>11s} {'bankconf/lds':>12s} "
      f"{'lds/wave':>9s} {'vmem/wave':>9s} {'valu/wave':>9s} {'salu/wave':>9s} {'actany/cyc':>10s} {'cyc/wave':>10s}")
for k, d in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    w = max(d.get("SQ_WAVES", 0.0), 1.0)
    cyc = max(d.get("SQ_WAVE_CYCLES", 0.0), 1.0)
    print(f"{k[:44]:44s} {w:9.0f} {d.get('SQ_WAIT_ANY', 0) / cyc:8.3f} {d.get('SQ_WAIT_INST_LDS', 0) / cyc:11.3f} "
          f"{d.get('SQ_LDS_BANK_CONFLICT', 0) / max(d.get('SQ_LDS_IDX_ACTIVE', 0), 1):12.3f} "
          f"{d.get('SQ_INSTS_LDS', 0) / w:9.1f} {d.get('SQ_INSTS_VMEM_RD', 0) / w:9.1f} "
          f"{d.get('SQ_INSTS_VALU', 0) / w:9.1f} {d.get('SQ_INSTS_SALU', 0) / w:9.1f} "
          f"{d.get('SQ_ACTIVE_INST_ANY', 0) / cyc:10.3f} {cyc / w:10.0f}")
