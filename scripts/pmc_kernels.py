"""Per-kernel fetched / written bytes and L2 hit rate of pmc_bulk.sh's passes
(one warmup + one timed step: per step = sum / 2; load-time kernels once).
fetched = 2 x FETCH_SIZE KB x 1024 (gfx950 correction, profiles/r02/c4/fetch_calibration.json),
written = WRITE_SIZE KB x 1024.
usage: python scripts/pmc_kernels.py gpurun_out/pmc_c4[_TAG]"""
import csv
import re
import sys
from collections import defaultdict

LOAD = ("k_urec", "k_sbound", "k_lrec", "k_llrec")


def sums(d, counters):
    out = defaultdict(lambda: defaultdict(float))
    with open(f"{d}/p_counter_collection.csv") as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] in counters:
                name = re.sub(r"\(anonymous namespace\)::|void |\(.*$", "", row["Kernel_Name"]).strip()
                out[name][row["Counter_Name"]] += float(row["Counter_Value"])
    return out


base = sys.argv[1]
fe = sums(base + "_fetch", ("FETCH_SIZE",))
wr = sums(base + "_write", ("WRITE_SIZE",))
tc = sums(base + "_tcc", ("TCC_HIT_sum", "TCC_MISS_sum"))
rows = []
for k in set(fe) | set(wr):
    div = 1 if any(k.startswith(x) for x in LOAD) else 2
    f = 2 * fe[k]["FETCH_SIZE"] * 1024 / div / 1e9
    w = wr[k]["WRITE_SIZE"] * 1024 / div / 1e9
    h, m = tc[k]["TCC_HIT_sum"], tc[k]["TCC_MISS_sum"]
    rows.append((f, w, h / (h + m) if h + m else 0.0, k + ("  (load, once)" if div == 1 else "")))
rows.sort(reverse=True)
print(f"{'kernel':55s} fetched GB/step  written GB/step  L2 hit")
for f, w, hr, k in rows:
    if f + w > 0.005:
        print(f"{k:55s} {f:15.2f} {w:16.2f} {hr:7.2f}")
step = [r for r in rows if "once" not in r[3]]
print(f"{'step total':55s} {sum(r[0] for r in step):15.2f} {sum(r[1] for r in step):16.2f}")
