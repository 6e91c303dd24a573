"""Wall time of one replay of an n-step C2 graph (n = 1 .. 40), closed by a
device-wide synchronize, against its device window (HIP events): how the
region's fixed cost splits into host submission (grows with n?) and the
launch / completion latency. One JSON line per n: median wall, median device
window, median host time of the hipGraphLaunch call, all in microseconds.

    python scripts/graph_size_probe.py [--regions 200] [--sizes 1,2,5,10,20,40]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from musicrecommendation_amd import synth  # noqa: E402
from musicrecommendation_amd.engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--regions", type=int, default=200)
    ap.add_argument("--sizes", default="1,2,5,10,20,40")
    a = ap.parse_args()
    ds = synth.config("c2").dataset()
    e = Engine(ds, device=0, out_dtype="f32", topk=10)
    for _ in range(5):
        e.run("ibm")
    e.sync()
    pc = time.perf_counter
    for n in [int(x) for x in a.sizes.split(",")]:
        e.graph_capture("ibm", n)
        e.graph_launch()
        e.sync()
        wall, dev, sub, wall_ev = [], [], [], []
        for _ in range(a.regions):
            torch.cuda.synchronize()
            t0 = pc()
            e.graph_launch()
            t1 = pc()
            torch.cuda.synchronize()
            t2 = pc()
            wall.append((t2 - t0) * 1e6)
            sub.append((t1 - t0) * 1e6)
            torch.cuda.synchronize()
            t0 = pc()
            e.timing_begin()
            e.graph_launch()
            e.timing_stop()
            torch.cuda.synchronize()
            t2 = pc()
            _k, ms = e.timing_end()
            wall_ev.append((t2 - t0) * 1e6)
            dev.append(ms * 1e3)
        print(json.dumps({"steps": n, "wall_us": statistics.median(wall), "wall_events_us": statistics.median(wall_ev),
                          "device_us": statistics.median(dev), "launch_call_us": statistics.median(sub),
                          "overhead_us": statistics.median(wall) - statistics.median(dev)}), flush=True)


if __name__ == "__main__":
    main()
