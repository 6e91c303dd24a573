"""The driver's 20-step C2 region as one 20-step graph replay vs one direct
mr_run followed by a 19-step graph replay (the first kernel's packet is
written without the graph launch's fixed host cost in front of it, which the
graph then pays while that kernel runs). Interleaved regions, closed by a
device-wide synchronize, the window's events around them as in bench.py.
One JSON line: median wall and device window per region, microseconds.

    python scripts/graph_head_probe.py [--steps 20] [--regions 300]
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--regions", type=int, default=300)
    a = ap.parse_args()
    ds = synth.config("c2").dataset()
    full = Engine(ds, device=0, out_dtype="f32", topk=10)
    head = Engine(ds, device=0, out_dtype="f32", topk=10)
    for e in (full, head):
        for _ in range(5):
            e.run("ibm")
        e.sync()
    full.graph_capture("ibm", a.steps)
    head.graph_capture("ibm", a.steps - 1)
    for e in (full, head):
        e.graph_launch()
        e.sync()
    pc = time.perf_counter

    def graph_only():
        t0 = pc()
        full.timing_begin()
        full.graph_launch()
        full.timing_stop()
        torch.cuda.synchronize()
        t1 = pc()
        _n, ms = full.timing_end()
        return t1 - t0, ms

    def run_then_graph():
        t0 = pc()
        head.timing_begin()
        head.run("ibm")
        head.graph_launch()
        head.timing_stop()
        torch.cuda.synchronize()
        t1 = pc()
        _n, ms = head.timing_end()
        return t1 - t0, ms

    variants = {"graph": graph_only, "run_then_graph": run_then_graph}
    res = {k: ([], []) for k in variants}
    for _ in range(a.regions):
        for k, fn in variants.items():
            torch.cuda.synchronize()
            w, ms = fn()
            res[k][0].append(w * 1e6)
            res[k][1].append(ms * 1e3)
    print(json.dumps({k: {"wall_us": statistics.median(v[0]), "wall_p10": sorted(v[0])[len(v[0]) // 10],
                          "device_us": statistics.median(v[1]), "wall_per_step": statistics.median(v[0]) / a.steps}
                      for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
