"""Fixed cost of the driver's timed region at C2 (bench.py --steps 20): wall
time per region of one 20-step graph replay, with and without the window's
HIP events around it, closed by a device-wide or an engine-stream wait.
Variants are interleaved so drift hits each alike; prints one JSON line with
the median / p10 wall microseconds per region and the host time of each call.

    python scripts/k20_region_probe.py [--steps 20] [--regions 300]
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
    e = Engine(ds, device=0, out_dtype="f32", topk=10)
    for _ in range(5):
        e.run("ibm")
    e.graph_capture("ibm", a.steps)
    e.graph_launch()
    e.sync()
    torch.cuda.synchronize()
    pc = time.perf_counter

    def events_dev():
        t0 = pc()
        e.timing_begin()
        t1 = pc()
        e.graph_launch()
        t2 = pc()
        e.timing_stop()
        torch.cuda.synchronize()
        t3 = pc()
        _n, ms = e.timing_end()
        return t3 - t0, {"begin": t1 - t0, "launch": t2 - t1, "dev_ms": ms}

    def plain_dev():
        t0 = pc()
        e.graph_launch()
        t1 = pc()
        torch.cuda.synchronize()
        return pc() - t0, {"launch": t1 - t0}

    def plain_stream():
        t0 = pc()
        e.graph_launch()
        e.sync()
        return pc() - t0, {}

    variants = {"events_device_sync": events_dev, "no_events_device_sync": plain_dev,
                "no_events_stream_sync": plain_stream}
    res = {k: [] for k in variants}
    extra = {k: {} for k in variants}
    for _ in range(a.regions):
        for k, fn in variants.items():
            torch.cuda.synchronize()
            w, x = fn()
            res[k].append(w * 1e6)
            for kk, vv in x.items():
                extra[k].setdefault(kk, []).append(vv * (1e3 if kk == "dev_ms" else 1e6))
    out = {"steps": a.steps, "regions": a.regions, "wall_us_per_region": {}}
    for k, v in res.items():
        v = sorted(v)
        out["wall_us_per_region"][k] = {
            "median": statistics.median(v), "p10": v[len(v) // 10], "mean": statistics.fmean(v),
            "median_per_step": statistics.median(v) / a.steps,
            **{kk + "_median_us": statistics.median(vv) for kk, vv in extra[k].items()}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
