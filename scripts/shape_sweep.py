"""Launch-shape sweep: device ms per run of each shape on bulk synthetic data.
Usage: python scripts/shape_sweep.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from musicrecommendation_amd import _lib, synth  # noqa: E402
from musicrecommendation_amd.engine import Engine  # noqa: E402

for n_tr, n_te in ((500, 10), (500, 32), (500, 64), (500, 128), (500, 256), (2000, 10), (2000, 32), (2000, 100), (2000, 1000), (5000, 1000), (10000, 300), (10000, 1000), (16000, 2000)):
    ds = synth.generate_bulk(n_tr, n_te, 3).dataset()
    row = [f"{n_tr:6d}/{n_te:5d} songs {ds.n_songs:6d}"]
    for shape in ("fused", "separate", "wide"):
        try:
            with Engine(ds, topk=10, stage1=shape) as e:
                e.run("ibm")
                e.sync()
                e.timing_begin()
                for _ in range(3):
                    e.run("ibm")
                _, ms = e.timing_end()
                row.append(f"{shape} {ms / 3:8.3f}")
        except _lib.EngineError:
            row.append(f"{shape}      n/a")
    print("  ".join(row), flush=True)
