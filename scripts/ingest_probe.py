"""Ingest at full scale: write a config's synthetic triplet
files, then time the native TSV ingest (mr_corpus_from_tsv via
Dataset.from_tsv) and mr_load's host index build + H2D, with a JSON summary.

    python scripts/ingest_probe.py --config c4 [--out gpurun_out/ingest_c4.json] [--load] [--check]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from musicrecommendation_amd import synth  # noqa: E402
from musicrecommendation_amd.dataset import Dataset  # noqa: E402
from musicrecommendation_amd.mr_par_info import usable_cores  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--load", action="store_true", help="also time mr_load (needs a GPU)")
    ap.add_argument("--check", action="store_true", help="compare with the numpy builder")
    ap.add_argument("--dir", default=None)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    t0 = time.perf_counter()
    trip = synth.config(args.config)
    gen_s = time.perf_counter() - t0
    print(f"generated {args.config} in {gen_s:.1f} s", flush=True)
    res = {"config": args.config, "cores": usable_cores(), "generate_s": gen_s}
    with tempfile.TemporaryDirectory(dir=args.dir) as td:
        paths = [os.path.join(td, n) for n in ("train.txt", "test.txt", "labels.txt")]
        t0 = time.perf_counter()
        res["tsv_bytes"] = trip.write_tsv(*paths)
        res["write_s"] = time.perf_counter() - t0
        print(f"wrote {res['tsv_bytes'] / 1e9:.2f} GB in {res['write_s']:.1f} s", flush=True)
        res["rows"] = int(trip.train_u.size + trip.test_u.size + trip.label_u.size)
        times = []
        ds = None
        for _ in range(args.reps):
            ds = None
            t0 = time.perf_counter()
            ds = Dataset.from_tsv(*paths)
            times.append(time.perf_counter() - t0)
            print(f"ingest {times[-1]:.2f} s", flush=True)
        res["ingest_s"] = sorted(times)[len(times) // 2]
        res["ingest_all_s"] = times
        res["shape"] = {"n_train": ds.n_train, "n_test": ds.n_test, "n_songs": ds.n_songs,
                        "nnz_train": int(ds.tr_off[-1])}
    if args.check:
        ref = trip.dataset()
        res["check"] = all(np.array_equal(getattr(ref, f), getattr(ds, f))
                           for f in ("tr_off", "tr_songs", "te_off", "te_songs", "song_count", "tr_len", "te_len",
                                     "lab_off", "lab_songs"))
    if args.load:
        import torch  # noqa: F401
        from musicrecommendation_amd.engine import Engine

        times = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            e = Engine(ds, device=0, topk=10, dense=False)
            times.append(time.perf_counter() - t0)
            print(f"mr_load {times[-1]:.2f} s", flush=True)
            e.close()
        res["mr_load_s"] = sorted(times)[len(times) // 2]
        res["mr_load_all_s"] = times
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
