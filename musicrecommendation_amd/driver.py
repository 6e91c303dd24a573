"""Spark-free equivalent of the reference's drivers (src/main/scala/main.scala
MN:8-123, src/main/scala/distributed.scala DS:55-602) on the MI355X engine.

    python -m musicrecommendation_amd.driver TRAIN_N TEST_N [--resources DIR]
        [--devices 0,1,...] [--song-shards G_s] [--user-blocks G_u] [--distributed] [--quiet]

Same flow and output as main.scala: load train_{N}_{M}.txt, test_{N}_{M}.txt,
test_labels_{N}_{M}.txt (MN:21-23), build the recommender (untimed, MN:27),
time the user- and item-based models (MN:37-40), sort them by (user, song,
-score) (MN:57-59), time the linear / aggregation / stochastic combinations
with 0.5 (MN:62-89), evaluate all five with the threshold mAP (MN:101-110) and
print the mAPs rounded to 10 decimals (MN:112-121). Times print as
MyUtils.time does (my_utils/MyUtils.scala:4-15). --distributed follows
distributed.scala instead: defaults 300 / 10 (DS:61-62) and its evaluation's
11 thresholds 0.0..1.0 (DS:395-415) for every mAP.

The models stay on the device as dense buffers (ensemble.DeviceEnsemble): the
combinations and the mAP run as HIP kernels, nothing is materialised as a
pair list. With --devices / --song-shards / --user-blocks the two similarity
models are ALSO scored through one multi-GPU group (mr_group_*, the
distributed.scala strategies 1/2 as a single call: song shards x user blocks,
in-library RCCL across GPUs) and checked bit for bit against the
single-context models. The reference's sequential/parallel pairs collapse into
one GPU run each (seq = par holds by construction, README.md:254-261).
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from typing import Callable, Optional, Sequence, TypeVar

T = TypeVar("T")


def timed(f: Callable[[], T], what: str, verbose: bool = True) -> T:
    """MyUtils.time (MyUtils.scala:4-15): run, print the elapsed wall time."""
    import torch

    t0 = time.perf_counter_ns()
    r = f()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    dt = time.perf_counter_ns() - t0
    if verbose:
        print(f"Elapsed time for {what}:\t{dt // 1_000_000}ms ({dt}ns)", flush=True)
    return r


def round_at(p: int, x: float) -> float:
    """MyUtils.roundAt (MyUtils.scala:17): math.round(x * 10^p) / 10^p."""
    import math

    s = 10 ** p
    return math.floor(x * s + 0.5) / s


def run(train_n: int, test_n: int, resources: str, devices: Optional[Sequence[int]] = None,
        song_shards: Optional[int] = None, user_blocks: int = 1, verbose: bool = True, seed: int = 1,
        distributed: bool = False) -> dict:
    import numpy as np

    from .dataset import Dataset
    from .engine import Engine
    from .ensemble import DeviceEnsemble

    n_thr = 11 if distributed else 10  # DS:395 vs MR:590
    if song_shards is None:  # one song shard per listed GPU and user block (DS:477-479's song partition)
        song_shards = max(1, len(devices) // max(1, user_blocks)) if devices else 1
    if verbose:
        print(f"Train users: {train_n}\nTest users: {test_n}", flush=True)
    paths = [os.path.join(resources, f"{k}_{train_n}_{test_n}.txt") for k in ("train", "test", "test_labels")]
    for p in paths:
        if not os.path.exists(p):
            raise FileNotFoundError(p)
    if verbose:
        print("Loaded files", flush=True)
    ds = Dataset.from_tsv(*paths)                                     # MN:27, untimed
    dev = devices[0] if devices else 0
    eng = Engine(ds, device=dev, out_dtype="f64", topk=10)
    ens = DeviceEnsemble(eng)
    if verbose:
        print("MusicRecommender instanced", flush=True)
    ubm = timed(lambda: ens.model("ubm"), "user-based model", verbose)     # MN:37-38
    ibm = timed(lambda: ens.model("ibm"), "item-based model", verbose)     # MN:39-40
    group_checked = None
    if devices and (len(devices) > 1 or song_shards > 1 or user_blocks > 1):
        from .group import Group

        with Group(ds, song_shards=song_shards, user_blocks=user_blocks, devices=devices, out_dtype="f64",
                   topk=10) as g:
            for name, t in (("user-based", ubm), ("item-based", ibm)):
                # run AND drain every context's stream inside the timed region
                timed(lambda: (g.run("ubm" if name == "user-based" else "ibm"), g.sync()),
                      f"{name} model ({g.transport}, {song_shards} song shards x {user_blocks} user blocks)",
                      verbose)
                if not np.array_equal(g.dense(), t.cpu().numpy(), equal_nan=True):
                    raise AssertionError(f"multi-GPU {name} model differs from the single-context model")
        group_checked = True
    # MN:57-59 sorts by (user, song, -score): the dense rows are in that order
    # already (lexicographic ids), the combinations index pairs in it.
    lcm = timed(lambda: ens.linear(ubm, ibm, 0.5), "linear-combination model", verbose)          # MN:62-69
    am = timed(lambda: ens.aggregation(ubm, ibm, 0.5), "aggregation model", verbose)             # MN:70-77
    scm = timed(lambda: ens.stochastic(ubm, ibm, 0.5, seed=seed), "stochastic-combination model", verbose)
    maps = {}
    for name, t in (("user-based", ubm), ("item-based", ibm), ("linear-combination", lcm), ("aggregation", am),
                    ("stochastic-combination", scm)):
        maps[name] = timed(lambda: ens.threshold_map(t, n_thresholds=n_thr), f"{name} model mAP", verbose)  # MN:101-110
    for name, v in maps.items():
        print(f"{name} model mAP: {round_at(10, v)}", flush=True)                              # MN:112-121
    eng.close()
    return {"mAP": maps, "multi_gpu_checked": group_checked, "thresholds": n_thr,
            "layout": (song_shards, user_blocks)}


def main(argv: Optional[Sequence[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("train_n", type=int, nargs="?", default=None)  # MN:15 default 100 (DS:61: 300)
    ap.add_argument("test_n", type=int, nargs="?", default=10)     # MN:16 / DS:62 default
    ap.add_argument("--resources", default=".", help="directory of the train/test/test_labels TSV files")
    ap.add_argument("--devices", default="", help="comma-separated GPU ids for the multi-GPU group")
    ap.add_argument("--song-shards", type=int, default=None,
                    help="default: one per listed device and user block")
    ap.add_argument("--user-blocks", type=int, default=1)
    ap.add_argument("--seed", type=int, default=1, help="stochastic combination seed (the reference's is unseeded)")
    ap.add_argument("--distributed", action="store_true",
                    help="distributed.scala's flow: defaults 300/10, 11-threshold mAP (DS:61-62, DS:395)")
    ap.add_argument("--quiet", action="store_true")
    a = ap.parse_args(argv)
    devices = [int(x) for x in a.devices.split(",") if x.strip()] if a.devices else None
    train_n = a.train_n if a.train_n is not None else (300 if a.distributed else 100)
    run(train_n, a.test_n, a.resources, devices, a.song_shards, a.user_blocks, verbose=not a.quiet, seed=a.seed,
        distributed=a.distributed)
    return 0


if __name__ == "__main__":
    sys.exit(main())
