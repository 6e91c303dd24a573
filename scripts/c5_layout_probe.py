"""C5 per-model layouts (sharding.EnsembleScorer) at N ranks, each rank's
slice built and timed alone on ONE GPU (the driver's 8-GPU node is not
available to this build's sessions): ubm on test-user block r, ibm on song
shard r, the placement of the all-to-all's received pieces into the block's
columns (the device copies; the transfer itself is modelled below), the three
combinations on the block and the five threshold mAPs' class counts + AP.

The all-to-all moves (N-1)/N of each rank's ibm shard out and as much in:
with xGMI point-to-point (7 links per GPU, ~153 GB/s each per the build
brief) every pair of ranks exchanges exchange_bytes / (N-1) over its own
link. Modelled at 50 % and 100 % of a 76.5 GB/s direction.
  python scripts/c5_layout_probe.py [N ...]   (default 8)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from musicrecommendation_amd import synth  # noqa: E402
from musicrecommendation_amd.sharding import EnsembleScorer  # noqa: E402

LINK_GBS = 153.0 / 2  # one direction of one xGMI link


def timed(fn, reps=2):
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        best = dt if best is None else min(best, dt)
    return best, out


def device_ms(eng, model, t, reps=2):
    best = None
    for _ in range(reps):
        eng.timing_begin()
        eng.run_into(model, t.data_ptr())
        _n, ms = eng.timing_end()
        best = ms if best is None else min(best, ms)
    return best


def main():
    ns = [int(x) for x in sys.argv[1:]] or [8]
    full = synth.config("c5").dataset()
    for n in ns:
        ranks = []
        t_all = time.time()
        for r in range(n):
            sc = EnsembleScorer(full, r, n, 0, out_dtype="f32")
            ens, ens_i = sc.ens, sc.ens_i
            ubm = ens.model("ubm")  # warm (neighbour lists allocated, kernels loaded)
            ibm_s = ens_i.model("ibm")
            ph = {"ubm_ms": device_ms(sc.eng_u, "ubm", ubm), "ibm_ms": device_ms(sc.eng_i, "ibm", ibm_s)}
            # the exchange's placement: a received buffer of the right size into the block's columns
            recv = torch.rand(sum(sc.recv_splits), dtype=torch.float32, device="cuda")  # (timing only)

            def place():
                out = ens.empty()
                off, nb = 0, sc.user_hi - sc.user_lo
                for (lo, hi), k in zip(sc.shards, sc.recv_splits):
                    out[:, lo:hi].copy_(recv[off:off + k].view(nb, hi - lo))
                    off += k
                return out
            ph["place_ms"], ibm = timed(place)

            def overlapped():  # EnsembleScorer.step's order: ubm queued, ibm beside it, the placement
                out_u = ens.empty()
                sc.eng_u.run_into("ubm", out_u.data_ptr())
                sc.eng_i.run_into("ibm", ibm_s.data_ptr())
                sc.eng_i.sync()
                o = place()
                sc.eng_u.sync()
                return o
            ov_ms, _ = timed(overlapped)
            ibm._mr_minmax = (ibm._version, 0.0, 1.0)
            ph["combinations_ms"], comb = timed(lambda: ens.combinations(ubm, ibm, 0.5, 0.5, 0.5, seed=1))
            models = {"ubm": ubm, "ibm": ibm, "lcm": comb[0], "am": comb[1], "scm": comb[2]}
            cls, cpos = ens._classes()
            blk = torch.empty((5, 2, cls.shape[0], 10), dtype=torch.int32, device="cuda")

            def evals():  # as DeviceEnsemble.threshold_maps, less its two all-reduces
                sc.eng_u.eval_class_counts([t.data_ptr() for t in models.values()], [0.0] * 5, [1.0] * 5,
                                           sc.ds_u.lab_off, sc.ds_u.lab_songs, cls, blk.data_ptr())
                return sc.eng_u.eval_map_counts(5, blk.data_ptr(), cpos, full.n_label_songs)
            ph["five_maps_ms"], _ = timed(evals)
            slice_ms = sum(ph.values())
            ph_ov = {"models_overlapped_ms": ov_ms,
                     "slice_overlapped_ms": ov_ms + ph["combinations_ms"] + ph["five_maps_ms"]}
            xb = sc.exchange_bytes
            per_link = xb / max(1, n - 1)
            ph_ex = {"exchange_bytes_per_rank": xb, "count_block_bytes": int(blk.numel() * 4),
                     "exchange_ms_link_full": per_link / (LINK_GBS * 1e9) * 1e3,
                     "exchange_ms_link_half": per_link / (0.5 * LINK_GBS * 1e9) * 1e3}
            ranks.append({"rank": r, "users": [sc.user_lo, sc.user_hi], "songs": [sc.song_lo, sc.song_hi],
                          "ibm_route": sc.ibm_route, **ph, "slice_ms": slice_ms, **ph_ov, **ph_ex})
            del ubm, ibm_s, ibm, comb, models, recv, blk
            sc.close()
            torch.cuda.empty_cache()
            print(json.dumps(ranks[-1]), flush=True)
        worst = max(x["slice_ms"] for x in ranks)
        ex = max(x["exchange_ms_link_half"] for x in ranks)
        print(json.dumps({"layout": f"models{n}", "max_slice_ms": worst,
                          "max_slice_overlapped_ms": max(x["slice_overlapped_ms"] for x in ranks),
                          "max_slice_overlapped_plus_exchange_half_ms": max(
                              x["slice_overlapped_ms"] + x["exchange_ms_link_half"] for x in ranks),
                          "max_slice_plus_exchange_half_ms": max(x["slice_ms"] + x["exchange_ms_link_half"]
                                                                  for x in ranks),
                          "max_exchange_half_ms": ex, "mean_slice_ms": float(np.mean([x["slice_ms"] for x in ranks])),
                          "wall_s": time.time() - t_all}), flush=True)


if __name__ == "__main__":
    main()
