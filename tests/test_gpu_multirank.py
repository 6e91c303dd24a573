"""GPU, two ranks on one card (gloo process group; RCCL needs one GPU per
rank): the song-sharded layouts end to end with real engine contexts —
* top-k exchange (all-gather + merge) = the single-context lists;
* DeviceEnsemble: per-shard combinations = the full model's columns, and the
  threshold mAP after the MIN/MAX + SUM reductions = the single-context value."""

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from helpers import pg_init_method

pytestmark = pytest.mark.gpu


def _dataset():
    from musicrecommendation_amd import synth
    return synth.config("c2", n_test=16).dataset()


def _worker(rank, world, init, out):
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        from musicrecommendation_amd import evaluation
        from musicrecommendation_amd.engine import Engine
        from musicrecommendation_amd.ensemble import DeviceEnsemble
        from musicrecommendation_amd.sharding import exchange_topk, merge_gathered_host, song_shards

        ds = _dataset()
        lo, hi = song_shards(ds, world)[rank]
        res = {}
        with Engine(ds, out_dtype="f64", topk=10, song_lo=lo, song_hi=hi) as e:
            e.run("ibm")
            s, _sc, k = e.topk()
            g_s, g_k = exchange_topk(torch.from_numpy(s), torch.from_numpy(k))
            ms, mk = merge_gathered_host(g_s, g_k)
            res["topk"] = (ms.tolist(), mk.tolist())
            ens = DeviceEnsemble(e, pos=evaluation.label_pos(ds), n_label_songs=ds.n_label_songs)
            u, i = ens.model("ubm"), ens.model("ibm")
            for name, t in (("ibm", i), ("lcm", ens.linear(u, i, 0.5)), ("am", ens.aggregation(u, i, 0.5)),
                            ("scm", ens.stochastic(u, i, 0.5, seed=2))):
                res["map_" + name] = ens.threshold_map(t)
                res["cols_" + name] = (lo, hi, t.cpu().numpy().tolist())
        out[rank] = res
    finally:
        dist.destroy_process_group()


def test_two_ranks_song_shards_on_one_gpu():
    from musicrecommendation_amd.engine import Engine
    from musicrecommendation_amd.ensemble import DeviceEnsemble

    world = 2
    ctx = mp.get_context("spawn")
    with ctx.Manager() as m:
        out = m.dict()
        mp.start_processes(_worker, args=(world, pg_init_method(), out), nprocs=world, join=True, start_method="spawn")
        res = dict(out)
    ds = _dataset()
    with Engine(ds, out_dtype="f64", topk=10) as e:
        e.run("ibm")
        s, _sc, k = e.topk()
        ens = DeviceEnsemble(e)
        u, i = ens.model("ubm"), ens.model("ibm")
        full = {"ibm": i, "lcm": ens.linear(u, i, 0.5), "am": ens.aggregation(u, i, 0.5),
                "scm": ens.stochastic(u, i, 0.5, seed=2)}
        maps = {n: ens.threshold_map(t) for n, t in full.items()}
        dense = {n: t.cpu().numpy() for n, t in full.items()}
    for r in range(world):
        assert res[r]["topk"] == (s.tolist(), k.tolist())
        for n in full:
            assert res[r]["map_" + n] == maps[n], n
            lo, hi, cols = res[r]["cols_" + n]
            assert np.array_equal(np.array(cols), dense[n][:, lo:hi], equal_nan=True), n
