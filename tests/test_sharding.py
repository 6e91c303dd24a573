"""Multi-GPU layouts on the CPU (gloo, world size 2): shard geometry and the
song-shard exchange (all-gather of per-shard top-k + merge) give exactly the
unsharded result. Per-shard partials come from the fixed-point oracle here
(no GPU); on the GPU box the same exchange runs over RCCL on engine outputs
(tests/test_gpu_parity.py::test_song_shards_merge_identical, bench --shard songs)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from musicrecommendation_amd import synth
from musicrecommendation_amd.sharding import exchange_topk, merge_gathered_host, song_shards, user_blocks
from oracle import native


def test_song_shards_cover_and_balance():
    ds = synth.config("c2").dataset()
    for g in (1, 2, 3, 8):
        sh = song_shards(ds, g)
        assert sh[0][0] == 0 and sh[-1][1] == ds.n_songs
        assert all(a < b for a, b in sh) and all(sh[i][1] == sh[i + 1][0] for i in range(g - 1))
        c_tr = np.bincount(ds.tr_songs, minlength=ds.n_songs) + 1
        cost = [int(c_tr[a:b].sum()) for a, b in sh]
        assert max(cost) <= 1.1 * sum(cost) / g + int(c_tr.max())


def test_user_blocks_partition():
    assert user_blocks(10, 3) == [(0, 3), (3, 6), (6, 10)]
    assert user_blocks(8, 8) == [(i, i + 1) for i in range(8)]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, model, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ds = synth.config("small").dataset()
        lo, hi = song_shards(ds, world)[rank]
        _, s, k = native.fp_model(ds, model, song_lo=lo, song_hi=hi, k=10, dense=False)
        g_s, g_k = exchange_topk(torch.from_numpy(s), torch.from_numpy(k))
        ms, mk = merge_gathered_host(g_s, g_k)
        out[rank] = (ms.tolist(), mk.tolist())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model", ["ibm", "ubm"])
def test_gloo_world2_song_shard_exchange(model):
    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, _free_port(), model, out), nprocs=world, join=True)
        res = dict(out)
    ds = synth.config("small").dataset()
    _, ts, tk = native.fp_model(ds, model, k=10, dense=False)
    for r in range(world):
        assert np.array_equal(np.array(res[r][0]), ts)
        assert np.array_equal(np.array(res[r][1]), tk)
