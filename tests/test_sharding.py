"""Multi-GPU layouts on the CPU (gloo, world size 2): shard geometry and the
song-shard exchange (all-gather of per-shard top-k + merge) give exactly the
unsharded result. Per-shard partials come from the fixed-point oracle here
(no GPU); on the GPU box the same exchange runs over RCCL on engine outputs
(tests/test_gpu_parity.py::test_song_shards_merge_identical, bench --shard songs)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from musicrecommendation_amd import synth
from musicrecommendation_amd.sharding import exchange_topk, merge_gathered_host, song_shards, user_blocks
from oracle import native
from helpers import pg_init_method


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


def _worker(rank, world, init, model, out):
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
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
        mp.spawn(_worker, args=(world, pg_init_method(), model, out), nprocs=world, join=True)
        res = dict(out)
    ds = synth.config("small").dataset()
    _, ts, tk = native.fp_model(ds, model, k=10, dense=False)
    for r in range(world):
        assert np.array_equal(np.array(res[r][0]), ts)
        assert np.array_equal(np.array(res[r][1]), tk)


def test_layout_2d():
    from musicrecommendation_amd.sharding import layout_2d

    assert layout_2d(8) == (8, 1)
    assert layout_2d(8, 2) == (2, 4)
    assert layout_2d(4, 4) == (4, 1)
    with pytest.raises(ValueError):
        layout_2d(6, 4)


def _worker_2d(rank, world, init, song_groups, model, out):
    """A rank of the 2-D layout with the oracle standing in for the engine:
    its (user block, song shard) cell's top-k, the all-gather inside the
    block's process group, the merge."""
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        from musicrecommendation_amd.sharding import block_group, layout_2d

        ds = synth.config("small").dataset()
        gs, gu = layout_2d(world, song_groups)
        grp = block_group(rank, world, song_groups)
        a, b = user_blocks(ds.n_test, gu)[rank // gs]
        lo, hi = song_shards(ds, gs)[rank % gs]
        _, s, k = native.fp_model(ds, model, song_lo=lo, song_hi=hi, user_lo=a, user_hi=b, k=10, dense=False)
        g_s, g_k = exchange_topk(torch.from_numpy(s), torch.from_numpy(k), grp)
        assert g_s.shape[0] == gs
        ms, mk = merge_gathered_host(g_s, g_k)
        out[rank] = (a, b, ms.tolist(), mk.tolist())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,song_groups", [(2, 1), (2, 2), (4, 2), (4, 4)])
def test_gloo_2d_layout_exchange(world, song_groups):
    model = "ibm"
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker_2d, args=(world, pg_init_method(), song_groups, model, out), nprocs=world, join=True)
        res = dict(out)
    ds = synth.config("small").dataset()
    _, ts, tk = native.fp_model(ds, model, k=10, dense=False)
    covered = np.zeros(ds.n_test, bool)
    for r in range(world):
        a, b, s, k = res[r]
        assert np.array_equal(np.array(s), ts[a:b]) and np.array_equal(np.array(k), tk[a:b]), r
        covered[a:b] = True
    assert covered.all()


def _worker_shared(rank, world, init, out):
    """bench.shared_bulk_dataset: rank 0 builds the dataset once, the others
    load its arrays after a barrier; the node-local file is removed."""
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        import bench

        ds, _s = bench.shared_bulk_dataset("small", world, rank)
        out[rank] = {k: np.asarray(getattr(ds, k)).tolist() for k in ds._ARRAYS} | {
            "sizes": [ds.n_train, ds.n_test, ds.n_songs, ds.n_label_songs, ds.n_extra_songs]}
    finally:
        dist.destroy_process_group()


def test_gloo_world2_shared_bulk_dataset(tmp_path, monkeypatch):
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker_shared, args=(world, pg_init_method(), out), nprocs=world, join=True)
        res = dict(out)
    ds = synth.config("small").dataset()
    for r in range(world):
        assert res[r]["sizes"] == [ds.n_train, ds.n_test, ds.n_songs, ds.n_label_songs, ds.n_extra_songs]
        for k in ds._ARRAYS:
            assert np.array_equal(np.array(res[r][k]), np.asarray(getattr(ds, k))), (r, k)
    assert list(tmp_path.iterdir()) == []  # rank 0 removed the shared file


def test_usable_cores_shared_by_local_ranks(monkeypatch):
    """Host pools per rank: the usable cores divided by LOCAL_WORLD_SIZE
    (csrc/mr_par.h and its Python twin)."""
    from musicrecommendation_amd.mr_par_info import usable_cores

    monkeypatch.delenv("MR_THREADS", raising=False)
    monkeypatch.delenv("LOCAL_WORLD_SIZE", raising=False)
    full = usable_cores()
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert usable_cores() == max(1, full // 8)
    monkeypatch.setenv("MR_THREADS", "3")
    assert usable_cores() == 3


def test_usable_cores_pinned_rank_keeps_its_mask(monkeypatch):
    """A launcher that pinned each rank to its own CPU set (affinity mask
    smaller than the node's share) already split the cores: no further
    division by LOCAL_WORLD_SIZE."""
    import os

    from musicrecommendation_amd import mr_par_info

    monkeypatch.delenv("MR_THREADS", raising=False)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    monkeypatch.setattr(mr_par_info.os, "cpu_count", lambda: 64)
    monkeypatch.setattr(mr_par_info.os, "sched_getaffinity", lambda pid: set(range(4)))
    real_open = open

    def no_cgroup(path, *a, **k):
        if str(path) == "/sys/fs/cgroup/cpu.max":
            raise OSError("no cgroup")
        return real_open(path, *a, **k)

    monkeypatch.setattr("builtins.open", no_cgroup)
    assert mr_par_info.usable_cores() == 4  # pinned to 4 of 64: kept
    monkeypatch.setattr(mr_par_info.os, "sched_getaffinity", lambda pid: set(range(64)))
    assert mr_par_info.usable_cores() == 16  # the whole machine: split 4 ways
    assert os.cpu_count() is not None
