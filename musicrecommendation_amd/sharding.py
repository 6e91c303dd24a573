"""Multi-GPU layouts: one process per GPU (torch.distributed over RCCL).

Two partitions of the model's (test user, song) pairs, both exact:

* song-range shards (the north star; the reference's Spark "strategy 2",
  distributed.scala:477-479 ``parallelize(songs, 4)``): every rank holds the
  whole train CSR (stage 1 is replicated) and scores songs [lo, hi). Dense
  rows stay sharded by column; the per-test-user top-k lists are exchanged
  with ONE all-gather of (int64 key, int32 song) and merged by
  (key desc, song asc). Fixed-point keys make the merge order-independent,
  so the result is bit-identical for any shard count.
* test-user blocks (Spark "strategy 1", distributed.scala:468-470): each rank
  scores its own test users over all songs; no exchange at all. This is the
  bench's weak-scaling layout (each GPU scores a C2-sized block).

Shard boundaries balance the stage-2 work Σ_s (c_tr(s) + 1) — listener
entries streamed plus one output element per song — not song counts
(SURVEY.md §8e).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np

from .dataset import Dataset


def song_shards(ds: Dataset, n_shards: int) -> List[Tuple[int, int]]:
    """[lo, hi) song ranges with ~equal Σ (c_tr(s) + 1)."""
    if n_shards < 1:
        raise ValueError("n_shards must be >= 1")
    c_tr = np.bincount(ds.tr_songs, minlength=ds.n_songs).astype(np.int64)
    cost = np.cumsum(c_tr + 1)
    total = int(cost[-1])
    bounds = [0]
    for g in range(1, n_shards):
        b = int(np.searchsorted(cost, total * g / n_shards, side="left")) + 1
        bounds.append(min(max(b, bounds[-1] + 1), ds.n_songs - (n_shards - g)))
    bounds.append(ds.n_songs)
    return [(bounds[g], bounds[g + 1]) for g in range(n_shards)]


def user_blocks(n_test: int, n_blocks: int) -> List[Tuple[int, int]]:
    """Contiguous test-user blocks [lo, hi), sizes differing by at most one."""
    return [(n_test * b // n_blocks, n_test * (b + 1) // n_blocks) for b in range(n_blocks)]


def exchange_topk(songs, keys, group=None):
    """All-gather per-rank top-k lists (torch tensors [n_test, k], int32 songs,
    int64 keys, song ids global) and merge them by (key desc, song asc).

    CUDA tensors: RCCL all-gather over xGMI + the engine's merge kernel (the
    caller passes ``engine``-backed merge via ``merge_device``). CPU tensors
    (gloo): the same all-gather + the engine library's host merge. Returns
    merged (songs, keys) tensors on the input device.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n_te, k = songs.shape
    g_songs = torch.empty((world * n_te, k), dtype=songs.dtype, device=songs.device)
    g_keys = torch.empty((world * n_te, k), dtype=keys.dtype, device=keys.device)
    if songs.is_cuda and dist.get_backend(group) != "nccl":  # gloo rehearsal: gather on the host
        gs, gk = exchange_topk(songs.cpu(), keys.cpu(), group)
        return gs.to(songs.device), gk.to(keys.device)
    dist.all_gather_into_tensor(g_songs, songs.contiguous(), group=group)
    dist.all_gather_into_tensor(g_keys, keys.contiguous(), group=group)
    return g_songs.view(world, n_te, k), g_keys.view(world, n_te, k)


def merge_gathered_host(g_songs, g_keys):
    from .engine import merge_topk_host

    s, _sc, k = merge_topk_host(g_songs.cpu().numpy(), g_keys.cpu().numpy())
    return s, k


class SongShardScorer:
    """One rank of a song-sharded run: Engine on [lo, hi) + the top-k exchange."""

    def __init__(self, ds: Dataset, rank: int, world: int, device: int, *, topk: int = 10, dense: bool = True,
                 out_dtype: str = "f32", time_kernels: bool = False,
                 shards: Optional[List[Tuple[int, int]]] = None):
        import torch
        from .engine import Engine

        self.shards = shards or song_shards(ds, world)
        lo, hi = self.shards[rank]
        self.rank, self.world = rank, world
        self.engine = Engine(ds, device=device, song_lo=lo, song_hi=hi, topk=topk, dense=dense,
                             out_dtype=out_dtype, time_kernels=time_kernels)
        self.device = torch.device("cuda", device)
        n_te = ds.n_test
        self.local_songs = torch.empty((n_te, topk), dtype=torch.int32, device=self.device)
        self.local_keys = torch.empty((n_te, topk), dtype=torch.int64, device=self.device)
        self.out_songs = torch.empty((n_te, topk), dtype=torch.int32, device=self.device)
        self.out_keys = torch.empty((n_te, topk), dtype=torch.int64, device=self.device)
        self.out_scores = torch.empty((n_te, topk), dtype=torch.float64, device=self.device)

    def step(self, model: str) -> None:
        """Score the shard, then exchange + merge top-k (ends synchronised)."""
        import torch

        e = self.engine
        e.run(model)
        if self.world == 1:
            return
        # D2D copy of the engine's lists into torch-owned send buffers; the
        # engine call returns after its stream has drained.
        torch.cuda.current_stream(self.device).synchronize()
        e.copy_topk_device(self.local_songs.data_ptr(), self.local_keys.data_ptr())
        g_songs, g_keys = exchange_topk(self.local_songs, self.local_keys)
        torch.cuda.current_stream(self.device).synchronize()
        e.merge_topk_device(self.world, g_songs.data_ptr(), g_keys.data_ptr(), self.out_songs.data_ptr(),
                            self.out_keys.data_ptr(), self.out_scores.data_ptr())

    def topk(self):
        """Merged (songs, keys) as numpy arrays (after step)."""
        if self.world == 1:
            s, _sc, k = self.engine.topk()
            return s, k
        return self.out_songs.cpu().numpy(), self.out_keys.cpu().numpy()
