"""Multi-GPU layouts: one process per GPU (torch.distributed over RCCL).

Partitions of the model's (test user, song) pairs, all exact (the 2-D
ShardScorer combines the first two; include/mr_engine.h mr_group_* is the same
layout inside the C ABI for single-process callers):

* song-range shards (the north star; the reference's Spark "strategy 2",
  distributed.scala:477-479 ``parallelize(songs, 4)``): every rank holds the
  whole train CSR and scores songs [lo, hi). On the ItemBasedModel's
  co-listening route nothing is replicated: each rank builds
  the index columns of its own songs only (on the two-hop route, stage 1 —
  the neighbour weights — is recomputed by every shard of a user block). Dense
  rows stay sharded by column; the per-test-user top-k lists travel as one
  record block per rank (int64 keys, then int32 songs) exchanged with ONE
  all-gather and merged by (key desc, song asc). Fixed-point keys make the merge order-independent,
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


def song_shards(ds: Dataset, n_shards: int, tile: int = 0) -> List[Tuple[int, int]]:
    """[lo, hi) song ranges with ~equal Σ (c_tr(s) + 1). tile > 0: then every
    boundary moves the least so that no shard is wider than
    ceil(ceil(n_songs / tile) / n_shards) tiles (mr_song_shards_tiled; the
    wide kernel walks a test user's neighbour list once per tile, so a shard a
    few songs past whole tiles pays a whole extra tile)."""
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
    if tile > 0:
        n_s = ds.n_songs
        tiles = (n_s + tile - 1) // tile
        cap = (tiles + n_shards - 1) // n_shards * tile  # songs per shard at most
        for g in range(1, n_shards):
            x = max(bounds[g], n_s - (n_shards - g) * cap)
            x = min(x, bounds[g - 1] + cap)
            x = max(x, bounds[g - 1] + 1)
            bounds[g] = min(x, n_s - (n_shards - g))
    return [(bounds[g], bounds[g + 1]) for g in range(n_shards)]


def shard_tile(n_train: int, n_test: int, *, topk: int = 10, stage1: str = "auto", block_songs: int = 0,
               stage1_chunk: int = 0, n_songs: int = 0, n_shards: int = 1) -> int:
    """The wide shape's song tile for a context scoring n_test x n_train users
    with these options (mr_shard_tile_songs), 0 when it would use another shape;
    with n_songs and n_shards > 1, narrowed so the shards hold equal whole
    numbers of tiles (mr_shard_tile_songs_n)."""
    import ctypes

    from . import _lib

    L = _lib.lib()
    opt = _lib.MrOptions()
    _lib.check(L.mr_options_default(ctypes.byref(opt)), "mr_options_default")
    opt.topk = topk
    opt.block_songs = block_songs
    opt.stage1 = _lib.STAGE1[stage1]
    opt.stage1_chunk = stage1_chunk
    out = ctypes.c_int32()
    if n_songs > 0 and n_shards > 1:
        _lib.check(L.mr_shard_tile_songs_n(ctypes.byref(opt), int(n_train), int(n_test), int(n_songs), int(n_shards),
                                           ctypes.byref(out)), "mr_shard_tile_songs_n")
    else:
        _lib.check(L.mr_shard_tile_songs(ctypes.byref(opt), int(n_train), int(n_test), ctypes.byref(out)),
                   "mr_shard_tile_songs")
    return out.value


def user_blocks(n_test: int, n_blocks: int) -> List[Tuple[int, int]]:
    """Contiguous test-user blocks [lo, hi), sizes differing by at most one."""
    return [(n_test * b // n_blocks, n_test * (b + 1) // n_blocks) for b in range(n_blocks)]


def pack_records(songs, keys):
    """One rank's lists as a record block (torch uint8): n int64 keys, then n
    int32 songs, padded to 16 B — the layout of mr_topk_record_bytes."""
    import torch

    n = songs.numel()
    rec = -(-12 * n // 16) * 16
    out = torch.zeros(rec, dtype=torch.uint8, device=songs.device)
    out[:8 * n] = keys.contiguous().reshape(-1).view(torch.uint8)
    out[8 * n:12 * n] = songs.contiguous().reshape(-1).view(torch.uint8)
    return out


def unpack_records(g_rec, world: int, n_te: int, k: int):
    """[world][rec] gathered blocks -> (songs [world, n_te, k], keys [world, n_te, k])."""
    import torch

    n = n_te * k
    blocks = g_rec.view(world, -1)
    keys = blocks[:, :8 * n].contiguous().view(torch.int64).view(world, n_te, k)
    songs = blocks[:, 8 * n:12 * n].contiguous().view(torch.int32).view(world, n_te, k)
    return songs, keys


def exchange_topk(songs, keys, group=None):
    """All-gather per-rank top-k lists (torch tensors [n_test, k], int32 songs,
    int64 keys, song ids global) as ONE collective over packed record blocks
    (pack_records); returns the gathered (songs, keys), each
    [world, n_test, k], on the input device, ready for a merge by (key desc,
    song asc) (merge_gathered_host, or the engine's record merge on a GPU).
    CUDA tensors under a gloo group are gathered on the host (rehearsals)."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n_te, k = songs.shape
    if songs.is_cuda and dist.get_backend(group) != "nccl":  # gloo rehearsal: gather on the host
        gs, gk = exchange_topk(songs.cpu(), keys.cpu(), group)
        return gs.to(songs.device), gk.to(keys.device)
    rec = pack_records(songs, keys)
    import torch

    g_rec = torch.empty(world * rec.numel(), dtype=torch.uint8, device=rec.device)
    dist.all_gather_into_tensor(g_rec, rec, group=group)
    return unpack_records(g_rec, world, n_te, k)


def merge_gathered_host(g_songs, g_keys):
    from .engine import merge_topk_host

    s, _sc, k = merge_topk_host(g_songs.cpu().numpy(), g_keys.cpu().numpy())
    return s, k


def layout_2d(world: int, song_groups: Optional[int] = None) -> Tuple[int, int]:
    """(G_s, G_u): song shards per user block and user blocks, G_s * G_u = world.
    Rank r holds user block r // G_s and song shard r % G_s. song_groups=None:
    all ranks shard songs (G_u = 1, the north star's layout)."""
    gs = world if song_groups is None else int(song_groups)
    if gs < 1 or world % gs:
        raise ValueError(f"song_groups={gs} does not divide world={world}")
    return gs, world // gs


def block_group(rank: int, world: int, song_groups: Optional[int] = None):
    """The process group of the ranks sharing this rank's user block (the
    all-gather of the exchange runs inside it). Every rank creates every
    block's group (torch.distributed.new_group is collective). None = the
    default group (one block)."""
    import torch.distributed as dist

    gs, gu = layout_2d(world, song_groups)
    if gu == 1:
        return None
    mine = None
    for b in range(gu):
        g = dist.new_group(list(range(b * gs, (b + 1) * gs)))
        if b == rank // gs:
            mine = g
    return mine


class ShardScorer:
    """One rank of a 2-D layout: test-user block b of G_u
    (contiguous, sizes within one) x song-range shard g of G_s (Σ(c_tr + 1)
    balanced). The ranks of a block exchange their per-user top-k lists with
    ONE all-gather over RCCL (inside the block's process group) and merge them
    on the device. G_u = 1 is the north star's song-shard layout (Spark strategy
    2, distributed.scala:477-479), G_s = 1 the test-user blocks of strategy 1
    (:468-470, no exchange); in between, stage 1 (replicated over the song
    shards of a block) is split G_u ways.

    No host synchronisation inside a step: the engine stream (run, list copy,
    merge) and torch's stream (the all-gather) are ordered with events."""

    def __init__(self, ds: Dataset, rank: int, world: int, device: int, *, song_groups: Optional[int] = None,
                 topk: int = 10, dense: bool = True, out_dtype: str = "f32", time_kernels: bool = False,
                 stage1: str = "auto", block_songs: int = 0, ibm_route: str = "auto"):
        import torch
        from .engine import Engine

        self.gs, self.gu = layout_2d(world, song_groups)
        self.rank, self.world = rank, world
        self.block, self.shard = rank // self.gs, rank % self.gs
        self.user_lo, self.user_hi = user_blocks(ds.n_test, self.gu)[self.block]
        tile = shard_tile(ds.n_train, ds.n_test // self.gu, topk=topk, stage1=stage1, block_songs=block_songs,
                          n_songs=ds.n_songs, n_shards=self.gs)
        self.song_lo, self.song_hi = song_shards(ds, self.gs, tile)[self.shard]
        self.full = ds
        self.ds = ds if self.gu == 1 else ds.subset_test_users(self.user_lo, self.user_hi)
        self.group = block_group(rank, world, self.gs) if world > 1 else None
        self.engine = Engine(self.ds, device=device, song_lo=self.song_lo, song_hi=self.song_hi, topk=topk,
                             dense=dense, out_dtype=out_dtype, time_kernels=time_kernels, stage1=stage1,
                             block_songs=block_songs, ibm_route=ibm_route)
        self.device = torch.device("cuda", device)
        n_te = self.ds.n_test
        # the exchange: this rank's lists as ONE record block (keys, then songs),
        # all-gathered in one collective into [G_s][rec] and merged on the device
        self.rec_bytes = self.engine.record_bytes()
        self.local_rec = torch.empty(self.rec_bytes // 8, dtype=torch.int64, device=self.device)
        self.g_rec = torch.empty(self.gs * (self.rec_bytes // 8), dtype=torch.int64, device=self.device)
        self.out_songs = torch.empty((n_te, topk), dtype=torch.int32, device=self.device)
        self.out_keys = torch.empty((n_te, topk), dtype=torch.int64, device=self.device)
        self.out_scores = torch.empty((n_te, topk), dtype=torch.float64, device=self.device)
        self._ext = torch.cuda.ExternalStream(self.engine.stream, device=self.device)
        # one song shard has nothing to exchange; True runs the all-gather +
        # merge anyway (a one-rank rehearsal of the N > 1 collective path)
        self.exchange_always = False

    @property
    def exchanges(self) -> bool:
        return self.gs > 1 or self.exchange_always

    def pairs(self) -> int:
        """Scored pairs of this rank: its users x its songs, minus the heard ones."""
        te_off, te_songs = self.ds.te_off, self.ds.te_songs
        heard = int(((te_songs >= self.song_lo) & (te_songs < self.song_hi)).sum())
        return self.ds.n_test * (self.song_hi - self.song_lo) - heard

    def step(self, model: str) -> None:
        """Score the (block, shard) cell, then exchange + merge the block's top-k
        lists. Asynchronous: returns with the work queued on the streams."""
        self.engine.run(model)
        if self.exchanges:
            self.exchange()

    def exchange(self) -> None:
        """The exchange step alone (after a run): this rank's record block
        copied out, ONE all-gather inside the block's group, the merge on the
        device. Asynchronous; the engine stream and torch's stream are ordered
        with events."""
        import torch
        import torch.distributed as dist

        e = self.engine
        e.copy_topk_record(self.local_rec.data_ptr())
        cur = torch.cuda.current_stream(self.device)
        cur.wait_stream(self._ext)  # lists copied before the all-gather reads them
        if dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(self.g_rec, self.local_rec, group=self.group)
        else:  # gloo rehearsal with CUDA tensors: gather on the host
            parts = [torch.empty_like(self.local_rec, device="cpu") for _ in range(self.gs)]
            dist.all_gather(parts, self.local_rec.cpu(), group=self.group)
            self.g_rec.copy_(torch.cat(parts))
        self._ext.wait_stream(cur)  # the merge reads the gathered blocks
        e.merge_topk_records(self.gs, self.g_rec.data_ptr(), self.rec_bytes, self.out_songs.data_ptr(),
                             self.out_keys.data_ptr(), self.out_scores.data_ptr())

    def sync(self) -> None:
        import torch

        self.engine.sync()
        torch.cuda.current_stream(self.device).synchronize()

    def topk(self):
        """Merged (songs, keys) of this rank's user block, numpy (after step)."""
        self.sync()
        if not self.exchanges:
            s, _sc, k = self.engine.topk()
            return s, k
        return self.out_songs.cpu().numpy(), self.out_keys.cpu().numpy()


class SongShardScorer(ShardScorer):
    """The north star's layout: every rank a song shard of all test users."""

    def __init__(self, ds: Dataset, rank: int, world: int, device: int, **kw):
        super().__init__(ds, rank, world, device, song_groups=world, **kw)


class EnsembleScorer:
    """Config C5 over N ranks (one process per GPU), each similarity model in
    the layout that splits it without replicated work:

    * ubm by test-user blocks (Spark strategy 1, distributed.scala:450-452):
      its two-hop walk (MR:140-166) is per test user, so a block's neighbour
      lists and stage-2 walks are 1/N of the job — over song shards every
      shard would rebuild the lists and re-walk them per tile;
    * ibm by song shards (strategy 2, distributed.scala:477-479): on the
      co-listening route (MR:230-257) the index columns split with the songs —
      over user blocks every block would rebuild the popular rows.

    The combinations (main.scala:57-89, MR:317-481) pair the two models
    element by element, so before them ONE all-to-all moves the ibm shard's
    rows into the user-block layout: rank r's [n_test x w_r] shard is already
    block-major (block b = rows [a_b, b_b), contiguous), rank b receives the
    [n_b x w_r] pieces of every shard and places them at columns [lo_r, hi_r).
    Then the combinations and the five threshold mAPs run on the user block
    (DeviceEnsemble.threshold_maps: one MAX and one SUM all-reduce in all).
    Every pair is scored by the same kernels as on one context: the models,
    the combinations and the mAPs are bit-identical for any N (tested).
    N = 1: one context scores both models (the single-GPU pipeline)."""

    def __init__(self, full: Dataset, rank: int, world: int, device: int, *, out_dtype: str = "f32",
                 topk: int = 10, ibm_route: str = "auto", group=None, collectives: Optional[bool] = None,
                 engine_factory=None):
        from . import evaluation
        from .engine import Engine
        from .ensemble import DeviceEnsemble

        make = engine_factory or Engine  # (tests: host stand-ins of the contexts)

        self.full, self.rank, self.world, self.group = full, rank, world, group
        self.blocks = user_blocks(full.n_test, world)
        self.user_lo, self.user_hi = self.blocks[rank]
        tile = shard_tile(full.n_train, full.n_test, topk=topk, n_songs=full.n_songs, n_shards=world)
        self.shards = song_shards(full, world, tile)
        self.song_lo, self.song_hi = self.shards[rank]
        pos = evaluation.label_pos(full)
        a = self.user_lo
        self.ds_u = full if world == 1 else full.subset_test_users(self.user_lo, self.user_hi)
        # the block's context scores ubm over all songs (no co-listening pool:
        # its ibm is never run when N > 1)
        self.eng_u = make(self.ds_u, device=device, out_dtype=out_dtype, topk=topk,
                          ibm_route=ibm_route if world == 1 else "two_hop")
        self.eng_i = self.eng_u if world == 1 else make(full, device=device, out_dtype=out_dtype, topk=topk,
                                                         song_lo=self.song_lo, song_hi=self.song_hi,
                                                         ibm_route=ibm_route)
        kw = dict(n_pairs=full.n_pairs(), pos=pos, n_label_songs=full.n_label_songs, group=group,
                  collectives=collectives)
        self.ens = DeviceEnsemble(self.eng_u, pair_base=a * full.n_songs - int(full.te_off[a]), **kw)
        self.ens_i = self.ens if world == 1 else DeviceEnsemble(self.eng_i, **kw)
        nb = [b - a for a, b in self.blocks]
        w = [hi - lo for lo, hi in self.shards]
        self.send_splits = [n * w[rank] for n in nb]          # my shard's rows of block b
        self.recv_splits = [nb[rank] * x for x in w]          # shard r's rows of my block
        self.exchange_bytes = sum(s for i, s in enumerate(self.send_splits) if i != rank) * \
            (8 if out_dtype == "f64" else 4)

    @property
    def ibm_route(self) -> str:
        return self.eng_i.ibm_route

    def ibm_to_blocks(self, ibm_shard):
        """The all-to-all: this rank's ibm columns of every block out, its own
        block's columns of every shard in, placed at their songs."""
        import torch
        import torch.distributed as dist

        if self.world == 1:
            return ibm_shard
        mn_mx = getattr(ibm_shard, "_mr_minmax", None)
        send = ibm_shard.reshape(-1)
        recv = torch.empty(sum(self.recv_splits), dtype=ibm_shard.dtype, device=ibm_shard.device)
        if send.is_cuda and dist.get_backend(self.group) != "nccl":  # gloo rehearsal: through the host
            r = recv.cpu()
            dist.all_to_all_single(r, send.cpu(), self.recv_splits, self.send_splits, group=self.group)
            recv.copy_(r)
        else:
            dist.all_to_all_single(recv, send, self.recv_splits, self.send_splits, group=self.group)
        out = self.ens.empty()
        off = 0
        n_b = self.user_hi - self.user_lo
        for (lo, hi), n in zip(self.shards, self.recv_splits):
            out[:, lo:hi].copy_(recv[off:off + n].view(n_b, hi - lo))
            off += n
        if mn_mx is not None:
            # the shard's extremes: shards and blocks both partition the model,
            # so the MIN / MAX all-reduce of threshold_maps gives its extremes
            out._mr_minmax = (out._version, mn_mx[1], mn_mx[2])
        return out

    def step(self, alpha: float = 0.5, ibm_percentage: float = 0.5, ibm_probability: float = 0.5,
             seed: int = 1, n_thresholds: int = 10):
        """One C5 pass: ibm on the song shard, its all-to-all, ubm on the user
        block, the three combinations and the five mAPs. Returns ({name: this
        rank's block of the model}, {name: mAP})."""
        if self.world == 1:
            ubm, ibm = self.ens.model("ubm"), self.ens.model("ibm")
        else:
            # ubm queued first on the block context's stream; the ibm shard on
            # the shard context's stream and its all-to-all on torch's stream
            # run beside the ubm walk
            ubm = self.ens.empty()
            self.ens._after_torch()
            self.eng_u.run_into("ubm", ubm.data_ptr())
            ibm_s = self.ens_i.model("ibm")
            ibm = self.ibm_to_blocks(ibm_s)
            del ibm_s
            self.eng_u.sync()
            mm = self.eng_u.dense_minmax()
            if mm is not None:
                ubm._mr_minmax = (ubm._version, mm[0], mm[1])
        lcm, am, scm = self.ens.combinations(ubm, ibm, alpha, ibm_percentage, ibm_probability, seed=seed)
        models = {"ubm": ubm, "ibm": ibm, "lcm": lcm, "am": am, "scm": scm}
        return models, self.ens.threshold_maps(models, n_thresholds)

    def close(self) -> None:
        if self.eng_i is not self.eng_u:
            self.eng_i.close()
        self.eng_u.close()
