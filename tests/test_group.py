"""Multi-GPU behind the C ABI (mr_group_*, the reference's getItemBasedModel2 /
getUserBasedModel2 fan-out, distributed.scala:459-479).

CPU: the shard boundaries of the library (mr_song_shards, and
mr_song_shards_tiled: no shard past the fewest whole wide tiles) equal
sharding.song_shards (Σ(c_tr + 1) balance); creating a group without a GPU
fails with an error code (never a crash or a CPU fallback).
GPU (one MI355X): G = song shards x user blocks logical contexts on device 0
(COPY transport: device-copy exchange) give top-k lists, keys and dense models
bit-identical to one context, for ubm and ibm; the dense all-gather assembles
full rows on every context; a 1-context RCCL group runs the real
ncclCommInitAll / ncclAllGather / merge sequence; and the multi-context RCCL
path (G = 2x1, 3x1, 2x2 communicators, one all-gather of packed top-k record
blocks per context, the dense all-gather) runs on the one GPU through
tests/fake_rccl (MR_RCCL_LIB: RCCL's collective semantics with device copies;
real RCCL refuses two ranks on one device), bitwise against one context."""
import ctypes
import os

import numpy as np
import pytest

from musicrecommendation_amd import _lib, synth
from musicrecommendation_amd.group import Group, song_shards_native
from musicrecommendation_amd.sharding import shard_tile, song_shards

from helpers import kat, dataset_from_lines, synth_fixture

FAKE_RCCL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fake_rccl", "libfake_rccl.so")


def test_fake_rccl_library_exports():
    """The fake RCCL is built (by __graft_entry__.build) and exports what the
    group loads; a 1-rank all-gather outside a group completes on the host
    side of the API (no GPU work for zero bytes)."""
    L = ctypes.CDLL(FAKE_RCCL)
    for name in ("ncclCommInitAll", "ncclCommDestroy", "ncclAllGather", "ncclGroupStart", "ncclGroupEnd",
                 "ncclGetErrorString"):
        assert getattr(L, name)
    L.ncclGetErrorString.restype = ctypes.c_char_p
    assert b"fake" in L.ncclGetErrorString(5)
    comms = (ctypes.c_void_p * 2)()
    assert L.ncclCommInitAll(comms, 2, (ctypes.c_int * 2)(0, 0)) == 0
    assert L.ncclGroupEnd() == 5  # unbalanced group end: invalid usage
    for c in comms:
        assert L.ncclCommDestroy(ctypes.c_void_p(c)) == 0


def _datasets():
    K = kat()
    yield "kat", dataset_from_lines(K["train"], K["test"], K["labels"])
    yield "small", synth_fixture("small")[0]
    yield "c2x24", synth.config("c2", n_test=24).dataset()


def test_native_song_shards_equal_python_rule():
    for name, ds in _datasets():
        for n in range(1, min(9, ds.n_songs) + 1):
            assert song_shards_native(ds, n) == song_shards(ds, n), (name, n)


def test_tiled_song_shards():
    """mr_song_shards_tiled = sharding.song_shards(..., tile): no shard wider
    than ceil(ceil(n_songs / tile) / n) tiles, boundaries otherwise the
    balanced ones; tile 0 = the plain balance."""
    for name, ds in _datasets():
        for n in range(1, min(9, ds.n_songs) + 1):
            assert song_shards_native(ds, n, 0) == song_shards(ds, n), (name, n)
            for tile in (1, 3, 7, 64, 256, 1000):
                got = song_shards(ds, n, tile)
                assert song_shards_native(ds, n, tile) == got, (name, n, tile)
                assert got[0][0] == 0 and got[-1][1] == ds.n_songs
                assert all(hi > lo for lo, hi in got) and all(a[1] == b[0] for a, b in zip(got, got[1:]))
                tiles = -(-ds.n_songs // tile)
                cap = -(-tiles // n) * tile  # songs per shard at most
                assert max(hi - lo for lo, hi in got) <= cap, (name, n, tile)
                if tile >= ds.n_songs:  # one tile holds every shard: the balance is kept
                    assert got == song_shards(ds, n)


def test_shard_tile_follows_the_shape_rule():
    # C4-sized train set: wide, the widest tile the LDS holds (k = 10)
    assert shard_tile(1_009_318, 10_000) == 19_456
    assert shard_tile(1_009_318, 10_000, block_songs=8192) == 8192
    # C2 (500 x 10): fused, no wide tile; forced wide: the widest tile
    assert shard_tile(500, 10) == 0
    assert shard_tile(500, 10, stage1="wide") == 19_456
    # k > 16 never takes the wide shape
    assert shard_tile(1_009_318, 10_000, topk=17) == 0
    with pytest.raises(_lib.EngineError):
        shard_tile(10, 0)
    # song shards: the tile count rounded up to a multiple of the shard count
    # (C4 over 8 shards: 24 tiles of 16,128, 3 per shard; 2 and 4 shards keep 20)
    assert shard_tile(1_009_318, 10_000, n_songs=384_546, n_shards=8) == 16_128
    assert shard_tile(1_009_318, 10_000, n_songs=384_546, n_shards=2) == 19_456
    assert shard_tile(1_009_318, 10_000, n_songs=384_546, n_shards=4) == 19_456
    assert shard_tile(1_009_318, 10_000, n_songs=384_546, n_shards=8, block_songs=8192) == 8192


def test_group_without_gpu_fails_cleanly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    ds = synth_fixture("tiny")[0]
    with pytest.raises(_lib.EngineError) as e:
        Group(ds, song_shards=2)
    assert e.value.code in (_lib.MR_E_HIP, _lib.MR_E_INVALID)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", [(2, 1), (3, 1), (1, 2), (2, 2), (3, 2)])
def test_copy_group_equals_one_context(layout):
    from musicrecommendation_amd.engine import Engine

    gs, gu = layout
    for name, ds in _datasets():
        if ds.n_songs < gs or ds.n_test < gu:
            continue
        with Engine(ds, out_dtype="f64", topk=7) as e:
            ref = {}
            for model in ("ibm", "ubm"):
                e.run(model)
                ref[model] = (e.dense(), *e.topk())
        with Group(ds, song_shards=gs, user_blocks=gu, out_dtype="f64", topk=7) as g:
            assert g.transport == "copy" and len(g.layout) == gs * gu
            shards = song_shards(ds, gs, shard_tile(ds.n_train, ds.n_test // gu, topk=7, n_songs=ds.n_songs,
                                                    n_shards=gs))
            for i, (slo, shi, ulo, uhi, dev) in enumerate(g.layout):
                assert (slo, shi) == shards[i % gs] and dev == 0
            for model in ("ibm", "ubm"):
                g.run(model)
                songs, scores, keys = g.topk()
                d_ref, s_ref, sc_ref, k_ref = ref[model]
                assert np.array_equal(songs, s_ref), (name, layout, model)
                assert np.array_equal(keys, k_ref), (name, layout, model)
                assert np.array_equal(scores, sc_ref, equal_nan=True), (name, layout, model)
                assert np.array_equal(g.dense(), d_ref, equal_nan=True), (name, layout, model)


@pytest.mark.gpu
def test_copy_group_dense_allgather_and_repeated_runs():
    import torch

    ds = synth.config("c2", n_test=24).dataset()
    from musicrecommendation_amd.engine import Engine

    with Engine(ds, out_dtype="f32", topk=10) as e:
        e.run("ibm")
        d_ref = e.dense()
        s_ref = e.topk()[0]
    with Group(ds, song_shards=3, user_blocks=2, out_dtype="f32", topk=10) as g:
        for _ in range(3):  # back-to-back runs without host syncs in between
            g.run("ubm")
            g.run("ibm")
        g.sync()
        assert np.array_equal(g.topk()[0], s_ref)
        bufs = [torch.empty((uhi - ulo, ds.n_songs), dtype=torch.float32, device="cuda")
                for (_slo, _shi, ulo, uhi, _d) in g.layout]
        torch.cuda.synchronize()
        g.allgather_dense([b.data_ptr() for b in bufs])
        for (slo, shi, ulo, uhi, _d), b in zip(g.layout, bufs):
            assert np.array_equal(b.cpu().numpy(), d_ref[ulo:uhi], equal_nan=True)


@pytest.mark.gpu
@pytest.mark.parametrize("dense", [True, False])
def test_rccl_group_single_device(dense):
    """The RCCL transport end to end on one GPU: a 1-rank communicator, the
    all-gather of the lists (and of the dense shard), the merge kernel."""
    import torch
    from musicrecommendation_amd.engine import Engine

    ds = synth.config("c2", n_test=24).dataset()
    with Engine(ds, out_dtype="f32", topk=10, dense=dense) as e:
        e.run("ibm")
        s_ref, sc_ref, k_ref = e.topk()
        d_ref = e.dense() if dense else None
    with Group(ds, transport="rccl", out_dtype="f32", topk=10, dense=dense) as g:
        assert g.transport == "rccl"
        g.run("ibm")
        songs, scores, keys = g.topk()
        assert np.array_equal(songs, s_ref) and np.array_equal(keys, k_ref)
        if dense:
            assert np.array_equal(g.dense(), d_ref, equal_nan=True)
            b = torch.empty((ds.n_test, ds.n_songs), dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            g.allgather_dense([b.data_ptr()])
            assert np.array_equal(b.cpu().numpy(), d_ref, equal_nan=True)


@pytest.mark.gpu
def test_group_errors():
    ds = synth_fixture("tiny")[0]
    with pytest.raises(_lib.EngineError):
        Group(ds, song_shards=2, transport="rccl")  # two contexts, one device
    with pytest.raises(_lib.EngineError):
        Group(ds, song_shards=ds.n_songs + 1)
    with pytest.raises(_lib.EngineError):
        Group(ds, user_blocks=ds.n_test + 1)


@pytest.mark.gpu
def test_c3_song_sharded_group_equals_one_context():
    """C3 ("User+ItemBased 10k/1k, song-id sharded across 2 MI355X with RCCL
    all-gather"): the same 2-shard layout through the group (device-copy
    transport on the 1-GPU box), both models, top-10 and the dense model
    gathered on the device, bitwise against one context."""
    import torch
    from musicrecommendation_amd.engine import Engine

    ds = synth.config("c3").dataset()
    with Engine(ds, out_dtype="f32", topk=10) as e:
        ref = {}
        for model in ("ubm", "ibm"):
            e.run(model)
            ref[model] = (e.dense(), e.topk()[0], e.topk()[2])
    with Group(ds, song_shards=2, out_dtype="f32", topk=10) as g:
        assert [(lo, hi) for lo, hi, *_ in g.layout] == song_shards(
            ds, 2, shard_tile(ds.n_train, ds.n_test, n_songs=ds.n_songs, n_shards=2))
        for model in ("ubm", "ibm"):
            g.run(model)
            songs, _scores, keys = g.topk()
            d_ref, s_ref, k_ref = ref[model]
            assert np.array_equal(songs, s_ref) and np.array_equal(keys, k_ref), model
            bufs = [torch.empty((ds.n_test, ds.n_songs), dtype=torch.float32, device="cuda") for _ in range(2)]
            torch.cuda.synchronize()
            g.allgather_dense([b.data_ptr() for b in bufs])
            for b in bufs:
                assert np.array_equal(b.cpu().numpy(), d_ref, equal_nan=True), model
            del bufs


@pytest.mark.gpu
def test_shard_tile_matches_the_loaded_contexts():
    """mr_shard_tile_songs (host, before any load) is the tile the loaded
    contexts use: every tiled shard of C3 holds ceil(width / tile) tiles."""
    from musicrecommendation_amd.engine import Engine

    ds = synth.config("c3").dataset()
    tile = shard_tile(ds.n_train, ds.n_test)
    assert tile > 0
    for gs in (2, 3, 5):
        for lo, hi in song_shards(ds, gs, tile):
            with Engine(ds, topk=10, dense=False, song_lo=lo, song_hi=hi) as e:
                assert e.shape == "wide" and e.block_songs <= tile
                assert e.n_tiles == -(-(hi - lo) // tile), (gs, lo, hi)


@pytest.mark.gpu
def test_group_uneven_blocks_and_topk_only():
    from musicrecommendation_amd.engine import Engine

    ds = synth.config("c2", n_test=23).dataset()  # 23 users over 3 blocks: 7 / 8 / 8
    with Engine(ds, out_dtype="f64", topk=16, dense=False) as e:
        e.run("ubm")
        s_ref, _sc, k_ref = e.topk()
    with Group(ds, song_shards=2, user_blocks=3, out_dtype="f64", topk=16, dense=False) as g:
        assert [(ulo, uhi) for _slo, _shi, ulo, uhi, _d in g.layout[::2]] == [(0, 7), (7, 15), (15, 23)]
        g.run("ubm")
        s, _sc, k = g.topk()
        assert np.array_equal(s, s_ref) and np.array_equal(k, k_ref)
        with pytest.raises(_lib.EngineError):
            g.dense()  # dense=0


@pytest.mark.gpu
@pytest.mark.parametrize("layout", [(2, 1), (3, 1), (2, 2)])
@pytest.mark.parametrize("dense", [True, False])
def test_multi_context_rccl_path_equals_one_context(layout, dense, monkeypatch):
    """The RCCL transport with G_s > 1 communicators per block (one
    ncclAllGather of the packed record blocks per context inside
    ncclGroupStart/End, the merge on every context) through the fake RCCL on
    one GPU: lists, keys, scores, the dense model and the dense all-gather
    bitwise equal to one context, ubm and ibm, back-to-back runs."""
    import torch
    from musicrecommendation_amd.engine import Engine

    monkeypatch.setenv("MR_RCCL_LIB", FAKE_RCCL)
    gs, gu = layout
    ds = synth.config("c2", n_test=24).dataset()
    with Engine(ds, out_dtype="f32", topk=10, dense=dense) as e:
        ref = {}
        for model in ("ibm", "ubm"):
            e.run(model)
            ref[model] = (e.dense() if dense else None, *e.topk())
    with Group(ds, song_shards=gs, user_blocks=gu, transport="rccl", out_dtype="f32", topk=10, dense=dense) as g:
        assert g.transport == "rccl" and len(g.layout) == gs * gu
        for _ in range(2):
            for model in ("ibm", "ubm"):
                g.run(model)
                songs, scores, keys = g.topk()
                d_ref, s_ref, sc_ref, k_ref = ref[model]
                assert np.array_equal(songs, s_ref) and np.array_equal(keys, k_ref), (layout, model)
                assert np.array_equal(scores, sc_ref, equal_nan=True), (layout, model)
                for i in range(len(g.layout)):  # every context holds its block's merged lists
                    ps, pk, _psc = g.device_topk(i)
                    assert ps and pk
                if dense:
                    assert np.array_equal(g.dense(), d_ref, equal_nan=True), (layout, model)
                    bufs = [torch.empty((uhi - ulo, ds.n_songs), dtype=torch.float32, device="cuda")
                            for (_slo, _shi, ulo, uhi, _d) in g.layout]
                    torch.cuda.synchronize()
                    g.allgather_dense([b.data_ptr() for b in bufs])
                    for (_slo, _shi, ulo, uhi, _d), b in zip(g.layout, bufs):
                        assert np.array_equal(b.cpu().numpy(), d_ref[ulo:uhi], equal_nan=True), (layout, model)


@pytest.mark.gpu
def test_real_rccl_by_path_keeps_the_distinct_device_check(monkeypatch):
    """MR_RCCL_LIB naming the real librccl does not lift the 'one distinct
    device per context' rule: only a library exporting the test marker
    (tests/fake_rccl) may be handed two contexts on one GPU."""
    import os

    real = "/opt/rocm/lib/librccl.so.1"
    if not os.path.exists(real):
        pytest.skip("no librccl in this image")
    monkeypatch.setenv("MR_RCCL_LIB", real)
    ds = synth_fixture("tiny")[0]
    with pytest.raises(_lib.EngineError) as e:
        Group(ds, song_shards=2, transport="rccl")
    assert e.value.code == _lib.MR_E_INVALID


@pytest.mark.gpu
@pytest.mark.parametrize("layout", [(2, 1), (3, 1), (2, 2)])
@pytest.mark.parametrize("transport", ["copy", "rccl"])
def test_group_colistening_route_equals_one_context(layout, transport, monkeypatch):
    """The ItemBasedModel's co-listening route (mr_options.ibm_route = 2) in
    every context of a group — each shard's index over its own songs, each
    user block's over its own users' songs — merged lists and the dense model
    bitwise equal to one two-hop context (copy transport, and the RCCL
    transport through the fake RCCL on one GPU)."""
    from musicrecommendation_amd.engine import Engine

    if transport == "rccl":
        monkeypatch.setenv("MR_RCCL_LIB", FAKE_RCCL)
    gs, gu = layout
    ds = synth.generate_bulk(20_000, 24, 6).dataset()
    with Engine(ds, out_dtype="f64", topk=10, ibm_route="two_hop") as e:
        e.run("ibm")
        d_ref, (s_ref, _sc, k_ref) = e.dense(), e.topk()
    with Group(ds, song_shards=gs, user_blocks=gu, transport=transport, out_dtype="f64", topk=10,
               ibm_route="cooc") as g:
        for _ in range(2):
            g.run("ibm")
            songs, _scores, keys = g.topk()
            assert np.array_equal(songs, s_ref) and np.array_equal(keys, k_ref), (layout, transport)
            assert np.array_equal(g.dense(), d_ref, equal_nan=True), (layout, transport)


@pytest.mark.gpu
def test_group_load_validates_before_sharding():
    """mr_group_load runs mr_load's checks before it reads the dataset itself
    (the shard balance indexes by song id): out-of-range ids, unsorted rows and
    decreasing offsets are MR_E_INVALID, not heap writes."""
    ds = synth_fixture("tiny")[0]
    for mutate in ("song_range", "unsorted", "offsets"):
        bad = synth_fixture("tiny")[0]
        bad.tr_songs = bad.tr_songs.copy()
        bad.tr_off = bad.tr_off.copy()
        if mutate == "song_range":
            bad.tr_songs[3] = ds.n_songs + 7
        elif mutate == "unsorted":
            bad.tr_songs[[0, 1]] = bad.tr_songs[[1, 0]]
        else:
            bad.tr_off[2] = bad.tr_off[1] - 1
        with pytest.raises(_lib.EngineError) as e:
            Group(bad, song_shards=2)
        assert e.value.code == _lib.MR_E_INVALID, mutate


@pytest.mark.gpu
def test_group_reload():
    """A second mr_group_load replaces the layout's data (old contexts freed
    first) and the next run scores the new dataset."""
    from musicrecommendation_amd.engine import Engine

    a = synth.config("c2", n_test=12).dataset()
    b = synth_fixture("small")[0]
    with Group(a, song_shards=2, topk=10, dense=False) as g:
        g.run("ibm")
        cd = b.c_struct()
        _lib.check(g._L.mr_group_load(g._h, ctypes.byref(cd)), "mr_group_load")
        g.dataset = b
        g.run("ibm")
        songs, _sc, keys = g.topk()
    with Engine(b, topk=10, dense=False) as e:
        e.run("ibm")
        s_ref, _sc, k_ref = e.topk()
    assert np.array_equal(songs, s_ref) and np.array_equal(keys, k_ref)
