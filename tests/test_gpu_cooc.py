"""GPU parity of the ItemBasedModel's co-listening route (mr_options.ibm_route = 2).

The route counts C[s2][s] = |L_tr(s2) ∩ L_tr(s)| (the distinct-user numerator
of MusicRecommender.scala:232-235) for every test-visible song s2 at the start
of each ibm run, then scores rank(u, s) = (1/sqrt c(s)) Σ_{s2 ∈ T(u)} q(s2)·C[s2][s]
(MR:249-257 in the engine's fixed point). That is the same integer sum as the
two-hop route's Σ_{v: s ∈ S(v)} Σ_{s2 ∈ T(u) ∩ S(v)} q(s2), so the bar is
bit-identity with the fixed-point oracle (oracle/fixedpoint.c) and with the
two-hop route, on every tile width, shard, k and launch.
"""
import ctypes
import os

import numpy as np
import pytest

from musicrecommendation_amd import _lib, synth
from musicrecommendation_amd.engine import Engine, merge_topk_host
from musicrecommendation_amd.sharding import song_shards
from oracle import native

from helpers import synth_fixture

pytestmark = pytest.mark.gpu


def run_route(ds, route, *, k=10, dense=True, **kw):
    with Engine(ds, out_dtype="f64", topk=k, dense=dense, stage1=kw.pop("stage1", "wide"), ibm_route=route,
                **kw) as e:
        assert e.ibm_route == ("cooc" if route == "cooc" else "two_hop")
        e.run("ibm")
        d = e.dense() if dense else None
        songs, _, keys = e.topk()
        return d, songs, keys, (e.song_lo, e.song_hi)


def check_route_exact(ds, *, k=10, **kw):
    d, songs, keys, (lo, hi) = run_route(ds, "cooc", k=k, **kw)
    exp, ts, tk = native.fp_model(ds, "ibm", song_lo=lo, song_hi=hi, k=k)
    assert np.array_equal(d, exp, equal_nan=True), "co-listening dense scores differ from the oracle"
    assert np.array_equal(songs, ts) and np.array_equal(keys, tk), "co-listening top-k differs from the oracle"
    return d, songs, keys


# Index build paths (engine environment read at mr_load): light rows by the
# LDS hash (default) or every row per (row, tile) (MR_COOC_LIGHT=0); tile
# segments dense when a third of the songs are non-zero (default), always
# (MR_COOC_DENSE_DIV=1000000) or never (0); MR_COOC_DENSE32=1 puts every heavy
# row on the u32-counter kernel (saturated u16 words + excess entries, the
# format of rows with >= 65536 listeners), MR_COOC_SAT lowers the saturation.
BUILD_PATHS = {
    "light": {},
    "tiled": {"MR_COOC_LIGHT": "0"},
    "sparse": {"MR_COOC_LIGHT": "0", "MR_COOC_DENSE_DIV": "0"},
    "dense16": {"MR_COOC_LIGHT": "0", "MR_COOC_DENSE_DIV": "1000000"},
    "dense32": {"MR_COOC_LIGHT": "0", "MR_COOC_DENSE_DIV": "1000000", "MR_COOC_DENSE32": "1"},
    # every heavy row on the u32-counter kernel, dense counts saturated at 2:
    # the excess entries after the u16 words (the format of >= 65536-listener rows)
    "dense_tail": {"MR_COOC_LIGHT": "0", "MR_COOC_DENSE_DIV": "1000000", "MR_COOC_DENSE32": "1",
                   "MR_COOC_SAT": "2"},
    "mixed_tail": {"MR_COOC_LIGHT": "0", "MR_COOC_DENSE32": "1", "MR_COOC_SAT": "3"},
    # heavy u16 rows per tile (k_cooc_build<512, true>) instead of by tile
    # groups (k_cooc_group, the default whenever the per-user records fit)
    "pertile": {"MR_COOC_LIGHT": "0", "MR_COOC_GROUP": "0"},
    "pertile_dense16": {"MR_COOC_LIGHT": "0", "MR_COOC_GROUP": "0", "MR_COOC_DENSE_DIV": "1000000"},
    # k_cooc_group with 512-thread workgroups and 2-tile groups: more groups per
    # row, and rows over 2048 listeners back on the per-group rows_walk (the
    # pipelined walk holds <= 4 listeners per lane group)
    "group512": {"MR_COOC_LIGHT": "0", "MR_COOC_GNT": "512", "MR_COOC_GRP": "2"},
}
COOC_ENV = ("MR_COOC_LIGHT", "MR_COOC_DENSE_DIV", "MR_COOC_DENSE32", "MR_COOC_SAT", "MR_COOC_GROUP",
            "MR_COOC_GNT", "MR_COOC_GRP")


@pytest.fixture(params=list(BUILD_PATHS))
def build_path(request, monkeypatch):
    for key in COOC_ENV:
        monkeypatch.delenv(key, raising=False)
    for key, val in BUILD_PATHS[request.param].items():
        monkeypatch.setenv(key, val)
    return request.param


@pytest.mark.parametrize("k", [1, 7, 10, 16])
@pytest.mark.parametrize("block", [256, 2048, 16384])
def test_fixtures_and_c2_exact(block, k, build_path):
    for ds in (synth_fixture("tiny")[0], synth_fixture("small")[0], synth.config("c2", n_test=13).dataset()):
        check_route_exact(ds, k=k, block_songs=block)


def test_routes_identical_and_auto(build_path):
    """Both routes bitwise equal to each other and to the oracle; auto picks
    one of them by its cost model (the choice never changes results)."""
    ds = synth.generate_bulk(40_000, 21, 4).dataset()
    with Engine(ds, out_dtype="f64", topk=10) as e:
        assert e.shape == "wide" and e.ibm_route in ("cooc", "two_hop")
    with Engine(ds, out_dtype="f64", topk=10, ibm_route="cooc") as e:
        assert e.cooc_rows > 0 and e.cooc_pool_entries > 0
    a = run_route(ds, "cooc")
    b = run_route(ds, "two_hop")
    assert np.array_equal(a[0], b[0], equal_nan=True)
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    exp, ts, tk = native.fp_model(ds, "ibm", k=10)
    assert np.array_equal(a[0], exp, equal_nan=True)
    assert np.array_equal(a[1], ts) and np.array_equal(a[2], tk)
    # ubm keeps the two-hop path in the same context
    with Engine(ds, out_dtype="f64", topk=10) as e:
        e.run("ubm")
        got = e.dense()
    assert np.array_equal(got, native.fp_model(ds, "ubm", k=10)[0], equal_nan=True)


@pytest.mark.parametrize("n_shards", [2, 3])
def test_song_shards(n_shards, build_path):
    """Per-shard index (rows over all test-visible songs, columns = the shard):
    merged lists identical to one context and to the oracle."""
    ds = synth.generate_bulk(40_000, 21, 4).dataset()
    _, ts, tk = native.fp_model(ds, "ibm", k=10)
    ss, kk = [], []
    for lo, hi in song_shards(ds, n_shards):
        d, s, k, _ = run_route(ds, "cooc", song_lo=lo, song_hi=hi)
        exp = native.fp_model(ds, "ibm", song_lo=lo, song_hi=hi, k=10)[0]
        assert np.array_equal(d, exp, equal_nan=True)
        ss.append(s)
        kk.append(k)
    ms, _, mk = merge_topk_host(np.stack(ss), np.stack(kk))
    assert np.array_equal(ms, ts) and np.array_equal(mk, tk)


def test_topk_only_graph_and_repeats():
    """dense = 0, f32, repeated runs and a captured graph of several steps
    (the per-run index rebuild, its row cursors reset inside the graph)."""
    ds = synth.generate_bulk(20_000, 64, 7).dataset()
    _, ts, tk = native.fp_model(ds, "ibm", k=10, dense=False)
    with Engine(ds, topk=10, dense=False, ibm_route="cooc") as e:
        for _ in range(3):
            e.run("ibm")
            s, _, k = e.topk()
            assert np.array_equal(s, ts) and np.array_equal(k, tk)
        e.graph_capture("ibm", 4)
        e.graph_launch()
        e.sync()
        s, _, k = e.topk()
        assert np.array_equal(s, ts) and np.array_equal(k, tk)
        # interleaved ubm run, then ibm again
        e.run("ubm")
        e.run("ibm")
        s, _, k = e.topk()
        assert np.array_equal(s, ts) and np.array_equal(k, tk)


def cold_heavy_dataset():
    """Test users whose songs have no train listener (empty rows), a test user
    with hundreds of songs (several descriptor passes), and one-song users."""
    rng = np.random.default_rng(11)
    base = synth.generate_bulk(20_000, 30, 9)
    heard = np.unique(base.train_s)
    K = 10 ** 9  # test-user keys past every generated user
    # user K: 900 distinct train-heard songs; K+1: one song no train user heard; K+2: the most popular song
    heavy = rng.choice(heard, 900, replace=False)
    cold = np.array([synth.N_SONG_UNIVERSE + 5])
    pop = np.array([np.bincount(base.train_s).argmax()])
    te_u = np.concatenate([np.full(heavy.size, K), [K + 1], [K + 2], base.test_u])
    te_s = np.concatenate([heavy, cold, pop, base.test_s])
    t = synth.Triplets(base.train_u, base.train_s, te_u, te_s, base.label_u[:0], base.label_s[:0], base.alpha)
    return t.dataset()


def test_cold_and_heavy_users(build_path):
    ds = cold_heavy_dataset()
    check_route_exact(ds, k=10)
    check_route_exact(ds, k=16, block_songs=4096)


@pytest.mark.parametrize("counters", ["u16_groups", "u16_pertile", "u32"])
def test_dense_excess_on_every_tile(counters, monkeypatch):
    """Regression test of the dc4df36 race (k_cooc_build's dense branch: a
    shared LDS word reset while other waves still read it). Every heavy row is
    built by k_cooc_build (no light rows), every tile segment is dense
    (MR_COOC_DENSE_DIV=1000000) and every count above 1 spills into the excess
    tail (MR_COOC_SAT=1), so the excess counter and the non-zero counter are
    both live on every tile of every row; the u16-pair counters by tile groups
    (k_cooc_group) and per tile, and the u32 counter kernel."""
    for key in COOC_ENV:
        monkeypatch.delenv(key, raising=False)
    monkeypatch.setenv("MR_COOC_LIGHT", "0")
    if counters == "u16_pertile":
        monkeypatch.setenv("MR_COOC_GROUP", "0")
    monkeypatch.setenv("MR_COOC_DENSE_DIV", "1000000")
    monkeypatch.setenv("MR_COOC_SAT", "1")
    if counters == "u32":
        monkeypatch.setenv("MR_COOC_DENSE32", "1")
    ds = cold_heavy_dataset()
    check_route_exact(ds, k=10)
    check_route_exact(ds, k=16, block_songs=4096)


def test_route_errors():
    """ibm_route 2 outside the wide shape is refused with a code; 3 is invalid."""
    ds, _ = synth_fixture("small")
    with pytest.raises(_lib.EngineError):
        Engine(ds, stage1="fused", ibm_route="cooc")
    with pytest.raises(_lib.EngineError):
        Engine(ds, stage1="separate", ibm_route="cooc")
    with Engine(ds, stage1="fused") as e:  # auto on another shape: two-hop
        assert e.ibm_route == "two_hop"
    o = _lib.MrOptions()
    _lib.check(_lib.lib().mr_options_default(ctypes.byref(o)), "defaults")
    o.ibm_route = 3
    h = ctypes.c_void_p()
    assert _lib.lib().mr_create(ctypes.byref(o), ctypes.byref(h)) == _lib.MR_E_INVALID


def test_cooc_stats_count_the_index(build_path):
    """mr_cooc_stats: the index's non-zeros, the entries the scoring reads and
    the build's reads, against a scipy count (bench.py's byte model uses them)."""
    import scipy.sparse as sp

    ds = synth.generate_bulk(20_000, 40, 3).dataset()
    with Engine(ds, topk=10, dense=False, ibm_route="cooc") as e:
        with pytest.raises(_lib.EngineError):
            e.cooc_stats()  # no ibm run yet
        e.run("ibm")
        e.run("ubm")  # the counts stay those of the latest ibm run
        index_nnz, consumed, reads = e.cooc_stats()
        cb = e.cooc_bytes()
        bs, n_tiles = e.block_songs, e.n_tiles
    tr_rows = np.repeat(np.arange(ds.n_train), np.diff(ds.tr_off))
    A = sp.csr_matrix((np.ones(tr_rows.size, np.int64), (tr_rows, ds.tr_songs)), shape=(ds.n_train, ds.n_songs))
    c_tr = np.asarray(A.sum(axis=0)).ravel()
    rows = np.unique(ds.te_songs)
    rows = rows[c_tr[rows] > 0]
    C = (A[:, rows].T @ A).tocsr()
    nnz_r = np.diff(C.indptr)
    users_r = np.bincount(np.searchsorted(rows, ds.te_songs[np.isin(ds.te_songs, rows)]), minlength=rows.size)
    deg = np.diff(ds.tr_off)
    assert index_nnz == int(nnz_r.sum())
    assert consumed == int((nnz_r * users_r).sum())
    assert reads == int(c_tr[rows].sum() + (A[:, rows].T @ deg).sum())
    # mr_cooc_bytes: per (row, tile) segment min(4 nnz, tile songs) bytes
    tile_of = C.indices // bs
    row_of = np.repeat(np.arange(rows.size), nnz_r)
    seg_nnz = np.bincount(row_of * n_tiles + tile_of, minlength=rows.size * n_tiles).reshape(rows.size, n_tiles)
    bw = np.minimum(bs, ds.n_songs - bs * np.arange(n_tiles))
    seg_min = np.minimum(4 * seg_nnz, bw[None, :]).sum(axis=1)
    assert cb["heavy_rows"] + cb["light_rows"] == rows.size
    assert cb["heavy_reads"] + cb["light_reads"] == reads
    if os.environ.get("MR_COOC_LIGHT") == "0":  # every row heavy: one walk per tile, or per tile group
        walks = n_tiles if (cb["group_tiles"] == 0 or os.environ.get("MR_COOC_DENSE32") == "1") else cb["n_groups"]
        assert cb["light_rows"] == 0 and cb["heavy_visits"] == int(c_tr[rows].sum()) * walks
    got_index = cb["heavy_index_bytes"] + cb["light_index_bytes"]
    if os.environ.get("MR_COOC_DENSE_DIV") is None:  # the build's own dense rule: exact
        assert got_index == int(seg_min.sum())
        assert cb["consumed_bytes"] == int((seg_min * users_r).sum())
    else:  # a test dense rule charges a sparse-enough dense segment its tile's songs
        assert got_index >= int(seg_min.sum())
        assert cb["consumed_bytes"] >= int((seg_min * users_r).sum())


@pytest.mark.parametrize("n_listeners,n_common", [(100, 5), (700, 9), (2000, 13)])
def test_light_rows_shared_songs_and_straddling_chunks(n_listeners, n_common, monkeypatch):
    """The light rows' LDS hash insert (light_insert_queue, MR:232-235's
    counts): every listener of the row holds the same n_common songs, so
    hundreds of lanes claim and add to the same slots at once (CAS-first, then
    an add on a tag match), and the listeners' rows have every length mod 8,
    so a lane's 16-B chunk often ends inside a listener's row with the NEXT
    listener's songs right behind it in sr_songs — the key batch a lane hands
    over is a prefix of m < 8 valid keys of ONE listener (distinct songs) and
    no key past m may be inserted (the invariant the reverted two-queue insert
    of r05 s43 broke). Counts up to 2000 per slot (< the 4095
    the 12 count bits hold; mr_load keeps rows with more listeners off the
    light path). Dense scores and top-k bitwise vs the oracle."""
    monkeypatch.delenv("MR_COOC_LIGHT", raising=False)
    tr, te = [], []
    for v in range(n_listeners):
        songs = ["hub"] + [f"c{j:02d}" for j in range(n_common)] + [f"p{v:05d}_{j}" for j in range(v % 8)]
        tr += [f"v{v:05d}\t{s}\t1" for s in songs]
    te = ["x0\thub\t1", "x1\tc00\t1", "x2\thub\t1", "x2\tp00003_1\t1", "x3\tp00007_6\t1"]
    from helpers import dataset_from_lines
    ds = dataset_from_lines(tr, te, [])
    for k in (1, 10):
        check_route_exact(ds, k=k)
    with Engine(ds, out_dtype="f64", topk=10, stage1="wide", ibm_route="cooc") as e:
        e.run("ibm")
        assert e.cooc_bytes()["light_rows"] >= 1  # the rows went through the hash tables
