"""Combination models and the threshold mAP, host side (no GPU):
* the stochastic model's seeded stream: product restatement = oracle restatement;
* the mAP fold of the counts (C mr_eval_map and numpy map_from_counts) = the
  literal restatement of MR:521-639 (oracle/reference_py.py) on the fixtures,
  with MR's 10 thresholds and with the distributed evaluation's 11
  (distributed.scala:395-415);
* the Model-array API mirror (MR:317-481) = the oracle's literal versions;
* the multi-rank reduction of DeviceEnsemble.threshold_map (gloo, world 2)
  over song shards and over test-user blocks = the single-process value."""

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from musicrecommendation_amd import evaluation
from musicrecommendation_amd.ensemble import DeviceEnsemble, eval_map, pair_uniform
from musicrecommendation_amd.recommender import MusicRecommender
from musicrecommendation_amd.sharding import song_shards
from oracle.reference_py import LiteralRecommender

from helpers import kat, pg_init_method, synth_fixture

MODELS = ("ibm", "ubm")


def test_stochastic_stream_matches_oracle_restatement():
    for seed in (0, 1, 7, 2 ** 63 + 11, 2 ** 64 - 1):
        for i in (0, 1, 2, 3, 1000, 2 ** 31, 2 ** 40 + 5):
            assert pair_uniform(seed, i) == LiteralRecommender.uniform(seed, i)
    u = np.array([pair_uniform(5, i) for i in range(40000)])
    assert 0 <= u.min() and u.max() < 1 and abs(u.mean() - 0.5) < 0.01


def _literal(name):
    if name == "kat":
        K = kat()
        lr = LiteralRecommender(K["train"], K["test"], K["labels"])
        from helpers import dataset_from_lines
        ds = dataset_from_lines(K["train"], K["test"], K["labels"])
        return lr, ds
    ds, z = synth_fixture(name)
    lr = LiteralRecommender(z["train"].tolist(), z["test"].tolist(), z["labels"].tolist())
    return lr, ds


def _dense_of(ds, model):
    si = {ds.song_names(i): i for i in range(ds.n_songs)}
    ui = {ds.test_names(i): i for i in range(ds.n_test)}
    d = np.full((ds.n_test, ds.n_songs), np.nan)
    for u, (s, x) in model:
        d[ui[u], si[s]] = x
    return d


@pytest.mark.parametrize("n_thr", [10, 11])
@pytest.mark.parametrize("name", ["kat", "tiny", "small"])
@pytest.mark.parametrize("model", MODELS)
def test_map_fold_matches_literal_evaluation(name, model, n_thr):
    ths = evaluation.THRESHOLDS if n_thr == 10 else evaluation.THRESHOLDS_DISTRIBUTED
    lr, ds = _literal(name)
    if name == "kat":
        m = lr.get_item_based_model() if model == "ibm" else lr.get_user_based_model()
        dense = _dense_of(ds, m)
    else:  # the committed literal model (tests/golden/make_golden.py) instead of re-scoring
        dense = synth_fixture(name)[1][model]
        m = [(ds.test_names(u), (ds.song_names(s), float(dense[u, s])))
             for s in range(ds.n_songs) for u in range(ds.n_test) if not np.isnan(dense[u, s])]
    ref = lr.evaluate_model(m, list(ths))
    host = evaluation.threshold_map(dense, ds, ths)
    valid = ~np.isnan(dense)
    pred, tp = evaluation.threshold_counts(dense, ds, dense[valid].min(), dense[valid].max(), ths)
    assert pred.shape[1] == n_thr
    c_map = eval_map(pred, tp, evaluation.label_pos(ds), ds.n_label_songs)
    assert c_map == host                       # C fold == numpy fold, bit for bit
    assert abs(host - ref) <= 1e-12            # == literal MR:521-639 (class order: ulps)
    if name == "kat":
        assert abs(host - 0.6666666666666666) < 1e-15  # SURVEY.md §4.2 (10 and 11 thresholds)


def test_eleven_thresholds_differ_from_ten():
    """The 11-threshold recurrence is not the 10-threshold one (it adds the
    (R_8 - R_9) P_8 + R_9 P_9 tail): on a fixture with mid-range scores the two
    mAPs differ, each equal to its literal restatement."""
    lr, ds = _literal("small")
    dense = synth_fixture("small")[1]["ibm"]
    m = [(ds.test_names(u), (ds.song_names(s), float(dense[u, s])))
         for s in range(ds.n_songs) for u in range(ds.n_test) if not np.isnan(dense[u, s])]
    a = evaluation.threshold_map(dense, ds, evaluation.THRESHOLDS)
    b = evaluation.threshold_map(dense, ds, evaluation.THRESHOLDS_DISTRIBUTED)
    assert a != b
    assert abs(b - lr.evaluate_model(m, lr.THRESHOLDS_DISTRIBUTED)) <= 1e-12
    with pytest.raises(Exception):
        eval_map(np.zeros((3, 9), np.int32), np.zeros((3, 9), np.int32), np.ones(3, np.int32), 3)


@pytest.mark.parametrize("name", ["kat", "tiny"])
def test_list_api_combinations_match_oracle(name):
    lr, ds = _literal(name)
    order = lambda m: sorted(m, key=lambda t: (t[0], t[1][0], -t[1][1]))  # noqa: E731  main.scala:57-59
    ubm, ibm = order(lr.get_user_based_model()), order(lr.get_item_based_model())
    rec = MusicRecommender.__new__(MusicRecommender)  # the list API needs no engine
    assert rec.getLinearCombinationModel(ubm, ibm, 0.3) == LiteralRecommender.linear_combination(ubm, ibm, 0.3)
    assert rec.getAggregationModel(ubm, ibm, 0.4) == LiteralRecommender.aggregation(ubm, ibm, 0.4)
    assert rec.getStochasticCombinationModel(ubm, ibm, 0.6, seed=9) == LiteralRecommender.stochastic(ubm, ibm, 0.6, 9)
    with pytest.raises(ValueError):
        rec.getAggregationModel(ubm, ibm, 1.5)
    with pytest.raises(ValueError):
        rec.getLinearCombinationModel(ubm, ibm[::-1], 0.5)


class _HostEngine:
    """Stands in for an Engine on one shard: eval_minmax / eval_counts by numpy
    over the shard's columns (the device kernels' twins)."""

    def __init__(self, ds, dense, lo, hi):
        self.dataset, self.dense, self.song_lo, self.song_hi = ds, dense, lo, hi
        self.dtype, self.n_test, self.width = np.float64, ds.n_test, hi - lo

        class _O:
            device = 0
        self.opt = _O()

    def eval_minmax(self, _ptr):
        x = self.dense[:, self.song_lo:self.song_hi]
        v = x[~np.isnan(x)]
        return (float(v.min()), float(v.max())) if v.size else (np.inf, -np.inf)

    def eval_counts(self, _ptr, mn, mx, lab_off, lab_songs, n_thresholds=10, **_bufs):
        ths = evaluation.THRESHOLDS if n_thresholds == 10 else evaluation.THRESHOLDS_DISTRIBUTED
        p, t = evaluation.threshold_counts(self.dense, self.dataset, mn, mx, ths)
        return p[self.song_lo:self.song_hi].astype(np.int32), t[self.song_lo:self.song_hi].astype(np.int32)


def _worker(rank, world, init, layout, out, n_thr=10):
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        ds, z = synth_fixture("small")
        dense = z["ibm"]
        full_pos = evaluation.label_pos(ds)
        if layout == "songs":
            lo, hi = song_shards(ds, world)[rank]
            eng = _HostEngine(ds, dense, lo, hi)
        elif layout == "2d":  # 2 user blocks x 2 song shards (sharding.ShardScorer's cells)
            from musicrecommendation_amd.sharding import user_blocks

            a, b = user_blocks(ds.n_test, 2)[rank // 2]
            lo, hi = song_shards(ds, 2)[rank % 2]
            eng = _HostEngine(ds.subset_test_users(a, b), dense[a:b], lo, hi)
        else:  # test-user blocks: each rank sees its users over all songs
            a, b = ds.n_test * rank // world, ds.n_test * (rank + 1) // world
            sub = ds.subset_test_users(a, b)
            eng = _HostEngine(sub, dense[a:b], 0, ds.n_songs)
        ens = DeviceEnsemble(eng, pos=full_pos, n_label_songs=ds.n_label_songs)

        class _Ptr:  # the host stand-in ignores the device pointer
            def data_ptr(self):
                return 0
        out[rank] = ens.threshold_map(_Ptr(), n_thresholds=n_thr)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("layout,n_thr", [("songs", 10), ("users", 10), ("2d", 10), ("songs", 11)])
def test_gloo_world2_threshold_map_reduction(layout, n_thr):
    world = 4 if layout == "2d" else 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, pg_init_method(), layout, out, n_thr), nprocs=world, join=True)
        res = dict(out)
    ds, z = synth_fixture("small")
    ref = evaluation.threshold_map(z["ibm"], ds,
                                   evaluation.THRESHOLDS if n_thr == 10 else evaluation.THRESHOLDS_DISTRIBUTED)
    assert all(res[r] == ref for r in range(world))


def test_carried_minmax_follows_the_tensor_version():
    """DeviceEnsemble._minmax: a min / max carried from the producing pass
    (combinations(), model() on the wide shape) is used while the tensor is
    unmodified, and recomputed (mr_eval_minmax_device) after an in-place edit
    or when none was carried."""
    import torch

    class FakeEngine:
        calls = 0

        def eval_minmax(self, ptr):
            FakeEngine.calls += 1
            return (-1.0, 1.0)

    ens = DeviceEnsemble.__new__(DeviceEnsemble)
    ens.e = FakeEngine()
    t = torch.zeros(4)
    assert ens._minmax(t) == (-1.0, 1.0) and FakeEngine.calls == 1  # nothing carried
    t._mr_minmax = (t._version, 0.25, 0.5)
    assert ens._minmax(t) == (0.25, 0.5) and FakeEngine.calls == 1  # carried, unchanged
    t.add_(1.0)
    assert ens._minmax(t) == (-1.0, 1.0) and FakeEngine.calls == 2  # edited in place
