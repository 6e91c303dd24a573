"""GPU: combination models (MR:317-481), the threshold mAP (MR:521-639) and the
dense top-k on the device, through the C ABI, against host restatements:
* combinations: bit-identical to the reference formulas applied in numpy to
  the same engine models (pair order of main.scala:57-59);
* threshold mAP: bit-identical to the host evaluation (same counts, same fold),
  and within 1e-9 of the literal restatement on the committed fixtures;
* dense top-k of a model = the engine's own top-k of that model (keys too);
* test-user blocks and song shards give the single-context results."""
import numpy as np
import pytest
import torch

from musicrecommendation_amd import _lib, evaluation, synth
from musicrecommendation_amd.engine import Engine, merge_topk_host
from musicrecommendation_amd.ensemble import DeviceEnsemble, pair_uniform
from musicrecommendation_amd.sharding import song_shards

from helpers import dataset_from_lines, kat, pair_index, reference_combination, synth_fixture

pytestmark = pytest.mark.gpu


def datasets():
    K = kat()
    yield "kat", dataset_from_lines(K["train"], K["test"], K["labels"])
    yield "small", synth_fixture("small")[0]
    yield "c2x24", synth.config("c2", n_test=24).dataset()


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_combinations_and_map_bit_identical(dtype):
    for name, ds in datasets():
        with Engine(ds, out_dtype=dtype, topk=4) as e:
            ens = DeviceEnsemble(e)
            ubm_t, ibm_t = ens.model("ubm"), ens.model("ibm")
            ubm, ibm = ubm_t.cpu().numpy().astype(np.float64), ibm_t.cpu().numpy().astype(np.float64)
            e.run("ubm")
            assert np.array_equal(e.dense().astype(np.float64), ubm, equal_nan=True)  # run_into == run
            idx = pair_index(ds)
            n_pairs = ds.n_pairs()
            cases = [("linear", ens.linear(ubm_t, ibm_t, 0.5), 0.5), ("linear", ens.linear(ubm_t, ibm_t, 0.3), 0.3),
                     ("aggregation", ens.aggregation(ubm_t, ibm_t, 0.5), 0.5),
                     ("aggregation", ens.aggregation(ubm_t, ibm_t, 0.37), 0.37),
                     ("stochastic", ens.stochastic(ubm_t, ibm_t, 0.5, seed=3), 0.5)]
            for kind, t, param in cases:
                got = t.cpu().numpy().astype(np.float64)
                exp = reference_combination(kind, ubm, ibm, param, idx, n_pairs, seed=3)
                if dtype == "f32":
                    exp = exp.astype(np.float32).astype(np.float64)
                assert np.array_equal(got, exp, equal_nan=True), (name, kind, param)
            for t in (ubm_t, ibm_t, cases[0][1], cases[2][1], cases[4][1]):
                host = evaluation.threshold_map(t.cpu().numpy().astype(np.float64), ds)
                assert ens.threshold_map(t) == host, name
            with pytest.raises(_lib.EngineError):
                ens.aggregation(ubm_t, ibm_t, 1.2)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_combinations_in_one_pass(dtype):
    """mr_combine_all_device: the three outputs bitwise equal to the separate
    calls, their min / max equal to mr_eval_minmax_device, the mAP through the
    carried min / max equal to the recomputed one; a block of test users and
    a song shard too; an in-place edit drops the carried min / max."""
    ds = synth.config("c2", n_test=24).dataset()
    n_pairs = ds.n_pairs()
    for song_lo, song_hi, a, b in [(0, ds.n_songs, 0, ds.n_test), (0, ds.n_songs, 7, 19), (3000, 9000, 0, ds.n_test)]:
        sub = ds if (a, b) == (0, ds.n_test) else ds.subset_test_users(a, b)
        base = a * ds.n_songs - int(ds.te_off[a])
        with Engine(sub, out_dtype=dtype, song_lo=song_lo, song_hi=song_hi) as e:
            ens = DeviceEnsemble(e, pair_base=base, n_pairs=n_pairs, pos=evaluation.label_pos(ds),
                                 n_label_songs=ds.n_label_songs)
            u_t, i_t = ens.model("ubm"), ens.model("ibm")
            lin, agg, sto = ens.combinations(u_t, i_t, 0.3, 0.37, 0.5, seed=5)
            sep = (ens.linear(u_t, i_t, 0.3), ens.aggregation(u_t, i_t, 0.37), ens.stochastic(u_t, i_t, 0.5, seed=5))
            for got, exp in zip((lin, agg, sto), sep):
                assert np.array_equal(got.cpu().numpy(), exp.cpu().numpy(), equal_nan=True)
                assert got._mr_minmax[1:] == e.eval_minmax(got.data_ptr())
            if (song_lo, song_hi, a, b) == (0, ds.n_songs, 0, ds.n_test):
                for got, exp in zip((lin, agg, sto), sep):
                    assert ens.threshold_map(got) == ens.threshold_map(exp)
                carried = lin._mr_minmax[1:]
                lin.mul_(2.0)  # in place: the carried min / max no longer apply
                # no host sync: _minmax orders the engine's stream after torch's pending mul_
                mm = ens._minmax(lin)
                assert mm == e.eval_minmax(lin.data_ptr()) != carried
                with pytest.raises(_lib.EngineError):
                    ens.combinations(u_t, i_t, 0.5, 1.5, 0.5)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("route", ["two_hop", "cooc"])
def test_dense_minmax_from_the_scoring_kernels(dtype, route):
    """mr_dense_minmax (wide shape: min / max kept by the scoring kernels while
    they store the model) equals mr_eval_minmax_device over the stored model,
    for both models and both ibm routes, over a song shard and user batches;
    threshold_map through it equals the recomputed one; a fused-shape run
    and a top-k-only context leave none."""
    ds = synth.config("c2", n_test=24).dataset()
    for lo, hi in [(0, ds.n_songs), (2000, 11000)]:
        with Engine(ds, out_dtype=dtype, stage1="wide", song_lo=lo, song_hi=hi, ibm_route=route) as e:
            ens = DeviceEnsemble(e)
            for model in ("ubm", "ibm"):
                t = ens.model(model)
                mm = e.dense_minmax()
                assert mm is not None and mm == e.eval_minmax(t.data_ptr()), (model, lo)
                assert t._mr_minmax[1:] == mm
                if (lo, hi) == (0, ds.n_songs):
                    host = evaluation.threshold_map(t.cpu().numpy().astype(np.float64), ds)
                    assert ens.threshold_map(t) == host
    with Engine(ds, out_dtype=dtype, stage1="fused") as e:
        e.run("ibm")
        assert e.dense_minmax() is None
    with Engine(ds, out_dtype=dtype, stage1="wide", dense=False) as e:
        e.run("ubm")
        assert e.dense_minmax() is None


def test_map_vs_literal_fixture():
    for name in ("tiny", "small"):
        ds, z = synth_fixture(name)
        with Engine(ds, out_dtype="f64") as e:
            ens = DeviceEnsemble(e)
            for model in ("ibm", "ubm"):
                got = ens.threshold_map(ens.model(model))
                assert abs(got - evaluation.threshold_map(z[model], ds)) < 1e-9


@pytest.mark.parametrize("model", ["ibm", "ubm"])
@pytest.mark.parametrize("k", [1, 10, 16])
def test_dense_topk_equals_engine_topk(model, k):
    ds = synth.config("c2", n_test=13).dataset()
    with Engine(ds, out_dtype="f64", topk=k) as e:
        e.run(model)
        s1, sc1, k1 = e.topk()
        ens = DeviceEnsemble(e)
        t = ens.model(model)
        s2, sc2, k2 = ens.topk(t)
        assert np.array_equal(s1, s2) and np.array_equal(k1, k2)
        # a combination model's top-k against a numpy top-k by (score desc, song asc)
        c = ens.linear(ens.model("ubm"), ens.model("ibm"), 0.5)
        s3, sc3, _ = ens.topk(c)
        x = c.cpu().numpy()
        for u in range(ds.n_test):
            row = x[u]
            cand = sorted((-row[j], j) for j in np.flatnonzero(~np.isnan(row)))[:k]
            assert s3[u].tolist() == [j for _, j in cand]


def test_user_blocks_and_song_shards():
    ds = synth.config("c2", n_test=24).dataset()
    n_pairs = ds.n_pairs()
    with Engine(ds, out_dtype="f64") as e:
        ens = DeviceEnsemble(e)
        u_t, i_t = ens.model("ubm"), ens.model("ibm")
        full_agg = ens.aggregation(u_t, i_t, 0.5).cpu().numpy()
        full_sto = ens.stochastic(u_t, i_t, 0.5, seed=5).cpu().numpy()
        full_map = ens.threshold_map(i_t)
    pos = evaluation.label_pos(ds)
    for a, b in [(0, 7), (7, 19), (19, 24)]:
        sub = ds.subset_test_users(a, b)
        base = a * ds.n_songs - int(ds.te_off[a])
        with Engine(sub, out_dtype="f64") as e:
            ens = DeviceEnsemble(e, pair_base=base, n_pairs=n_pairs, pos=pos, n_label_songs=ds.n_label_songs)
            u_t, i_t = ens.model("ubm"), ens.model("ibm")
            assert np.array_equal(ens.aggregation(u_t, i_t, 0.5).cpu().numpy(), full_agg[a:b], equal_nan=True)
            assert np.array_equal(ens.stochastic(u_t, i_t, 0.5, seed=5).cpu().numpy(), full_sto[a:b],
                                  equal_nan=True)
    # song shards: combinations are per-column; eval counts sum into the full table
    pred_full = np.zeros((ds.n_songs, 10), np.int64)
    tp_full = np.zeros_like(pred_full)
    mins, maxs = [], []
    for lo, hi in song_shards(ds, 3):
        with Engine(ds, out_dtype="f64", song_lo=lo, song_hi=hi) as e:
            ens = DeviceEnsemble(e)
            u_t, i_t = ens.model("ubm"), ens.model("ibm")
            assert np.array_equal(ens.aggregation(u_t, i_t, 0.5).cpu().numpy(), full_agg[:, lo:hi], equal_nan=True)
            mn, mx = e.eval_minmax(i_t.data_ptr())
            mins.append(mn)
            maxs.append(mx)
            shard_tensors = (e, i_t, lo, hi)
            p, t = e.eval_counts(i_t.data_ptr(), -1.0, -1.0, ds.lab_off, ds.lab_songs)  # placeholder extremes
        del shard_tensors
    mn, mx = min(mins), max(maxs)
    for lo, hi in song_shards(ds, 3):
        with Engine(ds, out_dtype="f64", song_lo=lo, song_hi=hi) as e:
            i_t = DeviceEnsemble(e).model("ibm")
            p, t = e.eval_counts(i_t.data_ptr(), mn, mx, ds.lab_off, ds.lab_songs)
            pred_full[lo:hi], tp_full[lo:hi] = p, t
    from musicrecommendation_amd.ensemble import eval_map
    assert eval_map(pred_full, tp_full, pos, ds.n_label_songs) == full_map


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_level_thresholds_exact_at_boundaries(dtype):
    """k_eval_pred compares scores against per-threshold floors found on the host
    (level_floor); scores one ulp either side of every (x - min)/(max - min) = t
    boundary must count exactly as the fp64 expression of MR:529 does."""
    ds = synth_fixture("small")[0]
    npt = np.float32 if dtype == "f32" else np.float64
    with Engine(ds, out_dtype=dtype) as e:
        ens = DeviceEnsemble(e)
        shape = (e.n_test, e.width)
        rng = np.random.default_rng(7)
        mn, mx = npt(0.0137), npt(0.7731)
        vals = [mn, mx]
        for t in (0.0, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9):
            x0 = npt(float(mn) + t * (float(mx) - float(mn)))
            lo = hi = x0
            for _ in range(3):
                lo, hi = np.nextafter(lo, npt(-1)), np.nextafter(hi, npt(2))
                vals += [lo, hi]
            vals.append(x0)
        vals = np.array(vals, dtype=npt)
        x = rng.choice(vals, size=shape).astype(npt)
        x[0, 0], x[0, 1] = mn, mx  # the range is exactly [mn, mx]
        x[ds.heard_mask()[:, :e.width]] = np.nan
        t = torch.from_numpy(x).cuda()
        got_mn, got_mx = e.eval_minmax(t.data_ptr())
        assert (got_mn, got_mx) == (float(np.nanmin(x)), float(np.nanmax(x)))
        pred, _tp = e.eval_counts(t.data_ptr(), got_mn, got_mx, ds.lab_off, ds.lab_songs)
        xd = x.astype(np.float64)
        with np.errstate(invalid="ignore"):
            v = (xd - got_mn) / (got_mx - got_mn)
            exp = np.stack([(v > thr).sum(axis=0) for thr in (0.0, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9)],
                           axis=1)
        assert np.array_equal(pred, exp.astype(np.int32))
        assert ens.threshold_map(t) == evaluation.threshold_map(xd, ds)


@pytest.mark.parametrize("n_thr", [10, 11])
@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_device_map_fold_equals_host_fold(dtype, n_thr):
    """mr_eval_map_device (counts + AP per class on the device, ordered host sum)
    == mr_eval_counts_device + mr_eval_map, bit for bit, and both == numpy;
    with MR's 10 thresholds and the distributed evaluation's 11
    (distributed.scala:395), whose counts also equal numpy's column for column."""
    from musicrecommendation_amd.ensemble import eval_map

    ths = evaluation.THRESHOLDS if n_thr == 10 else evaluation.THRESHOLDS_DISTRIBUTED
    for name, ds in datasets():
        with Engine(ds, out_dtype=dtype, topk=4) as e:
            ens = DeviceEnsemble(e)
            for t in (ens.model("ubm"), ens.model("ibm")):
                mn, mx = e.eval_minmax(t.data_ptr())
                pred, tp = e.eval_counts(t.data_ptr(), mn, mx, ds.lab_off, ds.lab_songs, n_thresholds=n_thr)
                x = t.cpu().numpy().astype(np.float64)
                np_pred, np_tp = evaluation.threshold_counts(x, ds, mn, mx, ths)
                assert np.array_equal(pred, np_pred) and np.array_equal(tp, np_tp), name
                host = eval_map(pred, tp, ens.pos, ds.n_label_songs)
                dev = e.eval_map(t.data_ptr(), mn, mx, ds.lab_off, ds.lab_songs, ens.pos, ds.n_label_songs,
                                 n_thresholds=n_thr)
                assert dev == host, name
                assert dev == evaluation.threshold_map(x, ds, ths), name
                assert ens.threshold_map(t, n_thresholds=n_thr) == dev, name
            with pytest.raises(ValueError):
                e.eval_map(t.data_ptr(), mn, mx, ds.lab_off, ds.lab_songs, ens.pos[:1], ds.n_label_songs)
