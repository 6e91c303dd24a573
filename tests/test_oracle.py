"""The oracle pinned before it is trusted (CPU only).

Parity anchors: the reference has no tests, fixtures or
golden vectors and cannot run here (Scala/Spark, no JVM), so the oracle is
pinned by the hand-derived known-answer test of SURVEY.md §4.2 and by
agreement of three independent restatements:
  * oracle/reference_py.py — line-by-line Python of the Scala (fixtures' source),
  * oracle/literal.c       — the same loop nests in C over string ids (timed CPU baseline),
  * oracle/fixedpoint.c    — two-hop identity in int64 fixed point (the GPU's bit-exact target).
"""
import math

import numpy as np
import pytest

from musicrecommendation_amd import synth
from oracle import native
from oracle.reference_py import LiteralRecommender, map_at_k

from helpers import dataset_from_lines, dense_from_pairs, kat, rel_err, synth_fixture, topk_consistent


def test_kat_python_literal_matches_hand_derivation():
    K = kat()
    rec = LiteralRecommender(K["train"], K["test"], K["labels"])
    for model, fn in (("ibm", rec.get_item_based_model), ("ubm", rec.get_user_based_model)):
        got = {f"{u}|{s}": x for u, (s, x) in fn()}
        assert got == K["expected"][model]  # bitwise, hand-derived numbers
        assert rec.evaluate_model(fn()) == K["expected"][f"map_{model}"]


def test_kat_catches_the_three_classic_mistakes():
    """train-only c(s), sqrt(a*b), scoring heard songs."""
    K = kat()
    assert 1 / math.sqrt(6) != K["expected"]["ibm"]["Y|s1"]             # sqrt(a*b)
    assert 1 / (1 * math.sqrt(2)) != K["expected"]["ibm"]["Y|s1"]       # train-only counts
    assert "X|s1" not in K["expected"]["ibm"] and "Y|s2" not in K["expected"]["ibm"]  # heard


@pytest.mark.parametrize("which", ["plain", "dup"])
@pytest.mark.parametrize("model", ["ibm", "ubm"])
def test_kat_c_literal_and_fixed_point(which, model):
    K = kat() if which == "plain" else kat()["dup"]
    ds = dataset_from_lines(K["train"], K["test"], K["labels"])
    exp = dense_from_pairs(ds, K["expected"][model])
    li = native.LiteralInputs(K["train"], K["test"])
    lit, n = li.model(model, threads=1)
    assert n == int((~np.isnan(exp)).sum())
    assert np.array_equal(lit, exp, equal_nan=True)  # same fp64 op order on 1-3 term sums
    fp, _, _ = native.fp_model(ds, model)
    assert rel_err(fp, exp) < 1e-9


@pytest.mark.parametrize("name", ["tiny", "small"])
@pytest.mark.parametrize("model", ["ibm", "ubm"])
def test_golden_fixtures_three_oracles_agree(name, model):
    ds, z = synth_fixture(name)
    tr, te = z["train"].tolist(), z["test"].tolist()
    li = native.LiteralInputs(tr, te)
    seq, n_seq = li.model(model, threads=1)
    par, n_par = li.model(model, threads=4)
    assert n_seq == n_par == ds.n_pairs()
    assert np.array_equal(seq, par, equal_nan=True)  # seq == par (README.md:254-261)
    assert rel_err(seq, z[model]) < 1e-13            # HashSet vs sorted summation order only
    fp, ts, _tk = native.fp_model(ds, model)
    assert rel_err(fp, z[model]) < 1e-7               # fixed-point rounding, F = 32
    topk_consistent(ts, z[model], 10)


def test_fixed_point_error_bound_scales_with_frac_bits():
    ds, z = synth_fixture("small")
    errs = []
    for F in (16, 24, 32):
        fp, _, _ = native.fp_model(ds, "ibm", frac_bits=F)
        errs.append(rel_err(fp, z["ibm"]))
    assert errs[0] > errs[1] > errs[2]
    assert errs[2] < 1e-8


def test_fixed_point_sharding_is_exact():
    ds, _ = synth_fixture("small")
    full, ts, tk = native.fp_model(ds, "ubm")
    parts = [native.fp_model(ds, "ubm", song_lo=lo, song_hi=hi)[0]
             for lo, hi in ((0, 700), (700, 701), (701, ds.n_songs))]
    assert np.array_equal(np.concatenate(parts, axis=1), full, equal_nan=True)


def test_c1_literal_vs_fixed_point_sample():
    """C1 (ubm 100/10/~4.8k songs, the CPU-path config) on a block of pairs."""
    ds = synth.config("c1").dataset()
    tr, te, _ = native.dataset_lines(ds)
    li = native.LiteralInputs(tr, te)
    lit, n = li.model("ubm", threads=8, pair_lo=0, pair_hi=4000)
    fp, _, _ = native.fp_model(ds, "ubm")
    sel = ~np.isnan(lit)
    assert n == sel.sum() > 3000
    err = np.abs(fp[sel] - lit[sel]) / np.maximum(np.abs(lit[sel]), 1e-300)
    assert err.max() < 1e-7


def test_reference_py_map_at_k_and_combinations():
    K = kat()
    rec = LiteralRecommender(K["train"], K["test"], K["labels"])
    ubm = sorted(rec.get_user_based_model(), key=lambda t: (t[0], t[1][0], -t[1][1]))
    ibm = sorted(rec.get_item_based_model(), key=lambda t: (t[0], t[1][0], -t[1][1]))
    lc = LiteralRecommender.linear_combination(ubm, ibm, 0.5)
    assert [x for _, (_, x) in lc] == [a * 0.5 + b * 0.5 for (_, (_, a)), (_, (_, b)) in zip(ubm, ibm)]
    ag = LiteralRecommender.aggregation(ubm, ibm, 0.5)
    assert len(ag) == len(ubm)
    # X: labels {s3,s5}; top-1 unheard by ibm is s3 -> AP@1 = 1/min(1,2)
    assert map_at_k(ibm, rec.test_labels, rec.test_users, 1) == 1.0
