"""GPU: the wide kernel's candidate-only tile top-k (wide_cand_topk).

Top-k-only runs (C4's north star: no dense model) rank an fp32 approximation
of every song's score (its integer accumulator times a 4-B 1/sqrt(c) table),
take the threshold over those, and compute the exact fp64 key — the oracle's
operations, MR:249-257 — for the songs within 2^-17 of it only. The bar is
bit-identity of songs AND keys with the all-songs path (MR_WIDE_CAND=0) and
with the fixed-point oracle, over both models, both ibm routes, k from 1 to
16, song shards, users whose tiles hold fewer than k positive scores (the
fallback to the all-songs path) and ties.
"""
import numpy as np
import pytest

from musicrecommendation_amd import synth
from musicrecommendation_amd.engine import Engine
from musicrecommendation_amd.sharding import song_shards
from oracle import native

from helpers import dataset_from_lines, synth_fixture

pytestmark = pytest.mark.gpu


def topk_lists(ds, model, k, cand, monkeypatch, route="auto", **kw):
    monkeypatch.setenv("MR_WIDE_CAND", "1" if cand else "0")
    with Engine(ds, topk=k, dense=False, stage1="wide", ibm_route=route, **kw) as e:
        assert e.shape == "wide" and e.candidate_topk == cand
        e.run(model)
        songs, scores, keys = e.topk()
        return songs, scores, keys, (e.song_lo, e.song_hi)


@pytest.fixture(scope="module")
def c3_64():
    return synth.config("c3", n_test=64).dataset()


@pytest.mark.parametrize("k", [1, 4, 10, 16])
@pytest.mark.parametrize("model,route", [("ibm", "cooc"), ("ibm", "two_hop"), ("ubm", "auto")])
def test_candidate_lists_bitwise(c3_64, model, route, k, monkeypatch):
    ds = c3_64
    s1, sc1, k1, (lo, hi) = topk_lists(ds, model, k, True, monkeypatch, route=route)
    s0, sc0, k0, _ = topk_lists(ds, model, k, False, monkeypatch, route=route)
    assert np.array_equal(s1, s0) and np.array_equal(k1, k0)
    assert np.array_equal(sc1, sc0, equal_nan=True)
    _, ts, tk = native.fp_model(ds, model, song_lo=lo, song_hi=hi, k=k, dense=False)
    assert np.array_equal(s1, ts) and np.array_equal(k1, tk)


@pytest.mark.parametrize("n_shards", [3, 8])
def test_candidate_lists_song_shards(c3_64, n_shards, monkeypatch):
    ds = c3_64
    for lo, hi in song_shards(ds, n_shards)[:2]:
        s1, _, k1, _ = topk_lists(ds, "ibm", 10, True, monkeypatch, song_lo=lo, song_hi=hi)
        _, ts, tk = native.fp_model(ds, "ibm", song_lo=lo, song_hi=hi, k=10, dense=False)
        assert np.array_equal(s1, ts) and np.array_equal(k1, tk)


@pytest.mark.parametrize("block", [256, 1024, 4096])
def test_candidate_fixture_tiles(block, monkeypatch):
    """Small tiles (many per user), the fixtures' tiny users: tiles with fewer
    than k unheard or positive songs take the all-songs fallback."""
    ds, _ = synth_fixture("small")
    for k in (3, 10, 16):
        s1, _, k1, (lo, hi) = topk_lists(ds, "ibm", k, True, monkeypatch, block_songs=block)
        _, ts, tk = native.fp_model(ds, "ibm", song_lo=lo, song_hi=hi, k=k, dense=False)
        assert np.array_equal(s1, ts) and np.array_equal(k1, tk)


def test_candidate_ties_and_empty_users(monkeypatch):
    """Songs with identical scores (same listeners, same c) straddling the
    k-th place, and a test user whose only visible song has no train
    listener (every score 0: tau = 0, the survivors overflow, fallback)."""
    tr = []
    for v in range(40):  # songs a0..a29 all heard by the same 40 users: equal scores
        tr += [f"v{v:03d}\ta{j:02d}\t1" for j in range(30)]
    for v in range(40, 60):
        tr += [f"v{v:03d}\tb{j:02d}\t1" for j in range(5)] + [f"v{v:03d}\ta00\t1"]
    te = ["x000\ta00\t1", "x001\tb00\t1", "x002\tzz\t1", "x003\ta05\t1", "x003\tb03\t1"]
    ds = dataset_from_lines(tr, te, [])
    for k in (1, 7, 10, 16):
        for model in ("ibm", "ubm"):
            s1, _, k1, (lo, hi) = topk_lists(ds, model, k, True, monkeypatch)
            s0, _, k0, _ = topk_lists(ds, model, k, False, monkeypatch)
            _, ts, tk = native.fp_model(ds, model, song_lo=lo, song_hi=hi, k=k, dense=False)
            assert np.array_equal(s1, ts) and np.array_equal(k1, tk), (model, k)
            assert np.array_equal(s0, ts) and np.array_equal(k0, tk), (model, k)


def test_candidate_mode_only_for_topk_only_wide(c3_64, monkeypatch):
    """Dense runs and the fused shape keep the all-songs path."""
    monkeypatch.delenv("MR_WIDE_CAND", raising=False)
    with Engine(c3_64, topk=10, dense=True, stage1="wide") as e:
        assert not e.candidate_topk
    with Engine(synth.config("c2").dataset(), topk=10, dense=False) as e:
        assert e.shape == "fused" and not e.candidate_topk
    with Engine(c3_64, topk=10, dense=False, stage1="wide") as e:
        assert e.candidate_topk


@pytest.mark.parametrize("nt,k,frac_bits,block", [(512, 10, 32, 8192), (512, 16, 32, 8192), (1024, 10, 40, 0),
                                                  (512, 10, 40, 8192)])
def test_candidate_cooc_kernel_variants(c3_64, nt, k, frac_bits, block, monkeypatch):
    """The co-listening scoring kernel at 512 threads (NG = 32, pass A spans
    20 x 512 songs; k up to the wide shape's 16) and the non-split dense pass of
    frac_bits > 32, candidate-only vs all-songs vs the oracle, bitwise.
    (MR_COOC_DS=16 is a compile-time A/B knob of the dense layout, not an
    option of the shipped library.)"""
    monkeypatch.setenv("MR_COOC_NT", str(nt))
    kw = dict(frac_bits=frac_bits)
    if block:
        kw["block_songs"] = block
    s1, _, k1, (lo, hi) = topk_lists(c3_64, "ibm", k, True, monkeypatch, route="cooc", **kw)
    s0, _, k0, _ = topk_lists(c3_64, "ibm", k, False, monkeypatch, route="cooc", **kw)
    assert np.array_equal(s1, s0) and np.array_equal(k1, k0)
    _, ts, tk = native.fp_model(c3_64, "ibm", song_lo=lo, song_hi=hi, k=k, dense=False, frac_bits=frac_bits)
    assert np.array_equal(s1, ts) and np.array_equal(k1, tk)
