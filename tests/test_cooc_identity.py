"""CPU check of the factorisation behind the ItemBasedModel's co-listening
route, against the fixed-point oracle (oracle/fixedpoint.c).

MusicRecommender.scala:230-257 scores rank(u, s) = Σ_{s2 ∈ T(u)} cos(s, s2)
with cos's numerator |L_tr(s) ∩ L_tr(s2)| (MR:232-235). In the engine's fixed
point the two-hop route sums q(s2) over (v, s2) with s, s2 ∈ S(v); the
co-listening route sums q(s2) · C[s2][s] with C = A_trᵀ A_tr. Both are the
same int64 sum, so the numpy restatement below (integer matmul, exact) must
equal the oracle's dense scores bit for bit — the property the GPU tests of
tests/test_gpu_cooc.py then check on the device.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from musicrecommendation_amd import synth
from oracle import native

from helpers import dataset_from_lines, kat, synth_fixture


def cooc_scores(ds, frac_bits=32):
    n_s = ds.n_songs
    tr_rows = np.repeat(np.arange(ds.n_train), np.diff(ds.tr_off))
    A = sp.csr_matrix((np.ones(tr_rows.size, np.int64), (tr_rows, ds.tr_songs)), shape=(ds.n_train, n_s))
    te_rows = np.repeat(np.arange(ds.n_test), np.diff(ds.te_off))
    rows = np.unique(ds.te_songs)                                   # the index rows (test-visible songs)
    C = (A[:, rows].T @ A).toarray().astype(np.int64)               # C[s2][s] = |L_tr(s2) ∩ L_tr(s)|
    sqrt_c = np.sqrt(ds.song_count.astype(np.float64))              # c(s): train + test lines (MR:237)
    q = np.rint(np.ldexp(1.0, frac_bits) / sqrt_c).astype(np.int64)  # q(s2) = rint(2^F / sqrt c(s2))
    W = np.zeros((ds.n_test, rows.size), np.int64)
    W[te_rows, np.searchsorted(rows, ds.te_songs)] = q[ds.te_songs]
    acc = W @ C                                                      # exact int64 sums
    score = acc.astype(np.float64) * np.ldexp(1.0, -frac_bits) / sqrt_c[None, :]
    score[te_rows, ds.te_songs] = np.nan                            # heard: no pair (MR:109)
    return score


def _datasets():
    K = kat()
    yield "kat", dataset_from_lines(K["train"], K["test"], K["labels"])
    Kd = K["dup"]
    yield "kat_dup", dataset_from_lines(Kd["train"], Kd["test"], Kd["labels"])
    yield "tiny", synth_fixture("tiny")[0]
    yield "small", synth_fixture("small")[0]
    yield "bulk", synth.generate_bulk(3000, 12, 8).dataset()


@pytest.mark.parametrize("frac_bits", [16, 32])
def test_colistening_sum_equals_fixed_point_oracle(frac_bits):
    for name, ds in _datasets():
        exp = native.fp_model(ds, "ibm", frac_bits=frac_bits, k=1)[0]
        got = cooc_scores(ds, frac_bits)
        assert np.array_equal(got, exp, equal_nan=True), name
