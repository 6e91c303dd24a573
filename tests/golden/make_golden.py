"""Regenerate the committed golden fixtures (tests/golden/*.json, *.npz).

The reference ships no tests, fixtures or golden vectors and cannot be run in
this image (Scala 2.12 + Spark 3.3.2, no JVM), so parity is
pinned by:
  1. kat.json — the hand-derivable known-answer test of SURVEY.md §4.2. Its
     expected numbers were derived by hand from MR:26-62, 105-111, 140-166,
     230-257 and 521-639; this script re-derives them with the pure-Python
     literal restatement (oracle/reference_py.py) and refuses to write the
     file if they disagree.
  2. synth_<name>.npz — seeded synthetic datasets (musicrecommendation_amd.synth)
     scored by that same literal restatement: inputs (triplet lines) and
     expected dense ubm/ibm models, threshold mAP and mAP@10.

Usage: python tests/golden/make_golden.py   (from the repository root)
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.reference_py import LiteralRecommender, map_at_k  # noqa: E402
from oracle.native import dataset_lines  # noqa: E402
from musicrecommendation_amd import synth  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))

KAT = {
    "train": ["A\ts1\t1", "A\ts2\t1", "A\ts3\t1", "B\ts2\t1", "B\ts3\t1", "C\ts3\t1", "C\ts4\t1"],
    "test": ["X\ts1\t1", "X\ts4\t1", "Y\ts2\t1"],
    "labels": ["X\ts3\t1", "X\ts5\t1", "Y\ts3\t1", "Y\ts1\t1"],
    # SURVEY.md §4.2, derived by hand (c = {s1:2, s2:3, s3:3, s4:2}, test listens counted)
    "expected": {
        "ibm": {"Y|s1": 0.40824829046386296, "X|s2": 0.40824829046386296, "X|s3": 0.8164965809277259,
                "Y|s3": 0.6666666666666667, "Y|s4": 0.0},
        "ubm": {"Y|s1": 0.5773502691896258, "X|s2": 0.40824829046386296, "X|s3": 0.9082482904638629,
                "Y|s3": 1.2844570503761732, "Y|s4": 0.0},
        "map_ibm": 0.6666666666666666,
        "map_ubm": 0.6666666666666666,
    },
}

# Same KAT with duplicate lines: reference lengths count duplicates (MR:44-46,
# MR:60-62), numerators count distinct users/songs (MR:142-145, MR:232-235).
KAT_DUP = {
    "train": KAT["train"] + ["A\ts1\t5", "C\ts4\t2"],
    "test": KAT["test"] + ["X\ts1\t3"],
    "labels": KAT["labels"],
}


def model_dict(model):
    return {f"{u}|{s}": x for u, (s, x) in model}


def make_kat():
    rec = LiteralRecommender(KAT["train"], KAT["test"], KAT["labels"])
    got = {"ibm": model_dict(rec.get_item_based_model()), "ubm": model_dict(rec.get_user_based_model())}
    for m in ("ibm", "ubm"):
        exp = KAT["expected"][m]
        if set(got[m]) != set(exp):
            raise SystemExit(f"KAT {m}: pairs {sorted(got[m])} != {sorted(exp)}")
        for k, v in exp.items():
            if got[m][k] != v:
                raise SystemExit(f"KAT {m} {k}: literal {got[m][k]!r} != hand-derived {v!r}")
    for m, fn in (("ibm", rec.get_item_based_model), ("ubm", rec.get_user_based_model)):
        mp = rec.evaluate_model(fn())
        if mp != KAT["expected"][f"map_{m}"]:
            raise SystemExit(f"KAT map {m}: {mp!r}")
    dup = LiteralRecommender(KAT_DUP["train"], KAT_DUP["test"], KAT_DUP["labels"])
    kat = dict(KAT)
    kat["dup"] = dict(KAT_DUP)
    kat["dup"]["expected"] = {"ibm": model_dict(dup.get_item_based_model()),
                              "ubm": model_dict(dup.get_user_based_model())}
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1, sort_keys=True)
    print("kat.json: hand-derived values reproduced")


def dense_from(model, songs, users):
    si = {s: i for i, s in enumerate(songs)}
    ui = {u: i for i, u in enumerate(users)}
    out = np.full((len(users), len(songs)), np.nan)
    for u, (s, x) in model:
        out[ui[u], si[s]] = x
    return out


def make_synth(name: str):
    t = synth.config(name)
    ds = t.dataset()
    tr, te, lab = dataset_lines(ds)
    rec = LiteralRecommender(tr, te, lab)
    songs = sorted(rec.songs)
    users = sorted(rec.test_users)
    ubm = rec.get_user_based_model()
    ibm = rec.get_item_based_model()
    np.savez_compressed(
        os.path.join(HERE, f"synth_{name}.npz"),
        train=np.array(tr), test=np.array(te), labels=np.array(lab),
        songs=np.array(songs), test_users=np.array(users),
        ubm=dense_from(ubm, songs, users), ibm=dense_from(ibm, songs, users),
        map_ubm=rec.evaluate_model(ubm), map_ibm=rec.evaluate_model(ibm),
        map10_ubm=map_at_k(ubm, rec.test_labels, rec.test_users, 10),
        map10_ibm=map_at_k(ibm, rec.test_labels, rec.test_users, 10),
        alpha=t.alpha,
    )
    print(f"synth_{name}.npz: {ds.n_train}/{ds.n_test}/{ds.n_songs}, {len(ibm)} pairs")


if __name__ == "__main__":
    make_kat()
    for name in sys.argv[1:] or ["tiny", "small"]:
        make_synth(name)
