"""The Spark-free driver (musicrecommendation_amd/driver.py ≙ main.scala
MN:8-123 / distributed.scala DS:55-602): file naming, MyUtils helpers, and on
the GPU the whole flow — models, combinations, five threshold mAPs — with the
multi-GPU group cross-check, against the literal restatement's mAPs."""
import os

import numpy as np
import pytest

from musicrecommendation_amd import driver, evaluation

from helpers import GOLDEN, synth_fixture


def _write_resources(tmp_path, name="small"):
    z = np.load(os.path.join(GOLDEN, f"synth_{name}.npz"))
    n_tr = len({l.split("\t")[0] for l in z["train"].tolist()})
    n_te = len({l.split("\t")[0] for l in z["test"].tolist()})
    for key, fn in (("train", "train"), ("test", "test"), ("labels", "test_labels")):
        (tmp_path / f"{fn}_{n_tr}_{n_te}.txt").write_text("".join(l + "\n" for l in z[key].tolist()))
    return n_tr, n_te


def test_round_at_and_missing_files(tmp_path):
    assert driver.round_at(10, 0.28097677601234567) == 0.280976776
    assert driver.round_at(2, 0.125) == 0.13  # math.round: half up
    with pytest.raises(FileNotFoundError):
        driver.run(7, 3, str(tmp_path), verbose=False)


@pytest.mark.gpu
def test_driver_flow_and_group_check(tmp_path, capsys):
    n_tr, n_te = _write_resources(tmp_path)
    out = driver.run(n_tr, n_te, str(tmp_path), devices=[0], song_shards=2, user_blocks=2)
    assert out["multi_gpu_checked"] is True
    ds, z = synth_fixture("small")
    for name, key in (("user-based", "ubm"), ("item-based", "ibm")):
        assert abs(out["mAP"][name] - evaluation.threshold_map(z[key], ds)) < 1e-9
    text = capsys.readouterr().out
    assert "Elapsed time for item-based model:" in text and "stochastic-combination model mAP:" in text
    assert len(out["mAP"]) == 5


@pytest.mark.gpu
def test_driver_distributed_mode_uses_eleven_thresholds(tmp_path):
    """--distributed: the mAPs follow distributed.scala's evaluation (11
    thresholds, DS:395-415); a device list alone gives one song shard per GPU."""
    n_tr, n_te = _write_resources(tmp_path)
    out = driver.run(n_tr, n_te, str(tmp_path), devices=[0], verbose=False, distributed=True)
    assert out["thresholds"] == 11 and out["layout"] == (1, 1)
    ds, z = synth_fixture("small")
    for name, key in (("user-based", "ubm"), ("item-based", "ibm")):
        ref = evaluation.threshold_map(z[key], ds, evaluation.THRESHOLDS_DISTRIBUTED)
        assert abs(out["mAP"][name] - ref) < 1e-9


def test_driver_default_layout_follows_devices(monkeypatch):
    """--devices 0,1 without --song-shards is a 2-shard group, not a
    one-context 'multi-GPU' check (the layout rule, without running)."""
    seen = {}

    def fake_run(train_n, test_n, resources, devices, song_shards, user_blocks, **kw):
        seen.update(train_n=train_n, devices=devices, song_shards=song_shards, distributed=kw["distributed"])
        return {}

    monkeypatch.setattr(driver, "run", fake_run)
    driver.main(["--devices", "0,1", "--distributed"])
    assert seen == {"train_n": 300, "devices": [0, 1], "song_shards": None, "distributed": True}
    driver.main(["50", "5"])
    assert seen["train_n"] == 50 and seen["distributed"] is False
